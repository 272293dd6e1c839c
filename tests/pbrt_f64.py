"""A second, independent restatement of the single-interface BSDFs in float64 numpy.

TEST INFRASTRUCTURE ONLY.  Written from the reference's PBRT headers (paths relative to
OptixPathtracer/source/Renderer/OptiX/), not from oracle/pt_oracle.c, so a misreading of a
formula in the C oracle shows up as a disagreement with the oracle's golden tuples
(tests/test_oracle_pins.py).  Everything is evaluated in float64; the C oracle rounds every
step to float32, so the two agree to a few float32 ulps where the formulas are well
conditioned.

    PBRT/SphericalGeometry.h:8-35   trig of shading-space directions
    PBRT/Microfacet.h:9-84          Trowbridge-Reitz D, Lambda, G, G1, visible-normal D(w, wm)
    Surface.h:22-29                 alpha = roughness^2, "effectively smooth" if alpha < 1e-3
    PBRT/Complex.h, Conductor.h:42-120   complex Fresnel (eta = 1, k from the albedo), f
    PBRT/Dielectric.h:20-343        dielectric Fresnel (eta = 1.5), f and PDF (Radiance mode)
    PBRT/LambertDiffuse.h:100-140   f, PDF
All functions take wo, wi as (n, 3) arrays in shading space (N = +z).
"""
from __future__ import annotations

import numpy as np

PI = 3.14159265359  # the reference's literal (Microfacet.h:10)
INV_PI = 0.31830988618379067154  # LambertDiffuse.h:105


def alpha_of(roughness: float) -> float:
    return roughness * roughness  # Surface.h:26-29


def smooth(alpha: float) -> bool:
    return alpha < 1e-3  # Surface.h:22-24


def cos2(w):
    return w[..., 2] ** 2


def sin2(w):
    return np.maximum(0.0, 1.0 - cos2(w))


def tan2(w):
    with np.errstate(divide="ignore", invalid="ignore"):
        return sin2(w) / cos2(w)


def cos_phi(w):
    s = np.sqrt(sin2(w))
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(s == 0.0, 1.0, np.clip(w[..., 0] / np.where(s == 0, 1, s), -1.0, 1.0))


def sin_phi(w):
    s = np.sqrt(sin2(w))
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(s == 0.0, 0.0, np.clip(w[..., 1] / np.where(s == 0, 1, s), -1.0, 1.0))


def D(wm, alpha):
    """Trowbridge-Reitz, Microfacet.h:9-20."""
    t2 = tan2(wm)
    c4 = cos2(wm) ** 2
    e = t2 * ((cos_phi(wm) / alpha) ** 2 + (sin_phi(wm) / alpha) ** 2)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = 1.0 / (PI * alpha * alpha * c4 * (1.0 + e) ** 2)
    return np.where(np.isinf(t2) | (c4 < 1e-16), 0.0, d)


def Lambda(w, alpha):
    """Microfacet.h:37-44."""
    t2 = tan2(w)
    a2 = (cos_phi(w) * alpha) ** 2 + (sin_phi(w) * alpha) ** 2
    with np.errstate(invalid="ignore"):
        lam = (np.sqrt(1.0 + a2 * t2) - 1.0) / 2.0
    return np.where(np.isinf(t2), 0.0, lam)


def G(wo, wi, alpha):
    return 1.0 / (1.0 + Lambda(wo, alpha) + Lambda(wi, alpha))


def G1(w, alpha):
    return 1.0 / (1.0 + Lambda(w, alpha))


def dot(a, b):
    return np.sum(a * b, axis=-1)


def D_vis(w, wm, alpha):
    """Visible-normal distribution D_w(wm) = G1(w) / |cos w| * D(wm) * |w . wm|, Microfacet.h:81-84."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return G1(w, alpha) / np.abs(w[..., 2]) * D(wm, alpha) * np.abs(dot(w, wm))


def normalize(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def same_hemisphere(a, b):
    return a[..., 2] * b[..., 2] > 0.0


# ---- Conductor (Conductor.h) --------------------------------------------------------------
def fresnel_complex(cos_i, albedo):
    """FresnelComplex / FrComplex, Conductor.h:42-91: eta = 1, k = 2 sqrt(r) / sqrt(1 - r),
    r = clamp(albedo, 0, 0.9999), per channel; returns (n, 3)."""
    r = np.clip(np.asarray(albedo, np.float64), 0.0, 0.9999)
    k = 2.0 * np.sqrt(r) / np.sqrt(np.maximum(1.0 - r, 0.0))
    eta = 1.0 + 1j * k  # (3,)
    c = np.clip(np.asarray(cos_i, np.float64), 0.0, 1.0)[..., None]
    s2i = 1.0 - c * c
    s2t = s2i / (eta * eta)
    ct = np.sqrt(1.0 - s2t)  # principal branch, as Complex::sqrt
    r_parl = (eta * c - ct) / (eta * c + ct)
    r_perp = (c - eta * ct) / (c + eta * ct)
    return (np.abs(r_parl) ** 2 + np.abs(r_perp) ** 2) / 2.0


def conductor_f(albedo, roughness, wo, wi):
    """Conductor::f, Conductor.h:97-120."""
    a = alpha_of(roughness)
    out = np.zeros(wo.shape[:-1] + (3,))
    if smooth(a):
        return out
    co, ci = np.abs(wo[..., 2]), np.abs(wi[..., 2])
    wm = wo + wi
    ok = same_hemisphere(wo, wi) & (co != 0) & (ci != 0) & (dot(wm, wm) != 0)
    wm = normalize(np.where(ok[..., None], wm, 1.0))
    F = fresnel_complex(np.abs(dot(wo, wm)), albedo)
    with np.errstate(divide="ignore", invalid="ignore"):
        val = (D(wm, a) * G(wo, wi, a) / (4.0 * ci * co))[..., None] * F
    return np.where(ok[..., None], val, 0.0)


def conductor_pdf(roughness, wo, wi):
    """The density of Conductor::Sample_f's direction, D_w(wo, wm) / (4 |wo . wm|) with wm the
    half vector (Conductor.h:156-163; PBRT-v4 ConductorBxDF::PDF)."""
    a = alpha_of(roughness)
    if smooth(a):
        return np.zeros(wo.shape[:-1])
    wm = wo + wi
    ok = same_hemisphere(wo, wi) & (dot(wm, wm) != 0)
    wm = normalize(np.where(ok[..., None], wm, 1.0))
    wm = np.where((wm[..., 2] < 0)[..., None], -wm, wm)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(ok, D_vis(wo, wm, a) / (4.0 * np.abs(dot(wo, wm))), 0.0)


# ---- Dielectric (Dielectric.h), eta = 1.5, Radiance transport -----------------------------
ETA = 1.5


def fresnel_dielectric(cos_i, eta=ETA):
    """Dielectric.h:20-43."""
    c = np.clip(np.asarray(cos_i, np.float64), -1.0, 1.0)
    e = np.where(c < 0, 1.0 / eta, eta)
    c = np.abs(c)
    s2t = (1.0 - c * c) / (e * e)
    with np.errstate(invalid="ignore"):
        ct = np.sqrt(np.maximum(1.0 - s2t, 0.0))
        r_parl = (e * c - ct) / (e * c + ct)
        r_perp = (c - e * ct) / (c + e * ct)
    return np.where(s2t >= 1.0, 1.0, (r_parl ** 2 + r_perp ** 2) / 2.0)


def _dielectric_half(wo, wi):
    co, ci = wo[..., 2], wi[..., 2]
    reflect = ci * co > 0
    etap = np.where(reflect, 1.0, np.where(co > 0, ETA, 1.0 / ETA))
    wm = wi * etap[..., None] + wo
    ok = (ci != 0) & (co != 0) & (dot(wm, wm) != 0)
    wm = normalize(np.where(ok[..., None], wm, 1.0))
    wm = np.where((wm[..., 2] < 0)[..., None], -wm, wm)  # glm::faceforward(-n, z, n): n toward +z
    ok &= ~((dot(wm, wi) * ci < 0) | (dot(wm, wo) * co < 0))  # back-facing microfacets
    return reflect, etap, wm, ok


def dielectric_f(roughness, wo, wi):
    """Dielectric::f, Dielectric.h:98-141 (Radiance mode: transmission divided by etap^2)."""
    a = alpha_of(roughness)
    if smooth(a):
        return np.zeros(wo.shape[:-1])
    reflect, etap, wm, ok = _dielectric_half(wo, wi)
    co, ci = wo[..., 2], wi[..., 2]
    F = fresnel_dielectric(dot(wo, wm))
    with np.errstate(divide="ignore", invalid="ignore"):
        fr = D(wm, a) * G(wo, wi, a) * F / np.abs(4.0 * ci * co)
        denom = (dot(wi, wm) + dot(wo, wm) / etap) ** 2 * ci * co
        ft = D(wm, a) * (1.0 - F) * G(wo, wi, a) * np.abs(dot(wi, wm) * dot(wo, wm) / denom) / etap ** 2
    return np.where(ok, np.where(reflect, fr, ft), 0.0)


def dielectric_pdf(roughness, wo, wi):
    """Dielectric::PDF, Dielectric.h:279-340 (both lobes allowed)."""
    a = alpha_of(roughness)
    if smooth(a):
        return np.zeros(wo.shape[:-1])
    reflect, etap, wm, ok = _dielectric_half(wo, wi)
    R = fresnel_dielectric(dot(wo, wm))
    T = 1.0 - R
    with np.errstate(divide="ignore", invalid="ignore"):
        pr = D_vis(wo, wm, a) / (4.0 * np.abs(dot(wo, wm))) * R / (R + T)
        denom = (dot(wi, wm) + dot(wo, wm) / etap) ** 2
        pt = D_vis(wo, wm, a) * np.abs(dot(wi, wm)) / denom * T / (R + T)
    return np.where(ok, np.where(reflect, pr, pt), 0.0)


# ---- Lambert (LambertDiffuse.h) ------------------------------------------------------------
def lambert_f(albedo, wo, wi):
    return np.where(same_hemisphere(wo, wi)[..., None], np.asarray(albedo, np.float64) * INV_PI, 0.0)


def lambert_pdf(wo, wi):
    return np.where(same_hemisphere(wi, wo), np.abs(wi[..., 2]) * INV_PI, 0.0)


# =============================================================================================
# Layered BSDF (GlossyDiffuse.h:141-524), stochastic, in float64 -- written from the header.
#
# Scalar Python floats (IEEE float64).  The random numbers are the reference's: TEA-16 / LCG
# (random.h:34-69) on u32 seeds, rnd = (lcg & 0xFFFFFF) / 2^24, which float64 holds exactly.
# Quantities the reference declares as float constants (pi, 0.01f thickness, invPi, ...) take
# their float32 values, and the private Russian-roulette streams are seeded from
# u32(float(w.x * 1000)) exactly as the float expression evaluates (a float32 product, then
# PTX cvt.rzi.u32.f32: truncation, saturating, NaN -> 0); everything else is float64.  Every
# `uc < threshold`, Russian-roulette or total-internal-reflection decision therefore sees the
# same random number as the oracle and a threshold within float32 rounding of the oracle's, so
# the two agree except where a threshold falls within a few ulp of the draw.
#
# `fault` seeds a misreading on purpose (tests/test_layered_f64.py shows the comparison catches
# it): "swap_exit" exchanges the exit / non-exit interface choice of f (:183-203),
# "no_flipmode" samples wis in Radiance instead of FlipMode(mode) = Importance (:238),
# "rr_main_seed" draws the Russian roulette from the path seed instead of the private stream
# (:215-222), "wo_seed_only" seeds f's private stream from wo alone (:215-218).
# =============================================================================================
import math

_F32 = np.float32
_PI_F = float(_F32(3.14159265359))  # `const float pi` (random.h:77, Microfacet.h:10)
_INV_PI_F = float(_F32(0.31830988618379067154))  # LambertDiffuse.h:90,111
_PI_OVER4_F = float(_F32(0.78539816339744830961))  # LambertDiffuse.h:36
_PI_OVER2_F = float(_F32(1.57079632679489661923))  # LambertDiffuse.h:37
_THICK_F = float(_F32(0.01))  # GlossyDiffuse.h:145,375
_FLT_MIN = float(np.finfo(np.float32).tiny)  # ::cuda::std::numeric_limits<float>::min()
_ETA_F = 1.5
_M32 = 0xFFFFFFFF
RADIANCE, IMPORTANCE = 0, 1


def tea16(v0: int, v1: int) -> int:
    """RandomOptix::tea<16> (random.h:34-48) on u32."""
    v0 &= _M32
    v1 &= _M32
    s0 = 0
    for _ in range(16):
        s0 = (s0 + 0x9E3779B9) & _M32
        v0 = (v0 + ((((v1 << 4) & _M32) + 0xA341316C) ^ (v1 + s0) ^ ((v1 >> 5) + 0xC8013EA4))) & _M32
        v1 = (v1 + ((((v0 << 4) & _M32) + 0xAD90777D) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7E95761E))) & _M32
    return v0


class Seed:
    """An `unsigned int&` seed advanced by RandomOptix::rnd (random.h:51-69)."""

    def __init__(self, s: int):
        self.s = s & _M32

    def rnd(self) -> float:
        self.s = (1664525 * self.s + 1013904223) & _M32
        return (self.s & 0xFFFFFF) / 16777216.0


def u32_of_times_1000(x: float) -> int:
    """unsigned(w.x * 1000) with w.x a float: float32 product, then PTX cvt.rzi.u32.f32."""
    p = float(_F32(x) * _F32(1000.0))
    if not (p > 0.0):
        return 0
    if p >= 4294967296.0:
        return _M32
    return int(p)


def _div(a: float, b: float) -> float:
    """IEEE division (no Python exception on zero)."""
    if b != 0.0:
        return a / b
    if a == 0.0 or a != a:
        return math.nan
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _neg(a):
    return (-a[0], -a[1], -a[2])


def _scale(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def _add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def _mulv(a, b):
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def _norm(a):
    return _scale(a, 1.0 / math.sqrt(_dot(a, a)))


def _cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _is_zero(c) -> bool:
    return c[0] == 0.0 and c[1] == 0.0 and c[2] == 0.0


def _sin2(w):
    return max(0.0, 1.0 - w[2] * w[2])  # SphericalGeometry.h:12


def _tan2(w):
    return _div(_sin2(w), w[2] * w[2])  # :16


def _cos_phi(w):
    s = math.sqrt(_sin2(w))
    return 1.0 if s == 0.0 else min(max(w[0] / s, -1.0), 1.0)  # :18-21


def _sin_phi(w):
    s = math.sqrt(_sin2(w))
    return 0.0 if s == 0.0 else min(max(w[1] / s, -1.0), 1.0)  # :22-25


def _same_hemi(a, b):
    return a[2] * b[2] > 0.0  # :27-29


def _D(wm, a):
    """D_Anisotropic with alpha (a, a), Microfacet.h:9-20."""
    t2 = _tan2(wm)
    if math.isinf(t2):
        return 0.0
    c4 = (wm[2] * wm[2]) ** 2
    if c4 < 1e-16:
        return 0.0
    e = t2 * ((_cos_phi(wm) / a) ** 2 + (_sin_phi(wm) / a) ** 2)
    return 1.0 / (_PI_F * a * a * c4 * (1.0 + e) ** 2)


def _Lambda(w, a):
    """Lambda_Anisotropic, Microfacet.h:46-52."""
    t2 = _tan2(w)
    if math.isinf(t2):
        return 0.0
    a2 = (_cos_phi(w) * a) ** 2 + (_sin_phi(w) * a) ** 2
    return (math.sqrt(1.0 + a2 * t2) - 1.0) / 2.0


def _G(wo, wi, a):
    return 1.0 / (1.0 + _Lambda(wo, a) + _Lambda(wi, a))  # :62-69


def _Dvis(w, wm, a):
    """D(w, wm) = G1(w) / |cos w| * D(wm) * |w . wm|, Microfacet.h:81-88 (= PDF_Isotropic)."""
    return _div(1.0 / (1.0 + _Lambda(w, a)), abs(w[2])) * _D(wm, a) * abs(_dot(w, wm))


def _sample_wm(seed: Seed, w, a):
    """Microfacet::Sample_wm, Microfacet.h:90-119 (polar disk sample: 2 draws, random.h:76-84)."""
    wh = _norm((a * w[0], a * w[1], w[2]))
    if wh[2] < 0:
        wh = _neg(wh)
    t1 = _norm(_cross((0.0, 0.0, 1.0), wh)) if wh[2] < 0.99999 else (1.0, 0.0, 0.0)
    t2 = _cross(wh, t1)
    u0 = seed.rnd()
    u1 = seed.rnd()
    r = math.sqrt(u0)
    th = 2.0 * _PI_F * u1
    px, py = r * math.cos(th), r * math.sin(th)
    h = math.sqrt(1.0 - px * px)
    x = (1.0 + wh[2]) / 2.0
    py = (1.0 - x) * h + x * py
    pz = math.sqrt(max(0.0, 1.0 - (px * px + py * py)))
    nh = _add(_add(_scale(t1, px), _scale(t2, py)), _scale(wh, pz))
    return _norm((a * nh[0], a * nh[1], max(1e-6, nh[2])))


def _fresnel(c, eta=_ETA_F):
    """Dielectric::FresnelDielectric, Dielectric.h:20-42."""
    c = min(max(c, -1.0), 1.0)
    if c < 0.0:
        eta = 1.0 / eta
        c = -c
    s2t = (1.0 - c * c) / (eta * eta)
    if s2t >= 1.0:
        return 1.0
    ct = math.sqrt(1.0 - s2t)
    rpa = (eta * c - ct) / (eta * c + ct)
    rpe = (c - eta * ct) / (c + eta * ct)
    return (rpa * rpa + rpe * rpe) / 2.0


def _refract(wi, n, eta):
    """Dielectric::Refract, Dielectric.h:68-92 -> (wt, etap) or None (total internal reflection)."""
    ci = _dot(n, wi)
    if ci < 0.0:
        eta = 1.0 / eta
        ci = -ci
        n = _neg(n)
    s2t = max(0.0, 1.0 - ci * ci) / (eta * eta)
    if s2t >= 1.0:
        return None
    ct = math.sqrt(1.0 - s2t)
    return _add(_scale(wi, -1.0 / eta), _scale(n, ci / eta - ct)), eta


class BS:
    """BSDFSample (BSDFSample.h): color (3), direction, pdf, reflection/transmission/specular."""

    __slots__ = ("color", "dir", "pdf", "refl", "trans", "spec")

    def __init__(self, color, d, pdf, refl, trans, spec):
        self.color, self.dir, self.pdf, self.refl, self.trans, self.spec = color, d, pdf, refl, trans, spec

    def bad(self):  # the `!ok || color == 0 || pdf == 0 || dir.z == 0` tests of GlossyDiffuse.h
        return _is_zero(self.color) or self.pdf == 0.0 or self.dir[2] == 0.0


def _dielectric_sample(seed: Seed, a, wo, mode, reflection, transmission):
    """Dielectric::Sample_f, Dielectric.h:146-288: uc first, then (rough) the microfacet normal."""
    uc = seed.rnd()
    if a < 1e-3:
        R = _fresnel(wo[2])
        T = 1.0 - R
        pr = R if reflection else 0.0
        pt = T if transmission else 0.0
        if pr == 0.0 and pt == 0.0:
            return None
        if uc < pr / (pr + pt):
            wi = (-wo[0], -wo[1], wo[2])
            c = _div(R, abs(wi[2]))
            return BS((c, c, c), wi, pr / (pr + pt), True, False, True)
        rr = _refract(wo, (0.0, 0.0, 1.0), _ETA_F)
        if rr is None:
            return None
        wi, etap = rr
        ft = _div(T, abs(wi[2]))
        if mode == RADIANCE:
            ft /= etap * etap
        return BS((ft, ft, ft), wi, pt / (pr + pt), False, True, True)
    wm = _sample_wm(seed, wo, a)
    R = _fresnel(_dot(wo, wm))
    T = 1.0 - R
    pr = R if reflection else 0.0
    pt = T if transmission else 0.0
    if pr == 0.0 and pt == 0.0:
        return None
    if uc < pr / (pr + pt):
        wi = _add(_neg(wo), _scale(wm, 2.0 * _dot(wm, wo)))  # glm::reflect(-wo, wm)
        if not _same_hemi(wo, wi):
            return None
        pdf = _div(_Dvis(wo, wm, a), 4.0 * abs(_dot(wo, wm))) * pr / (pr + pt)
        c = _div(_D(wm, a) * _G(wo, wi, a) * R, 4.0 * wi[2] * wo[2])
        return BS((c, c, c), wi, pdf, True, False, False)
    rr = _refract(wo, wm, _ETA_F)
    if rr is None:
        return None
    wi, etap = rr
    if _same_hemi(wo, wi) or wi[2] == 0.0:
        return None
    denom = (_dot(wi, wm) + _dot(wo, wm) / etap) ** 2
    pdf = _Dvis(wo, wm, a) * _div(abs(_dot(wi, wm)), denom) * pt / (pr + pt)
    ft = T * _D(wm, a) * _G(wo, wi, a) * abs(_div(_dot(wi, wm) * _dot(wo, wm), wi[2] * wo[2] * denom))
    if mode == RADIANCE:
        ft /= etap * etap
    return BS((ft, ft, ft), wi, pdf, False, True, False)


def _dielectric_half_s(wo, wi):
    co, ci = wo[2], wi[2]
    reflect = ci * co > 0
    etap = 1.0 if reflect else (_ETA_F if co > 0.0 else 1.0 / _ETA_F)
    wm = _add(_scale(wi, etap), wo)
    if ci == 0.0 or co == 0.0 or _dot(wm, wm) == 0.0:
        return None
    wm = _norm(wm)
    if wm[2] < 0.0:  # glm::faceforward(-n, (0,0,1), n)
        wm = _neg(wm)
    if _dot(wm, wi) * ci < 0.0 or _dot(wm, wo) * co < 0.0:
        return None
    return reflect, etap, wm


def _dielectric_f_s(a, wo, wi, mode):
    """Dielectric::f, Dielectric.h:96-139 (scalar)."""
    if a < 1e-3:
        return 0.0
    h = _dielectric_half_s(wo, wi)
    if h is None:
        return 0.0
    reflect, etap, wm = h
    F = _fresnel(_dot(wo, wm))
    if reflect:
        return _div(_D(wm, a) * _G(wo, wi, a) * F, abs(4.0 * wi[2] * wo[2]))
    denom = (_dot(wi, wm) + _dot(wo, wm) / etap) ** 2 * wi[2] * wo[2]
    ft = _D(wm, a) * (1.0 - F) * _G(wo, wi, a) * abs(_div(_dot(wi, wm) * _dot(wo, wm), denom))
    if mode == RADIANCE:
        ft /= etap * etap
    return ft


def _dielectric_pdf_s(a, wo, wi, reflection, transmission):
    """Dielectric::PDF, Dielectric.h:290-343 (scalar, with the sample flags)."""
    if a < 1e-3:
        return 0.0
    h = _dielectric_half_s(wo, wi)
    if h is None:
        return 0.0
    reflect, etap, wm = h
    R = _fresnel(_dot(wo, wm))
    T = 1.0 - R
    pr = R if reflection else 0.0
    pt = T if transmission else 0.0
    if pr == 0.0 and pt == 0.0:
        return 0.0
    if reflect:
        return _div(_Dvis(wo, wm, a), 4.0 * abs(_dot(wo, wm))) * pr / (pr + pt)
    denom = (_dot(wi, wm) + _dot(wo, wm) / etap) ** 2
    return _Dvis(wo, wm, a) * _div(abs(_dot(wi, wm)), denom) * pt / (pr + pt)


def _lambert_sample(seed: Seed, albedo, reflection):
    """LambertDiffuse::Sample_f, LambertDiffuse.h:110-132 (concentric disk, :35-61)."""
    if not reflection:
        return None
    ox = 2.0 * seed.rnd() - 1.0
    oy = 2.0 * seed.rnd() - 1.0
    if ox == 0.0 and oy == 0.0:
        dx = dy = 0.0
    else:
        if abs(ox) > abs(oy):
            r, th = ox, _PI_OVER4_F * (oy / ox)
        else:
            r, th = oy, _PI_OVER2_F - _PI_OVER4_F * (ox / oy)
        dx, dy = r * math.cos(th), r * math.sin(th)
    z = math.sqrt(max(0.0, 1.0 - dx * dx - dy * dy))
    d = _norm((dx, dy, abs(z)))
    return BS(_scale(albedo, _INV_PI_F), d, abs(d[2]) * _INV_PI_F, True, False, False)


def _layer_f(top, a, albedo, wo, wi, mode):  # GlossyDiffuse.h:110-117
    if top:
        c = _dielectric_f_s(a, wo, wi, mode)
        return (c, c, c)
    return _scale(albedo, _INV_PI_F) if _same_hemi(wo, wi) else (0.0, 0.0, 0.0)


def _layer_sample(top, seed, a, albedo, wo, mode, reflection, transmission):  # :119-126
    if top:
        return _dielectric_sample(seed, a, wo, mode, reflection, transmission)
    return _lambert_sample(seed, albedo, reflection)


def _layer_pdf(top, a, wo, wi, reflection, transmission):  # :128-135
    if top:
        return _dielectric_pdf_s(a, wo, wi, reflection, transmission)
    return abs(wi[2]) * _INV_PI_F if (reflection and _same_hemi(wi, wo)) else 0.0


def _transmittance(dz, w):  # :97-105
    if abs(dz) <= _FLT_MIN:
        return 1.0
    return math.exp(-abs(_div(dz, w[2])))


def _power(f, g):  # PowerHeuristic(1, f, 1, g), :91-95
    return _div(f * f, f * f + g * g)


def layered_f(seed: int, albedo, roughness: float, wo, wi, fault=None):
    """GlossyDiffuse::f (GlossyDiffuse.h:141-367) -> (f[3], seed')."""
    rs = Seed(seed)
    a = float(roughness) ** 2
    albedo = tuple(float(x) for x in albedo)
    wo = tuple(float(x) for x in wo)
    wi = tuple(float(x) for x in wi)
    n_samples, max_depth = 5, 10
    top_spec, bottom_spec = a < 1e-3, False
    if wo[2] < 0:  # twoSided
        wo, wi = _neg(wo), _neg(wi)
    entered_top = True
    through = _same_hemi(wo, wi) ^ entered_top  # exit through the bottom
    if fault == "swap_exit":
        through = not through
    if through:
        exit_top, nonexit_top, exit_spec, nonexit_spec = False, True, bottom_spec, top_spec
    else:
        exit_top, nonexit_top, exit_spec, nonexit_spec = True, False, top_spec, bottom_spec
    exit_z = 0.0 if (_same_hemi(wo, wi) ^ entered_top) else _THICK_F
    f = (0.0, 0.0, 0.0)
    if _same_hemi(wo, wi):
        f = _scale(_layer_f(entered_top, a, albedo, wo, wi, RADIANCE), float(n_samples))
    if fault == "wo_seed_only":
        ns = tea16(u32_of_times_1000(wo[0]), u32_of_times_1000(wo[1]))
    else:
        ns = tea16(u32_of_times_1000(wo[0]), u32_of_times_1000(wo[1]))
        ns = tea16(ns, u32_of_times_1000(wi[0]))
        ns = tea16(ns, u32_of_times_1000(wi[1]))
    ns = tea16(ns, rs.s)
    rr = rs if fault == "rr_main_seed" else Seed(ns)
    wis_mode = RADIANCE if fault == "no_flipmode" else IMPORTANCE
    for _ in range(n_samples):
        wos = _layer_sample(entered_top, rs, a, albedo, wo, RADIANCE, False, True)
        if wos is None or wos.bad():
            continue
        wis = _layer_sample(exit_top, rs, a, albedo, wi, wis_mode, False, True)
        if wis is None or wis.bad():
            continue
        beta = _scale(wos.color, abs(wos.dir[2]) / wos.pdf)
        z = _THICK_F if entered_top else 0.0
        w = wos.dir
        for depth in range(max_depth):
            if depth > 3 and max(beta) < 0.25:
                q = max(0.0, 1.0 - max(beta))
                if rr.rnd() < q:
                    break
                beta = _scale(beta, 1.0 / (1.0 - q))
            z = 0.0 if z == _THICK_F else _THICK_F
            beta = _scale(beta, _transmittance(_THICK_F, w))
            if z == exit_z:
                bs = _layer_sample(exit_top, rs, a, albedo, _neg(w), RADIANCE, True, False)
                if bs is None or bs.bad():
                    break
                beta = _mulv(beta, _scale(bs.color, abs(bs.dir[2]) / bs.pdf))
                w = bs.dir
            else:
                if not nonexit_spec:
                    wt = 1.0
                    if not exit_spec:
                        wt = _power(wis.pdf, _layer_pdf(nonexit_top, a, _neg(w), _neg(wis.dir), True, True))
                    fn = _layer_f(nonexit_top, a, albedo, _neg(w), _neg(wis.dir), RADIANCE)
                    k = abs(wis.dir[2]) * wt * _transmittance(_THICK_F, wis.dir)
                    f = _add(f, _scale(_mulv(_mulv(beta, fn), wis.color), k / wis.pdf))
                bs = _layer_sample(nonexit_top, rs, a, albedo, _neg(w), RADIANCE, True, False)
                if bs is None or bs.bad():
                    break
                beta = _mulv(beta, _scale(bs.color, abs(bs.dir[2]) / bs.pdf))
                w = bs.dir
                if not exit_spec:
                    fe = _layer_f(exit_top, a, albedo, _neg(w), wi, RADIANCE)
                    if not _is_zero(fe):
                        wt = 1.0
                        if not nonexit_spec:
                            wt = _power(bs.pdf, _layer_pdf(exit_top, a, _neg(w), wi, False, True))
                        f = _add(f, _scale(_mulv(beta, fe), _transmittance(_THICK_F, bs.dir) * wt))
    return _scale(f, 1.0 / n_samples), rs.s


def layered_sample(seed: int, albedo, roughness: float, wo, fault=None):
    """GlossyDiffuse::Sample_f (GlossyDiffuse.h:372-524) -> (ok, f[3], pdf, wi[3], flags, seed').
    flags: reflection 1 | transmission 2 | specular 4 | glossy 8 (the oracle's encoding).
    fault: "seed_before_entrance" seeds the private stream with the path seed as it was before
    the entrance sample (it is read after it, :417-418); "no_cos" drops the |cos| factor after
    an interface scattering (:521)."""
    rs = Seed(seed)
    seed0 = rs.s
    a = float(roughness) ** 2
    albedo = tuple(float(x) for x in albedo)
    wo = tuple(float(x) for x in wo)
    max_depth = 10
    flip = False
    if wo[2] < 0:
        wo = _neg(wo)
        flip = True
    entered_top = True
    bs = _layer_sample(entered_top, rs, a, albedo, wo, RADIANCE, True, True)
    if bs is None or bs.bad():
        return False, None, None, None, 0, rs.s
    if bs.refl:
        d = _neg(bs.dir) if flip else bs.dir
        flags = 1 | (2 if bs.trans else 0) | (4 if bs.spec else 8)
        return True, bs.color, bs.pdf, d, flags, rs.s
    w = bs.dir
    specular = bs.spec
    rr = Seed(tea16(tea16(u32_of_times_1000(wo[0]), u32_of_times_1000(wo[1])),
                    seed0 if fault == "seed_before_entrance" else rs.s))
    f = _scale(bs.color, abs(bs.dir[2]))
    pdf = bs.pdf
    z = _THICK_F if entered_top else 0.0
    for depth in range(max_depth):
        rr_beta = max(f) / pdf
        if depth > 3 and rr_beta < 0.25:
            q = max(0.0, 1.0 - rr_beta)
            if rr.rnd() < q:
                return False, None, None, None, 0, rs.s
            pdf *= 1.0 - q
        if w[2] == 0.0:
            return False, None, None, None, 0, rs.s
        z = 0.0 if z == _THICK_F else _THICK_F
        f = _scale(f, _transmittance(_THICK_F, w))
        top = z != 0.0
        bs = _layer_sample(top, rs, a, albedo, _neg(w), RADIANCE, True, True)
        if bs is None or bs.bad():
            return False, None, None, None, 0, rs.s
        f = _mulv(f, bs.color)
        pdf *= bs.pdf
        specular = specular and bs.spec
        w = bs.dir
        if bs.trans:
            if flip:
                w = _neg(w)
            refl = _same_hemi(wo, w)
            flags = (1 if refl else 2) | (4 if specular else 8)
            return True, f, pdf, w, flags, rs.s
        if fault != "no_cos":
            f = _scale(f, abs(bs.dir[2]))
    return False, None, None, None, 0, rs.s
