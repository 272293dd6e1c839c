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
