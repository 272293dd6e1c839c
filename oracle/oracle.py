"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (optixpathtracer_amd/) never does.  See pt_oracle.h for the parity
status ("parity unpinned" against the OptiX original, pinned by the reference's own unit
test known answers only).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"

_FP = C.POINTER(C.c_float)
_UP = C.POINTER(C.c_uint32)


class orc_mesh(C.Structure):
    _fields_ = [
        ("vertices", _FP),
        ("normals", _FP),
        ("indices", C.POINTER(C.c_int32)),
        ("n_vertices", C.c_int32),
        ("n_triangles", C.c_int32),
        ("model", C.c_float * 16),
        ("albedo", C.c_float * 3),
        ("metallic", C.c_float),
        ("roughness", C.c_float),
        ("texcoords", _FP),
        ("albedo_tex", C.c_int32),
        ("normal_tex", C.c_int32),
        ("metal_rough_tex", C.c_int32),
    ]


class orc_texture(C.Structure):
    _fields_ = [("rgba8", _UP), ("width", C.c_int32), ("height", C.c_int32)]


class orc_launch(C.Structure):
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("cam_pos", C.c_float * 3),
        ("inv_view", C.c_float * 16),
        ("inv_proj", C.c_float * 16),
        ("lights", _FP),
        ("n_lights", C.c_int32),
        ("max_bounces", C.c_int32),
        ("material_mode", C.c_int32),
    ]


BSDF = {"lambert": 0, "conductor": 1, "dielectric": 2, "layered": 3}

_lib = None


def math_eval(fn: str, x) -> np.ndarray:
    """The oracle's (and the kernels') sin / cos / exp / pow2.4 polynomials on float32 inputs."""
    lib = load()
    xs = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(xs)
    lib.orc_math_eval({"sin": 0, "cos": 1, "exp": 2, "pow2.4": 3}[fn], fp(xs), fp(out), xs.size)
    return out


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB.exists():
        build()
    lib = C.CDLL(str(LIB))
    lib.orc_tea16.restype = C.c_uint32
    lib.orc_tea16.argtypes = [C.c_uint32, C.c_uint32]
    lib.orc_rnd_seq.argtypes = [C.c_uint32, C.c_int32, _FP, _UP]
    lib.orc_math_eval.argtypes = [C.c_int32, _FP, _FP, C.c_int32]
    lib.orc_f2u_sat.restype = C.c_uint32
    lib.orc_f2u_sat.argtypes = [C.c_float]
    lib.orc_bsdf_sample.restype = C.c_int32
    lib.orc_bsdf_sample.argtypes = [C.c_int32, _UP, _FP, C.c_float, _FP, _FP]
    lib.orc_bsdf_eval.argtypes = [C.c_int32, _UP, _FP, C.c_float, _FP, _FP, _FP]
    lib.orc_bsdf_pdf.restype = C.c_float
    lib.orc_bsdf_pdf.argtypes = [C.c_int32, C.c_float, _FP, _FP]
    lib.orc_bsdf_sample_n.argtypes = [C.c_int32, _UP, _FP, C.c_float, _FP, C.c_int32, _FP, C.POINTER(C.c_int32)]
    lib.orc_bsdf_pdf_n.argtypes = [C.c_int32, C.c_float, _FP, _FP, C.c_int32, _FP]
    lib.orc_cos_theta.restype = C.c_float
    lib.orc_cos_theta.argtypes = [_FP]
    lib.orc_furnace.argtypes = [C.c_int32, _UP, _FP, C.c_float, _FP, C.c_int32, _FP]
    lib.orc_camera_from_blender.argtypes = [_FP, _FP, C.c_float, C.c_int32, C.c_int32, _FP, _FP, _FP]
    lib.orc_camera_ray.argtypes = [C.POINTER(orc_launch), C.c_int32, C.c_int32, _FP, _FP]
    lib.orc_scene_create.restype = C.c_void_p
    lib.orc_scene_create.argtypes = [C.POINTER(orc_mesh), C.c_int32, C.POINTER(orc_texture), C.c_int32]
    lib.orc_tex_sample.restype = None
    lib.orc_tex_sample.argtypes = [C.POINTER(orc_texture), C.c_float, C.c_float, C.c_int32, _FP]
    lib.orc_scene_destroy.argtypes = [C.c_void_p]
    lib.orc_scene_triangles.restype = C.c_int32
    lib.orc_scene_triangles.argtypes = [C.c_void_p]
    lib.orc_trace_closest.restype = C.c_int32
    lib.orc_trace_closest.argtypes = [C.c_void_p, _FP, _FP, C.c_float, C.c_float, _FP, _FP, _FP,
                                      C.POINTER(C.c_int32)]
    lib.orc_trace_any.restype = C.c_int32
    lib.orc_trace_any.argtypes = [C.c_void_p, _FP, _FP, C.c_float, C.c_float]
    lib.orc_render.argtypes = [C.c_void_p, C.POINTER(orc_launch), C.c_uint32, C.c_uint32, C.c_int32, C.c_int32,
                               C.c_int32, C.c_int32, _FP, C.c_int32, C.POINTER(C.c_uint64)]
    lib.orc_sample_path.argtypes = [C.c_void_p, C.POINTER(orc_launch), C.c_int32, C.c_int32, C.c_uint32, _FP,
                                    C.POINTER(C.c_int32)]
    lib.orc_sample_path_debug.restype = C.c_int32
    lib.orc_sample_path_debug.argtypes = [C.c_void_p, C.POINTER(orc_launch), C.c_int32, C.c_int32, C.c_uint32, _FP,
                                          C.c_int32, _FP]
    _lib = lib
    return lib


def _f(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def fp(a):
    return a.ctypes.data_as(_FP)


def tea16(a: int, b: int) -> int:
    return int(load().orc_tea16(a & 0xFFFFFFFF, b & 0xFFFFFFFF))


def rnd_seq(seed: int, n: int):
    out = np.empty(n, np.float32)
    s = C.c_uint32()
    load().orc_rnd_seq(seed & 0xFFFFFFFF, n, fp(out), C.byref(s))
    return out, int(s.value)


def bsdf_sample(model: str, seed: int, albedo, roughness: float, wo):
    s = C.c_uint32(seed & 0xFFFFFFFF)
    out = np.zeros(8, np.float32)
    ok = load().orc_bsdf_sample(BSDF[model], C.byref(s), fp(_f(albedo)), float(roughness), fp(_f(wo)), fp(out))
    return bool(ok), out, int(s.value)


def bsdf_eval(model: str, seed: int, albedo, roughness: float, wo, wi):
    s = C.c_uint32(seed & 0xFFFFFFFF)
    out = np.zeros(3, np.float32)
    load().orc_bsdf_eval(BSDF[model], C.byref(s), fp(_f(albedo)), float(roughness), fp(_f(wo)), fp(_f(wi)), fp(out))
    return out, int(s.value)


def bsdf_sample_n(model: str, seed: int, albedo, roughness: float, wo, n: int):
    """n samples of one wo with a running seed -> (ok[n] bool, out[n, 8], seed')."""
    s = C.c_uint32(seed & 0xFFFFFFFF)
    out = np.zeros((n, 8), np.float32)
    ok = np.zeros(n, np.int32)
    load().orc_bsdf_sample_n(BSDF[model], C.byref(s), fp(_f(albedo)), float(roughness), fp(_f(wo)), int(n), fp(out),
                             ok.ctypes.data_as(C.POINTER(C.c_int32)))
    return ok.astype(bool), out, int(s.value)


def bsdf_pdf(model: str, roughness: float, wo, wi) -> np.ndarray:
    """pdf of the model's Sample_f at directions wi (n, 3) for one wo."""
    wi = _f(wi).reshape(-1, 3)
    out = np.zeros(len(wi), np.float32)
    load().orc_bsdf_pdf_n(BSDF[model], float(roughness), fp(_f(wo)), fp(wi), len(wi), fp(out))
    return out


def cos_theta(w) -> float:
    return float(load().orc_cos_theta(fp(_f(w))))


def furnace(model: str, seed: int, albedo, roughness: float, wo, n: int):
    """mean of f*|cos|/pdf over n samples (UnitTests/SpherGeom_Test.cpp:28-252); returns (mean, seed')."""
    s = C.c_uint32(seed & 0xFFFFFFFF)
    out = np.zeros(3, np.float32)
    load().orc_furnace(BSDF[model], C.byref(s), fp(_f(albedo)), float(roughness), fp(_f(wo)), int(n), fp(out))
    return out, int(s.value)


def camera_from_blender(pos, rot, fov_deg, w, h):
    p, iv, ip = np.empty(3, np.float32), np.empty(16, np.float32), np.empty(16, np.float32)
    load().orc_camera_from_blender(fp(_f(pos)), fp(_f(rot)), float(fov_deg), int(w), int(h), fp(p), fp(iv), fp(ip))
    return p, iv, ip


def tex_sample(rgba8: np.ndarray, x: float, y: float, srgb: bool) -> np.ndarray:
    """tex2D of the reference's texture objects (+ SRGB8ToLinear when srgb)."""
    px = np.ascontiguousarray(rgba8, dtype=np.uint32)
    t = orc_texture(px.ctypes.data_as(_UP), px.shape[1], px.shape[0])
    out = np.zeros(4, np.float32)
    load().orc_tex_sample(C.byref(t), float(x), float(y), 1 if srgb else 0, fp(out))
    return out


class OracleScene:
    """The CPU restatement of the render path over one scene (product `Scene` objects)."""

    def __init__(self, scene):
        self.lib = load()
        self.scene = scene
        self._keep = []
        arr = (orc_mesh * max(1, len(scene.meshes)))()
        for i, m in enumerate(scene.meshes):
            v = _f(m.vertices)
            idx = np.ascontiguousarray(m.indices, dtype=np.int32)
            self._keep += [v, idx]
            arr[i].vertices = fp(v)
            arr[i].indices = idx.ctypes.data_as(C.POINTER(C.c_int32))
            if m.normals is not None:
                n = _f(m.normals)
                self._keep.append(n)
                arr[i].normals = fp(n)
            arr[i].n_vertices = len(v)
            arr[i].n_triangles = len(idx)
            arr[i].model[:] = [float(x) for x in _f(m.model).ravel()]
            arr[i].albedo[:] = [float(x) for x in m.albedo]
            arr[i].metallic = float(m.metallic)
            arr[i].roughness = float(m.roughness)
            if getattr(m, "texcoords", None) is not None:
                t = _f(m.texcoords)
                self._keep.append(t)
                arr[i].texcoords = fp(t)
            arr[i].albedo_tex = int(getattr(m, "albedo_tex", -1))
            arr[i].normal_tex = int(getattr(m, "normal_tex", -1))
            arr[i].metal_rough_tex = int(getattr(m, "metal_rough_tex", -1))
        texs = list(getattr(scene, "textures", []) or [])
        tarr = (orc_texture * max(1, len(texs)))()
        for i, t in enumerate(texs):
            px = np.ascontiguousarray(t, dtype=np.uint32)
            self._keep.append(px)
            tarr[i].rgba8 = px.ctypes.data_as(_UP)
            tarr[i].height, tarr[i].width = px.shape
        self.h = self.lib.orc_scene_create(arr, len(scene.meshes), tarr, len(texs))
        self._lights = None

    def launch(self, width, height, max_bounces, material_mode=None, lights=None, camera=None):
        lp = orc_launch()
        lp.width, lp.height = int(width), int(height)
        if camera is None:
            camera = camera_from_blender(self.scene.camera_blender_pos, self.scene.camera_blender_rot,
                                         self.scene.fov_deg, width, height)
        p, iv, ip = camera
        lp.cam_pos[:] = [float(x) for x in p]
        lp.inv_view[:] = [float(x) for x in iv]
        lp.inv_proj[:] = [float(x) for x in ip]
        L = _f(self.scene.lights if lights is None else lights).reshape(-1, 6)
        self._lights = L
        lp.lights = fp(L)
        lp.n_lights = len(L)
        lp.max_bounces = int(max_bounces)
        lp.material_mode = int(self.scene.material_mode if material_mode is None else material_mode)
        return lp

    def render(self, lp, first_frame, n_frames, rect=None, sum_rgb=None, threads=None):
        """Per-pixel radiance SUM over frame ids [first_frame, first_frame + n_frames)."""
        w, h = lp.width, lp.height
        if sum_rgb is None:
            sum_rgb = np.zeros((h, w, 3), np.float32)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, w, h)
        segs = C.c_uint64()
        # the host's CPU share: OMP_NUM_THREADS where the box sets it (16 per GPU), else all cores
        nt = threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or os.cpu_count() or 1
        self.lib.orc_render(self.h, C.byref(lp), int(first_frame), int(n_frames), x0, y0, x1, y1, fp(sum_rgb), nt,
                            C.byref(segs))
        return sum_rgb, int(segs.value)

    def sample_path(self, lp, x, y, frame):
        out = np.zeros(3, np.float32)
        segs = C.c_int32()
        self.lib.orc_sample_path(self.h, C.byref(lp), x, y, frame, fp(out), C.byref(segs))
        return out, int(segs.value)

    def sample_path_debug(self, lp, x, y, frame, max_bounces=64):
        """The debug pixel's per-bounce records (orc_sample_path_debug; ptamd.h pt_debug_bounce
        layout) as a (bounces, 22) float32 array (bounce and prim are int32 bits) and the path's
        radiance."""
        rec = np.zeros((max_bounces, 22), np.float32)
        rgb = np.zeros(3, np.float32)
        n = self.lib.orc_sample_path_debug(self.h, C.byref(lp), x, y, frame, fp(rec), max_bounces, fp(rgb))
        return rec[:n], rgb

    def trace(self, rays, any_hit=False):
        r = _f(rays).reshape(-1, 8)
        n = len(r)
        prim = np.full(n, -1, np.int32)
        t, u, v = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
        back = np.zeros(n, np.int32)
        for i in range(n):
            o, d = r[i, 0:3].copy(), r[i, 3:6].copy()
            if any_hit:
                prim[i] = 0 if self.lib.orc_trace_any(self.h, fp(o), fp(d), float(r[i, 6]), float(r[i, 7])) else -1
            else:
                tt, uu, vv, bb = C.c_float(), C.c_float(), C.c_float(), C.c_int32()
                prim[i] = self.lib.orc_trace_closest(self.h, fp(o), fp(d), float(r[i, 6]), float(r[i, 7]),
                                                     C.byref(tt), C.byref(uu), C.byref(vv), C.byref(bb))
                if prim[i] >= 0:
                    t[i], u[i], v[i], back[i] = tt.value, uu.value, vv.value, bb.value
        return prim, t, u, v, back

    def close(self):
        if self.h:
            self.lib.orc_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
