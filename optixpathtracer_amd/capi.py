"""ctypes binding of libptamd.so — the C ABI declared in include/ptamd.h.

The shared library is built in-tree (``optixpathtracer_amd/libptamd.so``, see
``__graft_entry__.build``).  There is no fallback: if the library is missing or a call
fails, a :class:`PTError` is raised.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "libptamd.so"

PT_MAT_DEFAULT, PT_MAT_LAMBERT, PT_MAT_CONDUCTOR, PT_MAT_DIELECTRIC, PT_MAT_LAYERED = range(5)
PT_KERNEL_MEGA, PT_KERNEL_WAVEFRONT, PT_KERNEL_AUTO = 0, 1, 2
PT_BVH_AUTO, PT_BVH_LBVH, PT_BVH_SAH, PT_BVH_PLOC, PT_BVH_SAH_GPU = 0, 1, 2, 3, 4
PT_OK, PT_ERR_INVALID, PT_ERR_HIP, PT_ERR_STATE, PT_ERR_NOMEM = 0, -1, -2, -3, -4

MATERIAL_MODES = {
    "default": PT_MAT_DEFAULT,
    "lambert": PT_MAT_LAMBERT,
    "conductor": PT_MAT_CONDUCTOR,
    "dielectric": PT_MAT_DIELECTRIC,
    "layered": PT_MAT_LAYERED,
}


class PTError(RuntimeError):
    """A libptamd call returned a negative status (`status`: PT_ERR_*)."""

    def __init__(self, msg: str, status: int = 0):
        super().__init__(msg)
        self.status = status


class pt_mesh(C.Structure):
    _fields_ = [
        ("vertices", C.POINTER(C.c_float)),
        ("normals", C.POINTER(C.c_float)),
        ("texcoords", C.POINTER(C.c_float)),
        ("indices", C.POINTER(C.c_int32)),
        ("n_vertices", C.c_int32),
        ("n_triangles", C.c_int32),
        ("model_matrix", C.c_float * 16),
        ("albedo", C.c_float * 3),
        ("metallic", C.c_float),
        ("roughness", C.c_float),
        ("albedo_tex", C.c_int32),
        ("normal_tex", C.c_int32),
        ("metal_rough_tex", C.c_int32),
    ]


class pt_texture(C.Structure):
    _fields_ = [("rgba8", C.POINTER(C.c_uint32)), ("width", C.c_int32), ("height", C.c_int32)]


class pt_scene(C.Structure):
    _fields_ = [
        ("meshes", C.POINTER(pt_mesh)),
        ("n_meshes", C.c_int32),
        ("textures", C.POINTER(pt_texture)),
        ("n_textures", C.c_int32),
    ]


class pt_point_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("color", C.c_float * 3)]


class pt_options(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("material_mode", C.c_int32),
        ("kernel", C.c_int32),
        ("bvh_builder", C.c_int32),
        ("n_devices", C.c_int32),
        ("reserved", C.c_int32 * 3),
        ("device_list", C.POINTER(C.c_int32)),
    ]


class pt_debug_bounce(C.Structure):
    _fields_ = [
        ("bounce", C.c_int32),
        ("prim", C.c_int32),
        ("position", C.c_float * 3),
        ("albedo", C.c_float * 3),
        ("shading_normal", C.c_float * 3),
        ("geometry_normal", C.c_float * 3),
        ("roughness", C.c_float),
        ("metallic", C.c_float),
        ("beta", C.c_float * 3),
        ("radiance", C.c_float * 3),
    ]


class pt_stats(C.Structure):
    _fields_ = [
        ("segments", C.c_uint64),
        ("samples", C.c_uint64),
        ("last_render_ms", C.c_double),
        ("total_render_ms", C.c_double),
        ("render_calls", C.c_uint64),
        ("kernel_launches", C.c_uint64),
        ("bvh_build_ms", C.c_double),
        ("bvh_nodes", C.c_int32),
        ("triangles", C.c_int32),
        ("frames_per_launch", C.c_int32),
        ("bvh_depth", C.c_int32),
        ("nodes_visited", C.c_uint64),
        ("tri_tests", C.c_uint64),
        ("rays", C.c_uint64),
        ("stack_overflows", C.c_uint64),
        ("trace_kernel_ms", C.c_double),
        ("trace_kernel_launches", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("trace_kernel_rays", C.c_uint64),
        ("trace_kernel_bytes", C.c_uint64),
        ("strict_retraces", C.c_uint64),
        ("wave_steps", C.c_uint64),
        ("wave_active_lanes", C.c_uint64),
        ("wave_node_steps", C.c_uint64),
        ("wave_tri_steps", C.c_uint64),
        ("wave_refills", C.c_uint64),
        ("lds_nodes_visited", C.c_uint64),
        ("shade_kernel_ms", C.c_double),
        ("shade_kernel_launches", C.c_uint64),
        ("shade_kernel_items", C.c_uint64),
        ("frames_rendered_ahead", C.c_uint64),
        ("frames_served_ahead", C.c_uint64),
        ("look_ahead_cancelled", C.c_uint64),
        ("pair_kernel_ms", C.c_double),
        ("pair_kernel_launches", C.c_uint64),
        ("pair_kernel_rays", C.c_uint64),
        ("pair_kernel_bytes", C.c_uint64),
        ("pair_kernel_shadow_rays", C.c_uint64),
        ("nee_unoccluded", C.c_uint64),
        ("queue_bytes", C.c_uint64),
        ("queue_budget", C.c_uint64),
        ("last_streams", C.c_int32),
        ("last_batch_frames", C.c_int32),
        ("look_ahead_held", C.c_uint64),
    ]


class _pt_launch_frame(C.Structure):
    _fields_ = [("color_buffer", C.c_void_p), ("size", C.c_int32 * 2), ("id", C.c_uint32)]


class _pt_launch_camera(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("inverse_view_matrix", C.c_float * 16),
                ("inverse_projection_matrix", C.c_float * 16)]


class pt_launch_params(C.Structure):
    """LaunchParams (Renderer/OptiX/LaunchParams.h:9-28); device pointers as in the reference."""
    _fields_ = [("frame", _pt_launch_frame), ("camera", _pt_launch_camera), ("point_lights", C.c_void_p),
                ("point_light_count", C.c_int32), ("max_bounces", C.c_int32)]


_FP = C.POINTER(C.c_float)
_IP = C.POINTER(C.c_int32)
_R = C.c_void_p  # pt_renderer*
_M = C.c_void_p  # pt_model*
# int decode(const uint8_t* data, size_t size, int32_t* w, int32_t* h, uint8_t* rgba_out, void* user)
pt_image_decode_fn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                 C.c_void_p, C.c_void_p)

# name -> (restype, argtypes); this is the complete exported surface of include/ptamd.h
SIGNATURES = {
    "pt_create": (C.c_int, [C.POINTER(pt_scene), C.POINTER(pt_options), C.POINTER(C.c_void_p)]),
    "pt_destroy": (C.c_int, [_R]),
    "pt_resize": (C.c_int, [_R, C.c_int32, C.c_int32]),
    "pt_set_camera": (C.c_int, [_R, _FP, _FP, _FP]),
    "pt_set_lights": (C.c_int, [_R, C.POINTER(pt_point_light), C.c_int32]),
    "pt_set_max_bounces": (C.c_int, [_R, C.c_int32]),
    "pt_set_material_mode": (C.c_int, [_R, C.c_int32]),
    "pt_set_kernel": (C.c_int, [_R, C.c_int32]),
    "pt_set_frames_per_launch": (C.c_int, [_R, C.c_int32]),
    "pt_set_render_ahead": (C.c_int, [_R, C.c_int32]),
    "pt_set_render_ahead_budget": (C.c_int, [_R, C.c_float]),
    "pt_set_queue_budget": (C.c_int, [_R, C.c_int64]),
    "pt_get_trace_coherence": (C.c_int, [_R, C.POINTER(C.c_uint64)]),
    "pt_set_debug_hold": (C.c_int, [_R, C.c_int32]),
    "pt_set_traversal_stats": (C.c_int, [_R, C.c_int32]),
    "pt_set_kernel_timing": (C.c_int, [_R, C.c_int32]),
    "pt_render": (C.c_int, [_R, _FP]),
    "pt_launch": (C.c_int, [_R, C.POINTER(pt_launch_params)]),
    "pt_accum_clear": (C.c_int, [_R]),
    "pt_render_frames": (C.c_int, [_R, C.c_uint32, C.c_uint32]),
    "pt_set_primary_dedup": (C.c_int, [_R, C.c_int32]),
    "pt_set_band_split": (C.c_int, [_R, C.c_int32]),
    "pt_set_wavefront_streams": (C.c_int, [_R, C.c_int32]),
    "pt_render_accumulate": (C.c_int, [_R, C.c_uint32, C.c_uint32, _FP]),
    "pt_set_accum_device_buffer": (C.c_int, [_R, C.c_void_p]),
    "pt_accum_device_ptr": (C.c_void_p, [_R]),
    "pt_accum_download": (C.c_int, [_R, _FP, C.c_float]),
    "pt_set_accum_fp64": (C.c_int, [_R, C.c_int32]),
    "pt_accum_device_ptr64": (C.c_void_p, [_R]),
    "pt_accum_download64": (C.c_int, [_R, C.POINTER(C.c_double)]),
    "pt_synchronize": (C.c_int, [_R]),
    "pt_stream": (C.c_void_p, [_R]),
    "pt_device_count": (C.c_int32, [_R]),
    "pt_devices": (C.c_int, [_R, C.POINTER(C.c_int32), C.c_int32]),
    "pt_frame_id": (C.c_uint32, [_R]),
    "pt_set_frame_id": (C.c_int, [_R, C.c_uint32]),
    "pt_get_stats": (C.c_int, [_R, C.POINTER(pt_stats)]),
    "pt_stats_reset": (C.c_int, [_R]),
    "pt_camera_from_blender": (C.c_int, [_FP, _FP, C.c_float, C.c_int32, C.c_int32, _FP, _FP, _FP]),
    "pt_trace_rays": (C.c_int, [_R, _FP, C.c_int32, _IP, _FP, _FP, _FP, _IP, C.c_int32]),
    "pt_bvh_download": (C.c_int, [_R, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]),
    "pt_set_debug_pixel": (C.c_int, [_R, C.c_int32, C.c_int32, C.c_uint32]),
    "pt_get_debug_path": (C.c_int, [_R, C.POINTER(pt_debug_bounce), C.c_int32, C.POINTER(C.c_int32)]),
    "pt_last_error": (C.c_char_p, []),
    "pt_version": (C.c_char_p, []),
    "pt_display_reset": (C.c_int, [_R, C.c_int32]),
    "pt_display_add_frame": (C.c_int, [_R, C.POINTER(C.c_int32)]),
    "pt_display_download": (C.c_int, [_R, _FP]),
    "pt_model_load_gltf": (C.c_int, [C.c_char_p, pt_image_decode_fn, C.c_void_p, C.POINTER(_M)]),
    "pt_model_scene": (C.POINTER(pt_scene), [_M]),
    "pt_model_mesh_name": (C.c_char_p, [_M, C.c_int32]),
    "pt_model_destroy": (C.c_int, [_M]),
    "pt_model_last_error": (C.c_char_p, []),
    "pt_image_decode_png": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                      C.c_void_p]),
    "pt_image_write_exr": (C.c_int, [C.c_char_p, _FP, C.c_int32, C.c_int32]),
    "pt_image_write_bmp": (C.c_int, [C.c_char_p, _FP, C.c_int32, C.c_int32]),
    "pt_image_write_pfm": (C.c_int, [C.c_char_p, _FP, C.c_int32, C.c_int32]),
    "pt_image_read": (C.c_int, [C.c_char_p, _FP, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "pt_image_mse": (C.c_double, [_FP, _FP, C.c_int64]),
    "pt_image_flip": (C.c_double, [_FP, _FP, C.c_int32, C.c_int32, C.c_float, _FP]),
    "pt_image_last_error": (C.c_char_p, []),
}

_lib = None


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libptamd.so (in-tree).  Raises PTError if it has not been built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # PTAMD_LIB selects an alternative in-tree build (kernel A/B variants, tools/).
    p = Path(path) if path else Path(os.environ.get("PTAMD_LIB", LIB_PATH))
    if not p.exists():
        raise PTError(
            f"{p} not found: the HIP extension is not built (run `python -c 'import __graft_entry__ as g; g.build()'`)"
        )
    lib = C.CDLL(str(p))
    variant = path is None and "PTAMD_LIB" in os.environ
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue  # an older A/B build (tools/ab.sh) may predate an entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = load().pt_last_error()
        raise PTError(f"{what} failed ({status}): {msg.decode() if msg else ''}", status)


def fptr(a):
    """float32 contiguous numpy array -> float*"""
    return a.ctypes.data_as(_FP)


def iptr(a):
    return a.ctypes.data_as(_IP)
