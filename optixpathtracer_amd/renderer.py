"""Host-side mirror of the reference's render interface, over the C ABI.

`OptixRenderer` keeps the method names and semantics of
`Renderer/OptiX/OptixRenderer.h:63-76` (Resize, Render, SetCamera, SetLights,
SetMaxBounces) so caller code reads like the reference's `OptixView`/`main`; the extra
methods expose the device-resident accumulation that replaces the per-spp download + GL
blend (`Renderer/OptixView.cpp:201-255`).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import capi
from .capi import check, fptr, load
from .scenes import Scene


def _f32(a, shape=None) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    if shape is not None:
        a = a.reshape(shape)
    return a


class _SceneBinding:
    """Owns the ctypes `pt_scene` and keeps every numpy buffer it points to alive."""

    def __init__(self, scene: Scene):
        self.keep = []
        meshes = (capi.pt_mesh * max(1, len(scene.meshes)))()
        for i, m in enumerate(scene.meshes):
            v = _f32(m.vertices)
            idx = np.ascontiguousarray(m.indices, dtype=np.int32)
            self.keep += [v, idx]
            pm = meshes[i]
            pm.vertices = fptr(v)
            pm.indices = idx.ctypes.data_as(C.POINTER(C.c_int32))
            if m.normals is not None:
                n = _f32(m.normals)
                self.keep.append(n)
                pm.normals = fptr(n)
            if m.texcoords is not None:
                t = _f32(m.texcoords)
                self.keep.append(t)
                pm.texcoords = fptr(t)
            pm.n_vertices = int(v.shape[0])
            pm.n_triangles = int(idx.shape[0])
            pm.model_matrix[:] = [float(x) for x in _f32(m.model).ravel()]
            pm.albedo[:] = [float(x) for x in m.albedo]
            pm.metallic = float(m.metallic)
            pm.roughness = float(m.roughness)
            pm.albedo_tex = int(getattr(m, "albedo_tex", -1))
            pm.normal_tex = int(getattr(m, "normal_tex", -1))
            pm.metal_rough_tex = int(getattr(m, "metal_rough_tex", -1))
        texs = list(getattr(scene, "textures", []) or [])
        tarr = (capi.pt_texture * max(1, len(texs)))()
        for i, t in enumerate(texs):
            px = np.ascontiguousarray(t, dtype=np.uint32)
            self.keep.append(px)
            tarr[i].rgba8 = px.ctypes.data_as(C.POINTER(C.c_uint32))
            tarr[i].height, tarr[i].width = int(px.shape[0]), int(px.shape[1])
        self.meshes = meshes
        self.textures = tarr
        self.scene = capi.pt_scene()
        self.scene.meshes = C.cast(meshes, C.POINTER(capi.pt_mesh))
        self.scene.n_meshes = len(scene.meshes)
        self.scene.textures = C.cast(tarr, C.POINTER(capi.pt_texture))
        self.scene.n_textures = len(texs)


def camera_from_blender(pos, rot, fov_deg: float, width: int, height: int):
    """Camera.cpp:6-70 + OptixRenderer::SetCamera: (position, inverse view, inverse projection)."""
    lib = load()
    p = np.empty(3, np.float32)
    iv = np.empty(16, np.float32)
    ip = np.empty(16, np.float32)
    check(lib.pt_camera_from_blender(fptr(_f32(pos)), fptr(_f32(rot)), float(fov_deg), int(width), int(height),
                                     fptr(p), fptr(iv), fptr(ip)), "pt_camera_from_blender")
    return p, iv, ip


class OptixRenderer:
    """Drop-in for `OptixRenderer` (OptixRenderer.h:8-110) backed by libptamd.so."""

    def __init__(self, ptx_path_or_none, model: Scene, device: int = 0, material_mode: int | None = None,
                 kernel: int = capi.PT_KERNEL_AUTO, bvh_builder: int = capi.PT_BVH_AUTO, devices=None):
        """devices: None = the single `device`; a list of ordinals = one renderer over all of them
        (frame ids of render_frames split across the devices, RCCL-summed onto devices[0])."""
        # ptxPath is accepted for signature compatibility and ignored (no PTX on gfx950).
        self.lib = load()
        self.model = model
        self._binding = _SceneBinding(model)
        opts = capi.pt_options()
        opts.device = int(device)
        opts.material_mode = int(model.material_mode if material_mode is None else material_mode)
        opts.kernel = int(kernel)
        opts.bvh_builder = int(bvh_builder)
        if devices is not None:
            self._devlist = (C.c_int32 * max(1, len(devices)))(*[int(d) for d in devices])
            opts.n_devices = len(devices)
            opts.device_list = self._devlist
        h = C.c_void_p()
        check(self.lib.pt_create(C.byref(self._binding.scene), C.byref(opts), C.byref(h)), "pt_create")
        self.h = h
        self.size = (0, 0)

    # ---- reference API --------------------------------------------------------------
    def Resize(self, new_size) -> None:  # OptixRenderer.cpp:649-660
        w, h = int(new_size[0]), int(new_size[1])
        check(self.lib.pt_resize(self.h, w, h), "pt_resize")
        if w and h:
            self.size = (w, h)

    def Render(self, h_pixels: np.ndarray | None = None) -> np.ndarray:  # :617-647
        w, h = self.size
        out = h_pixels if h_pixels is not None else np.zeros((h, w, 3), np.float32)
        if w == 0:
            return out
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.size == w * h * 3
        check(self.lib.pt_render(self.h, fptr(out)), "pt_render")
        return out

    def launch(self, color_buffer_ptr: int, size, frame_id: int, position, inverse_view, inverse_projection,
               lights_device_ptr: int, n_lights: int, max_bounces: int) -> None:
        """optixLaunch with a LaunchParams block (pt_launch): writes frame `frame_id`'s 1-spp
        radiance into the device buffer at color_buffer_ptr (W*H*3 fp32, row 0 = bottom).
        Asynchronous; call synchronize().  Device pointers, as in the reference."""
        lp = capi.pt_launch_params()
        lp.frame.color_buffer = C.c_void_p(int(color_buffer_ptr))
        lp.frame.size[0], lp.frame.size[1] = int(size[0]), int(size[1])
        lp.frame.id = int(frame_id)
        for dst, src in ((lp.camera.position, position), (lp.camera.inverse_view_matrix, inverse_view),
                         (lp.camera.inverse_projection_matrix, inverse_projection)):
            vals = _f32(src).ravel()
            for i, v in enumerate(vals):
                dst[i] = float(v)
        lp.point_lights = C.c_void_p(int(lights_device_ptr)) if lights_device_ptr else None
        lp.point_light_count = int(n_lights)
        lp.max_bounces = int(max_bounces)
        check(self.lib.pt_launch(self.h, C.byref(lp)), "pt_launch")

    def SetCamera(self, position, inverse_view, inverse_projection) -> None:  # :662-668
        check(self.lib.pt_set_camera(self.h, fptr(_f32(position)), fptr(_f32(inverse_view)),
                                     fptr(_f32(inverse_projection))), "pt_set_camera")

    def SetCameraBlender(self, pos, rot, fov_deg: float = 40.0) -> None:
        w, h = self.size
        p, iv, ip = camera_from_blender(pos, rot, fov_deg, w, h)
        self.SetCamera(p, iv, ip)

    def SetLights(self, lights) -> None:  # :670-675
        L = _f32(lights).reshape(-1, 6)
        arr = (capi.pt_point_light * max(1, len(L)))()
        for i, row in enumerate(L):
            arr[i].position[:] = [float(x) for x in row[:3]]
            arr[i].color[:] = [float(x) for x in row[3:]]
        check(self.lib.pt_set_lights(self.h, arr, len(L)), "pt_set_lights")

    def SetMaxBounces(self, n: int) -> None:  # :677-679
        check(self.lib.pt_set_max_bounces(self.h, int(n)), "pt_set_max_bounces")

    # ---- device-resident accumulation -------------------------------------------------
    def set_material_mode(self, mode: int) -> None:
        check(self.lib.pt_set_material_mode(self.h, int(mode)), "pt_set_material_mode")

    def set_kernel(self, kernel: int) -> None:
        check(self.lib.pt_set_kernel(self.h, int(kernel)), "pt_set_kernel")

    def set_render_ahead(self, frames: int) -> None:
        """pt_set_render_ahead: frames Render() may render ahead of the caller (1 = off)."""
        check(self.lib.pt_set_render_ahead(self.h, int(frames)), "pt_set_render_ahead")

    def set_render_ahead_budget(self, max_ms: float) -> None:
        """pt_set_render_ahead_budget: bound (ms of GPU time) on one render-ahead batch, 0 = none."""
        check(self.lib.pt_set_render_ahead_budget(self.h, float(max_ms)), "pt_set_render_ahead_budget")

    def set_frames_per_launch(self, frames: int) -> None:
        check(self.lib.pt_set_frames_per_launch(self.h, int(frames)), "pt_set_frames_per_launch")

    def set_queue_budget(self, nbytes: int) -> None:
        """pt_set_queue_budget: bytes for all streams' wavefront queues (0 = default, a quarter of the
        device memory; < 0 = none)."""
        check(self.lib.pt_set_queue_budget(self.h, int(nbytes)), "pt_set_queue_budget")

    def trace_coherence(self) -> dict:
        """pt_get_trace_coherence: wave steps of the trace kernels by the number of distinct global
        BVH nodes their lanes load (counted while traversal stats are on)."""
        h = (C.c_uint64 * 8)()
        check(self.lib.pt_get_trace_coherence(self.h, h), "pt_get_trace_coherence")
        keys = ["d1", "d2", "d3_4", "d5_8", "d9_16", "d17_64", "steps", "lanes"]
        return {k: int(v) for k, v in zip(keys, h)}

    def set_debug_hold(self, on: bool) -> None:
        """pt_set_debug_hold (tests): speculative look-ahead batches wait until cancelled or released."""
        check(self.lib.pt_set_debug_hold(self.h, 1 if on else 0), "pt_set_debug_hold")

    def set_traversal_stats(self, enable: bool) -> None:
        check(self.lib.pt_set_traversal_stats(self.h, 1 if enable else 0), "pt_set_traversal_stats")

    def set_kernel_timing(self, enable: bool = True) -> None:
        """Time every wavefront trace launch and every launch of the bounce's dominant shading
        kernel with its own HIP event pair (pt_stats trace_kernel_* / shade_kernel_*)."""
        check(self.lib.pt_set_kernel_timing(self.h, 1 if enable else 0), "pt_set_kernel_timing")

    # -- headless progressive view (OptixView accumulation on the device) -------------------
    def display_reset(self, max_samples: int = -1) -> None:
        check(self.lib.pt_display_reset(self.h, int(max_samples)), "pt_display_reset")

    def display_add_frame(self) -> int:
        n = C.c_int32(0)
        check(self.lib.pt_display_add_frame(self.h, C.byref(n)), "pt_display_add_frame")
        return n.value

    def display(self) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w, 3), dtype=np.float32)
        check(self.lib.pt_display_download(self.h, fptr(out)), "pt_display_download")
        return out

    def accum_clear(self) -> None:
        check(self.lib.pt_accum_clear(self.h), "pt_accum_clear")

    def render_frames(self, first_frame_id: int, n_frames: int) -> None:
        check(self.lib.pt_render_frames(self.h, int(first_frame_id), int(n_frames)), "pt_render_frames")

    def set_primary_dedup(self, enable: bool) -> None:
        check(self.lib.pt_set_primary_dedup(self.h, 1 if enable else 0), "pt_set_primary_dedup")

    def set_wavefront_streams(self, streams: int) -> None:
        check(self.lib.pt_set_wavefront_streams(self.h, int(streams)), "pt_set_wavefront_streams")

    def set_band_split(self, enable: bool) -> None:
        """One-frame calls: two row bands on two wavefront streams (pt_set_band_split, default on)."""
        check(self.lib.pt_set_band_split(self.h, 1 if enable else 0), "pt_set_band_split")

    def render_accumulate(self, spp: int, first_frame_id: int = 1) -> np.ndarray:
        """Clear, render frame ids first_frame_id .. +spp-1 and return the mean image
        (pt_render_accumulate); the sum stays in the device accumulator."""
        w, h = self.size
        out = np.empty((h, w, 3), np.float32)
        check(self.lib.pt_render_accumulate(self.h, int(spp), int(first_frame_id), fptr(out)),
              "pt_render_accumulate")
        return out

    def set_accum_device_buffer(self, ptr: int | None) -> None:
        check(self.lib.pt_set_accum_device_buffer(self.h, C.c_void_p(ptr) if ptr else None),
              "pt_set_accum_device_buffer")

    def accum(self, scale: float = 1.0) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w, 3), np.float32)
        check(self.lib.pt_accum_download(self.h, fptr(out), float(scale)), "pt_accum_download")
        return out

    def set_accum_fp64(self, enable: bool) -> None:
        """pt_set_accum_fp64: add the samples in fp64 (accum() then returns the fp64 sum rounded
        to fp32, accum64() the fp64 sum); off by default (the reference sums in fp32)."""
        check(self.lib.pt_set_accum_fp64(self.h, 1 if enable else 0), "pt_set_accum_fp64")

    def accum64(self) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w, 3), np.float64)
        check(self.lib.pt_accum_download64(self.h, out.ctypes.data_as(C.POINTER(C.c_double))), "pt_accum_download64")
        return out

    def synchronize(self) -> None:
        check(self.lib.pt_synchronize(self.h), "pt_synchronize")

    def stream(self) -> int:
        return int(self.lib.pt_stream(self.h) or 0)

    @property
    def frame_id(self) -> int:
        return int(self.lib.pt_frame_id(self.h))

    @frame_id.setter
    def frame_id(self, v: int) -> None:
        check(self.lib.pt_set_frame_id(self.h, int(v)), "pt_set_frame_id")

    def stats(self) -> dict:
        s = capi.pt_stats()
        check(self.lib.pt_get_stats(self.h, C.byref(s)), "pt_get_stats")
        return {k: getattr(s, k) for k, _ in capi.pt_stats._fields_}

    def stats_reset(self) -> None:
        check(self.lib.pt_stats_reset(self.h), "pt_stats_reset")

    def trace_rays(self, rays: np.ndarray, any_hit: bool = False):
        """rays: (n, 8) float32 = origin, dir, tmin, tmax -> (prim, t, u, v, backface)."""
        r = _f32(rays).reshape(-1, 8)
        n = len(r)
        prim = np.empty(n, np.int32)
        t, u, v = (np.empty(n, np.float32) for _ in range(3))
        back = np.empty(n, np.int32)
        check(self.lib.pt_trace_rays(self.h, fptr(r), n, prim.ctypes.data_as(C.POINTER(C.c_int32)), fptr(t),
                                     fptr(u), fptr(v), back.ctypes.data_as(C.POINTER(C.c_int32)),
                                     1 if any_hit else 0), "pt_trace_rays")
        return prim, t, u, v, back

    def set_debug_pixel(self, x: int, y: int, frame_id: int) -> None:
        """Record the per-bounce surface of pixel (x, y)'s path at frame_id (pt_set_debug_pixel;
        the reference's isDebugRay, devicePrograms.cu:637-644).  x < 0 turns it off."""
        check(self.lib.pt_set_debug_pixel(self.h, int(x), int(y), int(frame_id)), "pt_set_debug_pixel")

    def debug_path(self) -> list:
        """The recorded bounces as dicts of pt_debug_bounce fields."""
        recs = (capi.pt_debug_bounce * 64)()
        n = C.c_int32()
        check(self.lib.pt_get_debug_path(self.h, recs, 64, C.byref(n)), "pt_get_debug_path")
        out = []
        for k in range(n.value):
            r = recs[k]
            out.append({f: (list(getattr(r, f)) if isinstance(getattr(r, f), C.Array) else getattr(r, f))
                        for f, _ in capi.pt_debug_bounce._fields_})
        return out

    def devices(self) -> list:
        """Device ordinals this renderer drives (pt_devices)."""
        n = int(self.lib.pt_device_count(self.h))
        out = (C.c_int32 * max(1, n))()
        check(self.lib.pt_devices(self.h, out, n), "pt_devices")
        return [int(out[i]) for i in range(n)]

    def bvh_arrays(self):
        """(nodes, triangles): the BVH4 node array as (bvh_nodes, 32) uint32 words and the
        leaf-ordered triangle records as (triangles, 12) uint32 words (pt_bvh_download)."""
        st = self.stats()
        nodes = np.zeros((st["bvh_nodes"], 32), np.uint32)
        tris = np.zeros((st["triangles"], 12), np.uint32)
        check(self.lib.pt_bvh_download(self.h, nodes.ctypes.data, nodes.nbytes, tris.ctypes.data, tris.nbytes),
              "pt_bvh_download")
        return nodes, tris

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.pt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def setup_renderer(scene: Scene, width: int, height: int, max_bounces: int, device: int = 0,
                   kernel: int = capi.PT_KERNEL_AUTO, bvh_builder: int = capi.PT_BVH_AUTO,
                   devices=None) -> OptixRenderer:
    """The reference's main.cpp:95-113 sequence: construct, Resize, SetLights, SetMaxBounces, SetCamera."""
    r = OptixRenderer(None, scene, device=device, kernel=kernel, bvh_builder=bvh_builder, devices=devices)
    r.Resize((width, height))
    r.SetLights(scene.lights)
    r.SetMaxBounces(max_bounces)
    r.SetCameraBlender(scene.camera_blender_pos, scene.camera_blender_rot, scene.fov_deg)
    return r
