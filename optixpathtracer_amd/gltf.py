"""glTF 2.0 scene loading over the C ABI.

`load_gltf` is the counterpart of ModelLoader::LoadModel (ModelLoading/ModelLoader.cpp:10-244):
pt_model_load_gltf parses the file and decodes PNG textures in C++; any other image format
(JPEG, ... — stb_image in the reference) is decoded by the PIL callback below.  The result is
a `scenes.Scene` (meshes with world transforms, materials, texture ids, RGBA8 textures) that
OptixRenderer and the oracle consume like the procedural scenes.
"""
from __future__ import annotations

import ctypes as C
import io

import numpy as np

from . import capi
from .capi import PTError, load
from .scenes import Mesh, Scene


class _PilDecoder:
    """pt_image_decode_fn backed by PIL; decodes once, serves size then pixels."""

    def __init__(self):
        self.cache = {}
        self.cfn = capi.pt_image_decode_fn(self._decode)

    def _decode(self, data, size, w, h, out, user):  # noqa: ARG002
        try:
            raw = C.string_at(data, size)
            key = hash(raw)
            if key not in self.cache:
                from PIL import Image

                im = Image.open(io.BytesIO(raw)).convert("RGBA")
                self.cache = {key: np.ascontiguousarray(np.asarray(im, dtype=np.uint8))}
            px = self.cache[key]
            w[0], h[0] = px.shape[1], px.shape[0]
            if out:
                C.memmove(out, px.ctypes.data, px.nbytes)
            return 0
        except Exception:  # decoding errors are reported through the status code
            return 1


def load_gltf(path, lights=None, camera_blender_pos=(0.0, 0.0, 0.0), camera_blender_rot=(90.0, 0.0, 0.0),
              fov_deg: float = 40.0, material_mode: int = 0, use_pil: bool = True) -> Scene:
    lib = load()
    dec = _PilDecoder() if use_pil else None
    m = C.c_void_p()
    fn = dec.cfn if dec else capi.pt_image_decode_fn()
    st = lib.pt_model_load_gltf(str(path).encode(), fn, None, C.byref(m))
    if st != 0:
        msg = lib.pt_model_last_error()
        raise PTError(f"pt_model_load_gltf failed ({st}): {msg.decode() if msg else ''}")
    try:
        sc = lib.pt_model_scene(m).contents
        meshes = []
        for i in range(sc.n_meshes):
            pm = sc.meshes[i]
            nv, nt = pm.n_vertices, pm.n_triangles
            v = np.ctypeslib.as_array(pm.vertices, shape=(nv, 3)).copy()
            idx = np.ctypeslib.as_array(pm.indices, shape=(nt, 3)).copy()
            n = np.ctypeslib.as_array(pm.normals, shape=(nv, 3)).copy() if pm.normals else None
            uv = np.ctypeslib.as_array(pm.texcoords, shape=(nv, 2)).copy() if pm.texcoords else None
            name = lib.pt_model_mesh_name(m, i)
            meshes.append(Mesh(vertices=v, indices=idx, normals=n, texcoords=uv,
                               model=np.array(pm.model_matrix[:], np.float32), albedo=tuple(pm.albedo[:]),
                               metallic=float(pm.metallic), roughness=float(pm.roughness),
                               name=name.decode() if name else "", albedo_tex=pm.albedo_tex,
                               normal_tex=pm.normal_tex, metal_rough_tex=pm.metal_rough_tex))
        textures = []
        for i in range(sc.n_textures):
            t = sc.textures[i]
            textures.append(np.ctypeslib.as_array(t.rgba8, shape=(t.height, t.width)).copy())
    finally:
        lib.pt_model_destroy(m)
    L = np.zeros((0, 6), np.float32) if lights is None else np.asarray(lights, np.float32).reshape(-1, 6)
    return Scene(meshes=meshes, lights=L, camera_blender_pos=tuple(camera_blender_pos),
                 camera_blender_rot=tuple(camera_blender_rot), fov_deg=fov_deg, material_mode=material_mode,
                 name=str(path), textures=textures)


def decode_png(data: bytes) -> np.ndarray:
    """The loader's PNG decoder: (H, W, 4) uint8 RGBA, rows as stored."""
    lib = load()
    w, h = C.c_int32(0), C.c_int32(0)
    buf = C.create_string_buffer(data, len(data))
    if lib.pt_image_decode_png(buf, len(data), C.byref(w), C.byref(h), None) != 0:
        raise PTError(f"png decode failed: {lib.pt_model_last_error().decode()}")
    out = np.empty((h.value, w.value, 4), np.uint8)
    lib.pt_image_decode_png(buf, len(data), C.byref(w), C.byref(h), out.ctypes.data)
    return out
