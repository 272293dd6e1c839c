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


def write_glb(scene: Scene, path) -> int:
    """Write a `scenes.Scene` as one binary glTF 2.0 file (.glb): a JSON chunk and a BIN chunk with
    float32 POSITION / NORMAL / TEXCOORD_0, uint32 indices, the node matrix (column-major, the
    model matrix ModelLoader reads back, ModelLoader.cpp:199-245), the metallic-roughness material
    (baseColorFactor, metallicFactor, roughnessFactor, baseColorTexture, metallicRoughnessTexture,
    normalTexture; ModelLoader.cpp:171-197) and the RGBA8 textures embedded as PNG buffer views.
    The reference has no writer; this is the tool that hands the procedural scenes to the
    loader (pt_model_load_gltf) at full size.  Every value round-trips exactly (float32 in,
    float32 out).  Returns the file size in bytes."""
    import json
    import struct
    from pathlib import Path

    from PIL import Image

    chunks, views, accessors, meshes, nodes, materials, images = [], [], [], [], [], [], []
    off = 0

    def view(data: bytes) -> int:
        nonlocal off
        pad = (4 - len(data) % 4) % 4
        views.append({"buffer": 0, "byteOffset": off, "byteLength": len(data)})
        chunks.append(data + b"\0" * pad)
        off += len(data) + pad
        return len(views) - 1

    def accessor(arr, ctype, typ, count, minmax=False) -> int:
        a = {"bufferView": view(np.ascontiguousarray(arr).tobytes()), "componentType": ctype, "count": count,
             "type": typ}
        if minmax:  # POSITION needs its bounds (glTF 2.0 3.6.2.4)
            a["min"] = [float(x) for x in np.asarray(arr).min(axis=0)]
            a["max"] = [float(x) for x in np.asarray(arr).max(axis=0)]
        accessors.append(a)
        return len(accessors) - 1

    for m in scene.meshes:
        v = np.asarray(m.vertices, np.float32)
        attrs = {"POSITION": accessor(v, 5126, "VEC3", len(v), minmax=len(v) > 0)}
        if m.normals is not None:
            attrs["NORMAL"] = accessor(np.asarray(m.normals, np.float32), 5126, "VEC3", len(m.normals))
        if m.texcoords is not None:
            attrs["TEXCOORD_0"] = accessor(np.asarray(m.texcoords, np.float32), 5126, "VEC2", len(m.texcoords))
        idx = np.asarray(m.indices, np.uint32).ravel()
        pbr = {"baseColorFactor": [float(c) for c in m.albedo] + [1.0], "metallicFactor": float(m.metallic),
               "roughnessFactor": float(m.roughness)}
        mat = {"pbrMetallicRoughness": pbr}
        if m.albedo_tex >= 0:
            pbr["baseColorTexture"] = {"index": int(m.albedo_tex)}
        if m.metal_rough_tex >= 0:
            pbr["metallicRoughnessTexture"] = {"index": int(m.metal_rough_tex)}
        if m.normal_tex >= 0:
            mat["normalTexture"] = {"index": int(m.normal_tex)}
        materials.append(mat)
        prim = {"attributes": attrs, "indices": accessor(idx, 5125, "SCALAR", int(idx.size)),
                "material": len(materials) - 1}
        meshes.append({"primitives": [prim]})
        nodes.append({"name": m.name, "mesh": len(meshes) - 1,
                      "matrix": [float(x) for x in np.asarray(m.model, np.float32).ravel()]})
    for t in scene.textures:
        px = np.ascontiguousarray(t, dtype=np.uint32).view(np.uint8).reshape(t.shape[0], t.shape[1], 4)
        buf = io.BytesIO()
        Image.fromarray(px, "RGBA").save(buf, "PNG")
        images.append({"bufferView": view(buf.getvalue()), "mimeType": "image/png"})
    binbuf = b"".join(chunks)
    doc = {"asset": {"version": "2.0", "generator": "optixpathtracer_amd.gltf.write_glb"}, "scene": 0,
           "scenes": [{"nodes": list(range(len(nodes)))}], "nodes": nodes, "meshes": meshes,
           "materials": materials, "accessors": accessors, "bufferViews": views,
           "buffers": [{"byteLength": len(binbuf)}]}
    if images:
        doc["images"] = images
        doc["textures"] = [{"source": k} for k in range(len(images))]
    js = json.dumps(doc, separators=(",", ":")).encode()
    js += b" " * ((4 - len(js) % 4) % 4)
    total = 12 + 8 + len(js) + 8 + len(binbuf)
    with open(Path(path), "wb") as f:
        f.write(struct.pack("<4sII", b"glTF", 2, total))
        f.write(struct.pack("<II", len(js), 0x4E4F534A))
        f.write(js)
        f.write(struct.pack("<II", len(binbuf), 0x004E4942))
        f.write(binbuf)
    return total


def load_scene_glb(scene: Scene, folder) -> tuple:
    """`scene` written to `folder`/<name>.glb (write_glb) and loaded back through the C++ loader:
    (loaded scene, pt_model_load_gltf wall ms, file bytes).  The lights, camera and material mode
    come from `scene`, as the reference's Scene presets set them beside the loaded model
    (main.cpp:6-78)."""
    import time
    from pathlib import Path

    p = Path(folder) / f"{scene.name or 'scene'}.glb"
    size = write_glb(scene, p)
    t = time.perf_counter()
    loaded = load_gltf(p, lights=scene.lights, camera_blender_pos=scene.camera_blender_pos,
                       camera_blender_rot=scene.camera_blender_rot, fov_deg=scene.fov_deg,
                       material_mode=scene.material_mode, use_pil=False)
    ms = (time.perf_counter() - t) * 1e3
    loaded.name = scene.name
    return loaded, ms, size


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
