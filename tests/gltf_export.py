"""Test helper: write a `scenes.Scene` as glTF 2.0 (.gltf + .bin + PNG textures) following the
spec, so the C++ loader can be checked end to end on real renderable scenes."""
import io
import json

import numpy as np


def scene_to_gltf(scene, folder, name="scene"):
    from PIL import Image

    chunks, views, accessors, meshes, nodes, materials = [], [], [], [], [], []
    off = 0

    def add(arr, ctype, typ, count):
        nonlocal off
        data = np.ascontiguousarray(arr).tobytes()
        pad = (4 - len(data) % 4) % 4
        views.append({"buffer": 0, "byteOffset": off, "byteLength": len(data)})
        chunks.append(data + b"\0" * pad)
        off += len(data) + pad
        accessors.append({"bufferView": len(views) - 1, "componentType": ctype, "count": count, "type": typ})
        return len(accessors) - 1

    for m in scene.meshes:
        attrs = {"POSITION": add(np.asarray(m.vertices, np.float32), 5126, "VEC3", len(m.vertices))}
        if m.normals is not None:
            attrs["NORMAL"] = add(np.asarray(m.normals, np.float32), 5126, "VEC3", len(m.normals))
        if m.texcoords is not None:
            attrs["TEXCOORD_0"] = add(np.asarray(m.texcoords, np.float32), 5126, "VEC2", len(m.texcoords))
        idx = add(np.asarray(m.indices, np.uint32).ravel(), 5125, "SCALAR", int(np.asarray(m.indices).size))
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
        meshes.append({"primitives": [{"attributes": attrs, "indices": idx, "material": len(materials) - 1}]})
        nodes.append({"name": m.name, "mesh": len(meshes) - 1,
                      "matrix": [float(x) for x in np.asarray(m.model, np.float32).ravel()]})
    images = []
    for k, t in enumerate(scene.textures):
        px = np.ascontiguousarray(t, dtype=np.uint32).view(np.uint8).reshape(t.shape[0], t.shape[1], 4)
        buf = io.BytesIO()
        Image.fromarray(px, "RGBA").save(buf, "PNG")
        (folder / f"{name}_tex{k}.png").write_bytes(buf.getvalue())
        images.append({"uri": f"{name}_tex{k}.png"})
    binbuf = b"".join(chunks)
    (folder / f"{name}.bin").write_bytes(binbuf)
    doc = {"asset": {"version": "2.0"}, "scene": 0, "scenes": [{"nodes": list(range(len(nodes)))}],
           "nodes": nodes, "meshes": meshes, "materials": materials, "accessors": accessors,
           "bufferViews": views, "buffers": [{"byteLength": len(binbuf), "uri": f"{name}.bin"}],
           "textures": [{"source": k} for k in range(len(images))], "images": images}
    p = folder / f"{name}.gltf"
    p.write_text(json.dumps(doc))
    return p
