"""glTF loading (ModelLoader.cpp restated) and the PNG decoder — CPU only.

The fixtures are written here with json/numpy/PIL, following the glTF 2.0 spec; decoded
images are compared with PIL's decode of the same bytes."""
import base64
import io
import json
import struct

import numpy as np
import pytest

from optixpathtracer_amd import gltf
from optixpathtracer_amd.capi import PTError

PIL = pytest.importorskip("PIL.Image")


def _png(mode, size=(5, 3), seed=0, **kw):
    rng = np.random.default_rng(seed)
    if mode == "P":
        im = PIL.fromarray(rng.integers(0, 4, size=(size[1], size[0])).astype(np.uint8), "L").convert("P")
        im.putpalette([255, 0, 0, 0, 255, 0, 0, 0, 255, 9, 9, 9] + [0] * (768 - 12))
        im.info["transparency"] = bytes([255, 128, 0, 255])
        kw = {"transparency": bytes([255, 128, 0, 255])}
    elif mode == "1":
        im = PIL.fromarray(rng.integers(0, 2, size=(size[1], size[0])).astype(bool))
    else:
        ch = {"L": 1, "LA": 2, "RGB": 3, "RGBA": 4}[mode]
        a = rng.integers(0, 256, size=(size[1], size[0], ch)).astype(np.uint8)
        im = PIL.fromarray(a[..., 0] if ch == 1 else a, mode)
    buf = io.BytesIO()
    im.save(buf, "PNG", **kw)
    return buf.getvalue()


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P", "1"])
def test_png_decoder_matches_pil(mode):
    data = _png(mode, size=(13, 7), seed=3)
    got = gltf.decode_png(data)
    want = np.asarray(PIL.open(io.BytesIO(data)).convert("RGBA"))
    np.testing.assert_array_equal(got, want)


def test_png_decoder_16bit():
    a = (np.arange(6 * 4, dtype=np.uint16).reshape(4, 6) * 2731).astype(np.uint16)
    buf = io.BytesIO()
    PIL.fromarray(a).save(buf, "PNG")  # uint16 -> I;16
    got = gltf.decode_png(buf.getvalue())
    hi = (a >> 8).astype(np.uint8)  # 16-bit samples keep their high byte
    np.testing.assert_array_equal(got[..., 0], hi)
    np.testing.assert_array_equal(got[..., 3], 255)


def _quat_mat(q):
    x, y, z, w = [np.float32(c) for c in q]
    f = np.float32
    R = np.eye(4, dtype=np.float32)
    R[0, 0] = f(1) - f(2) * (y * y + z * z)
    R[1, 0] = f(2) * (x * y + w * z)
    R[2, 0] = f(2) * (x * z - w * y)
    R[0, 1] = f(2) * (x * y - w * z)
    R[1, 1] = f(1) - f(2) * (x * x + z * z)
    R[2, 1] = f(2) * (y * z + w * x)
    R[0, 2] = f(2) * (x * z + w * y)
    R[1, 2] = f(2) * (y * z - w * x)
    R[2, 2] = f(1) - f(2) * (x * x + y * y)
    return R


def _trs(t=(0, 0, 0), r=(0, 0, 0, 1), s=(1, 1, 1)):
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = t
    S = np.diag(np.array(list(s) + [1], np.float32))
    return T @ _quat_mat(r) @ S  # row-major numpy of the glm column-major matrix


def _write_scene(tmp_path, glb=False, data_uri=False):
    pos = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32)
    nrm = np.tile(np.array([0, 0, 1], np.float32), (4, 1))
    uv = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32)
    idx16 = np.array([0, 1, 2, 0, 2, 3], np.uint16)
    idx32 = np.array([2, 1, 0, 3, 2, 0], np.uint32)
    inter = np.concatenate([pos, nrm], axis=1).astype(np.float32)  # interleaved, byteStride 24
    chunks = [pos.tobytes(), nrm.tobytes(), uv.tobytes(), idx16.tobytes() + b"\0\0", idx32.tobytes(), inter.tobytes()]
    offs = np.cumsum([0] + [len(c) for c in chunks])
    binbuf = b"".join(chunks)
    png = _png("RGBA", size=(4, 4), seed=5)
    jpg_io = io.BytesIO()
    PIL.fromarray(np.random.default_rng(6).integers(0, 256, (8, 8, 3)).astype(np.uint8)).save(jpg_io, "JPEG")
    (tmp_path / "tex.png").write_bytes(png)
    (tmp_path / "tex b.jpg").write_bytes(jpg_io.getvalue())
    views = [{"buffer": 0, "byteOffset": int(offs[i]), "byteLength": len(chunks[i])} for i in range(6)]
    views[5]["byteStride"] = 24
    doc = {
        "asset": {"version": "2.0"},
        "scene": 0,
        "scenes": [{"nodes": [0]}],
        "nodes": [
            {"name": "root", "translation": [1.0, 2.0, 3.0], "children": [1]},
            {"name": "child", "mesh": 0, "rotation": [0.0, 0.38268343, 0.0, 0.9238795], "scale": [2.0, 1.0, 0.5]},
        ],
        "meshes": [{"primitives": [
            {"attributes": {"POSITION": 0, "NORMAL": 1, "TEXCOORD_0": 2}, "indices": 3, "material": 0},
            {"attributes": {"POSITION": 5, "NORMAL": 6}, "indices": 4},
            {"attributes": {"POSITION": 0}, "mode": 1},
        ]}],
        "accessors": [
            {"bufferView": 0, "componentType": 5126, "count": 4, "type": "VEC3"},
            {"bufferView": 1, "componentType": 5126, "count": 4, "type": "VEC3"},
            {"bufferView": 2, "componentType": 5126, "count": 4, "type": "VEC2"},
            {"bufferView": 3, "componentType": 5123, "count": 6, "type": "SCALAR"},
            {"bufferView": 4, "componentType": 5125, "count": 6, "type": "SCALAR"},
            {"bufferView": 5, "componentType": 5126, "count": 4, "type": "VEC3"},
            {"bufferView": 5, "byteOffset": 12, "componentType": 5126, "count": 4, "type": "VEC3"},
        ],
        "bufferViews": views,
        "materials": [{"pbrMetallicRoughness": {"baseColorFactor": [0.2, 0.4, 0.6, 1.0], "metallicFactor": 0.25,
                                                 "roughnessFactor": 0.75, "baseColorTexture": {"index": 0},
                                                 "metallicRoughnessTexture": {"index": 1}},
                       "normalTexture": {"index": 0}}],
        "textures": [{"source": 0}, {"source": 1}],
        "images": [{"uri": "tex.png"}, {"uri": "tex%20b.jpg"}],
    }
    if glb:
        doc["buffers"] = [{"byteLength": len(binbuf)}]
        js = json.dumps(doc).encode()
        js += b" " * ((4 - len(js) % 4) % 4)
        bb = binbuf + b"\0" * ((4 - len(binbuf) % 4) % 4)
        body = struct.pack("<II", len(js), 0x4E4F534A) + js + struct.pack("<II", len(bb), 0x004E4942) + bb
        p = tmp_path / "scene.glb"
        p.write_bytes(struct.pack("<4sII", b"glTF", 2, 12 + len(body)) + body)
    else:
        if data_uri:
            doc["buffers"] = [{"byteLength": len(binbuf),
                               "uri": "data:application/octet-stream;base64," + base64.b64encode(binbuf).decode()}]
        else:
            (tmp_path / "scene.bin").write_bytes(binbuf)
            doc["buffers"] = [{"byteLength": len(binbuf), "uri": "scene.bin"}]
        p = tmp_path / "scene.gltf"
        p.write_text(json.dumps(doc))
    return p, pos, nrm, uv, idx16, idx32, png, jpg_io.getvalue()


@pytest.mark.parametrize("variant", ["gltf", "glb", "data_uri"])
def test_load_gltf(tmp_path, variant):
    p, pos, nrm, uv, idx16, idx32, png, jpg = _write_scene(tmp_path, glb=variant == "glb",
                                                          data_uri=variant == "data_uri")
    sc = gltf.load_gltf(p)
    assert len(sc.meshes) == 2  # the line-list primitive is skipped
    m0, m1 = sc.meshes
    np.testing.assert_array_equal(m0.vertices, pos)
    np.testing.assert_array_equal(m0.normals, nrm)
    np.testing.assert_array_equal(m0.texcoords, uv)
    np.testing.assert_array_equal(m0.indices.ravel(), idx16.astype(np.int32))
    np.testing.assert_array_equal(m1.indices.ravel(), idx32.astype(np.int32))
    np.testing.assert_array_equal(m1.vertices, pos)  # interleaved with byteStride 24
    np.testing.assert_array_equal(m1.normals, nrm)
    assert m1.texcoords is None
    world = _trs(t=(1, 2, 3)) @ _trs(r=(0.0, 0.38268343, 0.0, 0.9238795), s=(2, 1, 0.5))
    np.testing.assert_allclose(m0.model.reshape(4, 4).T, world, rtol=0, atol=1e-6)
    assert m0.name == "child"
    assert m0.albedo == pytest.approx((0.2, 0.4, 0.6)) and m0.metallic == pytest.approx(0.25)
    assert m0.roughness == pytest.approx(0.75)
    assert (m0.albedo_tex, m0.metal_rough_tex, m0.normal_tex) == (0, 1, 0)
    assert m1.albedo == (1.0, 1.0, 1.0) and m1.metallic == 1.0 and m1.roughness == 1.0  # glTF default material
    assert (m1.albedo_tex, m1.metal_rough_tex, m1.normal_tex) == (-1, -1, -1)
    assert len(sc.textures) == 2
    want0 = np.asarray(PIL.open(io.BytesIO(png)).convert("RGBA")).view(np.uint32)[..., 0]
    want1 = np.asarray(PIL.open(io.BytesIO(jpg)).convert("RGBA")).view(np.uint32)[..., 0]
    np.testing.assert_array_equal(sc.textures[0], want0)
    np.testing.assert_array_equal(sc.textures[1], want1)


def test_load_gltf_errors(tmp_path):
    with pytest.raises(PTError):
        gltf.load_gltf(tmp_path / "missing.gltf")
    p = _write_scene(tmp_path)[0]
    with pytest.raises(PTError, match="not PNG"):
        gltf.load_gltf(p, use_pil=False)  # the JPEG needs a decoder
    bad = tmp_path / "bad.gltf"
    bad.write_text("{\"asset\": [1, 2,}")
    with pytest.raises(PTError, match="json"):
        gltf.load_gltf(bad)


def test_scene_round_trip_through_gltf(tmp_path):
    """A textured scene written as glTF loads back with identical geometry, materials (fp32),
    texture ids, transforms and texels."""
    from gltf_export import scene_to_gltf
    from optixpathtracer_amd import scenes

    f = np.float32
    sc = scenes.textured_scene("conductor")
    back = gltf.load_gltf(scene_to_gltf(sc, tmp_path))
    assert [m.name for m in back.meshes] == [m.name for m in sc.meshes]
    for a, b in zip(sc.meshes, back.meshes):
        np.testing.assert_array_equal(a.vertices, b.vertices)
        np.testing.assert_array_equal(a.normals, b.normals)
        np.testing.assert_array_equal(a.indices, b.indices)
        assert (a.texcoords is None) == (b.texcoords is None)
        if a.texcoords is not None:
            np.testing.assert_array_equal(a.texcoords, b.texcoords)
        assert (a.albedo_tex, a.normal_tex, a.metal_rough_tex) == (b.albedo_tex, b.normal_tex, b.metal_rough_tex)
        np.testing.assert_array_equal(np.asarray(a.albedo, f), np.asarray(b.albedo, f))
        assert f(a.metallic) == f(b.metallic) and f(a.roughness) == f(b.roughness)
        np.testing.assert_array_equal(np.asarray(a.model, f).ravel(), b.model.ravel())
    for t0, t1 in zip(sc.textures, back.textures):
        np.testing.assert_array_equal(t0, t1)


def _minimal(tmp_path, mutate):
    """A one-triangle glTF with an embedded buffer, mutated by `mutate(doc)` before writing."""
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32).tobytes()
    i = np.array([0, 1, 2], np.uint32).tobytes()
    buf = v + i
    doc = {
        "asset": {"version": "2.0"}, "scene": 0, "scenes": [{"nodes": [0]}],
        "nodes": [{"mesh": 0, "children": []}],
        "meshes": [{"primitives": [{"attributes": {"POSITION": 0}, "indices": 1}]}],
        "buffers": [{"byteLength": len(buf),
                     "uri": "data:application/octet-stream;base64," + base64.b64encode(buf).decode()}],
        "bufferViews": [{"buffer": 0, "byteOffset": 0, "byteLength": 36},
                        {"buffer": 0, "byteOffset": 36, "byteLength": 12}],
        "accessors": [{"bufferView": 0, "componentType": 5126, "count": 3, "type": "VEC3"},
                      {"bufferView": 1, "componentType": 5125, "count": 3, "type": "SCALAR"}],
        "textures": [], "images": [],
    }
    mutate(doc)
    p = tmp_path / "m.gltf"
    p.write_text(json.dumps(doc))
    return p


MALFORMED = {
    "huge-count": lambda d: d["accessors"][0].update(count=1e18),
    "wrapping-count": lambda d: d["accessors"][0].update(count=2 ** 62),
    "huge-stride": lambda d: d["bufferViews"][0].update(byteStride=2 ** 40),
    "small-stride": lambda d: d["bufferViews"][0].update(byteStride=4),
    "negative-offset": lambda d: d["accessors"][0].update(byteOffset=-8),
    "fractional-accessor": lambda d: d["meshes"][0]["primitives"][0]["attributes"].update(POSITION=0.5),
    "accessor-past-end": lambda d: d["meshes"][0]["primitives"][0]["attributes"].update(POSITION=7),
    "bufferview-past-end": lambda d: d["accessors"][0].update(bufferView=9),
    "buffer-past-end": lambda d: d["bufferViews"][0].update(buffer=3),
    "string-node": lambda d: d["scenes"][0].update(nodes=["0"]),
    "child-past-end": lambda d: d["nodes"][0].update(children=[5]),
    "negative-mesh": lambda d: d["nodes"][0].update(mesh=-1e300),
    "image-bufferview-past-end": lambda d: (d["textures"].append({"source": 0}),
                                            d["images"].append({"bufferView": 40})),
    "image-bad-buffer": lambda d: (d["textures"].append({"source": 0}), d["images"].append({"bufferView": 0}),
                                   d["bufferViews"][0].update(buffer=-1)),
    "texture-without-image": lambda d: d["textures"].append({"source": 2 ** 53}),
    "nan-bytelength": lambda d: d["buffers"][0].update(byteLength=-1),
}


@pytest.mark.parametrize("name", sorted(MALFORMED))
def test_load_gltf_rejects_malformed(tmp_path, name):
    """ADVICE round 1 (pt_gltf.cpp:692,806): untrusted indices, counts, offsets and strides are
    bounds-checked without overflow, so a malformed file is an error status, never a crash."""
    p = _minimal(tmp_path, MALFORMED[name])
    with pytest.raises(PTError):
        gltf.load_gltf(p)


def test_minimal_gltf_loads(tmp_path):
    sc = gltf.load_gltf(_minimal(tmp_path, lambda d: None))
    assert sc.n_triangles == 1


def _same_scene(a, b):
    assert len(a.meshes) == len(b.meshes) and len(a.textures) == len(b.textures)
    for ma, mb in zip(a.meshes, b.meshes):
        np.testing.assert_array_equal(np.asarray(ma.vertices, np.float32), mb.vertices)
        np.testing.assert_array_equal(np.asarray(ma.indices, np.int32), mb.indices)
        for fa, fb in ((ma.normals, mb.normals), (ma.texcoords, mb.texcoords)):
            assert (fa is None) == (fb is None)
            if fa is not None:
                np.testing.assert_array_equal(np.asarray(fa, np.float32), fb)
        np.testing.assert_array_equal(np.asarray(ma.model, np.float32), mb.model)
        assert np.float32(ma.metallic) == np.float32(mb.metallic)
        assert np.float32(ma.roughness) == np.float32(mb.roughness)
        np.testing.assert_array_equal(np.float32(ma.albedo), np.float32(mb.albedo))
        assert (ma.albedo_tex, ma.normal_tex, ma.metal_rough_tex) == (mb.albedo_tex, mb.normal_tex, mb.metal_rough_tex)
        assert ma.name == mb.name
    for ta, tb in zip(a.textures, b.textures):
        np.testing.assert_array_equal(ta, tb)


@pytest.mark.parametrize("name", ["textured_conductor", "sponza_class", "sponza_textured"])
def test_write_glb_round_trip(tmp_path, name):
    """the procedural scenes written as one .glb (gltf.write_glb, embedded
    PNG textures) and read back by the C++ loader (pt_model_load_gltf, ModelLoader::LoadModel's
    counterpart) give the same meshes, materials and textures bit for bit -- at full size for the
    250k-triangle atria (configs[4]), so bench.py --config 5 / 5t render the loaded scenes."""
    from optixpathtracer_amd import gltf, scenes

    sc = scenes.make_scene(name)
    loaded, ms, size = gltf.load_scene_glb(sc, tmp_path)
    assert size > 0 and ms > 0
    _same_scene(sc, loaded)
    assert loaded.n_triangles == sc.n_triangles and loaded.material_mode == sc.material_mode
