"""Image I/O (WriteImage.cpp restated) and the MSE parity metric — CPU only."""
import struct

import numpy as np
import pytest

from optixpathtracer_amd import imageio


def _img(h=5, w=7, seed=0):
    rng = np.random.default_rng(seed)
    return rng.uniform(-0.5, 3.0, size=(h, w, 3)).astype(np.float32)


def test_exr_round_trip_flip_and_nan(tmp_path):
    img = _img()
    img[2, 3, 1] = np.nan
    p = tmp_path / "a.exr"
    imageio.write_exr(p, img)
    back = imageio.read_image(p)
    want = img.copy()
    want[2, 3, :] = 0.0  # WriteImage.cpp:50-53: the whole pixel becomes 0
    np.testing.assert_array_equal(back, want)


def test_exr_layout(tmp_path):
    """Spec-level check: magic, B,G,R float channels, no compression, first scanline = top row."""
    img = _img(3, 4)
    p = tmp_path / "b.exr"
    imageio.write_exr(p, img)
    buf = p.read_bytes()
    assert buf[:4] == bytes([0x76, 0x2F, 0x31, 0x01]) and struct.unpack("<i", buf[4:8])[0] == 2
    assert b"channels\x00chlist\x00" in buf
    ch = buf.index(b"chlist\x00") + 7 + 4
    names = [buf[ch + 18 * k:ch + 18 * k + 1] for k in range(3)]
    assert names == [b"B", b"G", b"R"]
    assert all(struct.unpack("<i", buf[ch + 18 * k + 2:ch + 18 * k + 6])[0] == 2 for k in range(3))
    c = buf.index(b"compression\x00compression\x00") + len(b"compression\x00compression\x00") + 4
    assert buf[c] == 0
    hdr_end = buf.index(b"screenWindowWidth\x00float\x00") + len(b"screenWindowWidth\x00float\x00") + 8 + 1
    off0 = struct.unpack("<Q", buf[hdr_end:hdr_end + 8])[0]
    y, size = struct.unpack("<ii", buf[off0:off0 + 8])
    assert y == 0 and size == 4 * 4 * 3
    b_top = np.frombuffer(buf[off0 + 8:off0 + 8 + 16], dtype="<f4")
    np.testing.assert_array_equal(b_top, img[-1, :, 2])  # row 0 of the file is the top row (flip)


def test_exr_reader_half_channels(tmp_path):
    """An independently assembled half-float R,G,B EXR (as tinyexr/OpenEXR would write it)."""
    w, h = 2, 2
    vals = np.array([[[0.5, 1.0, 2.0], [0.25, 0.0, -1.0]], [[8.0, 0.125, 3.0], [1.5, 4.0, 0.75]]], np.float32)

    def attr(name, typ, payload):
        return name + b"\x00" + typ + b"\x00" + struct.pack("<i", len(payload)) + payload

    chl = b"".join(c + b"\x00" + struct.pack("<i", 1) + b"\x00\x00\x00\x00" + struct.pack("<ii", 1, 1)
                   for c in (b"B", b"G", b"R")) + b"\x00"
    hdr = struct.pack("<ii", 20000630, 2)
    hdr += attr(b"channels", b"chlist", chl)
    hdr += attr(b"compression", b"compression", b"\x00")
    hdr += attr(b"dataWindow", b"box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr(b"displayWindow", b"box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr(b"lineOrder", b"lineOrder", b"\x00")
    hdr += attr(b"pixelAspectRatio", b"float", struct.pack("<f", 1.0))
    hdr += attr(b"screenWindowCenter", b"v2f", struct.pack("<ff", 0, 0))
    hdr += attr(b"screenWindowWidth", b"float", struct.pack("<f", 1.0)) + b"\x00"
    rows = []
    for y in range(h):  # file row y = image row h-1-y (top-down)
        src = vals[h - 1 - y]
        data = b"".join(src[:, c].astype("<f2").tobytes() for c in (2, 1, 0))
        rows.append(struct.pack("<ii", y, len(data)) + data)
    table_end = len(hdr) + 8 * h
    offs, pos = [], table_end
    for r in rows:
        offs.append(pos)
        pos += len(r)
    p = tmp_path / "half.exr"
    p.write_bytes(hdr + b"".join(struct.pack("<Q", o) for o in offs) + b"".join(rows))
    np.testing.assert_array_equal(imageio.read_image(p), vals)


def test_pfm_round_trip(tmp_path):
    img = _img(4, 3, seed=2)
    p = tmp_path / "c.pfm"
    imageio.write_pfm(p, img)
    raw = p.read_bytes()
    assert raw.startswith(b"PF\n3 4\n-1.0\n")
    np.testing.assert_array_equal(imageio.read_image(p), img)


def test_bmp_quantisation(tmp_path):
    img = np.array([[[0.5, 1.5, -1.0], [1.0, 0.0, 0.999]]], np.float32)  # 1 row, 2 px
    p = tmp_path / "d.bmp"
    imageio.write_bmp(p, img)
    buf = p.read_bytes()
    assert buf[:2] == b"BM" and struct.unpack("<i", buf[18:22])[0] == 2 and struct.unpack("<i", buf[22:26])[0] == 1
    px = buf[54:54 + 6]
    assert list(px) == [0, 255, 127, 254, 0, 255]  # BGR, truncated clamp*255 (WriteImage.cpp:17-19)


def test_mse_definition():
    a = np.zeros((2, 2, 3), np.float32)
    b = np.zeros((2, 2, 3), np.float32)
    b[0, 0, 0] = 1.0
    b[1, 1] = 2.0
    assert imageio.mse(a, b) == pytest.approx((1.0 + 3 * 4.0) / 12.0)
    a[1, 1, 2] = np.nan  # a NaN pixel counts as 0 in every channel
    assert imageio.mse(a, b) == pytest.approx((1.0 + 3 * 4.0) / 12.0)
    assert imageio.mse(b, b) == 0.0
