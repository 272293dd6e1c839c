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


def _flip_numpy(ref, test, ppd=67.0):
    """Independent restatement of LDR-FLIP with full 2-D kernels (edge-clamped borders)."""
    M = np.array([[10135552 / 24577794, 8788810 / 24577794, 4435075 / 24577794],
                  [2613072 / 12288897, 8788810 / 12288897, 887015 / 12288897],
                  [1425312 / 73733382, 8788810 / 73733382, 70074185 / 73733382]])
    Minv = np.array([[3.241003275, -1.537398934, -0.498615861], [-0.969224334, 1.875930071, 0.041554224],
                     [0.055639423, -0.204011202, 1.057148933]])
    wp = M @ np.ones(3)

    def s2l(x):
        return np.where(x > 0.04045, ((x + 0.055) / 1.055) ** 2.4, x / 12.92)

    def l2s(x):
        return np.where(x > 0.0031308, 1.055 * np.power(np.maximum(x, 0), 1 / 2.4) - 0.055, 12.92 * x)

    def ycx(img):
        rgb = s2l(l2s(np.clip(np.nan_to_num(img.astype(np.float64)), 0, 1)))
        xyz = rgb @ M.T / wp
        return np.stack([116 * xyz[..., 1] - 16, 500 * (xyz[..., 0] - xyz[..., 1]), 200 * (xyz[..., 1] - xyz[..., 2])],
                        -1)

    def conv(img, k):
        r = k.shape[0] // 2
        p = np.pad(img, r, mode="edge")
        out = np.zeros_like(img)
        for dy in range(-r, r + 1):
            for dx in range(-r, r + 1):
                out += k[dy + r, dx + r] * p[r + dy:r + dy + img.shape[0], r + dx:r + dx + img.shape[1]]
        return out

    def hunt(rgb):
        xyz = rgb @ M.T / wp
        d = 6 / 29
        f = np.where(xyz > d ** 3, np.cbrt(xyz), xyz / (3 * d * d) + 4 / 29)
        L = 116 * f[..., 1] - 16
        return np.stack([L, 0.01 * L * 500 * (f[..., 0] - f[..., 1]), 0.01 * L * 200 * (f[..., 1] - f[..., 2])], -1)

    r = int(np.ceil(3 * np.sqrt(0.04 / (2 * np.pi ** 2)) * ppd))
    x = np.arange(-r, r + 1) / ppd
    z = x[None, :] ** 2 + x[:, None] ** 2
    csf = [(1, 0.0047, 0, 1e-5), (1, 0.0053, 0, 1e-5), (34.1, 0.04, 13.5, 0.025)]
    ks = []
    for a1, b1, a2, b2 in csf:
        g = a1 * np.sqrt(np.pi / b1) * np.exp(-np.pi ** 2 * z / b1) + a2 * np.sqrt(np.pi / b2) * np.exp(-np.pi ** 2 * z / b2)
        ks.append(g / g.sum())
    sd = 0.5 * 0.082 * ppd
    rf = int(np.ceil(3 * sd))
    xs = np.arange(-rf, rf + 1, dtype=np.float64)
    X, Y = np.meshgrid(xs, xs)
    g = np.exp(-(X ** 2 + Y ** 2) / (2 * sd * sd))
    e = -X * g
    e = e / e[e > 0].sum()
    pnt = (X ** 2 / sd ** 2 - 1) * g
    pnt = np.where(pnt > 0, pnt / pnt[pnt > 0].sum(), pnt / -pnt[pnt < 0].sum())
    labs, feats = [], []
    for img in (ref, test):
        c = ycx(img)
        f = np.stack([conv(c[..., k], ks[k]) for k in range(3)], -1)
        yy = (f[..., 0] + 16) / 116
        xyz = np.stack([f[..., 1] / 500 + yy, yy, yy - f[..., 2] / 200], -1) * wp
        labs.append(hunt(np.clip(xyz @ Minv.T, 0, 1)))
        yn = (c[..., 0] + 16) / 116
        feats.append((np.hypot(conv(yn, e), conv(yn, e.T)), np.hypot(conv(yn, pnt), conv(yn, pnt.T))))
    hg, hb = hunt(np.array([0.0, 1.0, 0.0])), hunt(np.array([0.0, 0.0, 1.0]))
    cmax = (abs(hg[0] - hb[0]) + np.hypot(hg[1] - hb[1], hg[2] - hb[2])) ** 0.7
    d = labs[0] - labs[1]
    dc = (np.abs(d[..., 0]) + np.hypot(d[..., 1], d[..., 2])) ** 0.7
    ec = np.where(dc < 0.4 * cmax, 0.95 / (0.4 * cmax) * dc, 0.95 + (dc - 0.4 * cmax) / (cmax - 0.4 * cmax) * 0.05)
    df = np.maximum(np.abs(feats[0][0] - feats[1][0]), np.abs(feats[0][1] - feats[1][1]))
    return ec ** (1 - np.sqrt(df / np.sqrt(2)))


def test_flip_matches_numpy_restatement():
    rng = np.random.default_rng(4)
    ref = rng.uniform(0, 1.2, size=(20, 24, 3)).astype(np.float32)
    test = np.clip(ref + rng.normal(0, 0.08, ref.shape), 0, 2).astype(np.float32)
    v, emap = imageio.flip(ref, test, pixels_per_degree=20.0, error_map=True)
    want = _flip_numpy(ref, test, ppd=20.0)
    np.testing.assert_allclose(emap, want, rtol=2e-4, atol=2e-5)
    assert v == pytest.approx(float(want.mean()), rel=1e-4)


def test_flip_properties():
    rng = np.random.default_rng(5)
    a = rng.uniform(0, 1, size=(32, 40, 3)).astype(np.float32)
    assert imageio.flip(a, a) == 0.0
    small = imageio.flip(a, np.clip(a + rng.normal(0, 0.02, a.shape), 0, 1).astype(np.float32))
    big = imageio.flip(a, np.clip(a + rng.normal(0, 0.2, a.shape), 0, 1).astype(np.float32))
    assert 0.0 < small < big <= 1.0
    bw = imageio.flip(np.zeros_like(a), np.ones_like(a))
    assert 0.9 < bw <= 1.0
