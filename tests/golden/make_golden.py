#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU oracle (oracle/liboracle.so).

The reference (Damo12320/OptixPathtracer) cannot be built or run here (OptiX/CUDA only;
host compilation of its headers was denied), so these vectors are the
build's own CPU restatement frozen as data: they pin the oracle against regressions and
give the GPU tests a committed target.  The restatement itself is pinned by the
reference's own known answers (tests/test_oracle.py: TEA/LCG constants, CosTheta KAT,
furnace bounds of UnitTests/SpherGeom_Test.cpp).

    python tests/golden/make_golden.py      # rewrites tests/golden/golden.npz
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import oracle as O  # noqa: E402
from optixpathtracer_amd import scenes  # noqa: E402

OUT = Path(__file__).resolve().parent / "golden.npz"

TEA_INPUTS = [(0, 0), (1, 1), (0xFFFFFFFF, 0xFFFFFFFF), (1920 * 540 + 960, 1), (12345, 678), (2730713777, 42)]
RND_SEEDS = [0, 1, 2730713777, 0xDEADBEEF]
BSDF_MODELS = ["lambert", "conductor", "dielectric", "layered"]
ROUGHNESS = [0.0, 0.2, 0.5, 1.0]


def directions(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d.astype(np.float32)


def make():
    g = {}
    g["tea_in"] = np.array(TEA_INPUTS, dtype=np.uint32)
    g["tea_out"] = np.array([O.tea16(a, b) for a, b in TEA_INPUTS], dtype=np.uint32)
    seqs, finals = [], []
    for s in RND_SEEDS:
        v, f = O.rnd_seq(s, 16)
        seqs.append(v)
        finals.append(f)
    g["rnd_seeds"] = np.array(RND_SEEDS, dtype=np.uint32)
    g["rnd_seq"] = np.array(seqs, dtype=np.float32)
    g["rnd_final"] = np.array(finals, dtype=np.uint32)

    # cameras: Scene1 at two sizes, Scene2 at 1080p
    cams = []
    for (pos, rot), (w, h) in [(scenes.SCENE1_CAMERA, (1920, 1080)), (scenes.SCENE1_CAMERA, (256, 256)),
                               (scenes.SCENE2_CAMERA, (1920, 1080))]:
        p, iv, ip = O.camera_from_blender(pos, rot, 40.0, w, h)
        cams.append(np.concatenate([p, iv, ip]))
    g["camera"] = np.array(cams, dtype=np.float32)

    # BSDF tuples: (model, roughness, seed, wo, wi) -> sample (ok, 8 floats, seed') and eval (3 floats, seed')
    wos = directions(12, 7)
    wis = directions(12, 8)
    rows_in, rows_sample, rows_eval = [], [], []
    albedo = np.array([0.7, 0.4, 0.2], np.float32)
    for mi, m in enumerate(BSDF_MODELS):
        for r in ROUGHNESS:
            for k in range(len(wos)):
                seed = 1000 * mi + 17 * k + int(r * 100)
                ok, out, s2 = O.bsdf_sample(m, seed, albedo, r, wos[k])
                ev, s3 = O.bsdf_eval(m, seed, albedo, r, wos[k], wis[k])
                rows_in.append([mi, r, seed, *wos[k], *wis[k]])
                rows_sample.append([float(ok), *out, float(s2)])
                rows_eval.append([*ev, float(s3)])
    g["bsdf_in"] = np.array(rows_in, dtype=np.float64)
    g["bsdf_sample"] = np.array(rows_sample, dtype=np.float64)
    g["bsdf_eval"] = np.array(rows_eval, dtype=np.float64)
    g["bsdf_albedo"] = albedo

    # tiny-scene images: 32x24, depth 4, frame ids 1..4, every variant (sum over frames)
    imgs = []
    for v in scenes.VARIANTS:
        sc = scenes.tiny_scene(v)
        o = O.OracleScene(sc)
        lp = o.launch(32, 24, 4)
        img, segs = o.render(lp, 1, 4, threads=1)
        imgs.append(img)
        o.close()
    g["tiny_variants"] = np.array(list(scenes.VARIANTS))
    g["tiny_images"] = np.array(imgs, dtype=np.float32)

    # textured tiny scene: albedo (sRGB, alpha cut-out), normal and
    # metal-rough maps; Lambert and Default modes
    timgs = []
    for v in ("diffuse", "conductor"):
        sc = scenes.textured_scene(v)
        o = O.OracleScene(sc)
        lp = o.launch(32, 24, 4)
        img, _ = o.render(lp, 1, 4, threads=1)
        timgs.append(img)
        o.close()
    g["textured_variants"] = np.array(["diffuse", "conductor"])
    g["textured_images"] = np.array(timgs, dtype=np.float32)
    # texture fetch: (texture, x, y, srgb) -> rgba over the checker texture
    sc = scenes.textured_scene("diffuse")
    pts = np.random.default_rng(11).uniform(-2.0, 3.0, size=(64, 2)).astype(np.float32)
    g["tex_pts"] = pts
    g["tex_rgba"] = np.array([[O.tex_sample(sc.textures[0], x, y, s) for x, y in pts] for s in (False, True)],
                             dtype=np.float32)
    return g


if __name__ == "__main__":
    g = make()
    np.savez_compressed(OUT, **g)
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")
