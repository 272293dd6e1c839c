#!/usr/bin/env python3
"""Render a scene through the C ABI and save the accumulated sum image (.npy), for bit-exact
A/B checks of kernel variants (select the library with PTAMD_LIB):

    PTAMD_LIB=... python tools/render_npy.py OUT.npy [--scene S] [--width W] [--height H] [--spp N]
    python tools/render_npy.py --compare A.npy B.npy
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--scene", default="sphere_box_layered")
    ap.add_argument("--width", type=int, default=480)
    ap.add_argument("--height", type=int, default=270)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--kernel", type=int, default=2)
    a = ap.parse_args()
    if a.compare:
        x, y = (np.load(p) for p in a.compare)
        same = x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
        diff = float(np.max(np.abs(x.astype(np.float64) - y))) if x.shape == y.shape else float("nan")
        print(f"bit-identical={same} max_abs_diff={diff:.3e} {a.compare[0]} {a.compare[1]}")
        sys.exit(0 if same else 1)
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(a.scene)
    r = setup_renderer(sc, a.width, a.height, a.depth, kernel=a.kernel)
    r.accum_clear()
    r.render_frames(1, a.spp)
    img = r.accum()
    r.close()
    np.save(a.out, img)
    print(f"{a.out}: mean={float(img.mean()) / a.spp:.6f}")


if __name__ == "__main__":
    main()
