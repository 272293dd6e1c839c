#!/usr/bin/env python3
"""Locate GPU-vs-oracle differences of one BASELINE config band (debug aid).
    python tools/diffpix.py SCENE Y0 Y1 SPP [MODE]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle.oracle import OracleScene  # noqa: E402
from optixpathtracer_amd import scenes  # noqa: E402
from optixpathtracer_amd.renderer import setup_renderer  # noqa: E402

scene, y0, y1, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
sc = scenes.make_scene(scene)
w, h, depth = 1920, 1080, 8
r = setup_renderer(sc, w, h, depth)
r.accum_clear()
r.render_frames(1, spp)
g = r.accum()[y0:y1]
o = OracleScene(sc)
lp = o.launch(w, h, depth)
ref, _ = o.render(lp, 1, spp, rect=(0, y0, w, y1))
ref = ref[y0:y1]
d = np.argwhere(g != ref)
print("differing values:", len(d))
for yy, xx, c in d[:10]:
    print("pixel", xx, y0 + yy, "ch", c, "gpu", repr(g[yy, xx, c]), "oracle", repr(ref[yy, xx, c]))
    # per-frame values of that pixel
    for f in range(1, spp + 1):
        r.accum_clear(); r.render_frames(f, 1)
        gv = r.accum()[y0 + yy, xx]
        ov, _ = o.render(lp, f, 1, rect=(xx, y0 + yy, xx + 1, y0 + yy + 1))
        ov = ov[y0 + yy, xx]
        if not np.array_equal(gv, ov):
            print("  frame", f, "gpu", gv.tolist(), "oracle", ov.tolist())
    break
