#!/usr/bin/env python3
"""Closest-hit order-independence check of the CPU oracle (diagnostic, test infrastructure).

Renders a band of a BASELINE config with the oracle while every closest-hit trace is repeated
without culling boxes by the running best t (only by [tmin, tmax]), and counts the traces whose
answers differ.  Round 1's oracle disagreed on 1 trace in 62.5 M of the config-5 band
(sponza_class rows 540..1079, 15 spp): a grazing ray accepted by Moller-Trumbore outside the
triangle's own box.  With the hit-acceptance rule (pt_oracle.c tri_accept) the count is 0.
    python tools/cullcheck.py SCENE Y0 Y1 SPP [THREADS]
"""
import ctypes as C
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from optixpathtracer_amd import scenes  # noqa: E402
from oracle.oracle import OracleScene, load  # noqa: E402

name, y0, y1, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
threads = int(sys.argv[5]) if len(sys.argv) > 5 else 8
sc = scenes.make_scene(name)
lib = load()
lib.orc_set_cull_check.argtypes = [C.c_int32]
lib.orc_cull_check_stats.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_float)]
o = OracleScene(sc)
lp = o.launch(1920, 1080, 8)
lib.orc_set_cull_check(1)
t = time.time()
o.render(lp, 1, spp, rect=(0, y0, 1920, y1), threads=threads)
st = (C.c_uint64 * 2)()
first = (C.c_float * 16)()
lib.orc_cull_check_stats(st, first)
lib.orc_set_cull_check(0)
print(f"{name} rows {y0}..{y1} spp {spp}: closest-hit traces {st[0]}, culled != exhaustive {st[1]}, "
      f"{time.time() - t:.1f} s")
if st[1]:
    print("first mismatch (o, d, tmin, tmax, prim, t, prim_exh, t_exh, u, v, u_exh, v_exh):", list(first))
