#!/usr/bin/env python3
"""The interactive path a viewer that moves the camera every frame gets: pt_render with
render-ahead off, one 1-spp wavefront batch and one 24.9 MB download per call (OptixView::DrawOptix,
OptixView.cpp:201-210).  Times calls into a fresh host array per call (bench.py's reference loop)
and into one reused array, and prints the trace / shading kernel split of a call.

    [PTAMD_LIB=...] python3 tools/one_frame.py [--scene sphere_box_diffuse] [--calls 64]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sphere_box_diffuse")
    ap.add_argument("--calls", type=int, default=64)
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first, as bench.py)

    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(a.scene)
    r = setup_renderer(sc, 1920, 1080, 8)
    r.set_material_mode(sc.material_mode)
    r.set_render_ahead(1)
    buf = np.empty((1080, 1920, 3), np.float32)
    for _ in range(8):
        r.Render(buf)
    out = {"scene": a.scene, "calls": a.calls}
    for band in (True, False):  # pt_set_band_split: the frame as two row bands on two streams
        r.set_band_split(band)
        best = None
        for _ in range(a.repeat):
            t = time.perf_counter()
            for _ in range(a.calls):
                r.Render(buf)
            r.synchronize()
            ms = (time.perf_counter() - t) / a.calls * 1e3
            best = ms if best is None else min(best, ms)
        out[f"ms_per_call_{'bands' if band else 'one_band'}"] = round(best, 3)
    r.set_band_split(True)
    for kind in ("fresh", "reuse"):
        best = None
        for _ in range(a.repeat):
            t = time.perf_counter()
            for _ in range(a.calls):
                r.Render(np.empty((1080, 1920, 3), np.float32) if kind == "fresh" else buf)
            r.synchronize()
            ms = (time.perf_counter() - t) / a.calls * 1e3
            best = ms if best is None else min(best, ms)
        out[f"ms_per_call_{kind}"] = round(best, 3)
    r.set_kernel_timing(True)
    r.stats_reset()
    for _ in range(16):
        r.Render(buf)
    s = r.stats()
    out["trace_ms_per_call"] = round(s["trace_kernel_ms"] / 16, 3)
    out["shade_ms_per_call"] = round(s["shade_kernel_ms"] / 16, 3)
    r.set_kernel_timing(False)
    # the render alone (no download): pt_render_frames of one frame per call
    r.accum_clear()
    r.synchronize()
    t = time.perf_counter()
    for k in range(a.calls):
        r.render_frames(1 + k, 1)
    r.synchronize()
    out["render_only_ms_per_call"] = round((time.perf_counter() - t) / a.calls * 1e3, 3)
    print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
