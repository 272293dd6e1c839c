#!/usr/bin/env python3
"""The reference's one-sample-per-call loop (bench.py value_reference_loop) for render-ahead
sizes and time budgets: calls/s as Msamples/s, and the latency of the first call after a camera
move in the steady state (median of 3).

    python tools/refloop_probe.py [--ahead 64,128] [--budget 50,100,0] [--calls 1024]"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sphere_box_diffuse")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--ahead", default="64,128")
    ap.add_argument("--budget", default="50,100,0")
    ap.add_argument("--calls", type=int, default=1024)
    a = ap.parse_args()
    import torch  # noqa: F401  (device init order as bench.py)
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(a.scene)
    r = setup_renderer(sc, a.width, a.height, a.depth)
    buf = lambda: np.empty((a.height, a.width, 3), np.float32)  # noqa: E731 (a fresh host array per call)
    for ahead in [int(x) for x in a.ahead.split(",")]:
        for budget in [float(x) for x in a.budget.split(",")]:
            r.set_render_ahead(ahead)
            r.set_render_ahead_budget(budget)
            r.SetCameraBlender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg)
            r.frame_id = 0
            r.Render()
            t = time.perf_counter()
            for _ in range(a.calls):
                r.Render(buf())
            r.synchronize()
            e = time.perf_counter() - t
            lat = []
            for k in range(3):
                r.SetCameraBlender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg)
                r.frame_id = 0
                for _ in range(200):
                    r.Render(buf())
                pos = np.asarray(sc.camera_blender_pos, np.float32) + np.float32(1e-3 * (k + 1))
                r.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)
                t = time.perf_counter()
                r.Render(buf())
                lat.append(time.perf_counter() - t)
            r.synchronize()
            print(json.dumps({"ahead": ahead, "budget_ms": budget, "calls": a.calls,
                              "msamples_s": round(a.width * a.height * a.calls / e / 1e6, 2),
                              "ms_per_call": round(e / a.calls * 1e3, 3),
                              "first_call_after_change_ms": round(1e3 * statistics.median(lat), 3)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
