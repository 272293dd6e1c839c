#!/usr/bin/env python3
"""Look-ahead cancellation probe: ramp pt_render to the 64-frame
look-ahead, move the camera while the speculative batch is in flight, and time the next call
against a one-frame call.   python tools/cancel_probe.py [--scene sphere_box_diffuse] [--width 1920]"""
import argparse
import json
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
    ap.add_argument("--budget", type=float, default=50.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--calls", type=int, default=70, help="calls after the synchronising stats read")
    ap.add_argument("--mode", type=int, default=-1)
    a = ap.parse_args()
    import torch  # noqa: F401  (device init order as bench.py)
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(a.scene)
    r = setup_renderer(sc, a.width, a.height, a.depth)
    r.set_render_ahead_budget(a.budget)
    if a.mode >= 0:
        r.set_material_mode(a.mode)
    buf = np.empty((a.height, a.width, 3), np.float32)
    out = {"scene": a.scene, "budget_ms": a.budget, "rounds": []}
    for k in range(a.rounds):
        r.SetCameraBlender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg)
        r.frame_id = 0
        t = time.perf_counter()
        for _ in range(200):
            r.Render(buf)
        steady = (time.perf_counter() - t) / 200
        s0 = r.stats()  # synchronises: the look-ahead batch in flight completes
        for _ in range(a.calls):  # into the next look-ahead batch without a synchronising call
            r.Render(buf)
        pos = np.asarray(sc.camera_blender_pos, np.float32) + np.float32(1e-3 * (k + 1))
        t = time.perf_counter()
        r.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)
        t1 = time.perf_counter()
        r.Render(buf)
        t2 = time.perf_counter()
        s1 = r.stats()
        out["rounds"].append({"steady_ms_per_call": round(steady * 1e3, 3), "set_camera_ms": round((t1 - t) * 1e3, 3),
                              "first_call_after_change_ms": round((t2 - t1) * 1e3, 3),
                              "cancelled": s1["look_ahead_cancelled"] - s0["look_ahead_cancelled"],
                              "rendered_ahead": s1["frames_rendered_ahead"], "served": s1["frames_served_ahead"]})
    r.set_render_ahead(1)
    r.Render(buf)
    t = time.perf_counter()
    for _ in range(20):
        r.Render(buf)
    out["one_frame_ms_per_call"] = round((time.perf_counter() - t) / 20 * 1e3, 3)
    print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
