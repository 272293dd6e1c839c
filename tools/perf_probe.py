#!/usr/bin/env python3
"""Quick performance probe: kernel time, Msamples/s and traversal statistics per config.

    python tools/perf_probe.py [--scene sphere_box_diffuse] [--spp 16] [--modes 1] [--stats]

Every run prints the device identity first, and every result line carries the per-kernel split
of the render (pt_set_kernel_timing: trace kernels and the dominant shading kernel, summed HIP
event time per launch), so an outlier run can be attributed to a kernel without a rerun
(VERDICT round 3 item 6).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sphere_box_diffuse")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--modes", default="")
    ap.add_argument("--kernels", default="2", help="0 = megakernel, 1 = wavefront, 2 = auto")
    ap.add_argument("--fpl", default="8")
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--builders", default="0", help="0 = default (SAH), 1 = LBVH, 2 = SAH, 3 = PLOC")
    ap.add_argument("--streams", default="", help="wavefront streams to sweep (pt_set_wavefront_streams)")
    a = ap.parse_args()
    import os
    import socket

    import torch  # before libptamd holds the device (torch's own HIP runtime must see it first)

    p = torch.cuda.get_device_properties(0)
    print(json.dumps({"device": p.name, "gcn_arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count,
                      "host": socket.gethostname(), "pid": os.getpid(),
                      "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")}),
          flush=True)
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(a.scene)
    modes = [int(m) for m in a.modes.split(",")] if a.modes else [sc.material_mode]
    for builder in [int(b) for b in a.builders.split(",")]:
        t0 = time.time()
        r = setup_renderer(sc, a.width, a.height, a.depth, bvh_builder=builder)
        r.set_kernel_timing(True)
        st = r.stats()
        print(json.dumps({"scene": a.scene, "tris": sc.n_triangles, "builder": builder,
                          "setup_s": round(time.time() - t0, 2),
                          "bvh_ms": round(st["bvh_build_ms"], 3), "bvh_nodes": st["bvh_nodes"],
                          "bvh_depth": st["bvh_depth"]}), flush=True)
        for kernel in [int(k) for k in a.kernels.split(",")]:
            for mode in modes:
                for fpl, nstr in [(int(f), int(x)) for f in a.fpl.split(",") for x in (a.streams.split(",") if a.streams else ["0"])]:
                    if nstr:
                        r.set_wavefront_streams(nstr)
                    r.set_kernel(kernel)
                    r.set_material_mode(mode)
                    r.set_frames_per_launch(fpl)
                    r.accum_clear()
                    r.render_frames(1, min(a.spp, fpl))  # warm (also sizes the wavefront queues)
                    r.synchronize()
                    best = None
                    runs = []
                    for rep in range(a.repeat):
                        r.stats_reset()
                        t0 = time.perf_counter()
                        r.render_frames(1 + 1000 * rep, a.spp)
                        r.synchronize()
                        ms = (time.perf_counter() - t0) * 1e3  # wall clock, as bench.py
                        s = r.stats()
                        tl, sl = max(1, s["trace_kernel_launches"]), max(1, s["shade_kernel_launches"])
                        # per-kernel split of this run: summed event windows per launch (with two
                        # streams a window includes the time it shares the GPU with the other stream)
                        runs.append({"wall_ms": round(ms, 2), "trace_ms": round(s["trace_kernel_ms"], 2),
                                     "trace_ms_per_launch": round(s["trace_kernel_ms"] / tl, 4),
                                     "shade_ms": round(s["shade_kernel_ms"], 2),
                                     "shade_ms_per_launch": round(s["shade_kernel_ms"] / sl, 4)})
                        best = ms if best is None else min(best, ms)
                    samples = a.width * a.height * a.spp
                    out = {"kernel": kernel, "mode": mode, "fpl": fpl, **({"streams": nstr} if nstr else {}),
                           "wall_ms": round(best, 2),
                           "msamples_s": round(samples / best / 1e3, 2),
                           "segments_per_sample": round(s["segments"] / samples, 4),
                           "runs": runs}
                    if a.stats:
                        r.set_traversal_stats(True)
                        r.stats_reset()
                        r.render_frames(1, max(1, a.spp // 4))
                        s = r.stats()
                        r.set_traversal_stats(False)
                        rays = max(1, s["rays"])
                        out.update({"nodes_per_ray": round(s["nodes_visited"] / rays, 2),
                                    "tris_per_ray": round(s["tri_tests"] / rays, 2),
                                    "rays_per_sample": round(rays / (a.width * a.height * max(1, a.spp // 4)), 3),
                                    "stack_overflows": s["stack_overflows"]})
                        ws = max(1, s["wave_steps"])
                        out.update({"wave_steps_per_ray": round(s["wave_steps"] * 64 / rays, 2),
                                    "active_frac": round(s["wave_active_lanes"] / (64 * ws), 3),
                                    "node_util": round(s["nodes_visited"] / (64 * max(1, s["wave_node_steps"])), 3),
                                    "tri_util": round(s["tri_tests"] / (64 * max(1, s["wave_tri_steps"])), 3),
                                    "node_step_frac": round(s["wave_node_steps"] / ws, 3),
                                    "tri_step_frac": round(s["wave_tri_steps"] / ws, 3),
                                    "refill_frac": round(s["wave_refills"] / ws, 3),
                                    # raw counters (a PT_CYCLE_PROBE build puts shader cycles per section here)
                                    "raw": {k: s[k] for k in ("wave_steps", "wave_active_lanes", "wave_node_steps",
                                                              "wave_tri_steps", "wave_refills", "rays")}})
                        # k_trace_pair per launch (the traffic classes of DESIGN.md §5): its rays, of
                        # them shadow rays, unoccluded shadow rays; the node visits of all trace
                        # kernels that loaded from global memory and their triangle tests
                        pl = max(1, s["pair_kernel_launches"])
                        out["pair_per_launch"] = {
                            "rays": s["pair_kernel_rays"] / pl, "shadow_rays": s["pair_kernel_shadow_rays"] / pl,
                            "unoccluded": s["nee_unoccluded"] / pl, "launches": s["pair_kernel_launches"],
                            "all_trace_rays": s["rays"], "global_node_visits": s["nodes_visited"] - s["lds_nodes_visited"],
                            "tri_tests": s["tri_tests"]}
                    print(json.dumps(out), flush=True)
        r.close()


if __name__ == "__main__":
    main()
