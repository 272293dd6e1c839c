#!/usr/bin/env python3
"""Coherence of the trace kernels' global BVH node loads.

    python tools/coherence_probe.py [--scene sphere_box_diffuse] [--spp 128] [--out FILE]

Renders one 128-frame batch at 1080p depth 8 with traversal statistics on and reports, for the
wave steps in which lanes load a BVH4 node from global memory (not from the LDS-staged top
levels), how many distinct nodes the lanes load (pt_get_trace_coherence).  A wave-uniform
scalar-cache node fetch only pays if steps with <= 2 distinct nodes are common (the bar: 20 %)."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sphere_box_diffuse")
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first, as bench.py)

    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer
    from optixpathtracer_amd.provenance import kernel_sources_sha

    sc = scenes.make_scene(a.scene)
    r = setup_renderer(sc, 1920, 1080, 8)
    r.set_traversal_stats(True)
    r.stats_reset()
    r.accum_clear()
    r.render_frames(1, a.spp)
    h = r.trace_coherence()
    st = r.stats()
    r.close()
    steps = max(1, h["steps"])
    out = {
        "scene": a.scene, "spp": a.spp, "sources_sha": kernel_sources_sha(),
        "what": "wave steps of k_extend / k_trace_pair / k_shadow_vis with global (non-LDS) BVH node loads, "
                "by the number of distinct nodes the wave's lanes load",
        "hist": {k: h[k] for k in ("d1", "d2", "d3_4", "d5_8", "d9_16", "d17_64")},
        "share": {k: round(h[k] / steps, 4) for k in ("d1", "d2", "d3_4", "d5_8", "d9_16", "d17_64")},
        "steps_le2_share": round((h["d1"] + h["d2"]) / steps, 4),
        "lanes_per_step": round(h["lanes"] / steps, 2),
        "global_node_visits": st["nodes_visited"] - st["lds_nodes_visited"],
        "lds_node_share": round(st["lds_nodes_visited"] / max(1, st["nodes_visited"]), 4),
        "rays": st["rays"],
    }
    print(json.dumps(out, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
