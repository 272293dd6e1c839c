#!/usr/bin/env python3
"""How often k_shade_nee's waves leave the layered walk's compile-time path (probe build only).

    PTAMD_LIB=optixpathtracer_amd/_variants/lib_neeprobe.so python tools/nee_probe.py --scene sponza_class

The probe library is built with -DPT_NEE_PROBE=1 (tools/build_variants.sh neeprobe
"-DPT_NEE_PROBE=1"): k_shade_nee then counts, with traversal statistics off, the waves that run
the layered walk, those of them with a lane whose light lies across the shading plane (the
run-time walk, layered_f_split) and those holding both top-interface kinds.  The counts share
the coherence counters, so they are read through pt_get_trace_coherence."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza_class")
    ap.add_argument("--spp", type=int, default=128)
    a = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first, as bench.py)

    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(a.scene)
    r = setup_renderer(sc, 1920, 1080, 8)
    r.stats_reset()
    r.accum_clear()
    r.render_frames(1, a.spp)
    h = r.trace_coherence()
    r.close()
    waves = max(1, h["d2"])
    print(json.dumps({"scene": a.scene, "spp": a.spp, "layered_waves": h["d2"],
                      "runtime_walk_waves": h["d1"], "runtime_share": round(h["d1"] / waves, 4),
                      "mixed_top_kind_waves": h["d3_4"], "mixed_top_share": round(h["d3_4"] / waves, 4),
                      "cross_lanes": h["d5_8"], "layered_lanes": h["d9_16"],
                      "cross_lane_share": round(h["d5_8"] / max(1, h["d9_16"]), 5)}))


if __name__ == "__main__":
    main()
