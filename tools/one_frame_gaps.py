#!/usr/bin/env python3
"""The interactive path: pt_render with render-ahead off (one 1-spp wavefront batch per call, as a
viewer that moves the camera every frame gets).  Run under rocprofv3 --kernel-trace --stats to
split a call's wall time into kernel time and gaps:

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- python3 tools/one_frame_gaps.py
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from optixpathtracer_amd import scenes  # noqa: E402
from optixpathtracer_amd.renderer import setup_renderer  # noqa: E402

sc = scenes.make_scene(sys.argv[1] if len(sys.argv) > 1 else "sphere_box_diffuse")
r = setup_renderer(sc, 1920, 1080, 8)
r.set_material_mode(sc.material_mode)
r.set_render_ahead(1)
buf = np.empty((1080, 1920, 3), np.float32)
for _ in range(8):
    r.Render(buf)
n = 64
t = time.perf_counter()
for _ in range(n):
    r.Render(buf)
wall = (time.perf_counter() - t) / n * 1e3
print(json.dumps({"scene": sc.name if hasattr(sc, "name") else None, "calls": n, "ms_per_call": round(wall, 3)}))
r.close()
