"""The exact configuration bench.py times, against the CPU oracle.

bench.py renders 1920x1080 at depth 8 through the library's shipped defaults: the default kernel
(PT_KERNEL_AUTO -> the wavefront), 128-frame batches (pt_set_frames_per_launch's default, lowered
to what the queue budget allows: 89 frames per batch when two streams share the default quarter of
the device memory), auto streams (one for Lambert, Default and Layered, two for Conductor and
Dielectric), the trace kernels' run-time ray pools, and the trace-kernel timing on.  Here the same
renderer state renders 130 frames -- a full batch and a ragged one -- and bands of rows must equal
the oracle's sum over the same frame ids bit for bit (the kernels and the oracle share the path's
arithmetic).  The test asserts the streams and batch size each mode actually ran
(pt_stats last_streams / last_batch_frames).  A second parametrisation keeps round 4's machinery:
64-frame batches forced onto two streams (64 + 64 + 2).

Scenes: configs[1] (Lambert), configs[2] (Default: conductor spheres + layered walls), configs[3]
(i) (Dielectric, lights x20), configs[3] (ii) (Layered) and configs[4] (the 249,740-triangle
Sponza-class atrium, Default mode: the bucketed NEE / sample queues over the big BVH).

Reference: SamplePath devicePrograms.cu:625-664 (the path loop), GlossyDiffuse.h:141-524 (the
layered BSDF of the Default / Layered modes) and OptixView.cpp:232-245 (accumulation in frame
order).
"""
import numpy as np
import pytest

from helpers import gpu_render, oracle_render

pytestmark = pytest.mark.gpu

W, H, DEPTH = 1920, 1080, 8
FRAMES = 130  # a full batch and a ragged one at the defaults; 64 + 64 + 2 with 64-frame batches
FIRST = 1
# rows (y0, y1) compared: a band through the spheres and one over the floor / lower spheres
BANDS = [(532, 540), (200, 206)]
SCENES = ["sphere_box_diffuse", "sphere_box_conductor", "sphere_box_dielectric20", "sphere_box_layered", "sponza_class"]

_oracle_cache = {}


def _oracle_band(scene_name, sc, y0, y1):
    key = (scene_name, y0, y1)
    if key not in _oracle_cache:
        _oracle_cache[key] = oracle_render(sc, W, H, DEPTH, FIRST, FRAMES, rect=(0, y0, W, y1))
    return _oracle_cache[key]


@pytest.mark.parametrize("machinery", ["defaults", "fpl64x2"])
@pytest.mark.parametrize("scene_name", SCENES)
def test_timed_configuration_bands_bit_exact(scene_name, machinery):
    from optixpathtracer_amd import scenes

    sc = scenes.make_scene(scene_name)
    if machinery == "defaults":
        img, st = gpu_render(sc, W, H, DEPTH, FIRST, FRAMES, kernel_timing=True)
        two = sc.material_mode in (2, 3)  # auto streams: Conductor and Dielectric take two
        assert st["last_streams"] == (2 if two else 1), st["last_streams"]
        # 128 frames unless the queue budget (default: a quarter of the device memory, all
        # streams together) holds fewer; pt_stats reports both
        per_frame = 208 * W * H
        fit = max(1, int(st["queue_budget"] // (st["last_streams"] * (per_frame + (1 << 16)))))
        assert st["last_batch_frames"] in (min(128, fit), min(128, fit + 1)), (st["last_batch_frames"], fit)
        assert st["queue_bytes"] <= st["queue_budget"]
        nbatch = -(-FRAMES // st["last_batch_frames"])
    else:
        img, st = gpu_render(sc, W, H, DEPTH, FIRST, FRAMES, frames_per_launch=64, streams=2, kernel_timing=True)
        assert st["last_streams"] == 2 and st["last_batch_frames"] == 64
        nbatch = 3
    assert st["samples"] == W * H * FRAMES
    assert np.isfinite(img).all()
    # fused modes trace depth + 1 times per batch, Default / Layered depth times
    per_batch = DEPTH if sc.material_mode in (0, 4) else DEPTH + 1
    assert st["trace_kernel_launches"] == nbatch * per_batch
    for y0, y1 in BANDS:
        ref, segs = _oracle_band(scene_name, sc, y0, y1)
        assert segs > (y1 - y0) * W * FRAMES  # paths bounce
        band = img[y0:y1]
        diff = band != ref[y0:y1]
        assert not diff.any(), (f"{scene_name} ({machinery}) rows {y0}..{y1 - 1}: {int(diff.any(axis=-1).sum())} "
                                f"pixels differ, max |d| {float(np.max(np.abs(band - ref[y0:y1])))}")
