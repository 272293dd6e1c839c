"""The exact configuration bench.py times, against the CPU oracle.

bench.py renders 1920x1080 at depth 8 through the default kernel (PT_KERNEL_AUTO -> the
wavefront) in 64-frame batches that alternate over two streams (k_shade0_pixel at bounce 0,
k_trace_pair after it, k_accum ordered across the streams by events), with the trace-kernel
timing on.  Here the same renderer state renders 130 frames -- batches of 64, 64 and a ragged 2,
so both streams run and the last batch is partial -- and bands of rows must equal the oracle's
sum over the same frame ids bit for bit (the kernels and the oracle share the path's
arithmetic).  Scenes: configs[1] (Lambert), configs[2] (Default: conductor
spheres + layered walls), configs[3] (i) (Dielectric, lights x20), configs[3] (ii) (Layered) and
configs[4] (the 249,740-triangle Sponza-class atrium, Default mode: the bucketed NEE / sample
queues over the big BVH).

Reference: SamplePath devicePrograms.cu:625-664 (the path loop), GlossyDiffuse.h:141-524 (the
layered BSDF of the Default / Layered modes) and OptixView.cpp:232-245 (accumulation in frame
order).
"""
import numpy as np
import pytest

from helpers import gpu_render, oracle_render

pytestmark = pytest.mark.gpu

W, H, DEPTH = 1920, 1080, 8
FRAMES = 130  # 64 + 64 + 2 frames: three batches over the two wavefront streams
FIRST = 1
# rows (y0, y1) compared: a band through the spheres and one over the floor / lower spheres
BANDS = [(532, 540), (200, 206)]


@pytest.mark.parametrize("scene_name", ["sphere_box_diffuse", "sphere_box_conductor", "sphere_box_dielectric20",
                                        "sphere_box_layered", "sponza_class"])
def test_timed_configuration_bands_bit_exact(scene_name):
    from optixpathtracer_amd import scenes

    sc = scenes.make_scene(scene_name)
    img, st = gpu_render(sc, W, H, DEPTH, FIRST, FRAMES, frames_per_launch=64, streams=2, kernel_timing=True)
    assert st["samples"] == W * H * FRAMES
    assert np.isfinite(img).all()
    # fused modes trace depth + 1 times per batch, Default depth times; 3 batches either way
    per_batch = DEPTH if sc.material_mode in (0, 4) else DEPTH + 1
    assert st["trace_kernel_launches"] == 3 * per_batch
    for y0, y1 in BANDS:
        ref, segs = oracle_render(sc, W, H, DEPTH, FIRST, FRAMES, rect=(0, y0, W, y1))
        assert segs > (y1 - y0) * W * FRAMES  # paths bounce
        band = img[y0:y1]
        diff = band != ref[y0:y1]
        assert not diff.any(), (f"{scene_name} rows {y0}..{y1 - 1}: {int(diff.any(axis=-1).sum())} pixels differ, "
                                f"max |d| {float(np.max(np.abs(band - ref[y0:y1])))}")
