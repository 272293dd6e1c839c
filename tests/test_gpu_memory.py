"""Device out-of-memory behaviour of the wavefront queues.

A batch's queues hold 208 B per path: 28 GB at 1920x1080 with 64 frames per batch, one queue set
per wavefront stream.  The tests take most of the card's free memory with a torch allocation
first, so the queues cannot all be allocated:

* when an extra stream's queues do not fit, the call renders on the streams that do (same image);
* when the first stream's queues do not fit, the call fails with PT_ERR_NOMEM and leaves no
  partial queue set behind, so lowering frames-per-launch and calling again renders correctly.
"""
import numpy as np
import pytest

from helpers import gpu_render

pytestmark = pytest.mark.gpu

W, H, DEPTH, FRAMES = 1920, 1080, 8, 130
QUEUE_BYTES_PER_PATH = 208


def _block(torch, leave_bytes):
    free, _ = torch.cuda.mem_get_info(0)
    n = free - int(leave_bytes)
    assert n > 0, (free, leave_bytes)
    return torch.empty(n, dtype=torch.uint8, device="cuda:0")


def test_queue_allocation_failures_fall_back_and_retry():
    import torch

    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PT_ERR_NOMEM, PTError
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene("sphere_box_diffuse")
    ref, sr = gpu_render(sc, W, H, DEPTH, 1, FRAMES, streams=1)
    per_stream = QUEUE_BYTES_PER_PATH * W * H * 64

    # room for one queue set and a half: the second stream's allocation fails -> one stream
    r = setup_renderer(sc, W, H, DEPTH)
    blk = _block(torch, 1.5 * per_stream)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    del blk
    torch.cuda.empty_cache()
    r.close()

    # room for half a queue set: PT_ERR_NOMEM, then a retry with smaller batches succeeds
    r = setup_renderer(sc, W, H, DEPTH)
    blk = _block(torch, 0.5 * per_stream)
    r.accum_clear()
    with pytest.raises(PTError) as ei:
        r.render_frames(1, FRAMES)
    assert ei.value.status == PT_ERR_NOMEM
    r.set_frames_per_launch(8)  # 3.5 GB per stream
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    assert r.stats()["samples"] == W * H * FRAMES
    del blk
    torch.cuda.empty_cache()
    # and with the memory back, the original batch size works on the same renderer
    r.set_frames_per_launch(64)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    r.close()
