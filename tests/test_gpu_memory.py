"""Device out-of-memory behaviour of the wavefront queues.

A batch's queues hold 208 B per path: 28 GB at 1920x1080 with 64 frames per batch, one queue set
per wavefront stream.  The tests take most of the card's free memory with a hipMalloc first
(through the HIP runtime libptamd.so links: torch ships a second HIP runtime, which finds no GPU
once ours holds the device in the same process), so the queues cannot all be allocated:

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


class _Block:
    """hipMalloc of all free device memory but `leave_bytes`, freed by release()."""

    def __init__(self, leave_bytes):
        import ctypes

        from optixpathtracer_amd import capi

        capi.load()  # the HIP runtime libptamd.so links, already initialised by the renderer
        self.hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
        free, total = ctypes.c_size_t(), ctypes.c_size_t()
        assert self.hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
        n = free.value - int(leave_bytes)
        assert n > 0, (free.value, leave_bytes)
        self.ptr = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(n)) == 0

    def release(self):
        if self.ptr:
            assert self.hip.hipFree(self.ptr) == 0
            self.ptr = None


def test_queue_allocation_failures_fall_back_and_retry():
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PT_ERR_NOMEM, PTError
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene("sphere_box_diffuse")
    ref, sr = gpu_render(sc, W, H, DEPTH, 1, FRAMES, streams=1)
    per_stream = QUEUE_BYTES_PER_PATH * W * H * 64

    # room for one queue set and a half: the second stream's allocation fails -> one stream
    r = setup_renderer(sc, W, H, DEPTH)
    blk = _Block(1.5 * per_stream)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    blk.release()
    r.close()

    # room for half a queue set: PT_ERR_NOMEM, then a retry with smaller batches succeeds
    r = setup_renderer(sc, W, H, DEPTH)
    blk = _Block(0.5 * per_stream)
    r.accum_clear()
    with pytest.raises(PTError) as ei:
        r.render_frames(1, FRAMES)
    assert ei.value.status == PT_ERR_NOMEM
    r.set_frames_per_launch(8)  # 3.5 GB per stream
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    assert r.stats()["samples"] == W * H * FRAMES
    blk.release()
    # and with the memory back, the original batch size works on the same renderer
    r.set_frames_per_launch(64)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    r.close()
