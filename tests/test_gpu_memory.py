"""Device out-of-memory behaviour of the wavefront queues.

A batch's queues hold 208 B per path: 56 GB at 1920x1080 with 128 frames per batch (the
default), one queue set per wavefront stream.  The tests take most of the card's free memory with a hipMalloc first
(through the HIP runtime libptamd.so links: torch ships a second HIP runtime, which finds no GPU
once ours holds the device in the same process), so the queues cannot all be allocated:

* when an extra stream's queues do not fit, the call renders on the streams that do (same image);
* when the first stream's queues do not fit, the call halves its batch until they do (the same
  image); only when one frame's queues do not fit does it fail with PT_ERR_NOMEM, leaving no
  partial queue set behind, so the same renderer renders once the memory is back.
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
    per_frame = QUEUE_BYTES_PER_PATH * W * H

    # 64-frame batches on two streams, room for one queue set and a half: the second stream's
    # allocation fails -> one stream
    r = setup_renderer(sc, W, H, DEPTH)
    r.set_frames_per_launch(64)
    r.set_wavefront_streams(2)
    blk = _Block(1.5 * per_stream)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    blk.release()
    r.close()

    # the default batch (128 frames) with room for half a 64-frame queue set: the call halves its
    # batch until the first stream's queues fit (32 or 16 frames) and renders the same image
    r = setup_renderer(sc, W, H, DEPTH)
    blk = _Block(0.5 * per_stream)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    assert r.stats()["samples"] == W * H * FRAMES
    blk.release()
    r.close()

    # room for half of one frame's queues: PT_ERR_NOMEM with no partial queue set left behind,
    # and with the memory back the same renderer renders the full batch
    r = setup_renderer(sc, W, H, DEPTH)
    blk = _Block(0.5 * per_frame)
    r.accum_clear()
    with pytest.raises(PTError) as ei:
        r.render_frames(1, FRAMES)
    assert ei.value.status == PT_ERR_NOMEM
    blk.release()
    r.set_frames_per_launch(128)  # clears the cap the halving left
    r.accum_clear()
    r.render_frames(1, FRAMES)
    np.testing.assert_array_equal(r.accum(), ref)
    r.close()


def test_queue_budget_bounds_the_batch():
    """pt_set_queue_budget bounds the queues of all streams together.  The
    default (a quarter of the device memory) keeps the 128-frame 1080p batch of one stream; a
    smaller budget lowers the frames per batch (the same image); -1 lifts it."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene("sphere_box_diffuse")
    ref, _ = gpu_render(sc, W, H, DEPTH, 1, FRAMES, streams=1)
    P = W * H
    r = setup_renderer(sc, W, H, DEPTH)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    st = r.stats()
    assert st["queue_budget"] > 0 and st["queue_bytes"] <= st["queue_budget"]
    assert st["last_streams"] == 1 and st["last_batch_frames"] == 128
    np.testing.assert_array_equal(r.accum(), ref)
    for streams, frames in ((1, 20), (2, 20), (2, 7)):
        budget = frames * QUEUE_BYTES_PER_PATH * P + (1 << 20)  # room for the counters
        r.set_queue_budget(budget)
        r.set_wavefront_streams(streams)
        r.accum_clear()
        r.render_frames(1, FRAMES)
        st = r.stats()
        assert st["queue_budget"] == budget
        assert st["queue_bytes"] <= budget, (streams, frames, st["queue_bytes"])
        assert st["last_streams"] == streams
        assert st["last_batch_frames"] == max(1, frames // streams), (streams, frames, st["last_batch_frames"])
        np.testing.assert_array_equal(r.accum(), ref)
    r.set_queue_budget(-1)  # none: the full batch on both streams
    r.accum_clear()
    r.render_frames(1, FRAMES)
    st = r.stats()
    assert st["queue_budget"] == 0 and st["last_batch_frames"] == 128 and st["last_streams"] == 2
    np.testing.assert_array_equal(r.accum(), ref)
    r.close()


def test_out_of_memory_frees_idle_stream_queues_first():
    """queues held by streams a call does not use (an earlier two-stream Conductor
    call's) are freed before the first stream's batch is halved, so a renderer does not stay on
    small batches because of memory it holds itself."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PT_MAT_CONDUCTOR, PT_MAT_LAMBERT
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene("sphere_box_diffuse")
    ref, _ = gpu_render(sc, W, H, DEPTH, 1, FRAMES, streams=1)
    per_stream = QUEUE_BYTES_PER_PATH * W * H * 64
    r = setup_renderer(sc, W, H, DEPTH)
    r.set_queue_budget(-1)  # this test is about the out-of-memory path, not the budget
    r.set_material_mode(PT_MAT_CONDUCTOR)
    r.set_frames_per_launch(64)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    st = r.stats()
    assert st["last_streams"] == 2 and st["queue_bytes"] >= 2 * per_stream
    blk = _Block(0.2 * per_stream)  # free: a fifth of a 64-frame set; held: two of them
    r.set_material_mode(PT_MAT_LAMBERT)  # one stream, 128 frames: needs both sets' memory
    r.set_frames_per_launch(128)
    r.accum_clear()
    r.render_frames(1, FRAMES)
    st = r.stats()
    assert st["last_streams"] == 1 and st["last_batch_frames"] == 128
    np.testing.assert_array_equal(r.accum(), ref)
    blk.release()
    r.close()
