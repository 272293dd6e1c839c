"""Render-ahead of pt_render / pt_display_add_frame (pt_set_render_ahead, pt_capi.cpp
render_frame_image): the reference's viewer renders one sample per Render() call
(OptixView::DrawOptix -> OptixRenderer::Render, OptixView.cpp:201-210, OptixRenderer.cpp:617-647).
With render-ahead the library renders the following frame ids in one wavefront batch while the
render state stays the same; every call must still return exactly the 1-spp image of its own frame
id under the state current at that call -- the same array, bit for bit, as a renderer without
render-ahead -- across camera, light, bounce and size changes and frame-id jumps."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, DEPTH = 64, 48, 5


def _pair(sc, mode):
    from optixpathtracer_amd.renderer import setup_renderer

    a = setup_renderer(sc, W, H, DEPTH)  # render-ahead on (default 64 frames)
    b = setup_renderer(sc, W, H, DEPTH)
    b.set_render_ahead(1)  # one frame per call
    for r in (a, b):
        r.set_material_mode(mode)
    return a, b


def _same_calls(a, b, n, shape=(H, W, 3)):
    for _ in range(n):
        fa = a.Render(np.empty(shape, np.float32)).copy()
        fb = b.Render(np.empty(shape, np.float32)).copy()
        assert a.frame_id == b.frame_id
        np.testing.assert_array_equal(fa, fb)


@pytest.mark.parametrize("mode", [1, 0], ids=["lambert", "default"])
def test_render_ahead_matches_frame_by_frame(mode):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import camera_from_blender

    sc = scenes.tiny_scene("layered")
    a, b = _pair(sc, mode)
    _same_calls(a, b, 40)  # ramps 1, 2, 4, 8, 16 frames ahead
    # a camera move: the frames rendered ahead under the old camera must not be used
    pos = np.asarray(sc.camera_blender_pos, np.float32) + np.float32(0.05)
    for r in (a, b):
        r.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)
    _same_calls(a, b, 9)
    # new light colours in the same device array
    lights = sc.lights.copy()
    lights[:, 3:6] *= np.float32(0.5)
    for r in (a, b):
        r.SetLights(lights)
    _same_calls(a, b, 5)
    for r in (a, b):
        r.SetMaxBounces(3)
    _same_calls(a, b, 5)
    # a jump back in frame ids (pt_set_frame_id), then forward past the ring
    for r in (a, b):
        r.frame_id = 3
    _same_calls(a, b, 4)
    for r in (a, b):
        r.frame_id = 500
    _same_calls(a, b, 3)
    # resize drops the ring; the camera is rebuilt for the new aspect
    p, iv, ip = camera_from_blender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg, 40, 30)
    for r in (a, b):
        r.Resize((40, 30))
        r.SetCamera(p, iv, ip)
    _same_calls(a, b, 6, shape=(30, 40, 3))
    # a frame rendered ahead equals a fresh renderer's frame of that id
    from optixpathtracer_amd.renderer import setup_renderer

    c = setup_renderer(sc, 40, 30, 3)
    c.set_material_mode(mode)
    c.SetCamera(p, iv, ip)
    c.SetLights(lights)
    c.set_render_ahead(1)
    c.frame_id = a.frame_id
    np.testing.assert_array_equal(a.Render(np.empty((30, 40, 3), np.float32)), c.Render(np.empty((30, 40, 3), np.float32)))
    for r in (a, b, c):
        r.close()


@pytest.mark.parametrize("mode", [1, 2], ids=["lambert", "dielectric"])
def test_look_ahead_long_sequence(mode):
    """Past the ramp (1+2+...+64 frames) pt_render serves from one ring slot while the next 64
    frame ids render into the other (look-ahead, downloads on their own stream).  300 sequential
    calls cross four look-ahead batches; then a camera move in the middle of a slot (the batch in
    flight is discarded), a second long run, a jump back into the older slot and stats."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("layered")
    a, b = _pair(sc, mode)
    _same_calls(a, b, 300)
    for r in (a, b):
        r.SetCameraBlender(np.asarray(sc.camera_blender_pos, np.float32) + np.float32(0.03), sc.camera_blender_rot,
                           sc.fov_deg)
    _same_calls(a, b, 200)
    back = a.frame_id - 70  # into the slot before the current one, if still held
    for r in (a, b):
        r.frame_id = back
    _same_calls(a, b, 80)
    assert a.stats()["samples"] >= b.stats()["samples"]
    for r in (a, b):
        r.close()


def test_render_ahead_display_path():
    """pt_display_add_frame takes its frames from the same ring: the progressive view after 20
    frames is identical with and without render-ahead."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("layered")
    a, b = _pair(sc, 1)
    for r in (a, b):
        r.display_reset(-1)
        for _ in range(20):
            r.display_add_frame()
    np.testing.assert_array_equal(a.display(), b.display())
    with pytest.raises(Exception):
        a.set_render_ahead(0)
    for r in (a, b):
        r.close()


def test_render_ahead_stats_exact():
    """pt_get_stats counts the frames rendered ahead and the calls served from the
    ring separately, and exactly.  Every call of `a` is served from the ring; `b` renders its own."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("layered")
    a, b = _pair(sc, 1)
    calls = 37  # the ramp 1 + 2 + 4 + 8 + 16 (+ 32 rendered ahead, 6 of them served)
    _same_calls(a, b, calls)
    sa, sb = a.stats(), b.stats()
    assert sa["frames_served_ahead"] == calls
    assert sa["frames_rendered_ahead"] >= calls
    assert sa["samples"] == sa["frames_rendered_ahead"] * W * H  # no call rendered outside the ring
    assert sb["frames_served_ahead"] == 0 and sb["frames_rendered_ahead"] == 0
    assert sb["samples"] == calls * W * H
    for r in (a, b):
        r.close()


def test_render_ahead_time_budget():
    """A batch's estimated duration stays within pt_set_render_ahead_budget: with a budget below one
    frame's time every call renders exactly its own frame into the ring (no frame is rendered that
    no call asked for), and the images stay bit-identical."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("layered")
    a, b = _pair(sc, 1)
    a.set_render_ahead_budget(1e-6)
    _same_calls(a, b, 2)  # the first batch is measured before the budget can apply
    a.stats_reset()
    _same_calls(a, b, 20)
    sa = a.stats()
    assert sa["frames_served_ahead"] == 20
    assert sa["frames_rendered_ahead"] == 20
    a.set_render_ahead_budget(0)  # no bound: the ramp runs again
    _same_calls(a, b, 40)
    assert a.stats()["frames_rendered_ahead"] > 60
    with pytest.raises(Exception):
        a.set_render_ahead_budget(-1.0)
    for r in (a, b):
        r.close()


def test_render_ahead_debug_pixel():
    """with a debug pixel set every call renders its own frame (no ring), so the
    debug records belong to the call that rendered the debug frame, also after pt_set_debug_pixel
    is called again with the same arguments."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("layered")
    a, b = _pair(sc, 0)
    _same_calls(a, b, 12)  # the ring holds frames ahead of the debug frame
    target = a.frame_id + 3
    for r in (a, b):
        r.set_debug_pixel(W // 2, H // 2, target)
    served = a.stats()["frames_served_ahead"]
    _same_calls(a, b, 5)
    assert a.stats()["frames_served_ahead"] == served
    ra, rb = a.debug_path(), b.debug_path()
    assert len(ra) > 0 and ra == rb
    for r in (a, b):  # the same arguments again: records cleared and rewritten by the next call
        r.frame_id = target - 1
        r.set_debug_pixel(W // 2, H // 2, target)
    _same_calls(a, b, 1)
    assert a.debug_path() == rb
    for r in (a, b):
        r.set_debug_pixel(-1, -1, 0)
    _same_calls(a, b, 10)
    assert a.stats()["frames_served_ahead"] > served
    for r in (a, b):
        r.close()


@pytest.mark.parametrize("mode", [0, 1], ids=["default", "lambert"])
def test_look_ahead_cancelled_by_camera_move(mode):
    """a camera move while the look-ahead batch is in
    flight cancels it (pt_capi.cpp cancel_look_ahead; its kernels stop at their next poll,
    pt_wavefront.hip wf_cancel_poll), and the next call's frame is the fresh render of the new
    camera, bit for bit.  With no time budget the ramp is 1, 2, ..., 64 frames, so call 64 is
    served from the first 64-frame slot and enqueues the next 64 frames on speculation.  The
    debug hold (pt_set_debug_hold) makes that batch wait in k_hold until it is cancelled, so the
    move provably finds it in flight, whatever the GPU's speed (round 5 sized the image so the
    batch would still be running, and a fast box finished it first).  The renderer without
    render-ahead replays the same calls afterwards for the bit-for-bit comparison."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("conductor")
    w, h, depth = 320, 180, 8
    shape = (h, w, 3)
    a = setup_renderer(sc, w, h, depth)
    b = setup_renderer(sc, w, h, depth)
    b.set_render_ahead(1)
    for r in (a, b):
        r.set_material_mode(mode)
    a.set_render_ahead_budget(0)  # no time bound: the ramp reaches 64 frames
    a.set_debug_hold(True)
    pos = np.asarray(sc.camera_blender_pos, np.float32) + np.float32(0.02)
    fa = [a.Render(np.empty(shape, np.float32)).copy() for _ in range(64)]
    a.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)  # the look-ahead batch waits in k_hold
    fa += [a.Render(np.empty(shape, np.float32)).copy() for _ in range(2)]
    st = a.stats()
    assert st["look_ahead_held"] == 1
    assert st["look_ahead_cancelled"] == 1
    a.set_debug_hold(False)
    for k in range(66):
        if k == 64:
            b.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)
        np.testing.assert_array_equal(fa[k], b.Render(np.empty(shape, np.float32)))
    # a fresh renderer with the new camera renders the same frame
    c = setup_renderer(sc, w, h, depth)
    c.set_material_mode(mode)
    c.set_render_ahead(1)
    c.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)
    c.frame_id = a.frame_id
    np.testing.assert_array_equal(a.Render(np.empty(shape, np.float32)), c.Render(np.empty(shape, np.float32)))
    b.frame_id = a.frame_id
    # the ring ramps again under the new camera, and a new-lights change while the next look-ahead
    # batch may be in flight leaves every image bit-identical
    _same_calls(a, b, 130, shape=shape)
    lights = sc.lights.copy()
    lights[:, 3:6] *= np.float32(0.75)
    for r in (a, b):
        r.SetLights(lights)
    _same_calls(a, b, 10, shape=shape)
    for r in (a, b, c):
        r.close()


def test_served_look_ahead_frame_survives_camera_move():
    """pt_display_add_frame can take its frame from the speculative batch that
    pt_render enqueued, and queues the blend behind it without waiting.  A camera move after that
    must not cancel the batch (the blend would mix a partly rendered frame into the view): a batch
    a call has taken a frame from is no longer cancellable.  The hold keeps the batch in flight
    across the move; the progressive view must equal the one of a renderer without render-ahead."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("conductor")
    w, h, depth = 320, 180, 8
    shape = (h, w, 3)
    a = setup_renderer(sc, w, h, depth)
    b = setup_renderer(sc, w, h, depth)
    b.set_render_ahead(1)
    a.set_render_ahead_budget(0)
    a.set_debug_hold(True)
    for r in (a, b):
        r.set_material_mode(1)
        r.display_reset(-1)
    _same_calls(a, b, 64, shape=shape)  # call 64 enqueues frames 65..128 on speculation (held)
    for r in (a, b):
        r.display_add_frame()  # frame 65: a takes it from the held batch
    pos = np.asarray(sc.camera_blender_pos, np.float32) + np.float32(0.02)
    for r in (a, b):
        r.SetCameraBlender(pos, sc.camera_blender_rot, sc.fov_deg)
    a.set_debug_hold(False)
    np.testing.assert_array_equal(a.display(), b.display())
    st = a.stats()
    assert st["look_ahead_held"] == 1 and st["look_ahead_cancelled"] == 0
    # both go on under the new camera
    for r in (a, b):
        r.display_add_frame()
    np.testing.assert_array_equal(a.display(), b.display())
    _same_calls(a, b, 3, shape=shape)
    for r in (a, b):
        r.close()
