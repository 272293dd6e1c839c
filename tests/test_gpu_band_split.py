"""One-frame calls in two row bands (pt_set_band_split, pt_capi.cpp launch_frames): a call that
renders a single frame -- pt_render without render-ahead (the reference's one-Render-per-frame
viewer with a camera that moves every frame, OptixView.cpp:201-210), pt_launch, pt_render_frames
of one frame -- splits the frame's rows into two bands on the two wavefront streams.  A pixel's
path depends only on its (pixel, frame id) seed and the camera ray through its pixel centre
(devicePrograms.cu:601-631), so the banded image must equal the unbanded one and the oracle's
bit for bit, in every material mode, for odd heights, textured scenes and the debug pixel."""
import numpy as np
import pytest

from helpers import oracle_render

pytestmark = pytest.mark.gpu


def _renderer(sc, w, h, depth, mode, band):
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(sc, w, h, depth)
    r.set_material_mode(mode)
    r.set_render_ahead(1)  # every pt_render call renders its own frame
    r.set_band_split(band)
    return r


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 0])
def test_band_split_render_bit_identical(mode):
    from optixpathtracer_amd import scenes

    sc = scenes.sphere_in_box("conductor" if mode == 0 else "diffuse")
    w, h = 96, 67  # odd height: bands of 33 and 34 rows
    a = _renderer(sc, w, h, 8, mode, True)
    b = _renderer(sc, w, h, 8, mode, False)
    for _ in range(5):
        fa = a.Render(np.empty((h, w, 3), np.float32)).copy()
        fb = b.Render(np.empty((h, w, 3), np.float32)).copy()
        np.testing.assert_array_equal(fa, fb)
    sa, sb = a.stats(), b.stats()
    assert sa["segments"] == sb["segments"]
    a.close()
    b.close()


@pytest.mark.parametrize("variant,mode", [("diffuse", 1), ("layered", 0), ("dielectric20", 3)])
def test_band_split_one_frame_matches_oracle(variant, mode):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.tiny_scene(variant)
    w, h, depth, frame = 64, 49, 6, 7
    r = setup_renderer(sc, w, h, depth)
    r.set_material_mode(mode)
    assert r.stats()  # the renderer is live
    r.accum_clear()
    r.render_frames(frame, 1)  # one frame: two bands
    g = r.accum()
    o, _ = oracle_render(sc, w, h, depth, frame, 1, mode=mode)
    np.testing.assert_array_equal(g, o)
    r.close()


def test_band_split_textured_and_display():
    from optixpathtracer_amd import scenes

    sc = scenes.textured_scene("diffuse")
    w, h = 80, 45
    a = _renderer(sc, w, h, 6, 0, True)
    b = _renderer(sc, w, h, 6, 0, False)
    for r in (a, b):
        r.display_reset(1000)
    for _ in range(4):
        fa = a.Render(np.empty((h, w, 3), np.float32)).copy()
        fb = b.Render(np.empty((h, w, 3), np.float32)).copy()
        np.testing.assert_array_equal(fa, fb)
        a.display_add_frame()
        b.display_add_frame()
    np.testing.assert_array_equal(a.display(), b.display())
    a.close()
    b.close()


def test_band_split_launch_params():
    """pt_launch (LaunchParams + optixLaunch) renders one frame into the caller's device buffer."""
    from test_gpu_parity import _HipBuffers

    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import camera_from_blender

    sc = scenes.tiny_scene("conductor")
    w, h, depth = 72, 41, 5
    p, iv, ip = camera_from_blender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg, w, h)
    out = []
    for band in (True, False):
        r = _renderer(sc, w, h, depth, 0, band)
        hb = _HipBuffers()
        lights = hb.alloc(sc.lights.nbytes)
        hb.upload(lights, sc.lights.astype(np.float32))
        buf = hb.alloc(w * h * 3 * 4)
        hb.upload(buf, np.full((h, w, 3), np.nan, np.float32))  # overwritten, not added
        r.launch(buf, (w, h), 9, p, iv, ip, lights, len(sc.lights), depth)
        r.synchronize()
        out.append(hb.download(buf, (h, w, 3)))
        hb.free()
        r.close()
    assert np.isfinite(out[0]).all()
    np.testing.assert_array_equal(out[0], out[1])


def test_band_split_debug_pixel_both_bands():
    from optixpathtracer_amd import scenes

    sc = scenes.sphere_in_box("conductor")
    w, h = 96, 64
    recs = {}
    for band in (True, False):
        r = _renderer(sc, w, h, 8, 0, band)
        got = []
        for x, y in [(20, 10), (70, 50)]:  # one pixel in each band
            r.set_debug_pixel(x, y, r.frame_id + 1)
            r.Render(np.empty((h, w, 3), np.float32))
            got.append([tuple(sorted((k, str(v)) for k, v in d.items())) for d in r.debug_path()])
        r.set_debug_pixel(-1, 0, 0)
        recs[band] = got
        r.close()
    assert recs[True] == recs[False]
    assert all(len(g) > 0 for g in recs[True])


def test_band_state_cleared_for_megakernel_calls():
    """A banded call followed by a megakernel call: the second call's download must wait for its
    own render, not for the earlier call's first-band event."""
    from optixpathtracer_amd import scenes

    sc = scenes.sphere_in_box("diffuse")
    w, h = 96, 64
    a = _renderer(sc, w, h, 6, 1, True)
    b = _renderer(sc, w, h, 6, 1, True)
    b.set_kernel(0)
    a.Render(np.empty((h, w, 3), np.float32))  # banded wavefront frame 1
    b.Render(np.empty((h, w, 3), np.float32))
    a.set_kernel(0)  # megakernel from frame 2 on
    for _ in range(3):
        fa = a.Render(np.empty((h, w, 3), np.float32)).copy()
        fb = b.Render(np.empty((h, w, 3), np.float32)).copy()
        np.testing.assert_array_equal(fa, fb)
    a.close()
    b.close()
