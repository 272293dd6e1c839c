"""Headless progressive view (OptixView accumulation on the device) and image output of a
render — GPU.  The blend is checked bit for bit against the same fp32 arithmetic in numpy
(AddPathtracedFrame.frag:18-24), fed with the individual pt_render frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene():
    from optixpathtracer_amd import scenes

    return scenes.tiny_scene("diffuse")


def _frames(scene, n, w=48, h=32):
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(scene, w, h, 4)
    out = [r.Render().copy() for _ in range(n)]
    r.close()
    return out


@pytest.mark.parametrize("max_samples", [-1, 5])
def test_display_matches_frag_shader(scene, max_samples):
    from optixpathtracer_amd.renderer import setup_renderer

    n = 5
    frames = _frames(scene, n)
    r = setup_renderer(scene, 48, 32, 4)
    r.display_reset(max_samples)
    for k in range(n):
        assert r.display_add_frame() == k + 1
    got = r.display()
    r.close()
    one = np.float32(1.0)
    fb = np.ones_like(frames[0])  # glClearColor(1,1,1,1)
    for k, f in enumerate(frames, start=1):
        if max_samples < 0:
            w = one / np.float32(k)
            fb = fb * (one - w) + f * w  # mix(fb, new, 1/n)
        else:
            w = one / np.float32(max_samples)
            fb = fb + f * w
    np.testing.assert_array_equal(got, fb)
    assert np.isfinite(got).all() and got.mean() > 0


def test_display_requires_reset(scene):
    from optixpathtracer_amd.capi import PTError
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(scene, 16, 16, 2)
    with pytest.raises(PTError):
        r.display_add_frame()
    r.display_reset(-1)
    r.display_add_frame()
    r.Resize((8, 8))  # a resize invalidates the view buffer, like a new GL framebuffer
    with pytest.raises(PTError):
        r.display_add_frame()
    r.close()


def test_render_exr_round_trip_and_mse(scene, tmp_path):
    from helpers import gpu_render, oracle_render
    from optixpathtracer_amd import imageio

    img, _ = gpu_render(scene, 40, 30, 4, 1, 4, kernel=1)
    ref, _ = oracle_render(scene, 40, 30, 4, 1, 4)
    p = tmp_path / "render.exr"
    imageio.write_exr(p, img / 4.0)
    back = imageio.read_image(p)
    np.testing.assert_array_equal(back, img / 4.0)
    assert imageio.mse(back, ref / 4.0) <= 1e-5
