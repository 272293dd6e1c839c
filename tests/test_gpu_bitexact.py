"""GPU images equal to the CPU oracle's bit for bit.

The kernels and the oracle keep glm's association order, compile without FMA contraction,
use correctly rounded division and square root, and evaluate the path's transcendentals
(sin / cos / exp / pow) with the same fixed fused polynomials (pt_math.h, pt_oracle.c).  So
at identical (pixel, frame id) seeds every path makes the same decisions and every radiance
sum rounds the same way: the images must be identical, not merely within the MSE bar.
"""
import numpy as np
import pytest

from helpers import gpu_render, oracle_render

pytestmark = pytest.mark.gpu


def assert_identical(g, o, what):
    diff = g != o
    if diff.any():
        idx = np.argwhere(diff)[:5]
        raise AssertionError(f"{what}: {int(diff.sum())} of {diff.size} values differ, first at {idx.tolist()}: "
                             f"gpu {g[tuple(idx[0])]!r} oracle {o[tuple(idx[0])]!r}")


@pytest.mark.parametrize("kernel", [0, 1], ids=["mega", "wavefront"])
@pytest.mark.parametrize("variant", ["diffuse", "conductor", "dielectric20", "layered"])
def test_tiny_scenes_bit_exact(variant, kernel):
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene(variant)
    g, sg = gpu_render(sc, 64, 48, 6, 1, 8, kernel=kernel)
    o, so = oracle_render(sc, 64, 48, 6, 1, 8)
    assert_identical(g, o, variant)
    assert sg["segments"] == so


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 0])
def test_sphere_box_all_modes_bit_exact(mode):
    from optixpathtracer_amd import scenes

    sc = scenes.sphere_in_box("conductor" if mode == 0 else "diffuse")
    g, sg = gpu_render(sc, 96, 64, 8, 3, 6, mode=mode, kernel=1)
    o, so = oracle_render(sc, 96, 64, 8, 3, 6, mode=mode)
    assert_identical(g, o, f"mode {mode}")
    assert sg["segments"] == so


def test_config1_bit_exact():
    """BASELINE config 1 (256x256, 16 spp, depth 4, Lambert) through the default kernel."""
    from optixpathtracer_amd import scenes

    sc = scenes.sphere_in_box("diffuse")
    g, _ = gpu_render(sc, 256, 256, 4, 1, 16, kernel=2)
    o, _ = oracle_render(sc, 256, 256, 4, 1, 16)
    assert_identical(g, o, "config 1")


def test_sponza_class_band_bit_exact():
    """The 250k-triangle mixed-material scene (config 5, light colour 100) at full HD and
    depth 8: a 12-row band of the GPU image against the oracle's render of that band."""
    from optixpathtracer_amd import scenes

    sc = scenes.sponza_class()
    w, h, y0, y1 = 1920, 1080, 600, 612
    g, _ = gpu_render(sc, w, h, 8, 1, 4, kernel=2)
    o, _ = oracle_render(sc, w, h, 8, 1, 4, rect=(0, y0, w, y1))
    assert_identical(g[y0:y1], o[y0:y1], "sponza band")


@pytest.mark.parametrize("variant", ["diffuse", "conductor"])
def test_textured_scene_bit_exact(variant):
    """sRGB albedo (pow), alpha cut-out, normal and metal/rough maps."""
    from optixpathtracer_amd import scenes

    sc = scenes.textured_scene(variant)
    g, _ = gpu_render(sc, 48, 32, 5, 1, 6, kernel=1)
    o, _ = oracle_render(sc, 48, 32, 5, 1, 6)
    assert_identical(g, o, f"textured {variant}")


@pytest.mark.parametrize("mode", [1, 0])
def test_sah_builder_images_bit_exact(mode):
    """The host binned-SAH builder (PT_BVH_SAH) gives a different BVH4; the images stay the
    oracle's bit for bit (the closest hit does not depend on the tree)."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("conductor" if mode == 0 else "diffuse")
    r = setup_renderer(sc, 96, 64, 8, bvh_builder=2)
    r.set_material_mode(mode)
    r.accum_clear()
    r.render_frames(3, 6)
    g = r.accum()
    r.close()
    o, _ = oracle_render(sc, 96, 64, 8, 3, 6, mode=mode)
    assert_identical(g, o, f"sah builder, mode {mode}")
