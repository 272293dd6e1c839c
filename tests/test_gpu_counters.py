"""The per-kernel counters bench.py builds its roofline from (pt_stats.pair_kernel_*, nee_unoccluded;
DESIGN.md §4): consistent with each other and with the work of the render, and the counting
kernel instances render the same image as the timed ones."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [1, 2, 3], ids=["lambert", "conductor", "dielectric"])
def test_pair_kernel_counters(mode):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("diffuse")
    r = setup_renderer(sc, 96, 64, 4)
    r.set_material_mode(mode)
    r.set_frames_per_launch(8)
    r.set_kernel_timing(True)
    imgs = []
    for stats in (False, True):
        r.set_traversal_stats(stats)
        r.stats_reset()
        r.accum_clear()
        r.render_frames(1, 16)
        imgs.append(r.accum())
        st = r.stats()
        # k_trace_pair: 48 algorithmic bytes per ray, shadow rays a part of its rays
        assert st["pair_kernel_launches"] > 0
        assert st["pair_kernel_bytes"] == 48 * st["pair_kernel_rays"]
        assert 0 <= st["pair_kernel_shadow_rays"] < st["pair_kernel_rays"]
        if mode != 3:  # a smooth dielectric queues no shadow rays after bounce 0
            assert st["pair_kernel_shadow_rays"] > 0
        assert st["pair_kernel_rays"] <= st["trace_kernel_rays"]
        assert st["pair_kernel_shadow_rays"] <= st["shadow_rays"]
        if stats and st["pair_kernel_shadow_rays"]:
            # counted only by the traversal-statistics instances: some lights are blocked, most not
            assert 0 < st["nee_unoccluded"] < st["pair_kernel_shadow_rays"]
        else:
            assert st["nee_unoccluded"] == 0
    np.testing.assert_array_equal(imgs[0], imgs[1])
    r.close()
