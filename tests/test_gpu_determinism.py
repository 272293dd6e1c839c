"""Closest-hit determinism (round-1 VERDICT "What's weak" 2 / "Next round" 1).

Round 1 saw one non-repeating one-ulp GPU-vs-oracle difference in the config-5 band.  Its
cause: a grazing ray (cos 0.038 to the surface) that Moller-Trumbore accepts on triangle B at a
point outside B's own box, with the neighbouring triangle A hit a few ulps farther on.  B's box
passes the cull only while `best` is still large, so the answer was A or B depending on which
triangle the traversal tested first -- which depends on the wave's postponed-leaf schedule and
the queue order (block atomics), i.e. on the run.  The oracle's own binary BVH had the same
order dependence (tools/cullcheck.py: 1 trace in 62.5 M of the band disagreed with an
exhaustive search).  Both sides now take only ACCEPTABLE hits (t inside the triangle's own
padded slab interval, pt_device.h tri_accept / pt_oracle.c tri_accept) and cull boxes with the
same slab arithmetic and slack, which makes the answer independent of BVH and visit order.

These tests pin that: the exact ray of the round-1 event, grazing and far-origin rays at shared
edges against the oracle, BVH builds that are identical bit for bit, and renders whose queue
layout differs (frames per launch) staying identical.
"""
import numpy as np
import pytest

from helpers import shared_edge_rays

pytestmark = pytest.mark.gpu

# the round-1 config-5 event: origin, direction, tmin, tmax (tools/cullcheck.py output)
EVENT_RAY = np.array([[-7.9992828369140625, 1.2957302331924438, -4.999000072479248, 0.9340350031852722,
                       -0.0061589255928993225, 0.3571285903453827, 0.0, 100.0]], np.float32)


@pytest.fixture(scope="module")
def sponza():
    from optixpathtracer_amd import scenes

    return scenes.sponza_class()


def _compare(r, o, rays):
    gp, gt, gu, gv, gb = r.trace_rays(rays)
    op, ot, ou, ov, ob = o.trace(rays)
    np.testing.assert_array_equal(gp, op)
    hit = op >= 0
    np.testing.assert_array_equal(gt[hit], ot[hit])
    np.testing.assert_array_equal(gu[hit], ou[hit])
    np.testing.assert_array_equal(gv[hit], ov[hit])
    np.testing.assert_array_equal(gb[hit], ob[hit])
    ga = r.trace_rays(rays, any_hit=True)[0] >= 0
    oa = o.trace(rays, any_hit=True)[0] >= 0
    np.testing.assert_array_equal(ga, oa)
    return hit.mean()


@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_round1_event_ray(sponza, builder):
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    r = setup_renderer(sponza, 32, 32, 2, bvh_builder=builder)
    o = OracleScene(sponza)
    _compare(r, o, EVENT_RAY)
    # the acceptable minimum: triangle 81823 at t = 20.41062 (not 81918 two ulps later)
    assert int(r.trace_rays(EVENT_RAY)[0][0]) == 81823
    r.close()
    o.close()


@pytest.mark.parametrize("far", [False, True], ids=["grazing", "far-origin"])
@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_shared_edge_rays_bit_exact(sponza, builder, far):
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    rays = shared_edge_rays(sponza, 4000, seed=11 + far, far=far)
    r = setup_renderer(sponza, 32, 32, 2, bvh_builder=builder)
    o = OracleScene(sponza)
    assert _compare(r, o, rays) > 0.9
    r.close()
    o.close()


def test_shared_edge_rays_sphere_box_bit_exact():
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    sc = scenes.sphere_in_box("diffuse")
    rays = np.concatenate([shared_edge_rays(sc, 3000, seed=5), shared_edge_rays(sc, 1000, seed=6, far=True)])
    r = setup_renderer(sc, 32, 32, 2)
    o = OracleScene(sc)
    assert _compare(r, o, rays) > 0.9
    r.close()
    o.close()


@pytest.mark.parametrize("scene_name", ["sphere_box_diffuse", "sponza_class"])
@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_bvh_build_deterministic(scene_name, builder):
    """Two builds of one scene give the same node and triangle arrays bit for bit (BVH4 slots are
    numbered breadth-first by a prefix sum, not by atomic arrival order)."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.make_scene(scene_name)
    arrays = []
    for _ in range(2):
        r = setup_renderer(sc, 16, 16, 1, bvh_builder=builder)
        arrays.append(r.bvh_arrays())
        r.close()
    (n0, t0), (n1, t1) = arrays
    assert n0.shape[0] > 0 and t0.shape[0] == sc.n_triangles
    np.testing.assert_array_equal(n0, n1)
    np.testing.assert_array_equal(t0, t1)


def test_sponza_band_identical_across_batch_layouts(sponza):
    """The same frames rendered with different wavefront batch sizes (different queue orders,
    different wave neighbours for every ray) are identical bit for bit."""
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(sponza, 480, 270, 8)
    imgs = []
    for fpl in (7, 3, 1):
        r.set_frames_per_launch(fpl)
        r.accum_clear()
        r.render_frames(1, 7)
        imgs.append(r.accum().copy())
    r.close()
    np.testing.assert_array_equal(imgs[0], imgs[1])
    np.testing.assert_array_equal(imgs[0], imgs[2])
