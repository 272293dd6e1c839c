"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on identical seeds.

Bar (north_star / SURVEY.md §8(c)): per-image MSE of the radiance (mean over pixels and
channels, NaN -> 0) <= 1e-5 against the oracle render at identical (pixel, frame id)
seeds.  Traversal results (integer primitive ids, hit flags) must be bit-exact.  Since the
kernels and the oracle share the path's transcendental polynomials the images are in fact
identical (tests/test_gpu_bitexact.py); the MSE / close-fraction bars here are the contract
the north star states, kept as the looser check.
"""
import numpy as np
import pytest

from helpers import gpu_render, image_mse, oracle_render, random_rays

pytestmark = pytest.mark.gpu

MSE_TOL = 1e-5
# Paths that never diverge agree to a few ulps; a path whose discrete decision flips on a
# transcendental ulp differs by O(1).  Require almost every pixel to be ulp-close.
CLOSE_RTOL = 1e-4
CLOSE_MIN = 0.97


def close_fraction(g, o):
    return float(np.mean(np.abs(g - o) <= CLOSE_RTOL * (1.0 + np.abs(o))))


@pytest.fixture(scope="module")
def diffuse_scene():
    from optixpathtracer_amd import scenes

    return scenes.sphere_in_box("diffuse")


@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_trace_closest_bit_exact(diffuse_scene, builder):
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    rays = random_rays(diffuse_scene, 3000, seed=1)
    r = setup_renderer(diffuse_scene, 64, 64, 4, bvh_builder=builder)
    gp, gt, gu, gv, gb = r.trace_rays(rays)
    o = OracleScene(diffuse_scene)
    op, ot, ou, ov, ob = o.trace(rays)
    assert (gp >= 0).sum() > 1000
    np.testing.assert_array_equal(gp, op)
    hit = op >= 0
    np.testing.assert_array_equal(gt[hit], ot[hit])
    np.testing.assert_array_equal(gu[hit], ou[hit])
    np.testing.assert_array_equal(gv[hit], ov[hit])
    np.testing.assert_array_equal(gb[hit], ob[hit])
    # any-hit (shadow rays) agree on occlusion
    ga = r.trace_rays(rays, any_hit=True)[0] >= 0
    oa = o.trace(rays, any_hit=True)[0] >= 0
    np.testing.assert_array_equal(ga, oa)
    r.close()


@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_trace_sponza_class_bit_exact(builder):
    """~250k triangles: deeper trees, many PLOC iterations, LDS-stack spills."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    sc = scenes.sponza_class()
    rays = random_rays(sc, 2000, seed=7)
    r = setup_renderer(sc, 32, 32, 2, bvh_builder=builder)
    gp, gt, gu, gv, gb = r.trace_rays(rays)
    st = r.stats()
    o = OracleScene(sc)
    op, ot, ou, ov, ob = o.trace(rays)
    assert (gp >= 0).sum() > 500
    np.testing.assert_array_equal(gp, op)
    hit = op >= 0
    np.testing.assert_array_equal(gt[hit], ot[hit])
    np.testing.assert_array_equal(gu[hit], ou[hit])
    np.testing.assert_array_equal(gv[hit], ov[hit])
    ga = r.trace_rays(rays, any_hit=True)[0] >= 0
    oa = o.trace(rays, any_hit=True)[0] >= 0
    np.testing.assert_array_equal(ga, oa)
    assert st["bvh_nodes"] > 0 and st["triangles"] == sc.n_triangles
    r.close()
    o.close()


@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_trace_two_triangles(builder):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import OptixRenderer

    two = scenes.Mesh(vertices=np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32),
                      indices=np.array([[0, 1, 2], [0, 2, 3]], np.int32),
                      normals=np.array([[0, 0, 1]] * 4, np.float32))
    sc = scenes.Scene(meshes=[two], lights=np.zeros((0, 6), np.float32), camera_blender_pos=(0, 0, 0),
                      camera_blender_rot=(0, 0, 0))
    r = OptixRenderer(None, sc, bvh_builder=builder)
    rays = np.array([[0.75, 0.25, 1, 0, 0, -1, 0, 10], [0.25, 0.75, 1, 0, 0, -1, 0, 10],
                     [2, 2, 1, 0, 0, -1, 0, 10]], dtype=np.float32)
    p = r.trace_rays(rays)[0]
    assert list(p) == [0, 1, -1]
    r.close()


@pytest.mark.parametrize("builder", [3, 1, 2, 4], ids=["ploc", "lbvh", "sah", "sah_gpu"])
def test_trace_empty_and_single_triangle(builder):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import OptixRenderer

    one = scenes.Mesh(vertices=np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32),
                      indices=np.array([[0, 1, 2]], np.int32),
                      normals=np.array([[0, 0, 1]] * 3, np.float32))
    sc = scenes.Scene(meshes=[one], lights=np.zeros((0, 6), np.float32), camera_blender_pos=(0, 0, 0),
                      camera_blender_rot=(0, 0, 0))
    r = OptixRenderer(None, sc, bvh_builder=builder)
    rays = np.array([[0.2, 0.2, 1, 0, 0, -1, 0, 100], [2, 2, 1, 0, 0, -1, 0, 100],
                     [0.2, 0.2, -1, 0, 0, 1, 0, 100]], np.float32)
    p, t, u, v, b = r.trace_rays(rays)
    assert list(p) == [0, -1, 0]
    assert t[0] == pytest.approx(1.0) and b[0] == 0 and b[2] == 1
    assert u[0] == pytest.approx(0.2) and v[0] == pytest.approx(0.2)
    r.close()
    empty = scenes.Scene(meshes=[], lights=np.zeros((0, 6), np.float32), camera_blender_pos=(0, 0, 0),
                         camera_blender_rot=(0, 0, 0))
    r = OptixRenderer(None, empty, bvh_builder=builder)
    assert list(r.trace_rays(rays)[0]) == [-1, -1, -1]
    r.Resize((8, 8))
    r.SetCameraBlender((0, 0, 0), (90, 0, 0))
    r.SetMaxBounces(4)
    img = r.Render()
    assert np.all(img == 0)
    r.close()


@pytest.mark.parametrize("variant", ["diffuse", "conductor", "dielectric20", "layered"])
def test_tiny_scene_parity(variant):
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene(variant)
    g, st = gpu_render(sc, 64, 48, 4, 1, 8)
    o, segs = oracle_render(sc, 64, 48, 4, 1, 8)
    assert np.isfinite(g).all()
    mse = image_mse(g / 8, o / 8)
    assert mse <= MSE_TOL, mse
    close = close_fraction(g, o)
    print(f"{variant}: mse={mse:.3e} close={close:.4f} exact={np.mean(g == o):.4f}")
    assert close >= CLOSE_MIN, close
    # segment counts agree to within the rare divergent paths
    assert abs(st["segments"] - segs) <= 0.01 * segs


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 0])
def test_all_material_modes_diffuse_scene(diffuse_scene, mode):
    g, _ = gpu_render(diffuse_scene, 48, 32, 3, 5, 4, mode=mode)
    o, _ = oracle_render(diffuse_scene, 48, 32, 3, 5, 4, mode=mode)
    mse = image_mse(g / 4, o / 4)
    close = close_fraction(g, o)
    print(f"mode {mode}: mse={mse:.3e} close={close:.4f}")
    assert mse <= MSE_TOL
    assert close >= CLOSE_MIN


def test_config1_parity(diffuse_scene):
    """BASELINE config 1: 256x256, 16 spp (frame ids 1..16), depth 4, Lambert mode."""
    g, st = gpu_render(diffuse_scene, 256, 256, 4, 1, 16)
    o, segs = oracle_render(diffuse_scene, 256, 256, 4, 1, 16)
    mse = image_mse(g / 16, o / 16)
    assert mse <= MSE_TOL, mse
    close = close_fraction(g, o)
    print(f"config1: mse={mse:.3e} close={close:.4f} exact={np.mean(g == o):.4f}")
    assert close >= CLOSE_MIN, close


def test_render_api_semantics(diffuse_scene):
    """Render() = 1 spp with frame.id++ (OptixRenderer.cpp:617-647); chunked accumulation
    is bit-identical to one pass; no-op before Resize."""
    from optixpathtracer_amd.renderer import OptixRenderer, setup_renderer

    r0 = OptixRenderer(None, diffuse_scene)
    out = np.full((1, 1, 3), 7.0, np.float32)
    r0.Render(out)  # no Resize yet: no-op
    assert np.all(out == 7.0)
    r0.close()

    r = setup_renderer(diffuse_scene, 40, 30, 4)
    assert r.frame_id == 0
    f1 = r.Render().copy()
    f2 = r.Render().copy()
    assert r.frame_id == 2
    r.accum_clear()
    r.render_frames(1, 1)
    np.testing.assert_array_equal(r.accum(), f1)
    r.accum_clear()
    r.render_frames(2, 1)
    np.testing.assert_array_equal(r.accum(), f2)
    r.accum_clear()
    r.render_frames(1, 11)
    one = r.accum()
    r.accum_clear()
    r.render_frames(1, 3)
    r.render_frames(4, 8)
    np.testing.assert_array_equal(r.accum(), one)
    # mean download
    np.testing.assert_allclose(r.accum(scale=1.0 / 11), one / 11, rtol=1e-6)
    # pt_render_accumulate = clear + render_frames + mean download; the sum stays on the device
    mean = r.render_accumulate(11, 1)
    np.testing.assert_array_equal(mean, (one * np.float32(1.0 / 11)).astype(np.float32))
    np.testing.assert_array_equal(r.accum(), one)
    r.close()


def test_determinism_fullhd_properties(diffuse_scene):
    """Config 2 geometry at 1920x1080: two runs bit-identical, no NaN, and a 16-row band
    matches the oracle on the same seeds."""
    g1, st1 = gpu_render(diffuse_scene, 1920, 1080, 8, 1, 2)
    g2, _ = gpu_render(diffuse_scene, 1920, 1080, 8, 1, 2)
    np.testing.assert_array_equal(g1, g2)
    assert np.isfinite(g1).all()
    assert st1["segments"] > 1920 * 1080 * 2
    o, _ = oracle_render(diffuse_scene, 1920, 1080, 8, 1, 2, rect=(0, 532, 1920, 548))
    band = slice(532, 548)
    assert image_mse(g1[band] / 2, o[band] / 2) <= MSE_TOL


@pytest.mark.parametrize("variant", ["diffuse", "conductor", "dielectric20", "layered"])
def test_wavefront_bit_identical_to_megakernel(variant):
    """Both kernel designs add each path's NEE terms in bounce order and accumulate frames
    in order, so their images must agree bit for bit (and hence with the oracle parity)."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene(variant)
    a, sa = gpu_render(sc, 64, 48, 5, 3, 6, kernel=0)
    b, sb = gpu_render(sc, 64, 48, 5, 3, 6, kernel=1)
    np.testing.assert_array_equal(a, b)
    assert sa["segments"] == sb["segments"]


@pytest.mark.parametrize("mode", [1, 3, 0])
def test_wavefront_frame_batching_bit_identical(mode):
    """The wavefront keeps the paths of a batch of frames in flight together (path = f * P +
    pixel) and k_accum adds the batch's frames in order, so any batch size -- including a
    ragged last batch (11 frames = 4 + 4 + 3) -- gives the accumulator of one frame at a time."""
    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("diffuse")
    ref, sr = gpu_render(sc, 48, 40, 5, 7, 11, mode=mode, kernel=1, frames_per_launch=1)
    for fpl in (4, 16):
        img, st = gpu_render(sc, 48, 40, 5, 7, 11, mode=mode, kernel=1, frames_per_launch=fpl)
        np.testing.assert_array_equal(img, ref)
        assert st["segments"] == sr["segments"]
    mega, _ = gpu_render(sc, 48, 40, 5, 7, 11, mode=mode, kernel=0)
    np.testing.assert_array_equal(mega, ref)
    # primary dedup off: every frame traces its own copy of the camera rays
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(sc, 48, 40, 5, kernel=1)
    r.set_material_mode(mode)
    r.set_frames_per_launch(4)
    r.set_primary_dedup(False)
    r.accum_clear()
    r.render_frames(7, 11)
    np.testing.assert_array_equal(r.accum(), ref)
    r.close()


@pytest.mark.parametrize("mode", [1, 0])
def test_wavefront_config1_parity(diffuse_scene, mode):
    g, st = gpu_render(diffuse_scene, 256, 256, 4, 1, 16, mode=mode, kernel=1)
    o, segs = oracle_render(diffuse_scene, 256, 256, 4, 1, 16, mode=mode)
    mse = image_mse(g / 16, o / 16)
    assert mse <= MSE_TOL, mse
    assert close_fraction(g, o) >= CLOSE_MIN
    m, _ = gpu_render(diffuse_scene, 256, 256, 4, 1, 16, mode=mode, kernel=0)
    np.testing.assert_array_equal(g, m)


def test_trace_textured_alpha_cutout_bit_exact():
    """AlphaCutout (devicePrograms.cu:518-561) inside the traversal: closest and any-hit rays
    through cut-out texels agree with the oracle bit for bit."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    sc = scenes.textured_scene("diffuse")
    rays = random_rays(sc, 4000, seed=5)
    r = setup_renderer(sc, 32, 32, 2)
    gp, gt, gu, gv, gb = r.trace_rays(rays)
    o = OracleScene(sc)
    op, ot, ou, ov, ob = o.trace(rays)
    np.testing.assert_array_equal(gp, op)
    hit = op >= 0
    np.testing.assert_array_equal(gt[hit], ot[hit])
    np.testing.assert_array_equal(gu[hit], ou[hit])
    np.testing.assert_array_equal(gv[hit], ov[hit])
    ga = r.trace_rays(rays, any_hit=True)[0] >= 0
    oa = o.trace(rays, any_hit=True)[0] >= 0
    np.testing.assert_array_equal(ga, oa)
    # the cut-outs matter: without textures some of these rays hit the checker walls
    plain = OracleScene(scenes.tiny_scene("diffuse"))
    assert (plain.trace(rays)[0] != op).sum() > 20
    r.close()
    o.close()
    plain.close()


@pytest.mark.parametrize("variant", ["diffuse", "conductor"])
@pytest.mark.parametrize("kernel", [0, 1], ids=["mega", "wavefront"])
def test_textured_scene_parity(variant, kernel):
    """Albedo (sRGB), alpha cut-out, normal and metal/rough textures."""
    from optixpathtracer_amd import scenes

    from pathlib import Path
    golden = np.load(Path(__file__).resolve().parent / "golden" / "golden.npz")
    want = golden["textured_images"][list(golden["textured_variants"]).index(variant)]
    sc = scenes.textured_scene(variant)
    img, st = gpu_render(sc, 32, 24, 4, 1, 4, kernel=kernel)
    assert image_mse(img / 4.0, want / 4.0) <= MSE_TOL
    assert close_fraction(img, want) >= CLOSE_MIN
    ref, _ = oracle_render(sc, 32, 24, 4, 1, 4)
    np.testing.assert_array_equal(ref, want)


@pytest.mark.parametrize("n_lights", [4, 6])
@pytest.mark.parametrize("depth", [0, 1, 2])
@pytest.mark.parametrize("mode", [1, 3, 0])
def test_shallow_depth_and_light_count(depth, mode, n_lights):
    """Edge cases of the bounce loop (devicePrograms.cu:646): depth 0 renders black, depth 1
    is a bounce-0-only path whose BSDF sample is skipped (its ray would never be traced),
    and more lights than frames per batch turns the bounce-0 shadow table off.  Wavefront
    (batched and not) and megakernel agree bit for bit and match the oracle."""
    import dataclasses

    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene("diffuse")
    lights = np.concatenate([sc.lights, sc.lights[:1] * np.array([1, 1, 1, 0.5, 0.5, 0.5], np.float32)])
    while len(lights) < n_lights:
        extra = lights[-1:].copy()
        extra[0, 0] += 0.1 * len(lights)
        lights = np.concatenate([lights, extra])
    sc = dataclasses.replace(sc, lights=np.ascontiguousarray(lights[:n_lights], np.float32))
    wf, sw = gpu_render(sc, 40, 32, depth, 3, 5, mode=mode, kernel=1, frames_per_launch=4)
    wf1, _ = gpu_render(sc, 40, 32, depth, 3, 5, mode=mode, kernel=1, frames_per_launch=1)
    mega, sm = gpu_render(sc, 40, 32, depth, 3, 5, mode=mode, kernel=0)
    np.testing.assert_array_equal(wf, mega)
    np.testing.assert_array_equal(wf1, mega)
    assert sw["segments"] == sm["segments"]
    if depth == 0:
        assert np.all(wf == 0) and sw["segments"] == 0
        return
    o, segs = oracle_render(sc, 40, 32, depth, 3, 5, mode=mode)
    assert image_mse(wf / 5, o / 5) <= MSE_TOL
    assert close_fraction(wf, o) >= CLOSE_MIN
    assert abs(sw["segments"] - segs) <= 0.01 * segs + 2


@pytest.mark.parametrize("mode", [1, 3, 0])
def test_wavefront_two_streams_bit_identical(mode):
    """pt_set_wavefront_streams(2) (the auto default's choice for Conductor and Dielectric) alternates
    the batches of a call between two streams with their own queues; k_accum still adds the
    batches in frame order, so the sum -- fp32 and fp64 -- equals the one-stream sum bit for bit,
    also across calls and with the trace-kernel timing on (11 frames = batches of 4 + 4 + 3).
    0 (auto) gives the same image."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.tiny_scene("conductor" if mode == 0 else "diffuse")
    out = {}
    for streams in (1, 2, 3, 0):
        for fp64 in (False, True):
            r = setup_renderer(sc, 48, 40, 5, kernel=1)
            r.set_material_mode(mode)
            r.set_frames_per_launch(4)
            r.set_wavefront_streams(streams)
            r.set_kernel_timing(True)
            if fp64:
                r.set_accum_fp64(True)
            r.accum_clear()
            r.render_frames(7, 11)
            r.render_frames(18, 5)  # a second call continues the sum
            out[streams, fp64] = (r.accum(), r.stats())
            r.close()
    for fp64 in (False, True):
        for streams in (2, 3, 0):
            (a, sa), (b, sb) = out[1, fp64], out[streams, fp64]
            np.testing.assert_array_equal(a, b)
            assert sa["segments"] == sb["segments"]
            assert sa["trace_kernel_launches"] == sb["trace_kernel_launches"] > 0
    from optixpathtracer_amd.capi import PTError

    r = setup_renderer(sc, 16, 16, 2, kernel=1)
    for bad in (5, -1):  # 0 (auto) or 1 to 4 streams
        with pytest.raises(PTError):
            r.set_wavefront_streams(bad)
    r.close()
    mega, _ = gpu_render(sc, 48, 40, 5, 7, 11, mode=mode, kernel=0)
    one, _ = gpu_render(sc, 48, 40, 5, 7, 11, mode=mode, kernel=1, frames_per_launch=4)
    np.testing.assert_array_equal(one, mega)


@pytest.mark.parametrize("n_lights", [0, 1])
@pytest.mark.parametrize("variant,mode", [("conductor", 0), ("layered", 4), ("conductor", 4), ("diffuse", 0)])
def test_bucketed_shading_queues(variant, mode, n_lights):
    """Default / Layered shading runs over bucketed NEE and sample queues (k_shade_a ->
    k_shadow_vis -> k_nee_compact -> k_shade_nee -> k_shade_smp; buckets: conductor, smooth-top
    and rough-top layered).  No lights (no NEE items at all), one light (the bounce-0 table with
    batching, shadow rays without), conductor and layered items mixed or alone: the images equal
    the megakernel's (one thread per path, no queues) bit for bit, with equal segment counts."""
    import dataclasses

    from optixpathtracer_amd import scenes

    sc = scenes.tiny_scene(variant)
    sc = dataclasses.replace(sc, lights=np.ascontiguousarray(sc.lights[:n_lights], np.float32).reshape(n_lights, 6))
    mega, sm = gpu_render(sc, 48, 40, 4, 2, 6, mode=mode, kernel=0)
    for fpl in (1, 6):
        wf, sw = gpu_render(sc, 48, 40, 4, 2, 6, mode=mode, kernel=1, frames_per_launch=fpl)
        np.testing.assert_array_equal(wf, mega)
        assert sw["segments"] == sm["segments"]
    if n_lights == 0:
        assert np.all(mega == 0)
    else:
        o, segs = oracle_render(sc, 48, 40, 4, 2, 6, mode=mode)
        np.testing.assert_array_equal(mega, o)


@pytest.mark.parametrize("mode", [1, 0])
def test_trace_kernel_timing_counts_every_launch(mode):
    """pt_set_kernel_timing brackets every trace launch with an event pair (bench.py's
    roofline): fused modes trace max_bounces + 1 times per batch (k_extend, then one
    k_trace_pair per bounce), Default / Layered max_bounces times (k_extend per bounce)."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PTError
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.tiny_scene("diffuse")
    depth, spp, fpl = 3, 10, 4
    r = setup_renderer(sc, 32, 24, depth, kernel=1)
    r.set_material_mode(mode)
    r.set_frames_per_launch(fpl)
    r.set_kernel_timing(True)
    r.accum_clear()
    r.render_frames(1, spp)
    r.synchronize()
    st = r.stats()
    batches = -(-spp // fpl)
    per_batch = depth + 1 if mode == 1 else depth
    assert st["trace_kernel_launches"] == batches * per_batch
    assert st["trace_kernel_ms"] > 0.0
    with pytest.raises(PTError):
        r.SetMaxBounces(-1)
    r.close()


class _HipBuffers:
    """Device buffers from the HIP runtime libptamd itself links (no second runtime in the
    test process: torch bundles its own)."""

    def __init__(self):
        import ctypes as C

        self.C = C
        self.hip = C.CDLL("libamdhip64.so.7")
        self.ptrs = []

    def alloc(self, nbytes: int) -> int:
        p = self.C.c_void_p()
        assert self.hip.hipMalloc(self.C.byref(p), self.C.c_size_t(nbytes)) == 0
        self.ptrs.append(p.value)
        return p.value

    def upload(self, ptr: int, arr: np.ndarray) -> None:
        arr = np.ascontiguousarray(arr)
        assert self.hip.hipMemcpy(self.C.c_void_p(ptr), arr.ctypes.data_as(self.C.c_void_p),
                                  self.C.c_size_t(arr.nbytes), 1) == 0  # hipMemcpyHostToDevice

    def download(self, ptr: int, shape) -> np.ndarray:
        out = np.empty(shape, np.float32)
        assert self.hip.hipMemcpy(out.ctypes.data_as(self.C.c_void_p), self.C.c_void_p(ptr),
                                  self.C.c_size_t(out.nbytes), 2) == 0  # hipMemcpyDeviceToHost
        return out

    def free(self):
        for p in self.ptrs:
            self.hip.hipFree(self.C.c_void_p(p))


def test_launch_params_matches_render():
    """pt_launch (optixLaunch with a LaunchParams block, device colour buffer and device
    lights) writes the same 1-spp image as Render() for that frame id, leaves the renderer's
    own state alone, and rejects invalid parameters."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PTError
    from optixpathtracer_amd.renderer import camera_from_blender, setup_renderer

    sc = scenes.tiny_scene("layered")
    w, h, depth = 64, 48, 5
    r = setup_renderer(sc, w, h, depth)
    r.set_material_mode(0)
    ref = r.Render()  # frame.id 1
    p, iv, ip = camera_from_blender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg, w, h)
    hb = _HipBuffers()
    lights = hb.alloc(sc.lights.nbytes)  # pt_point_light[] on the device
    hb.upload(lights, sc.lights.astype(np.float32))
    buf = hb.alloc(w * h * 3 * 4)
    hb.upload(buf, np.full((h, w, 3), np.nan, np.float32))  # overwritten, not added
    r.launch(buf, (w, h), 1, p, iv, ip, lights, len(sc.lights), depth)
    r.synchronize()
    np.testing.assert_array_equal(hb.download(buf, (h, w, 3)), ref)
    # a different size and depth in the launch block; the renderer's own state is unchanged
    small = hb.alloc(32 * 24 * 3 * 4)
    p2, iv2, ip2 = camera_from_blender(sc.camera_blender_pos, sc.camera_blender_rot, sc.fov_deg, 32, 24)
    r.launch(small, (32, 24), 7, p2, iv2, ip2, lights, len(sc.lights), 2)
    r.synchronize()
    img = hb.download(small, (24, 32, 3))
    assert np.isfinite(img).all() and np.abs(img).sum() > 0
    again = r.Render()  # frame.id 2 at 64x48, depth 5
    r2 = setup_renderer(sc, w, h, depth)
    r2.set_material_mode(0)
    r2.Render()
    np.testing.assert_array_equal(again, r2.Render())
    r2.close()
    for bad in (dict(n=-1, d=depth), dict(n=len(sc.lights), d=-1)):
        with pytest.raises(PTError):
            r.launch(buf, (w, h), 1, p, iv, ip, lights, bad["n"], bad["d"])
    with pytest.raises(PTError):
        r.launch(0, (w, h), 1, p, iv, ip, lights, len(sc.lights), depth)
    r.launch(0, (0, 0), 1, p, iv, ip, 0, 0, depth)  # empty grid: no-op
    r.close()
    hb.free()


@pytest.mark.parametrize("mode", [1, 0])
def test_fullhd_largest_batch_bit_identical(diffuse_scene, mode):
    """Maximum queue size at the headline resolution: 1920x1080 with frames_per_launch far
    above the renderer's cap of 2^28 paths per batch (129 frames, 56 GB of queues: one batch of
    129 frames and a ragged one of 1) gives the accumulator of 64-frame batches (64 + 64 + 2)
    bit for bit, with the same segment count."""
    n = 130
    ref, sr = gpu_render(diffuse_scene, 1920, 1080, 8, 1, n, mode=mode, kernel=1, frames_per_launch=64)
    big, sb = gpu_render(diffuse_scene, 1920, 1080, 8, 1, n, mode=mode, kernel=1, frames_per_launch=4096)
    np.testing.assert_array_equal(big, ref)
    assert sb["segments"] == sr["segments"]
    assert np.isfinite(ref).all()
    assert sr["samples"] == 1920 * 1080 * n


@pytest.mark.parametrize("builder", [2, 4, 3], ids=["sah", "sah_gpu", "ploc"])
def test_degenerate_triangles_build_and_trace(builder):
    """Zero-area, duplicate-centroid and NaN-vertex triangles among valid ones: every builder
    finishes, and rays at the valid triangles hit them as the oracle says."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import OptixRenderer
    from oracle.oracle import OracleScene

    rng = np.random.default_rng(7)
    v = rng.uniform(-1, 1, size=(300, 3)).astype(np.float32)
    idx = np.arange(300, dtype=np.int32).reshape(100, 3)
    v[3:6] = v[3]            # triangle 1: a point
    v[6:9] = [[0, 0, 0], [1, 1, 1], [2, 2, 2]]  # triangle 2: a segment
    v[9:12] = v[12:15] + np.float32(1e-7)  # triangles 3 and 4 nearly coincide
    v[15] = np.nan           # triangle 5: a NaN vertex
    mesh = scenes.Mesh(vertices=v, indices=idx, normals=np.tile(np.float32([0, 0, 1]), (300, 1)))
    sc = scenes.Scene(meshes=[mesh], lights=np.zeros((0, 6), np.float32), camera_blender_pos=(0, 0, 0),
                      camera_blender_rot=(0, 0, 0))
    r = OptixRenderer(None, sc, bvh_builder=builder)
    tri = v[idx[20:60]]
    o = tri.mean(axis=1) + np.float32([0, 0, 3])
    rays = np.concatenate([o, np.tile(np.float32([0, 0, -1]), (40, 1)), np.zeros((40, 1), np.float32),
                           np.full((40, 1), 100, np.float32)], axis=1).astype(np.float32)
    p, t, u, vv, b = r.trace_rays(rays)
    r.close()
    ref = OracleScene(sc).trace(rays)
    np.testing.assert_array_equal(p, ref[0])
    np.testing.assert_array_equal(t, ref[1])
