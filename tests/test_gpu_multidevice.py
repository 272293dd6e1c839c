"""Multi-GPU inside libptamd (SURVEY.md §8(b) threading row, §8(e); round-1 VERDICT "Next round" 3).

A renderer created with a device list (pt_options.n_devices) drives every listed device with its
own stream, scene copy and BVH, splits the frame ids of pt_render_frames into contiguous blocks
and sums the per-device fp32 sums with one ncclReduce (RCCL) onto the first device.  On a box
with one visible GPU the list is that one device: the RCCL communicator is still created and the
reduce still runs (a single-rank reduce), and the image must equal the plain single-device
renderer's bit for bit.  With N devices the image equals it up to the fp32 order of the N-way sum.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _visible_devices():
    import torch

    return list(range(max(1, torch.cuda.device_count())))


@pytest.mark.parametrize("mode", [1, 0], ids=["lambert", "default"])
def test_device_list_matches_single_device(mode):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("diffuse")
    devs = _visible_devices()
    w, h, spp = 320, 180, 13
    single = setup_renderer(sc, w, h, 8)
    single.set_material_mode(mode)
    single.set_frames_per_launch(4)
    single.accum_clear()
    single.render_frames(5, spp)
    ref = single.accum()
    st_ref = single.stats()
    single.close()

    multi = setup_renderer(sc, w, h, 8, devices=devs)
    assert multi.devices() == devs
    multi.set_material_mode(mode)
    multi.set_frames_per_launch(4)
    multi.accum_clear()
    multi.render_frames(5, spp)
    img = multi.accum()
    st = multi.stats()
    # accumulate a second call on top (the per-device sums are cumulative; the reduce re-sums)
    multi.render_frames(5 + spp, 3)
    img2 = multi.accum()
    multi.close()
    assert st["segments"] == st_ref["segments"] and st["samples"] == st_ref["samples"]
    if len(devs) == 1:
        np.testing.assert_array_equal(img, ref)
    else:
        np.testing.assert_allclose(img, ref, rtol=2e-6 * len(devs), atol=1e-7)
    assert (img2 >= img).all() and img2.sum() > img.sum()


def test_device_list_render_accumulate_mean():
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.tiny_scene("diffuse")
    a = setup_renderer(sc, 64, 48, 4)
    b = setup_renderer(sc, 64, 48, 4, devices=_visible_devices())
    ma = a.render_accumulate(8, 1)
    mb = b.render_accumulate(8, 1)
    a.close()
    b.close()
    np.testing.assert_allclose(mb, ma, rtol=1e-5, atol=1e-7)


def test_device_list_rejects_repeats_and_bad_ordinals():
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PTError
    from optixpathtracer_amd.renderer import OptixRenderer

    sc = scenes.tiny_scene("diffuse")
    with pytest.raises(PTError, match="repeats"):
        OptixRenderer(None, sc, devices=[0, 0])
    with pytest.raises(PTError, match="out of range"):
        OptixRenderer(None, sc, devices=[0, 999])


def test_fp64_accumulation_is_split_independent():
    """pt_set_accum_fp64 (round-1 VERDICT "missing" 6): the frames' fp32 radiance is summed in
    fp64, so a split of the frame ids over devices or processes -- partial fp64 sums added in
    fp64, as the ncclFloat64 reduce does -- gives the single-call image bit for bit after the
    final rounding to fp32, where the fp32 sums only agree to ~1e-6 relative."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("diffuse")
    w, h, first, spp = 320, 180, 3, 40
    r = setup_renderer(sc, w, h, 8)
    r.set_frames_per_launch(8)
    # the fp32 sum of the plain renderer, for the fp32-vs-fp64 comparison below
    r.accum_clear()
    r.render_frames(first, spp)
    ref32 = r.accum()
    r.set_accum_fp64(True)
    r.accum_clear()
    r.render_frames(first, spp)
    whole64, whole32 = r.accum64(), r.accum()
    np.testing.assert_array_equal(whole32, whole64.astype(np.float32))
    np.testing.assert_allclose(whole32, ref32, rtol=1e-5, atol=1e-7)
    # the same frames in 3 uneven shards (as 3 devices / ranks would render them)
    parts = []
    for a, b in [(0, 7), (7, 25), (25, spp)]:
        r.accum_clear()
        r.render_frames(first + a, b - a)
        parts.append(r.accum64())
    total = parts[0] + parts[1] + parts[2]
    mism = int((total.astype(np.float32) != whole32).sum())
    assert mism == 0, f"{mism} channels differ after the fp64 split sum"
    # cumulative calls: the fp64 sum keeps accumulating across pt_render_frames
    r.accum_clear()
    r.render_frames(first, 20)
    r.render_frames(first + 20, spp - 20)
    np.testing.assert_array_equal(r.accum(), whole32)
    r.close()


def test_fp64_accumulation_through_the_device_list():
    """The multi-device renderer reduces its fp64 partial sums (ncclFloat64) onto the first
    device and converts the total to the fp32 sum buffer: equal to the single-device fp64 image."""
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    sc = scenes.sphere_in_box("diffuse")
    w, h, spp = 256, 144, 11
    single = setup_renderer(sc, w, h, 8)
    single.set_accum_fp64(True)
    single.accum_clear()
    single.render_frames(2, spp)
    ref = single.accum()
    single.close()
    multi = setup_renderer(sc, w, h, 8, devices=_visible_devices())
    multi.set_accum_fp64(True)
    multi.accum_clear()
    multi.render_frames(2, spp)
    img = multi.accum()
    multi.close()
    np.testing.assert_array_equal(img, ref)


def test_fp64_accumulation_rejects_megakernel():
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.capi import PT_KERNEL_MEGA, PTError
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(scenes.tiny_scene("diffuse"), 32, 24, 4)
    r.set_accum_fp64(True)
    r.set_kernel(PT_KERNEL_MEGA)
    r.accum_clear()
    with pytest.raises(PTError, match="wavefront"):
        r.render_frames(1, 2)
    r.close()
