"""The debug pixel (the reference's isDebugRay, devicePrograms.cu:637-644, printed at :428-437)
as data: the GPU's per-bounce records of one path equal the CPU oracle's bit for bit, in the
megakernel and the wavefront (fused and RNG-coupled material modes, textured scenes)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ["position", "albedo", "shading_normal", "geometry_normal", "roughness", "metallic", "beta", "radiance"]


def _gpu_records(r):
    out = []
    for d in r.debug_path():
        row = [np.int32(d["bounce"]).view(np.float32), np.int32(d["prim"]).view(np.float32)]
        for f in FIELDS:
            v = d[f]
            row += v if isinstance(v, list) else [v]
        out.append(row)
    return np.array(out, np.float32).reshape(-1, 22)


@pytest.mark.parametrize("kernel", [0, 1], ids=["mega", "wavefront"])
@pytest.mark.parametrize("scene_name,mode", [("tiny:diffuse", 1), ("tiny:conductor", 0), ("sphere_box_diffuse", 1),
                                             ("sphere_box_conductor", 0), ("textured:diffuse", 0),
                                             ("sphere_box_dielectric20", 3)])
def test_debug_path_matches_oracle(kernel, scene_name, mode):
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer
    from oracle.oracle import OracleScene

    if scene_name.startswith("tiny:"):
        sc = scenes.tiny_scene(scene_name[5:])
    elif scene_name.startswith("textured:"):
        sc = scenes.textured_scene(scene_name[9:])
    else:
        sc = scenes.make_scene(scene_name)
    w, h, depth = 96, 64, 8
    r = setup_renderer(sc, w, h, depth, kernel=kernel)
    r.set_material_mode(mode)
    r.set_frames_per_launch(3)
    o = OracleScene(sc)
    lp = o.launch(w, h, depth, material_mode=mode)
    checked = 0
    for x, y, frame in [(48, 32, 10), (10, 5, 3), (90, 60, 7), (33, 47, 1)]:
        r.set_debug_pixel(x, y, frame)
        r.accum_clear()
        r.render_frames(1, 12)  # the debug frame is one of several in its batch
        g = _gpu_records(r)
        ref, _ = o.sample_path_debug(lp, x, y, frame)
        assert g.shape == ref.shape, (x, y, frame, g.shape, ref.shape)
        np.testing.assert_array_equal(g.view(np.uint32), ref.view(np.uint32))
        checked += len(ref)
    assert checked >= 1  # at least one shaded bounce compared
    r.set_debug_pixel(-1, 0, 0)
    r.close()
    o.close()
