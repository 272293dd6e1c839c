"""glTF end to end on the GPU: a textured scene written as glTF 2.0, loaded by the C++
loader (pt_model_load_gltf), renders bit-identically to the in-memory scene and matches
the oracle (SURVEY.md §8(f) rows f1 + f2)."""
import numpy as np
import pytest

from gltf_export import scene_to_gltf
from helpers import gpu_render, image_mse, oracle_render

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["diffuse", "conductor"])
def test_gltf_round_trip_render(tmp_path, variant):
    from optixpathtracer_amd import gltf, scenes

    sc = scenes.textured_scene(variant)
    p = scene_to_gltf(sc, tmp_path)
    loaded = gltf.load_gltf(p, lights=sc.lights, camera_blender_pos=sc.camera_blender_pos,
                            camera_blender_rot=sc.camera_blender_rot, material_mode=sc.material_mode)
    assert len(loaded.meshes) == len(sc.meshes) and len(loaded.textures) == len(sc.textures)
    for t0, t1 in zip(sc.textures, loaded.textures):
        np.testing.assert_array_equal(t0, t1)
    a, _ = gpu_render(sc, 40, 30, 4, 1, 3, kernel=1)
    b, _ = gpu_render(loaded, 40, 30, 4, 1, 3, kernel=1)
    np.testing.assert_array_equal(a, b)
    ref, _ = oracle_render(loaded, 40, 30, 4, 1, 3)
    assert image_mse(b / 3.0, ref / 3.0) <= 1e-5
