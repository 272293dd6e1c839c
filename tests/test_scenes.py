"""Synthetic scene construction: sizes, winding, normals."""
import numpy as np

from optixpathtracer_amd import scenes


def _tri_normals(m):
    v = m.vertices[m.indices]
    return np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])


def test_sphere_box_size_and_materials():
    sc = scenes.sphere_in_box("diffuse")
    assert len(sc.meshes) == 36 + 5
    assert sc.n_triangles == 36 * 960 + 10 == 34570
    assert sc.lights.shape == (4, 6)
    spheres = [m for m in sc.meshes if m.name.startswith("sphere")]
    assert sorted({round(m.roughness, 3) for m in spheres}) == [0.0, 0.2, 0.4, 0.6, 0.8, 1.0]
    assert scenes.sphere_in_box("conductor").meshes[0].metallic == 1.0
    assert scenes.sphere_in_box("dielectric20").lights[0, 3] == 20.0


def test_sphere_winding_outward_and_smooth_normals():
    sc = scenes.sphere_in_box("diffuse")
    m = sc.meshes[7]
    c = m.vertices.mean(0)
    v = m.vertices[m.indices]
    n = _tri_normals(m)
    assert np.all(np.einsum("ij,ij->i", n, v.mean(1) - c) > 0)
    np.testing.assert_allclose(np.linalg.norm(m.normals, axis=1), 1.0, atol=1e-6)
    assert np.all(np.einsum("ij,ij->i", m.normals, m.vertices - c) > 0)


def test_box_walls_face_inward():
    sc = scenes.sphere_in_box("diffuse")
    centre = np.array([0.9, 1.0, 0.0], np.float32)  # engine coords inside the box
    for m in sc.meshes:
        if m.name.startswith("sphere"):
            continue
        v = m.vertices[m.indices]
        n = _tri_normals(m)
        assert np.all(np.einsum("ij,ij->i", n, centre - v.mean(1)) > 0), m.name


def test_blender_to_engine():
    np.testing.assert_array_equal(scenes.blender_to_engine([1.0, 2.0, 3.0]), [1.0, 3.0, -2.0])


def test_sponza_class_scale():
    sc = scenes.sponza_class()
    assert 240_000 <= sc.n_triangles <= 260_000
    assert len({m.metallic for m in sc.meshes}) == 2
    assert sc.lights[0, 3] == 100.0
    for m in sc.meshes[:20]:
        assert m.indices.max() < len(m.vertices)
