"""The GPU binned-SAH builder (PT_BVH_SAH_GPU, pt_sah_gpu.hip) against the
host builder it restates (PT_BVH_SAH, pt_sah.cpp): the downloaded BVH4 nodes and leaf-ordered
triangle records must be identical bit for bit -- the same binned-SAH decisions at every node, the
same stable partitions and middle cuts, hence the same DFS leaf order and the same collapse.  Both
replace optixAccelBuild (OptixRenderer.cpp:306-456).  Scenes cover both phases of the GPU build
(large nodes level by level, subtrees of <= 64 triangles per wave) and the degenerate inputs the
host build handles (coincident centroids, points, segments, NaN and infinite vertices)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SAH, SAH_GPU = 2, 4


def _soup(v, name="soup"):
    from optixpathtracer_amd import scenes

    v = np.ascontiguousarray(v, np.float32).reshape(-1, 3)
    idx = np.arange(len(v), dtype=np.int32).reshape(-1, 3)
    mesh = scenes.Mesh(vertices=v, indices=idx, normals=np.tile(np.float32([0, 0, 1]), (len(v), 1)))
    return scenes.Scene(meshes=[mesh], lights=np.zeros((0, 6), np.float32), camera_blender_pos=(0, 0, 0),
                        camera_blender_rot=(0, 0, 0))


def _bvh(sc, builder):
    from optixpathtracer_amd.renderer import OptixRenderer

    r = OptixRenderer(None, sc, bvh_builder=builder)
    nodes, tris = r.bvh_arrays()
    st = r.stats()
    r.close()
    return nodes, tris, st


def _same_bvh(sc):
    n0, t0, s0 = _bvh(sc, SAH)
    n1, t1, s1 = _bvh(sc, SAH_GPU)
    assert s0["bvh_nodes"] == s1["bvh_nodes"] and s0["bvh_depth"] == s1["bvh_depth"]
    np.testing.assert_array_equal(n1, n0)
    np.testing.assert_array_equal(t1, t0)
    return s0, s1


@pytest.mark.parametrize("name", ["tiny_layered", "sphere_box_diffuse", "textured_layered"])
def test_scenes_identical(name):
    from optixpathtracer_amd import scenes

    _same_bvh(scenes.make_scene(name))


def test_sponza_class_identical_and_fast():
    """configs[4]'s 250k-triangle scene: the same BVH4, and the GPU build (binary tree, leaf gather,
    collapse: pt_stats.bvh_build_ms) well inside the round-5 bar of 25 ms."""
    from optixpathtracer_amd import scenes

    s_host, s_gpu = _same_bvh(scenes.make_scene("sponza_class"))
    assert s_gpu["bvh_build_ms"] < 25.0, s_gpu["bvh_build_ms"]


@pytest.mark.parametrize("n", [2, 3, 5, 31, 32, 33, 64, 65, 127, 128, 129, 511, 512, 513, 1025, 5000])
def test_random_soups_identical(n):
    """Sizes at the phase boundaries (one wave builds subtrees of <= 64 triangles; PT_SAH_SMALL variants of 32-512 passed the same list), clustered and
    sliver triangles."""
    rng = np.random.default_rng(n)
    c = rng.normal(size=(n, 1, 3)).astype(np.float32) * np.float32(3)
    c[: n // 3] *= np.float32(0.01)  # a dense cluster
    v = c + rng.normal(size=(n, 3, 3)).astype(np.float32) * np.float32(0.05)
    v[n // 2:, 2] = v[n // 2:, 1] + np.float32(1e-6)  # slivers
    _same_bvh(_soup(v))


def test_coincident_and_degenerate_identical():
    """Copies of one triangle (no binned split: middle cuts), points, segments, a NaN and an
    infinite vertex, and a grid of centroids on one plane."""
    rng = np.random.default_rng(3)
    tri = rng.uniform(-1, 1, size=(1, 3, 3)).astype(np.float32)
    parts = [np.repeat(tri, 700, axis=0)]                       # 700 coincident triangles
    p = rng.uniform(-1, 1, size=(200, 1, 3)).astype(np.float32)
    parts.append(np.repeat(p, 3, axis=1))                       # points
    g = np.stack(np.meshgrid(np.arange(30), np.arange(30), indexing="ij"), -1).reshape(-1, 2).astype(np.float32)
    grid = np.zeros((len(g), 3, 3), np.float32)
    grid[:, :, :2] = g[:, None, :]
    grid[:, 1, 0] += 1
    grid[:, 2, 1] += 1                                          # 900 triangles, centroids on z = 0
    parts.append(grid)
    odd = rng.uniform(-1, 1, size=(40, 3, 3)).astype(np.float32)
    odd[3, 1, 2] = np.nan
    odd[7, 0, 0] = np.inf
    odd[9, 2, 1] = -np.inf
    parts.append(odd)
    _same_bvh(_soup(np.concatenate(parts)))


def test_default_builder_is_gpu_sah():
    """PT_BVH_AUTO resolves to the GPU SAH build: the default BVH equals the host SAH build's."""
    from optixpathtracer_amd import scenes

    sc = scenes.make_scene("tiny_layered")
    n0, t0, _ = _bvh(sc, 0)
    n1, t1, _ = _bvh(sc, SAH)
    np.testing.assert_array_equal(n0, n1)
    np.testing.assert_array_equal(t0, t1)


def test_signed_zero_coordinates_identical():
    """the GPU builder merges boxes with ordered-int atomics (-0 below +0) where the
    host's std::min / std::max keep the first zero seen; both now take -0 as +0, so a mesh whose
    coordinates mix -0 and +0 gives the same BVH4 bit for bit."""
    rng = np.random.default_rng(11)
    g = np.stack(np.meshgrid(np.arange(24), np.arange(24), indexing="ij"), -1).reshape(-1, 2).astype(np.float32)
    grid = np.zeros((len(g), 3, 3), np.float32)
    grid[:, :, :2] = g[:, None, :] - np.float32(12)
    grid[:, 1, 0] += 1
    grid[:, 2, 1] += 1
    # z = +0 or -0 per vertex, and some x / y coordinates at -0 as well
    grid[:, :, 2] = np.where(rng.random((len(g), 3)) < 0.5, np.float32(-0.0), np.float32(0.0))
    zx = grid[:, :, 0] == 0
    grid[:, :, 0][zx] = np.where(rng.random(int(zx.sum())) < 0.5, np.float32(-0.0), np.float32(0.0))
    assert np.signbit(grid).any()
    _same_bvh(_soup(grid))
