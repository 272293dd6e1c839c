"""Shared helpers for the parity tests: run the same config through the HIP product (C ABI)
and through the CPU oracle, and compare."""
from __future__ import annotations

import numpy as np


def image_mse(a: np.ndarray, b: np.ndarray) -> float:
    """Mean over pixels x channels of the squared difference, NaN -> 0 (the reference's EXR
    writer zeroes NaN pixels, Renderer/Images/WriteImage.cpp:52-55)."""
    a = np.nan_to_num(np.asarray(a, np.float64), nan=0.0)
    b = np.nan_to_num(np.asarray(b, np.float64), nan=0.0)
    return float(np.mean((a - b) ** 2))


def gpu_render(scene, width, height, max_bounces, first_frame, n_frames, mode=None, kernel=2, device=0,
               frames_per_launch=None, streams=None, kernel_timing=False):
    """Render through the C ABI.  kernel 2 (PT_KERNEL_AUTO, the default) is the product path
    bench.py times: the wavefront with the library's default batches (128 frames, within the queue
    budget) on auto streams (two for Conductor / Dielectric, one otherwise), unless
    frames_per_launch / streams override them."""
    from optixpathtracer_amd.renderer import setup_renderer

    r = setup_renderer(scene, width, height, max_bounces, device=device, kernel=kernel)
    if mode is not None:
        r.set_material_mode(mode)
    if frames_per_launch is not None:
        r.set_frames_per_launch(frames_per_launch)
    if streams is not None:
        r.set_wavefront_streams(streams)
    if kernel_timing:
        r.set_kernel_timing(True)
    r.accum_clear()
    r.render_frames(first_frame, n_frames)
    img = r.accum()
    st = r.stats()
    r.close()
    return img, st


def oracle_render(scene, width, height, max_bounces, first_frame, n_frames, mode=None, rect=None):
    from oracle.oracle import OracleScene

    o = OracleScene(scene)
    lp = o.launch(width, height, max_bounces, material_mode=mode)
    img, segs = o.render(lp, first_frame, n_frames, rect=rect)
    o.close()
    return img, segs


def random_rays(scene, n, seed=0, tmax=100.0):
    """Rays from random points in the scene bounds toward random directions, plus rays aimed
    at random triangle interiors/edges/vertices (edge and vertex hits exercise the tie rule)."""
    rng = np.random.default_rng(seed)
    verts = np.concatenate([m.vertices for m in scene.meshes])
    lo, hi = verts.min(0), verts.max(0)
    o = rng.uniform(lo - 0.5, hi + 0.5, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    # aim a third at triangle points (vertices, edge midpoints, interiors)
    tris = np.concatenate([m.vertices[m.indices] for m in scene.meshes])
    k = n // 3
    ti = rng.integers(0, len(tris), size=k)
    w = rng.dirichlet([1.0, 1.0, 1.0], size=k)
    w[: k // 3] = np.eye(3)[rng.integers(0, 3, size=k // 3)]  # vertices
    w[k // 3: 2 * k // 3] = [0.5, 0.5, 0.0]  # edge midpoints
    tgt = np.einsum("ij,ijk->ik", w, tris[ti])
    d[:k] = tgt - o[:k]
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    # axis-aligned rays (the other components +0 or -0) aimed at triangle points from outside:
    # exercise the slab test's zero-direction handling and the near/far plane selection
    k2 = n // 6
    if k2 > 0:
        ti = rng.integers(0, len(tris), size=k2)
        w = rng.dirichlet([1.0, 1.0, 1.0], size=k2)
        w[: k2 // 2] = np.eye(3)[rng.integers(0, 3, size=k2 // 2)]
        tgt = np.einsum("ij,ijk->ik", w, tris[ti]).astype(np.float32)
        axis = rng.integers(0, 3, size=k2)
        sign = rng.choice([-1.0, 1.0], size=k2)
        dd = np.where(rng.random((k2, 3)) < 0.5, np.float32(-0.0), np.float32(0.0)).astype(np.float32)
        dd[np.arange(k2), axis] = sign
        oo = tgt.copy()
        oo[np.arange(k2), axis] -= (sign * rng.uniform(0.5, 3.0, size=k2)).astype(np.float32)
        o[k: k + k2] = oo
        d[k: k + k2] = dd
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = o
    rays[:, 3:6] = d
    rays[:, 6] = 0.0
    rays[:, 7] = tmax
    return rays


def shared_edge_rays(scene, n, seed=0, tmax=100.0, far=False):
    """Rays aimed at points on edges shared by two triangles of a mesh, at grazing incidence
    (cos in [1e-3, 0.08] to the first triangle's plane) from 0.5 to 90 units away -- or, with
    far=True, from 40 to 95 units away in any direction.  These are the rays whose
    Moller-Trumbore answer can lie outside the triangle's own box (the config-5 event of
    round 1): both triangles of the edge may accept the hit with t a few ulps apart."""
    rng = np.random.default_rng(seed)
    pairs = []
    for m in scene.meshes:
        idx = np.asarray(m.indices)
        edges = {}
        for t, (a, b, c) in enumerate(idx):
            for u, v in ((a, b), (b, c), (c, a)):
                key = (min(u, v), max(u, v))
                edges.setdefault(key, []).append(t)
        shared = [(k, ts) for k, ts in edges.items() if len(ts) == 2]
        if shared:
            pairs.append((m, shared))
    rays = np.zeros((n, 8), np.float32)
    for i in range(n):
        m, shared = pairs[rng.integers(len(pairs))]
        (u, v), (ta, _) = shared[rng.integers(len(shared))]
        V = np.asarray(m.vertices, np.float64)
        s = rng.uniform(0.05, 0.95)
        p = V[u] * (1 - s) + V[v] * s
        tri = V[np.asarray(m.indices)[ta]]
        nrm = np.cross(tri[1] - tri[0], tri[2] - tri[0])
        nrm /= np.linalg.norm(nrm)
        if far:
            d = rng.normal(size=3)
            dist = rng.uniform(40.0, 95.0)
        else:
            tng = np.cross(nrm, rng.normal(size=3))
            tng /= np.linalg.norm(tng)
            c = rng.uniform(1e-3, 0.08)
            d = -np.sign(rng.uniform(-1, 1)) * c * nrm + np.sqrt(1 - c * c) * tng
            dist = rng.uniform(0.5, 90.0)
        d = d / np.linalg.norm(d)
        rays[i, 0:3] = p - dist * d
        rays[i, 3:6] = d
        rays[i, 7] = tmax
    return rays
