#!/usr/bin/env python3
"""Generate tests/golden/layered.npz: Layered BSDF tuples from the CPU oracle.

GlossyDiffuse::f and ::Sample_f (GlossyDiffuse.h:141-524) are stochastic random walks that
advance the path seed; these tuples freeze the oracle's answers so that tests/test_layered_f64.py
can hold them against the independent float64 restatement of tests/pbrt_f64.py (written from the
reference header, not from oracle/pt_oracle.c).

    eval:   (wo, wi, roughness, albedo, seed) -> (f[3], seed')
    sample: (wo, roughness, albedo, seed)     -> (ok, f[3], pdf, wi[3], flags, seed')

    python tests/golden/make_layered_golden.py      # rewrites tests/golden/layered.npz
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent / "layered.npz"
N = 1200
# smooth top (alpha = r^2 < 1e-3: 0, 0.02, 0.031), both sides of the threshold, rough tops
ROUGHNESS = np.array([0.0, 0.02, 0.031, 0.033, 0.1, 0.2, 0.3, 0.5, 0.7, 0.8, 1.0], np.float32)


def directions(rng, n):
    d = rng.normal(size=(n, 3))
    # a tenth at grazing incidence (|z| < 0.02) on either side
    g = rng.random(n) < 0.1
    d[g, 2] = rng.uniform(-0.02, 0.02, size=g.sum()) * np.linalg.norm(d[g, :2], axis=1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d.astype(np.float32)


def make():
    rng = np.random.default_rng(20261016)
    wo, wi = directions(rng, N), directions(rng, N)
    rough = ROUGHNESS[np.arange(N) % len(ROUGHNESS)]
    albedo = rng.uniform(0.0, 1.0, size=(N, 3)).astype(np.float32)
    albedo[::17] = 1.0  # the reference's furnace albedo
    albedo[5::53] = 0.0  # black bottom layer: every bottom sample is rejected
    seed = rng.integers(0, 2**32, size=N, dtype=np.uint64).astype(np.uint32)
    ev = np.zeros((N, 3), np.float32)
    ev_seed = np.zeros(N, np.uint32)
    sm = np.zeros((N, 8), np.float32)
    sm_ok = np.zeros(N, np.int32)
    sm_seed = np.zeros(N, np.uint32)
    for k in range(N):
        ev[k], ev_seed[k] = O.bsdf_eval("layered", int(seed[k]), albedo[k], float(rough[k]), wo[k], wi[k])
        ok, out, s2 = O.bsdf_sample("layered", int(seed[k]), albedo[k], float(rough[k]), wo[k])
        sm_ok[k], sm[k], sm_seed[k] = int(ok), out, s2
    return dict(wo=wo, wi=wi, roughness=rough, albedo=albedo, seed=seed, eval_f=ev, eval_seed=ev_seed,
                sample_ok=sm_ok, sample_out=sm, sample_seed=sm_seed)


if __name__ == "__main__":
    np.savez_compressed(OUT, **make())
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")
