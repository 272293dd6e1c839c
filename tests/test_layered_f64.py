"""A second, independent reading of the Layered BSDF.

GlossyDiffuse::f and ::Sample_f (GlossyDiffuse.h:141-524) are the dominant cost of the Default and
Layered configs, and the kernels (pt_bsdf.h) and the oracle (oracle/pt_oracle.c) share one
reading of them.  tests/pbrt_f64.py restates both in float64 from the header alone, driven by
the same TEA/LCG draws: the path seed for the interface samples, the private Russian-roulette
streams tea(tea(tea(tea(u32(wo.x*1000), u32(wo.y*1000)), u32(wi.x*1000)), u32(wi.y*1000)), seed)
(f) and tea(tea(u32(wo.x*1000), u32(wo.y*1000)), seed) (Sample_f).  Here the restatement is held
against tests/golden/layered.npz, 1,200 eval and 1,200 sample tuples frozen from the oracle
(tests/golden/make_layered_golden.py), which the oracle must still reproduce bit for bit.

Bars.  The restatement sees the same random numbers as the oracle and float64 thresholds within
float32 rounding of the oracle's, so a discrete decision (R vs T, Russian roulette, total
internal reflection) can differ only when a draw falls within a few ulp of its threshold: at most
FLIP_FRAC of the tuples may disagree on the consumed seed, ok or flags (0 of 2,400 do today).
All others must agree on the seed exactly and on the values:
  * eval f (relative to the largest component):                 F_RTOL
  * sample direction (absolute, unit vectors):                  DIR_ATOL
  * sample weight f / pdf (the estimator's factor):             F_RTOL
  * sample f and pdf separately, where D is well conditioned:   F_RTOL
The last bar excludes the near-specular rough tops (1e-3 <= alpha < 0.04), where the
Trowbridge-Reitz D of a microfacet normal within a degree of +z is evaluated through
sin^2 = 1 - cos^2 and float32 leaves only a few significant bits (f and pdf reach 1e10..1e22 and
move together by up to ~25 %; their ratio still meets F_RTOL).  Measured worst cases: eval 2.6e-5,
direction 5.1e-6, weight 4.0e-5, f / pdf 4.9e-5.

Each seeded fault of the restatement (a misreading a shared C/HIP reading could carry) must
fail these bars.
"""
from pathlib import Path

import numpy as np
import pytest

import pbrt_f64 as P

GOLDEN = Path(__file__).resolve().parent / "golden" / "layered.npz"
FLIP_FRAC = 0.005
F_RTOL = 1e-4
DIR_ATOL = 2e-5


@pytest.fixture(scope="module")
def g():
    return np.load(GOLDEN)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = np.max(np.abs(b))
    if scale == 0.0:
        return float(np.max(np.abs(a)) > 0.0)
    return float(np.max(np.abs(a - b)) / scale)


def eval_agreement(g, fault=None):
    """(fraction with a different seed', list of value errors of the others)."""
    n = len(g["seed"])
    flips, errs = 0, []
    for k in range(n):
        f, s = P.layered_f(int(g["seed"][k]), g["albedo"][k], float(g["roughness"][k]), g["wo"][k], g["wi"][k],
                           fault=fault)
        if s != int(g["eval_seed"][k]):
            flips += 1
            continue
        errs.append(_rel(f, g["eval_f"][k]))
    return flips / n, np.array(errs)


def sample_agreement(g, fault=None):
    """(fraction with a different seed' / ok / flags, direction errors, weight errors, f/pdf errors
    where D is well conditioned)."""
    n = len(g["seed"])
    flips, ed, ew, efp = 0, [], [], []
    for k in range(n):
        a = float(g["roughness"][k]) ** 2
        ok, f, pdf, d, flags, s = P.layered_sample(int(g["seed"][k]), g["albedo"][k], float(g["roughness"][k]),
                                                   g["wo"][k], fault=fault)
        o = g["sample_out"][k].astype(np.float64)
        if s != int(g["sample_seed"][k]) or int(ok) != int(g["sample_ok"][k]) or (ok and flags != int(o[7])):
            flips += 1
            continue
        if not ok:
            continue
        ed.append(float(np.max(np.abs(np.array(d) - o[4:7]))))
        ew.append(_rel(np.array(f) / pdf, o[:3] / o[3]))
        if not (1e-3 <= a < 0.04):
            efp.append(max(_rel(f, o[:3]), abs(pdf - o[3]) / abs(o[3])))
    return flips / n, np.array(ed), np.array(ew), np.array(efp)


def test_oracle_reproduces_layered_golden(g):
    """The frozen tuples are the oracle's current answers, bit for bit."""
    from oracle import oracle as O

    for k in range(0, len(g["seed"]), 7):
        f, s = O.bsdf_eval("layered", int(g["seed"][k]), g["albedo"][k], float(g["roughness"][k]), g["wo"][k],
                           g["wi"][k])
        np.testing.assert_array_equal(f, g["eval_f"][k])
        assert s == int(g["eval_seed"][k])
        ok, out, s2 = O.bsdf_sample("layered", int(g["seed"][k]), g["albedo"][k], float(g["roughness"][k]),
                                    g["wo"][k])
        assert int(ok) == int(g["sample_ok"][k]) and s2 == int(g["sample_seed"][k])
        np.testing.assert_array_equal(out, g["sample_out"][k])


def test_golden_covers_the_walks(g):
    """The tuples reach every branch worth pinning: reflection and transmission evals, smooth
    and rough tops, zero values, successful and failed samples, reflected (entrance) and
    transmitted (walk) samples.  A transmission eval (wo, wi in opposite hemispheres: the exit
    interface is the bottom) is always 0: its wis sample asks the Lambert bottom for a
    transmission, which LambertDiffuse::Sample_f refuses without drawing (LambertDiffuse.h:113),
    so every one of the 5 samples continues (GlossyDiffuse.h:238-240)."""
    same = g["wo"][:, 2] * g["wi"][:, 2] > 0
    nonzero = np.any(g["eval_f"] != 0, axis=1)
    assert (same & nonzero).sum() > 300 and (~same).sum() > 300
    assert not (~same & nonzero).any()
    smooth = g["roughness"].astype(np.float64) ** 2 < 1e-3
    assert (smooth & nonzero).sum() > 100 and (~smooth & nonzero).sum() > 300
    ok = g["sample_ok"] == 1
    flags = g["sample_out"][:, 7].astype(int)
    assert ok.sum() > 600 and (~ok).sum() > 100
    assert ((flags & 1) & ok).sum() > 100 and ((flags & 2) > 0).sum() > 100
    assert ((flags & 4) > 0).sum() > 50 and ((flags & 8) > 0).sum() > 300


def test_layered_f_matches_independent_reading(g):
    flips, errs = eval_agreement(g)
    print(f"eval: seed flips {flips:.4f}, f error max {errs.max():.3e} p99 {np.quantile(errs, 0.99):.3e}")
    assert flips <= FLIP_FRAC
    assert np.mean(errs <= F_RTOL) >= 1.0 - FLIP_FRAC, np.sort(errs)[-5:]


def test_layered_sample_matches_independent_reading(g):
    flips, ed, ew, efp = sample_agreement(g)
    print(f"sample: flips {flips:.4f}, dir {ed.max():.3e}, weight {ew.max():.3e}, f/pdf {efp.max():.3e}")
    assert flips <= FLIP_FRAC
    for e, tol in ((ed, DIR_ATOL), (ew, F_RTOL), (efp, F_RTOL)):
        assert np.mean(e <= tol) >= 1.0 - FLIP_FRAC, np.sort(e)[-5:]


def _passes_eval(g, fault):
    flips, errs = eval_agreement(g, fault)
    return flips <= FLIP_FRAC and np.mean(errs <= F_RTOL) >= 1.0 - FLIP_FRAC


def _passes_sample(g, fault):
    flips, ed, ew, efp = sample_agreement(g, fault)
    return flips <= FLIP_FRAC and all(np.mean(e <= t) >= 1.0 - FLIP_FRAC
                                      for e, t in ((ed, DIR_ATOL), (ew, F_RTOL), (efp, F_RTOL)))


@pytest.mark.parametrize("fault", ["swap_exit", "no_flipmode", "rr_main_seed", "wo_seed_only"])
def test_seeded_eval_fault_is_caught(g, fault):
    """Exit / non-exit interfaces swapped (:183-203), wis sampled without FlipMode (:238), Russian
    roulette on the path seed (:220-222), private stream without wi (:215-218): each fails."""
    assert not _passes_eval(g, fault)


@pytest.mark.parametrize("fault", ["seed_before_entrance", "no_cos"])
def test_seeded_sample_fault_is_caught(g, fault):
    """Private stream seeded before the entrance sample (:417-418), |cos| dropped (:521)."""
    assert not _passes_sample(g, fault)
