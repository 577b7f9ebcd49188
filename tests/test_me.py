"""f2 full-resolution motion search (x265amd_motion_search).

Parity chain: the reference's own MotionEstimate::motionEstimate (motion.cpp:571-1172,
driven through oracle/ref_shim.cpp with its own BitCost tables) -> golden hashes (the `me`
cases of cases.all_cases: every luma PU shape with HEX / subme 2 as at --preset medium,
DIA and subme 0 / 1 on the square sizes; STAR / UMH and subme 3-7 checked by the oracle
against the reference here and by the GPU against the oracle) -> oracle restatement (xo_motion_search) [CPU]
-> gfx950 kernel k_motion_search [GPU].  Output MVs and costs bit-exact.
"""
import numpy as np
import pytest

from cases import LUMA_PU, case_me, me_cases, run_cpu, run_gpu, seed_of
from pyoracle import CpuOracle, available


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_me_oracle_matches_reference(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    for (w, h) in ((8, 8), (16, 16), (64, 64), (32, 8), (12, 16)):
        for method, subme in ((1, 2), (0, 1), (2, 3), (2, 4), (1, 5), (2, 6), (2, 7), (3, 2), (3, 3)):
            c = case_me(w, h, method, subme, 57 if method else 16, depth, 64, seed_of("me-r", depth, w, h, method))
            a, b = run_cpu(c, orc), run_cpu(c, ref)
            for k in c.outs:
                assert np.array_equal(a[k], b[k]), (c.key(), k)


def far_cases(depth, n=24):
    """MVP far off the motion and the range boxed around it, so the search usually starts at MV 0 outside the
    range (motion.cpp:615-624): every search method, whose patterns then cost points beside the out-of-range
    origin on the sides the reference does not check (STAR's per-point checks, :367-561)"""
    return [case_me(w, h, m, s, 57, depth, n, seed_of("me-far", depth, w, h, m), box=16, far=24)
            for (w, h) in ((8, 8), (16, 16), (32, 32), (64, 64), (32, 16), (8, 32))
            for m, s in ((0, 2), (1, 2), (2, 2), (2, 3), (3, 2))]


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_me_far_oracle_matches_reference(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    starts_outside = 0
    for c in far_cases(depth):
        a, b = run_cpu(c, orc), run_cpu(c, ref)
        for k in c.outs:
            assert np.array_equal(a[k], b[k]), (c.key(), k)
        rng = c.bufs["rng"].reshape(-1, 4)
        starts_outside += int(((rng[:, 0] > 0) | (rng[:, 2] < 0) | (rng[:, 1] > 0) | (rng[:, 3] < 0)).sum())
    assert starts_outside > 100


def full_cases(depth, n=16):
    """--me full (method 4) over MVP +- 16 (the exhaustive search is slow on the CPU), every luma PU shape,
    subme 2 and (with chroma SATD) 3"""
    return [case_me(w, h, 4, 2 + (i & 1), 16, depth, n, seed_of("me-full", depth, w, h), box=16)
            for i, (w, h) in enumerate(LUMA_PU[1:])]


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_me_full_oracle_matches_reference(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    for c in full_cases(depth):
        a, b = run_cpu(c, orc), run_cpu(c, ref)
        for k in c.outs:
            assert np.array_equal(a[k], b[k]), (c.key(), k)


@pytest.mark.parametrize("depth", [8, 10])
def test_me_cases_exercise_search(oracle_libs, depth):
    """results include quarter-pel, half-pel and full-pel MVs and MVs away from the MVP"""
    orc = CpuOracle("oracle", depth)
    mvs = np.concatenate([run_cpu(c, orc)["out_mv"].reshape(-1, 2) for c in me_cases(depth)[:8]])
    frac = mvs & 3
    assert (frac == 1).any() or (frac == 3).any()
    assert (frac == 2).any() and (frac == 0).all(axis=1).any()


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_me_gpu_matches_oracle(gpu_prims, oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    cases = me_cases(depth) + [case_me(w, h, 1, 2, 57, depth, 512, seed_of("me-g", depth, w, h))
                               for (w, h) in ((8, 8), (16, 16), (32, 32), (64, 64))]
    # --me umh (method 3): every luma PU shape, plus the sub-pel levels with chroma SATD
    cases += [case_me(w, h, 3, 2, 57, depth, 48, seed_of("me-umh", depth, w, h)) for (w, h) in LUMA_PU[1:]]
    cases += [case_me(w, h, 3, s, 57, depth, 128, seed_of("me-umh-s", depth, w, h, s))
              for (w, h) in ((8, 8), (32, 32), (64, 64)) for s in (3, 5)]
    # --me full (method 4): the exhaustive search kernel, then the lockstep refine
    cases += full_cases(depth, 32)
    # the search origin outside the MV range (MV 0 against a far MVP), every method
    cases += far_cases(depth)
    cases += [case_me(w, h, 4, 2, 57, depth, 24, seed_of("me-full-g", depth, w, h), box=57)
              for (w, h) in ((8, 8), (64, 64), (24, 32))]
    bad = []
    for c in cases:
        got, exp = run_gpu(c, gpu_prims), run_cpu(c, orc)
        for k in c.outs:
            if not np.array_equal(got[k], exp[k]):
                bad.append((c.key(), k, int((got[k] != exp[k]).sum())))
    assert not bad, bad[:6]


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_me_gpu_multi_batch_call(gpu_prims, oracle_libs, depth):
    """Several PU sizes in ONE x265amd_motion_search call (they run concurrently on the library's
    internal streams, joined back into the caller's stream): every batch equals the oracle."""
    import torch

    orc = CpuOracle("oracle", depth)
    cases = [case_me(w, h, m, 2, 57, depth, 384, seed_of("me-m", depth, w, h, m))
             for (w, h, m) in ((8, 8, 1), (16, 16, 0), (32, 32, 1), (64, 64, 2), (12, 16, 1), (64, 16, 1))]
    dv = lambda v: torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) else v
    jobs, keep = [], []
    for c in cases:
        b = {k: dv(v) for k, v in c.bufs.items()}
        p = c.params
        jobs.append(dict(w=p["w"], h=p["h"], method=p["method"], subme=p["subme"], merange=p["merange"],
                         max_cand=p["max_cand"], f=b["f"], fs=b["fs"], fo=b["fo"], r=b["r"], rs=b["rs"], ro=b["ro"],
                         rng=b["rng"], mvp=b["mvp"], mvc=b["mvc"], numc=b["numc"], tab=b["tab"], tab_off=b["tab_off"],
                         out_mv=b["out_mv"], out_cost=b["out_cost"]))
        keep.append(b)
    gpu_prims.motion_search_multi(depth, jobs)
    torch.cuda.synchronize()
    for c, b in zip(cases, keep):
        exp = run_cpu(c, orc)
        for k in c.outs:
            np.testing.assert_array_equal(b[k].cpu().numpy(), exp[k])


def window_cases(depth, n=96):
    """Round 6: with X265AMD_ME_LDS_R = r, PUs of 128 or more 4x4 units searched by DIA / HEX stage the
    reference within r pixels of the search start in LDS (k_motion_search<P, G, true>).  With the range boxed
    to the MVP +- merange, as Search::setSearchRange makes it, and r = merange the window (2 merange + w + 17)^2
    fits the launch's LDS (merange 57 at 8-bit: 195 x 195 bytes; merange 32 at 10-bit), so every candidate
    reads LDS; with r = 8 searches step out of the window and mix LDS and plane reads, as do the far cases
    (MV 0 outside the box)."""
    m = 57 if depth == 8 else 32
    out = [case_me(w, h, meth, s, m, depth, n, seed_of("me-win", depth, w, h, meth, s), box=m)
           for (w, h) in ((64, 64), (64, 32), (32, 64), (48, 64), (64, 48))
           for meth, s in ((1, 2), (0, 0), (0, 1), (1, 3))]
    out += [case_me(w, h, meth, 2, m, depth, n, seed_of("me-win-far", depth, w, h, meth), box=16, far=24)
            for (w, h) in ((64, 64), (64, 32)) for meth in (0, 1)]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
@pytest.mark.parametrize("reach", [8, 57])
def test_me_gpu_lds_window_matches_oracle(gpu_prims, oracle_libs, depth, reach, monkeypatch):
    monkeypatch.setenv("X265AMD_ME_LDS_R", str(reach))     # read by the library at every launch
    orc = CpuOracle("oracle", depth)
    bad = []
    for c in window_cases(depth):
        got, exp = run_gpu(c, gpu_prims), run_cpu(c, orc)
        for k in c.outs:
            if not np.array_equal(got[k], exp[k]):
                bad.append((c.key(), k, int((got[k] != exp[k]).sum())))
    assert not bad, bad[:6]


@pytest.mark.parametrize("depth", [8, 10])
def test_me_window_cases_fit_the_window(depth):
    """host-side arithmetic of the window launch (me.hip launch_me): the boxed cases' windows fit"""
    for c in window_cases(depth):
        p = c.params
        if p.get("far"):
            continue
        rng = c.bufs["rng"].reshape(-1, 4).astype(np.int64)
        sz = 1 if depth == 8 else 2
        ww, wh = 2 * p["merange"] + p["w"] + 17, 2 * p["merange"] + p["h"] + 17
        cap = ((ww * sz + 6) >> 2) * 4 * wh
        assert cap <= 64 * 1024
        assert (rng[:, 2] - rng[:, 0] <= 2 * p["merange"]).all() and (rng[:, 3] - rng[:, 1] <= 2 * p["merange"]).all()
