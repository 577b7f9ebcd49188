"""f1 lookahead lowres pipeline (x265amd_lowres_init / x265amd_lowres_intra).

Parity chain:
  reference frameInitLowres + extendPicBorder (lowres.cpp:151-162) and
  LookaheadTLD::lowresIntraEstimate (slicetype.cpp:230-330), run through
  oracle/ref_shim.cpp on the caller's buffers
    -> golden hashes (tests/golden, lowres cases of cases.all_cases)
    -> oracle restatement (x265_oracle.c xo_lowres_*)          [CPU tests]
    -> gfx950 kernels (csrc/lowres.hip)                         [GPU tests]
Outputs compared whole: the four border-extended planes (sentinel-filled
buffers, so any write outside them shows), per-CU intra cost / mode / lowres
cost, per-row SATD sums and the frame cost estimates, with and without AQ.
"""
import numpy as np
import pytest

from cases import case_lowres, lowres_cases, run_cpu, run_gpu, seed_of
from pyoracle import CpuOracle, available


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_lowres_oracle_matches_reference(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    for (W, H, n, aq) in ((96, 64, 2, True), (232, 136, 1, False), (1920, 1080, 1, True)):
        c = case_lowres(W, H, n, aq, depth, seed_of("lr-r", depth, W, H))
        a, b = run_cpu(c, orc), run_cpu(c, ref)
        for k in c.outs:
            assert np.array_equal(a[k], b[k]), (c.key(), k)


@pytest.mark.parametrize("depth", [8, 10])
def test_lowres_modes_cover_families(oracle_libs, depth):
    """the committed cases pick DC, planar and angular modes (all three code paths are pinned)"""
    orc = CpuOracle("oracle", depth)
    modes = np.concatenate([run_cpu(c, orc)["im"] for c in lowres_cases(depth)])
    assert (modes == 0).any() and (modes == 1).any() and (modes >= 2).any()


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_lowres_gpu_matches_oracle(gpu_prims, oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    cases = lowres_cases(depth) + [case_lowres(1920, 1080, 3, True, depth, seed_of("lr-g", depth)),
                                   case_lowres(3840, 2160, 1, False, depth, seed_of("lr-g4k", depth))]
    bad = []
    for c in cases:
        got, exp = run_gpu(c, gpu_prims), run_cpu(c, orc)
        for k in c.outs:
            if not np.array_equal(got[k], exp[k]):
                bad.append((c.key(), k, int((got[k] != exp[k]).sum())))
    assert not bad, bad[:6]


# ---------------------------------------------------------------- P-frame cost estimate (motion search)
from cases import MVCOST_RANGE, case_lowres_pcost, lowres_pcost_cases, mvcost_table  # noqa: E402


@pytest.mark.parametrize("depth", [8, 10])
def test_mvcost_table_matches_reference_fixture(oracle_libs, depth):
    """the oracle's BitCost restatement == the reference's table committed by make_golden.py"""
    assert np.array_equal(CpuOracle("oracle", depth).mvcost_table(MVCOST_RANGE), mvcost_table(depth))


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_pcost_oracle_matches_reference(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    for (W, H, n, rps, ns, aq) in ((192, 128, 1, 0, 0, False), (1920, 1080, 1, 10, 6, True),
                                   (1280, 720, 1, 0, 0, True)):
        c = case_lowres_pcost(W, H, n, rps, ns, aq, depth, seed_of("lp-r", depth, W, H))
        a, b = run_cpu(c, orc), run_cpu(c, ref)
        for k in c.outs:
            assert np.array_equal(a[k], b[k]), (c.key(), k)


@pytest.mark.parametrize("depth", [8, 10])
def test_pcost_cases_exercise_search(oracle_libs, depth):
    """the committed cases choose intra and inter CUs, sub-pel and full-pel MVs, non-zero MVs"""
    orc = CpuOracle("oracle", depth)
    mbs, mvs, lc = [], [], []
    for c in lowres_pcost_cases(depth):
        o = run_cpu(c, orc)
        mbs.append(o["mbs"]), mvs.append(o["mvs"].reshape(-1, 2)), lc.append(o["lc"])
    mvs, lc = np.concatenate(mvs), np.concatenate(lc)
    assert np.concatenate(mbs).sum() > 0
    assert ((lc >> 14) == 1).any() and ((lc >> 14) == 0).any()
    assert (mvs != 0).any() and ((mvs & 3) != 0).any() and ((mvs & 3) == 0).all(axis=1).any()


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_pcost_gpu_matches_oracle(gpu_prims, oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    cases = lowres_pcost_cases(depth) + [
        case_lowres_pcost(1920, 1080, 2, 10, 6, True, depth, seed_of("lp-g", depth)),
        case_lowres_pcost(1920, 1080, 1, 0, 0, False, depth, seed_of("lp-g1", depth))]
    bad = []
    for c in cases:
        got, exp = run_gpu(c, gpu_prims), run_cpu(c, orc)
        for k in c.outs:
            if not np.array_equal(got[k], exp[k]):
                bad.append((c.key(), k, int((got[k] != exp[k]).sum())))
    assert not bad, bad[:6]
