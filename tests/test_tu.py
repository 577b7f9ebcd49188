"""f3 fused TU pipeline (include/x265_amd.h x265amd_tu_pipeline).

Parity chain:
  reference Quant::transformNxN / invtransformNxN (quant.cpp:397-546, driven by
  oracle/ref_shim.cpp exactly as search.cpp:689-706 chains them)
    -> golden hashes (tests/golden, tu cases of cases.all_cases)
    -> oracle restatement (x265_oracle.c xo_tu_pipeline)      [CPU tests]
    -> gfx950 kernel k_tu (csrc/tu.hip)                       [GPU tests]
All outputs (residual buffer, coefficients, reconstruction, numSig) bit-exact.
"""
import numpy as np
import pytest

from cases import case_tu, run_cpu, run_gpu, seed_of, tu_cases, tu_scan_allowed
from pyoracle import CpuOracle, available

SIZES = (2, 3, 4, 5)


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_scan_tables_match_reference(oracle_libs, depth):
    """generated scan orders == the reference's g_scanOrder (constants.cpp:445-450)"""
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    for typ in range(3):
        for log2 in SIZES:
            if typ and log2 > 3:
                continue
            assert np.array_equal(orc.scan_table(typ, log2), ref.scan_table(typ, log2)), (typ, log2)


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_tu_oracle_matches_reference_random(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    for log2 in SIZES:
        for luma, intra in ((1, 1), (1, 0), (0, 1), (0, 0)):
            for sh in (1, 0):
                c = case_tu(log2, luma, intra, 1 - intra, sh, depth, 160, seed_of("tu-r", depth, log2, luma, intra, sh))
                a, b = run_cpu(c, orc), run_cpu(c, ref)
                for k in c.outs:
                    assert np.array_equal(a[k], b[k]), (c.key(), k)


@pytest.mark.parametrize("depth", [8, 10])
def test_tu_cases_exercise_every_branch(oracle_libs, depth):
    """the committed cases reach numSig 0 / 1 / >= 2, the DC shortcut, and sign
    hiding actually changes coefficients (so the parity tests cover those paths)"""
    orc = CpuOracle("oracle", depth)
    changed = 0
    sigs = []
    for log2 in SIZES:
        on = case_tu(log2, 1, 1, 0, 1, depth, 256, seed_of("tu-br", depth, log2))
        off = case_tu(log2, 1, 1, 0, 0, depth, 256, seed_of("tu-br", depth, log2))
        a, b = run_cpu(on, orc), run_cpu(off, orc)
        changed += int((a["c"] != b["c"]).sum())
        sigs += a["sig"].tolist()
    sigs = np.array(sigs)
    assert changed > 0
    assert (sigs == 0).any() and (sigs == 1).any() and (sigs >= 2).any()


def test_tu_scan_rule():
    assert tu_scan_allowed(2, 1, 1) and tu_scan_allowed(3, 1, 1) and tu_scan_allowed(2, 0, 1)
    assert not tu_scan_allowed(4, 1, 1) and not tu_scan_allowed(3, 0, 1) and not tu_scan_allowed(2, 1, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_tu_gpu_matches_oracle(gpu_prims, oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    cases = tu_cases(depth)
    for log2 in SIZES:
        for luma, intra in ((1, 1), (0, 0)):
            cases.append(case_tu(log2, luma, intra, 0, 1, depth, 4096, seed_of("tu-g", depth, log2, luma, intra)))
    bad = []
    for c in cases:
        got, exp = run_gpu(c, gpu_prims), run_cpu(c, orc)
        for k in c.outs:
            if not np.array_equal(got[k], exp[k]):
                bad.append((c.key(), k, int((got[k] != exp[k]).sum())))
    assert not bad, bad[:6]


@pytest.mark.gpu
def test_tu_without_residual_output(gpu_prims, oracle_libs):
    """resi == NULL: coefficients / recon / numSig unchanged, nothing else written"""
    import torch

    orc = CpuOracle("oracle", 8)
    c = case_tu(4, 1, 0, 0, 1, 8, 512, seed_of("tu-nores"))
    exp = run_cpu(c, orc)
    b = {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) else v)
         for k, v in c.bufs.items()}
    p = c.params
    gpu_prims.tu_pipeline(8, p["log2"], p["luma"], p["intra"], p["islice"], p["sh"], b["f"], b["fs"], b["fo"], b["p"],
                          b["ps"], b["po"], None, 0, None, b["c"], b["co"], b["rc"], b["rcs"], b["rco"], b["sig"],
                          b["qp"], b["scan"])
    torch.cuda.synchronize()
    for k in ("c", "rc", "sig"):
        assert np.array_equal(b[k].cpu().numpy(), exp[k]), k
