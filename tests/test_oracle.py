"""CPU-side parity of the oracle restatement (no GPU).

* every case of cases.all_cases() — all primitive families x every block
  shape of the reference table x the TestBench input classes — reproduces the
  golden hashes generated from the reference x265 1.9 C primitives
  (tests/golden/make_golden.py);
* when the reference library oracle/_ref is present, larger random batches
  are cross-checked against it directly.
"""
import json
import os

import numpy as np
import pytest

from cases import all_cases, case_interp, case_pixelcmp, case_transform, run_cpu, seed_of, LUMA_PU, SATD, SA8D, \
    HVPP, DCT, IDCT, TU_SQ
from pyoracle import CpuOracle, available

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_golden(depth):
    with open(os.path.join(GOLDEN, f"golden_d{depth}.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("depth", [8, 10])
def test_golden_covers_all_cases(depth):
    g = load_golden(depth)
    keys = [(e["family"], json.dumps(e["params"], sort_keys=True)) for e in g["cases"]]
    mine = [(c.family, json.dumps(c.params, sort_keys=True)) for c in all_cases(depth)]
    assert keys == mine


@pytest.mark.parametrize("depth", [8, 10])
def test_oracle_matches_golden(oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    g = load_golden(depth)
    bad = []
    for c, e in zip(all_cases(depth), g["cases"]):
        outs = run_cpu(c, orc)
        if c.output_hashes(outs) != e["sha256"]:
            bad.append(c.key())
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
@pytest.mark.parametrize("depth", [8, 10])
def test_oracle_matches_reference_random(oracle_libs, depth):
    orc, ref = CpuOracle("oracle", depth), CpuOracle("ref", depth)
    cases = []
    for (w, h) in LUMA_PU:
        cases.append(case_pixelcmp(SATD, w, h, depth, 64, seed_of("r", depth, w, h)))
        cases.append(case_interp(HVPP, 8, w, h, depth, 32, seed_of("rhv", depth, w, h)))
    for n in (8, 16, 32, 64):
        cases.append(case_pixelcmp(SA8D, n, n, depth, 64, seed_of("rs", depth, n)))
    for n in TU_SQ:
        cases.append(case_transform(DCT, n, depth, 64, seed_of("rd", depth, n)))
        cases.append(case_transform(IDCT, n, depth, 64, seed_of("ri", depth, n)))
    for c in cases:
        a, b = run_cpu(c, orc), run_cpu(c, ref)
        for k in c.outs:
            assert np.array_equal(a[k], b[k]), c.key()
