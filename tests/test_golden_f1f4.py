"""Reference-generated golden vectors for f1 B estimates and the f4 loop filters (VERDICT r1
weak item 1: the GPU must see reference-produced vectors for these rows, not only the oracle).

* (no GPU) the fixture covers every case, and the oracle restatement reproduces every hash;
* (GPU) the gfx950 kernels reproduce every hash of tests/golden/golden_f1f4.json.
"""
import pytest

import golden_f1f4 as G


def _cases():
    return G.cases(8) + G.cases(10)


def test_fixture_covers_cases():
    assert sorted(G.load()) == sorted(G.key(*c) for c in _cases())


@pytest.mark.parametrize("case", _cases(), ids=lambda c: G.key(*c))
def test_oracle_reproduces_reference_hashes(oracle_libs, case):
    want = G.load()[G.key(*case)]
    got = {k: G.sha(v) for k, v in G.run_cpu("oracle", case).items()}
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("case", _cases(), ids=lambda c: G.key(*c))
def test_gpu_reproduces_reference_hashes(gpu_prims, case):
    want = G.load()[G.key(*case)]
    got = {k: G.sha(v) for k, v in G.run_gpu(gpu_prims, case).items()}
    bad = [k for k in want if got.get(k) != want[k]]
    assert not bad, bad
