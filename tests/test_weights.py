"""f1 weighted-prediction analysis:
LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495) with weightCostLuma (:338-368) and the
weight_pp primitive (pixel.cpp:463-488).

* (no GPU) the oracle restatement equals the reference's own weightsAnalyse (driven on real
  Lowres objects by oracle/ref_shim.cpp) — decision, weighted planes and cost delta;
* (GPU) x265amd_weights_analyse (device weight_pp and SATD cost passes, the reference's float
  decisions on the host) equals the oracle.
"""
import numpy as np
import pytest

from pyoracle import Weights, available
from weights_cases import KINDS, weights_case

SIZES = [(416, 240), (1920, 1080)]


def _oracle(kind, lib, depth, W, H, seed):
    g, fb, rb, intra, st = weights_case(kind, W, H, depth, seed)
    wb = np.zeros_like(rb)
    out, delta = Weights(lib, depth).analyse(g["width"], g["lines"], g["stride"], g["padded"], g["padoff"], fb, rb,
                                             intra, wb, *st)
    return out, delta, wb


@pytest.mark.skipif(not available("ref"), reason="reference library not built")
@pytest.mark.parametrize("depth", [8, 10])
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("size", SIZES)
def test_weights_oracle_matches_reference(oracle_libs, depth, kind, size):
    a = _oracle(kind, "oracle", depth, *size, seed=depth)
    b = _oracle(kind, "ref", depth, *size, seed=depth)
    assert a[0][0] == b[0][0], (a[0], b[0])
    if a[0][0]:
        assert a[1] == b[1]
        np.testing.assert_array_equal(a[2], b[2])
    if kind == "fade":
        assert a[0][0] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
@pytest.mark.parametrize("kind", KINDS)
def test_weights_gpu_matches_oracle(gpu_prims, oracle_libs, depth, kind):
    import torch

    W, H = 1920, 1080
    g, fb, rb, intra, st = weights_case(kind, W, H, depth, seed=depth)
    out, delta, wb = _oracle(kind, "oracle", depth, W, H, seed=depth)
    t = lambda a: torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a).cuda()
    dfb, drb, dint = t(fb), t(rb), t(intra)
    dwb = torch.zeros_like(drb)
    res = gpu_prims.weights_analyse(depth, g["width"], g["lines"], g["stride"], g["padded"], g["padoff"], dfb, drb,
                                    dint, dwb, *st)
    assert res["weighted"] == out[0]
    if out[0]:
        assert (res["scale"], res["denom"], res["offset"]) == tuple(out[1:4])
        assert res["cost_delta"] == delta
        got = dwb.cpu().numpy()
        np.testing.assert_array_equal(got.view(np.uint16) if depth > 8 else got, wb)
