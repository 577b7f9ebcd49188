"""f1 cuTree propagation: Lookahead::estimateCUPropagate
(slicetype.cpp:1738-1836) with the propagateCost primitive (pixel.cpp:846-872).

* (no GPU) the oracle restatement equals the reference's own estimateCUPropagate (driven on
  real Lowres objects by oracle/ref_shim.cpp, the reference compiled here) bit for bit;
* (GPU) x265amd_cutree_propagate equals the oracle.
"""
import numpy as np
import pytest

from cutree_cases import CASES, cutree_case
from pyoracle import CuTree, available


def _run(lib, wcu, hcu, bp0, p1b, ref, wb, fn, fd, avg, c):
    out = {k: c[k].copy() for k in ("prop", "ref0", "ref1")}
    lib.propagate(wcu, hcu, bp0, p1b, ref, wb, fn, fd, avg, out["prop"], c["intra"], c["lowres"], c["invq"],
                  c["mvs0"], c["mvs1"], out["ref0"], out["ref1"])
    return out


@pytest.mark.skipif(not available("ref"), reason="reference library not built")
@pytest.mark.parametrize("case", range(len(CASES)))
def test_cutree_oracle_matches_reference(oracle_libs, case):
    wcu, hcu, bp0, p1b, ref, wb, fn, fd, avg = CASES[case]
    c = cutree_case(wcu, hcu, bp0, p1b, ref, 100 + case)
    a = _run(CuTree("oracle"), *CASES[case], c)
    b = _run(CuTree("ref"), *CASES[case], c)
    for k in ("ref0", "ref1", "prop"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert (a["ref0"] != c["ref0"]).any()


def gpu_fps_factor(fn, fd, avg):
    clip = lambda f: min(max(f, 0.01), 1.0)              # ratecontrol.h:45-47 CLIP_DURATION
    return clip(fd / fn) / clip(avg)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)))
def test_cutree_gpu_matches_oracle(gpu_prims, oracle_libs, case):
    import torch

    wcu, hcu, bp0, p1b, ref, wb, fn, fd, avg = CASES[case]
    c = cutree_case(wcu, hcu, bp0, p1b, ref, 100 + case)
    want = _run(CuTree("oracle"), *CASES[case], c)
    p0, b, p1 = 0, bp0, bp0 + p1b
    ds = (((b - p0) << 8) + ((p1 - p0) >> 1)) // (p1 - p0)
    w0 = 64 - (ds >> 2) if wb else 32
    t = lambda a: torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a).cuda()
    d = {k: t(c[k].copy()) for k in ("intra", "lowres", "invq", "mvs0", "mvs1", "prop", "ref0", "ref1")}
    if not ref:
        d["prop"][:wcu] = 0
    scratch = torch.empty(2 * wcu * hcu, dtype=torch.int64, device="cuda")
    gpu_prims.cutree_propagate([dict(wcu=wcu, hcu=hcu, prop=d["prop"] if ref else None, intra=d["intra"],
                                     lowres=d["lowres"], invq=d["invq"], mvs=(d["mvs0"], d["mvs1"] if p1b else None),
                                     fps_factor=gpu_fps_factor(fn, fd, avg), weights=(w0, 64 - w0),
                                     refs=(d["ref0"], d["ref1"] if p1b else None), scratch=scratch)])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d["ref0"].cpu().numpy().view(np.uint16), want["ref0"])
    if p1b:
        np.testing.assert_array_equal(d["ref1"].cpu().numpy().view(np.uint16), want["ref1"])
