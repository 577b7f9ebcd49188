"""f1 lookahead B estimates (x265amd_lowres_bcost): CostEstimateGroup::estimateFrameCost for
p0 < b < p1 (estimateCUCost with bBidir, slicetype.cpp:2068-2225).

CPU: the restatement (oracle/x265_oracle.c xo_lowres_bcost) equals the reference's own
estimateCUCost run by oracle/ref_shim.cpp — both lists searched, one list reused from a
previous estimate (bDoSearch false), coop slices and whole frames, AQ on / off.  GPU: the gfx950
kernel equals the restatement on the same estimates, batched.
"""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as po
from cases import Det, _lowres_planes_np, lowres_geometry, mvcost_table, pixel_dtype

MVR = 1 << 14


def make_case(W, H, n, depth, seed, aq=True):
    """n B estimates; estimate e uses frames (3e, 3e+1, 3e+2) = (p0, b, p1) of the synthetic
    sequence (pan + moving object + noise, a noise band so some blocks have no good match)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from src.x265_amd.synth import SyntheticSource

    det = Det(seed)
    g = lowres_geometry(W, H)
    pmax = (1 << depth) - 1
    src = SyntheticSource(W, H, 3 * n, depth, seed=seed % 100000)
    psize = g["ls"] * (g["lines"] + 2 * g["my"])
    planes = []
    for f in range(3 * n):
        y = src.frame(f)[0].astype(np.int64)
        band = slice(H // 3, H // 3 + max(16, H // 10))
        y[band] = det.ints(0, pmax + 1, y[band].size).reshape(y[band].shape)
        planes.append(_lowres_planes_np(y, g, pixel_dtype(depth)))
    planes = np.concatenate(planes)
    org = g["my"] * g["ls"] + g["mx"]
    fo = np.array([4 * (3 * e + 1) * psize + org for e in range(n)], np.int64)
    r0o = np.array([(4 * (3 * e) + k) * psize + org for e in range(n) for k in range(4)], np.int64)
    r1o = np.array([(4 * (3 * e + 2) + k) * psize + org for e in range(n) for k in range(4)], np.int64)
    ncu = g["wcu"] * g["hcu"]
    iq = det.ints(64, 512, n * ncu).astype(np.int32) if aq else None
    return g, planes, fo, r0o, r1o, iq


def oracle_run(lib, g, planes, fo, r0o, r1o, iq, tab, ds, rps, ns, mvs0, mc0, mvs1, mc1):
    n = len(fo)
    ncu, hcu = g["wcu"] * g["hcu"], g["hcu"]
    lc = np.zeros(n * ncu, np.uint16)
    rs = np.zeros(n * hcu, np.int32)
    ce = np.zeros(2 * n, np.int64)
    for e in range(n):
        sl = slice(e * ncu, (e + 1) * ncu)
        lib.bcost(g["wcu"], g["hcu"], rps, ns, planes, g["ls"], fo[e], r0o[4 * e:4 * e + 4], r1o[4 * e:4 * e + 4],
                  None if iq is None else iq[sl], tab.ctypes.data + 2 * MVR, int(ds[2 * e]), int(ds[2 * e + 1]),
                  mvs0[2 * e * ncu:2 * (e + 1) * ncu], mc0[sl], mvs1[2 * e * ncu:2 * (e + 1) * ncu], mc1[sl], lc[sl],
                  rs[e * hcu:(e + 1) * hcu], ce[2 * e:2 * e + 2])
    return lc, rs, ce


def _views(arr, n, per):
    return [arr[i * per:(i + 1) * per] for i in range(n)]


CASES = [(256, 160, 2, 0, 0, True), (480, 272, 1, 4, 2, False), (640, 360, 1, 10, 2, True)]


@pytest.mark.parametrize("depth", [8, 10])
@pytest.mark.parametrize("case", CASES)
def test_bcost_oracle_vs_reference(oracle_libs, depth, case):
    if not po.available("ref", depth):
        pytest.skip("reference library not built (make -C oracle ref)")
    W, H, n, rps, ns, aq = case
    g, planes, fo, r0o, r1o, iq = make_case(W, H, n, depth, 1000 * depth + W, aq)
    tab = mvcost_table(depth)
    ncu = g["wcu"] * g["hcu"]
    O, R = po.LowresB("oracle", depth), po.LowresB("ref", depth)
    st = {}
    for name, lib in (("o", O), ("r", R)):
        mvs0, mvs1 = np.zeros(2 * n * ncu, np.int16), np.zeros(2 * n * ncu, np.int16)
        mc0, mc1 = np.zeros(n * ncu, np.int32), np.zeros(n * ncu, np.int32)
        first = oracle_run(lib, g, planes, fo, r0o, r1o, iq, tab, np.ones(2 * n, np.uint8), rps, ns, mvs0, mc0, mvs1,
                           mc1)
        # a second estimate reusing list 0 (bDoSearch[0] false) with list 1 searched again from scratch
        mvs1b, mc1b = np.zeros_like(mvs1), np.zeros_like(mc1)
        second = oracle_run(lib, g, planes, fo, r0o, r1o, iq, tab, np.tile([0, 1], n).astype(np.uint8), rps, ns,
                            mvs0, mc0, mvs1b, mc1b)
        st[name] = (first, second, mvs0, mc0, mvs1, mc1, mvs1b, mc1b)
    for a, b in zip(st["o"][0] + st["o"][1] + st["o"][2:], st["r"][0] + st["r"][1] + st["r"][2:]):
        np.testing.assert_array_equal(a, b)
    lc = st["r"][0][0]
    assert len(np.unique(lc >> 14)) >= 3        # list 0, list 1 and bidir all win somewhere


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_bcost(gpu_prims, depth):
    import torch

    O = po.LowresB("oracle", depth)
    tab = mvcost_table(depth)
    T = torch.from_numpy(tab).cuda()
    for (W, H, n, rps, ns, aq) in CASES + [(1920, 1080, 3, 10, 6, True)]:
        g, planes, fo, r0o, r1o, iq = make_case(W, H, n, depth, 7 * depth + W, aq)
        ncu, hcu = g["wcu"] * g["hcu"], g["hcu"]
        pl = torch.from_numpy(planes.view(np.int16) if planes.dtype == np.uint16 else planes).cuda()
        dv = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda()
        for ds in (np.ones(2 * n, np.uint8), np.tile([1, 0], n).astype(np.uint8)):
            # stored list-1 results for the reuse pass come from a first full pass on both sides
            mvs0, mvs1 = np.zeros(2 * n * ncu, np.int16), np.zeros(2 * n * ncu, np.int16)
            mc0, mc1 = np.zeros(n * ncu, np.int32), np.zeros(n * ncu, np.int32)
            if not ds[1]:
                oracle_run(O, g, planes, fo, r0o, r1o, iq, tab, np.ones(2 * n, np.uint8), rps, ns, mvs0, mc0, mvs1, mc1)
                mvs0[:], mc0[:] = 0, 0
            d = dict(m0=dv(mvs0), c0=dv(mc0), m1=dv(mvs1), c1=dv(mc1))
            lc = torch.zeros(n * ncu, dtype=torch.int16, device="cuda")
            rs = torch.zeros(n * hcu, dtype=torch.int32, device="cuda")
            ce = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
            gpu_prims.lowres_bcost(depth, n, g["wcu"], hcu, rps, ns, pl, g["ls"], dv(fo), dv(r0o), dv(r1o), dv(ds),
                                   dv(iq), T.data_ptr() + 2 * MVR, d["m0"], d["c0"], d["m1"], d["c1"], lc, rs, ce)
            torch.cuda.synchronize()
            e_lc, e_rs, e_ce = oracle_run(O, g, planes, fo, r0o, r1o, iq, tab, ds, rps, ns, mvs0, mc0, mvs1, mc1)
            np.testing.assert_array_equal(lc.cpu().numpy().view(np.uint16), e_lc)
            np.testing.assert_array_equal(rs.cpu().numpy(), e_rs)
            np.testing.assert_array_equal(ce.cpu().numpy(), e_ce)
            for k, ref in (("m0", mvs0), ("c0", mc0), ("m1", mvs1), ("c1", mc1)):
                np.testing.assert_array_equal(d[k].cpu().numpy(), ref)
