"""Reference-generated golden vectors for the caller-level rows f1 (lookahead B estimates) and f4
(deblocking, SAO apply, SAO statistics; 4:2:0 / 4:2:2 / 4:4:4).

The inputs are regenerated bit-identically from seeds (tests/test_lowres_b.make_case,
tests/f4cases); the fixture tests/golden/golden_f1f4.json stores the SHA-256 of every output
buffer produced by the REFERENCE (oracle/_ref, the reference's own estimateCUCost / Deblock / SAO
classes driven by oracle/ref_shim.cpp), written by tests/golden/make_golden_f1f4.py.  The same
output buffers are produced here by any CPU library (`run_cpu`) or by the gfx950 kernels
(`run_gpu`), so the GPU is checked against reference-produced vectors directly.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

import f4cases as F
import pyoracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_f1f4.json")

BCOST_CASES = [(256, 160, 2, 0, 0, True), (480, 272, 1, 4, 2, False)]
F4_CASES = [(200, 136, 6, 1), (128, 64, 5, 2), (96, 48, 4, 3), (256, 128, 6, 2), (192, 128, 6, 3)]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def cases(depth):
    out = [("bcost", depth, c) for c in BCOST_CASES]
    out += [("f4", depth, c) for c in F4_CASES]
    return out


def key(kind, depth, c):
    return f"{kind}:{depth}:" + ",".join(str(int(v)) for v in c)


# ------------------------------------------------------------------ f1 B estimates
def _bcost_inputs(depth, c):
    from test_lowres_b import make_case

    W, H, n, rps, ns, aq = c
    return make_case(W, H, n, depth, 4000 + 10 * depth + W, aq)


def bcost_cpu(kind, depth, c):
    from cases import mvcost_table
    from test_lowres_b import oracle_run

    W, H, n, rps, ns, aq = c
    g, planes, fo, r0o, r1o, iq = _bcost_inputs(depth, c)
    ncu = g["wcu"] * g["hcu"]
    mvs0, mvs1 = np.zeros(2 * n * ncu, np.int16), np.zeros(2 * n * ncu, np.int16)
    mc0, mc1 = np.zeros(n * ncu, np.int32), np.zeros(n * ncu, np.int32)
    lc, rs, ce = oracle_run(po.LowresB(kind, depth), g, planes, fo, r0o, r1o, iq, mvcost_table(depth),
                            np.ones(2 * n, np.uint8), rps, ns, mvs0, mc0, mvs1, mc1)
    return {"lowres_costs": lc, "row_satd": rs, "cost_est": ce, "mvs0": mvs0, "mv_costs0": mc0, "mvs1": mvs1,
            "mv_costs1": mc1}


def bcost_gpu(prims, depth, c):
    import torch

    from cases import mvcost_table
    from test_lowres_b import MVR

    W, H, n, rps, ns, aq = c
    g, planes, fo, r0o, r1o, iq = _bcost_inputs(depth, c)
    ncu, hcu = g["wcu"] * g["hcu"], g["hcu"]
    T = torch.from_numpy(mvcost_table(depth)).cuda()
    pl = torch.from_numpy(planes.view(np.int16) if planes.dtype == np.uint16 else planes).cuda()
    dv = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda()
    m0, m1 = dv(np.zeros(2 * n * ncu, np.int16)), dv(np.zeros(2 * n * ncu, np.int16))
    c0, c1 = dv(np.zeros(n * ncu, np.int32)), dv(np.zeros(n * ncu, np.int32))
    lc = torch.zeros(n * ncu, dtype=torch.int16, device="cuda")
    rs = torch.zeros(n * hcu, dtype=torch.int32, device="cuda")
    ce = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    prims.lowres_bcost(depth, n, g["wcu"], hcu, rps, ns, pl, g["ls"], dv(fo), dv(r0o), dv(r1o),
                       dv(np.ones(2 * n, np.uint8)), dv(iq), T.data_ptr() + 2 * MVR, m0, c0, m1, c1, lc, rs, ce)
    torch.cuda.synchronize()
    h = lambda t: t.cpu().numpy()
    return {"lowres_costs": h(lc).view(np.uint16), "row_satd": h(rs), "cost_est": h(ce), "mvs0": h(m0),
            "mv_costs0": h(c0), "mvs1": h(m1), "mv_costs1": h(c1)}


# ------------------------------------------------------------------ f4 loop filters
def _f4_inputs(depth, c):
    W, H, cl, csp = c
    rng = np.random.default_rng(9000 + 17 * W + H + depth + 101 * csp)
    pl = F.frame_planes(W, H, depth, rng, csp=csp)
    U = F.deblock_units(W, H, cl, depth, rng, "B", 0.1)
    dp = F.deblock_params(rng, "B", 1)
    prm = F.sao_params(W, H, cl, depth, rng)
    fenc = F.frame_planes(W, H, depth, rng, csp=csp)
    return pl, U, dp, prm, fenc


def f4_cpu(kind, depth, c):
    """deblock -> SAO apply on the deblocked picture; SAO statistics of fenc vs the deblocked picture"""
    W, H, cl, csp = c
    L = po.FrameFilters(kind, depth)
    pl, U, dp, prm, fenc = _f4_inputs(depth, c)
    dbk = F.copy_planes(pl)
    L.deblock(W, H, cl, dbk, F.MARGIN, U, dp, csp=csp)
    sao = F.copy_planes(dbk)
    L.sao_apply(W, H, cl, sao, F.MARGIN, prm, 1, 1, csp=csp)
    st, cn = L.sao_stats(W, H, cl, fenc, dbk, F.MARGIN, 0, csp=csp)
    M = F.MARGIN
    out = {f"deblock{p}": dbk[p][M:-M, M:-M] for p in range(3)}
    out.update({f"sao{p}": sao[p][M:-M, M:-M] for p in range(3)})
    out.update(stats=st, count=cn)
    return out


def f4_gpu(prims, depth, c):
    import torch

    from src.x265_amd.native import DeblockFrame, SaoFrame, SaoStatsFrame

    W, H, cl, csp = c
    pl, U, dp, prm, fenc = _f4_inputs(depth, c)
    dev = lambda planes: tuple(torch.from_numpy(p.view(np.int16) if p.dtype == np.uint16 else p).cuda()
                               for p in planes)
    M = F.MARGIN
    org = lambda t: t.data_ptr() + (M * t.shape[1] + M) * t.element_size()
    d = dev(pl)
    du = torch.from_numpy(U.view(np.uint8).reshape(U.shape[0], -1)).cuda()
    fr = DeblockFrame()
    fr.width, fr.height, fr.chroma_format = W, H, csp
    for p in range(3):
        fr.plane[p] = org(d[p])
    fr.stride, fr.cstride = d[0].shape[1], d[1].shape[1]
    fr.units, fr.unit_stride = du.data_ptr(), U.shape[1]
    fr.is_p, fr.beta_offset_div2, fr.tc_offset_div2 = dp.is_p, dp.beta_offset_div2, dp.tc_offset_div2
    fr.cb_qp_offset, fr.cr_qp_offset, fr.tq_bypass_enabled = dp.cb_qp_offset, dp.cr_qp_offset, dp.tq_bypass_enabled
    for lst in range(2):
        for k in range(16):
            fr.ref_poc[lst][k] = dp.ref_poc[lst][k]
    prims.deblock(depth, [fr])
    out_t = dev(tuple(np.zeros_like(p) for p in pl))
    dprm = torch.from_numpy(prm.view(np.uint8)).cuda()
    sf = SaoFrame()
    sf.width, sf.height, sf.ctu_log2, sf.luma_on, sf.chroma_on, sf.chroma_format = W, H, cl, 1, 1, csp
    for p in range(3):
        sf.src[p], sf.dst[p] = org(d[p]), org(out_t[p])
    sf.stride, sf.cstride, sf.params = d[0].shape[1], d[1].shape[1], dprm.data_ptr()
    prims.sao_apply(depth, [sf])
    df = dev(fenc)
    ctu = 1 << cl
    nctu = ((W + ctu - 1) // ctu) * ((H + ctu - 1) // ctu)
    st = torch.full((nctu, 3, 5, 33), -7, dtype=torch.int32, device="cuda")
    cn = torch.full((nctu, 3, 5, 33), -7, dtype=torch.int32, device="cuda")
    tf = SaoStatsFrame()
    tf.width, tf.height, tf.ctu_log2, tf.non_deblocked, tf.chroma_format = W, H, cl, 0, csp
    for p in range(3):
        tf.fenc[p], tf.rec[p] = org(df[p]), org(d[p])
    tf.fenc_stride, tf.fenc_cstride = df[0].shape[1], df[1].shape[1]
    tf.rec_stride, tf.rec_cstride = d[0].shape[1], d[1].shape[1]
    tf.stats, tf.count = st.data_ptr(), cn.data_ptr()
    prims.sao_stats(depth, [tf])
    torch.cuda.synchronize()
    h = lambda t: (t.cpu().numpy().view(np.uint16) if depth > 8 else t.cpu().numpy())
    out = {f"deblock{p}": h(d[p])[M:-M, M:-M] for p in range(3)}
    out.update({f"sao{p}": h(out_t[p])[M:-M, M:-M] for p in range(3)})
    out.update(stats=st.cpu().numpy(), count=cn.cpu().numpy())
    return out


def run_cpu(kind, case):
    k, depth, c = case
    return bcost_cpu(kind, depth, c) if k == "bcost" else f4_cpu(kind, depth, c)


def run_gpu(prims, case):
    k, depth, c = case
    return bcost_gpu(prims, depth, c) if k == "bcost" else f4_gpu(prims, depth, c)


def load():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]
