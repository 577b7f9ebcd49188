"""Caller-level rates for bench.py on the bench's own
resolution and synthetic source: how fast the GPU runs, per frame, the lookahead's lowres
pipeline (plane init, intra estimate, one P estimate; B estimates separately), the main encoder's 2Nx2N motion search
(HEX, subme 2, merange 57: --preset medium; every PU of 8x8 .. 64x64 against one reference) and
the fused residual-coding chain for a frame's worth of TUs.  Informational: the census replay
stays the headline workload.  Product path only (no oracle)."""
from __future__ import annotations

import os

import numpy as np
import torch

from .synth import SyntheticSource

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _time(fn, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def caller_rates(prims, width: int, height: int, depth: int = 8, dev: str = "cuda") -> dict:
    if depth != 8:
        return {}
    out = {}
    syn = SyntheticSource(width, height, 9, depth)
    frames = [syn.frame(i) for i in range(9)]
    # ---- f1: lowres planes + intra estimate for 8 frames, P estimates of frames 1..8 against their predecessor
    mx, my = 96, 80
    w2, l2 = width // 2, height // 2
    ls = w2 + 2 * mx
    ls += (32 - ls % 32) % 32
    wcu, hcu = (w2 + 7) // 8, (l2 + 7) // 8
    lw, ll = wcu * 8, hcu * 8
    ss = 2 * lw + 32
    srows = 2 * ll + 4
    nf = 9
    src = np.zeros((nf, srows, ss), np.uint8)
    for i, f in enumerate(frames):
        y = np.pad(f[0], ((0, srows - height), (0, ss - width)), mode="edge")
        src[i] = y
    S = _t(src.reshape(-1), dev)
    so = _t(np.arange(nf, dtype=np.int64) * srows * ss, dev)
    psize = ls * (ll + 2 * my)
    org = my * ls + mx
    PL = torch.empty(4 * nf * psize, dtype=torch.uint8, device=dev)
    po = _t(np.arange(4 * nf, dtype=np.int64) * psize + org, dev)
    ncu = wcu * hcu
    IC = torch.empty(nf * ncu, dtype=torch.int32, device=dev)
    IM = torch.empty(nf * ncu, dtype=torch.uint8, device=dev)
    LC = torch.empty(nf * ncu, dtype=torch.int16, device=dev)
    RS = torch.empty(nf * hcu, dtype=torch.int32, device=dev)
    CE = torch.empty(2 * nf, dtype=torch.int64, device=dev)
    tab = np.load(os.path.join(ROOT, "tests", "golden", "mvcost_lookahead_d8.npy"))
    TAB = _t(tab, dev)
    ne = nf - 1
    rps = max(hcu // 8, 10)
    ns = max(1, hcu // rps)
    MV = torch.empty(2 * ne * ncu, dtype=torch.int16, device=dev)
    MC = torch.empty(ne * ncu, dtype=torch.int32, device=dev)
    PLC = torch.empty(ne * ncu, dtype=torch.int16, device=dev)
    PRS = torch.empty(ne * hcu, dtype=torch.int32, device=dev)
    PCE = torch.empty(2 * ne, dtype=torch.int64, device=dev)
    MB = torch.empty(ne, dtype=torch.int32, device=dev)
    p0 = po[0::4].contiguous()
    fo = po[4::4].contiguous()
    ro = po[:4 * ne].contiguous()

    def lookahead():
        prims.lowres_init(8, nf, lw, ll, mx, my, S, ss, so, PL, ls, po)
        prims.lowres_intra(8, nf, wcu, hcu, PL, ls, p0, None, IC, IM, LC, RS, CE)
        prims.lowres_pcost(8, ne, wcu, hcu, rps, ns, PL, ls, fo, ro, IC[ncu:], None, TAB.data_ptr() + 2 * (1 << 14),
                           MV, MC, PLC, PRS, PCE, MB)
    ms = _time(lookahead)
    out["lookahead_lowres_frames_per_s"] = round(ne / (ms * 1e-3), 1)
    out["lookahead_note"] = (f"{nf} frames: lowres planes + intra estimate, {ne} P estimates "
                             f"({ns} coop slices of {rps} rows)")
    # B estimates (p0, b, p1) = (f, f+1, f+2) on the same planes, both lists searched
    nb = nf - 2
    fob = po[4:4 * (nb + 1):4].contiguous()
    r0b = po[:4 * nb].contiguous()
    r1b = po[8:8 + 4 * nb].contiguous()
    DS = torch.ones(2 * nb, dtype=torch.uint8, device=dev)
    BM = [torch.empty(2 * nb * ncu, dtype=torch.int16, device=dev) for _ in range(2)]
    BC = [torch.empty(nb * ncu, dtype=torch.int32, device=dev) for _ in range(2)]
    BLC = torch.empty(nb * ncu, dtype=torch.int16, device=dev)
    BRS = torch.empty(nb * hcu, dtype=torch.int32, device=dev)
    BCE = torch.empty(2 * nb, dtype=torch.int64, device=dev)
    ms = _time(lambda: prims.lowres_bcost(8, nb, wcu, hcu, rps, ns, PL, ls, fob, r0b, r1b, DS, None,
                                          TAB.data_ptr() + 2 * (1 << 14), BM[0], BC[0], BM[1], BC[1], BLC, BRS, BCE))
    out["lookahead_b_estimates_per_s"] = round(nb / (ms * 1e-3), 1)
    # ---- f2: every 2Nx2N PU of one frame (8 .. 64) against the previous frame, HEX / subme 2 / merange 57
    M = 96
    st = width + 2 * M
    f1 = np.pad(frames[1][0], M, mode="edge").reshape(-1)
    f0 = np.pad(frames[0][0], M, mode="edge").reshape(-1)
    F1, F0 = _t(f1, dev), _t(f0, dev)
    tq = np.load(os.path.join(ROOT, "tests", "golden", "mvcost_qp_d8.npy"))
    TQ = _t(tq.reshape(-1), dev)
    R = (tq.shape[1] - 1) // 2
    jobs = []
    rng = np.random.default_rng(5)
    for s_ in (8, 16, 32, 64):
        xs, ys = np.meshgrid(np.arange(0, width - s_ + 1, s_), np.arange(0, height - s_ + 1, s_))
        xs, ys = xs.reshape(-1), ys.reshape(-1)
        n = xs.size
        mvp = np.stack([-8 + rng.integers(-4, 5, n), -4 + rng.integers(-4, 5, n)], 1)
        rg = np.stack([np.maximum(-xs - 40, (mvp[:, 0] >> 2) - 57), np.maximum(-ys - 40, (mvp[:, 1] >> 2) - 57),
                       np.minimum(width - xs - s_ + 40, (mvp[:, 0] >> 2) + 57),
                       np.minimum(height - ys - s_ + 40, (mvp[:, 1] >> 2) + 57)], 1)
        jobs.append(dict(s=s_, n=n, fo=_t(((ys + M) * st + xs + M).astype(np.int64), dev),
                         rg=_t(rg.astype(np.int16).reshape(-1), dev), mvp=_t(mvp.astype(np.int16).reshape(-1), dev),
                         mvc=_t(rng.integers(-16, 17, 4 * n).astype(np.int16), dev),
                         nc=_t(np.full(n, 2, np.uint8), dev),
                         to=_t(np.full(n, 2 * (2 * R + 1) + R, np.int64), dev),
                         om=torch.empty(2 * n, dtype=torch.int16, device=dev),
                         oc=torch.empty(n, dtype=torch.int32, device=dev)))

    multi = [dict(w=j["s"], h=j["s"], method=1, subme=2, merange=57, max_cand=2, f=F1, fs=st, fo=j["fo"], r=F0, rs=st,
                  ro=j["fo"], rng=j["rg"], mvp=j["mvp"], mvc=j["mvc"], numc=j["nc"], tab=TQ, tab_off=j["to"],
                  out_mv=j["om"], out_cost=j["oc"]) for j in jobs]
    ms = _time(lambda: prims.motion_search_multi(8, multi))     # the four PU sizes in one call
    out["me_2Nx2N_frames_per_s"] = round(1.0 / (ms * 1e-3), 1)
    out["me_pus_per_frame"] = int(sum(j["n"] for j in jobs))
    # ---- f3: a frame's worth of 8x8 luma TUs through the fused residual-coding chain
    xs, ys = np.meshgrid(np.arange(0, width - 7, 8), np.arange(0, height - 7, 8))
    n = xs.size
    off = _t(((ys.reshape(-1) + M) * st + xs.reshape(-1) + M).astype(np.int64), dev)
    RES = torch.empty(f1.size, dtype=torch.int16, device=dev)
    REC = torch.empty(f1.size, dtype=torch.uint8, device=dev)
    CO = torch.empty(64 * n, dtype=torch.int16, device=dev)
    coff = torch.arange(n, dtype=torch.int64, device=dev) * 64
    SIG = torch.empty(n, dtype=torch.int32, device=dev)
    QP = torch.full((n,), 32, dtype=torch.uint8, device=dev)
    ms = _time(lambda: prims.tu_pipeline(8, 3, 1, 0, 0, 1, F1, st, off, F0, st, off, RES, st, off, CO, coff, REC, st,
                                         off, SIG, QP, None))
    out["tu_pipeline_8x8_tus_per_s"] = round(n / (ms * 1e-3), 1)
    out.update(_loop_filter_rate(prims, frames[1:], width, height, dev))
    return out


# x265amd_deblock_unit / x265amd_sao_param (include/x265_amd.h)
_UNIT = np.dtype([("cu_log2", np.uint8), ("tu_log2", np.uint8), ("part", np.uint8), ("flags", np.uint8),
                  ("qp", np.int8), ("ref_idx", np.int8, 2), ("pad", np.uint8), ("mv", np.int16, (2, 2))])
_SAO = np.dtype([("type", np.int8), ("band", np.uint8), ("offset", np.int8, 4)])


def _loop_filter_rate(prims, frames, width, height, dev):
    """f4: deblock -> SAO statistics -> SAO apply -> border extension of 8 recon frames per call
    (a synthetic CU layout: 16x16 CUs of 8x8 TUs, a quarter intra, P-slice MVs)."""
    from .native import BorderPlane, DeblockFrame, SaoFrame, SaoStatsFrame

    rng = np.random.default_rng(9)
    hu, wu = height // 4, width // 4
    U = np.zeros((hu, wu), _UNIT)
    cu = rng.random((hu // 4 + 1, wu // 4 + 1)) < 0.25
    U["cu_log2"], U["tu_log2"], U["qp"] = 4, 3, 32
    U["flags"] = np.repeat(np.repeat(cu, 4, 0), 4, 1)[:hu, :wu].astype(np.uint8) | (rng.random((hu, wu)) < 0.5) * 2
    U["ref_idx"][..., 0], U["ref_idx"][..., 1] = 0, -1
    mv = np.repeat(np.repeat(rng.integers(-6, 7, (hu // 4 + 1, wu // 4 + 1, 2)), 4, 0), 4, 1)[:hu, :wu]
    U["mv"][..., 0, :] = mv
    ctu = 64
    nctu = ((width + ctu - 1) // ctu) * ((height + ctu - 1) // ctu)
    prm = np.zeros(3 * nctu, _SAO)
    prm["type"] = rng.integers(-1, 5, 3 * nctu)
    prm["type"][2 * nctu:] = prm["type"][nctu:2 * nctu]
    prm["band"] = rng.integers(0, 32, 3 * nctu)
    prm["offset"] = rng.integers(-3, 4, (3 * nctu, 4))
    M = 16
    planes, recs = [], []
    for f in frames:
        planes.append([_t(np.pad(p, M, mode="edge"), dev) for p in f[:3]])
        recs.append([p.clone() for p in planes[-1]])
    outs = [[torch.empty_like(p) for p in pl] for pl in planes]
    du = _t(U.view(np.uint8).reshape(hu, -1), dev)
    dprm = _t(prm.view(np.uint8), dev)
    stats = torch.empty(len(frames) * nctu * 3 * 5 * 33, dtype=torch.int32, device=dev)
    count = torch.empty_like(stats)

    def org(t):
        return t.data_ptr() + (M * t.shape[1] + M) * t.element_size()

    dbk, sst, sao, bor = [], [], [], []
    for i, (src, rec, dst) in enumerate(zip(planes, recs, outs)):
        d = DeblockFrame()
        d.width, d.height, d.is_p = width, height, 1
        for p in range(3):
            d.plane[p] = org(rec[p])
        d.stride, d.cstride, d.units, d.unit_stride = rec[0].shape[1], rec[1].shape[1], du.data_ptr(), wu
        d.ref_poc[0][0] = 0
        dbk.append(d)
        s = SaoStatsFrame()
        s.width, s.height, s.ctu_log2 = width, height, 6
        for p in range(3):
            s.fenc[p], s.rec[p] = org(src[p]), org(rec[p])
        s.fenc_stride, s.fenc_cstride, s.rec_stride, s.rec_cstride = (src[0].shape[1], src[1].shape[1],
                                                                      rec[0].shape[1], rec[1].shape[1])
        s.stats = stats.data_ptr() + i * nctu * 3 * 5 * 33 * 4
        s.count = count.data_ptr() + i * nctu * 3 * 5 * 33 * 4
        sst.append(s)
        a = SaoFrame()
        a.width, a.height, a.ctu_log2, a.luma_on, a.chroma_on = width, height, 6, 1, 1
        for p in range(3):
            a.src[p], a.dst[p] = org(rec[p]), org(dst[p])
        a.stride, a.cstride, a.params = rec[0].shape[1], rec[1].shape[1], dprm.data_ptr()
        sao.append(a)
        for p in range(3):
            b = BorderPlane()
            b.plane, b.stride = org(dst[p]), dst[p].shape[1]
            b.width, b.height = (width, height) if p == 0 else (width // 2, height // 2)
            b.margin_x = b.margin_y = M
            bor.append(b)

    def chain():
        prims.deblock(8, dbk)
        prims.sao_stats(8, sst)
        prims.sao_apply(8, sao)
        prims.extend_border(8, bor)
    ms = _time(chain)
    return {"loop_filter_frames_per_s": round(len(frames) / (ms * 1e-3), 1),
            "loop_filter_note": f"{len(frames)} frames per call: deblock, SAO statistics, SAO apply, border extension"}
