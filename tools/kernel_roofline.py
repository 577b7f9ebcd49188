#!/usr/bin/env python3
"""Kernel-level roofline of the gfx950 primitive kernels.

Each kernel runs on a batch of independent calls with DISJOINT operand
blocks tiled in raster order through buffers of >= --gb GB (default 1.5 GB,
about 4x the 32 MiB of L2 plus the 256 MiB Infinity Cache), so caches cannot
inflate bandwidth.  achieved = algorithmic bytes per launch (§8(d) formulas)
/ mean launch time (HIP events on the launch stream), against the 8 TB/s HBM
peak of MI355X_MICROARCH.md.  Writes one JSON object per kernel to stdout and
the table to --out.

    python tools/kernel_roofline.py --out profiles/kernel_roofline_r01.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM = 8000.0
SAD, SATD, SA8D, SSE_PP = 0, 1, 2, 3
HPP, HPS, VPP, VPS, VSP, VSS, HVPP = range(7)
DCT, IDCT = 0, 1


def tiled_offsets(n, bw, bh, pitch_w, pitch_h, width_px, margin=0):
    """raster tiling of n blocks with pitch (pitch_w x pitch_h) in a plane of width_px"""
    per_row = max(1, (width_px - 2 * margin) // pitch_w)
    j = np.arange(n, dtype=np.int64)
    x = margin + (j % per_row) * pitch_w
    y = margin + (j // per_row) * pitch_h
    rows = int(y.max()) + pitch_h + margin
    return x, y, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="")
    a = ap.parse_args()

    import torch

    from src.x265_amd import Primitives, capture_graph

    prims = Primitives(device=0)
    dev = "cuda"
    W = 8192  # plane width in pixels
    results = []

    def timeit(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        evs = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        return sum(x.elapsed_time(y) for x, y in evs) / len(evs)

    def record(name, nbytes, ms, n, desc=0):
        gbs = nbytes / (ms * 1e-3) / 1e9
        r = {"kernel": name, "jobs": n, "bytes_per_launch": int(nbytes), "ms": round(ms, 4),
             "achieved_GBps": round(gbs, 1), "frac_of_8TBps": round(gbs / HBM, 3)}
        if desc:
            # the C ABI's per-job descriptors (int64 offsets, per-job scalars) the kernel must also read
            r["descriptor_bytes_per_job"] = desc
            r["frac_incl_descriptors"] = round((nbytes + desc * n) / (ms * 1e-3) / 1e9 / HBM, 3)
        results.append(r)
        print(json.dumps(r), flush=True)

    def want(name):
        return not a.only or any(s in name for s in a.only.split(","))

    def rand_u8(numel):
        return torch.randint(0, 256, (numel,), dtype=torch.uint8, device=dev)

    # ---------------------------------------------------------------- pixel compare
    for op, opname, sizes in ((SAD, "sad", [8, 16, 32, 64]), (SATD, "satd", [8, 16, 64]),
                              (SA8D, "sa8d", [8, 16, 32]), (SSE_PP, "sse_pp", [8, 32])):
        for s in sizes:
            name = f"{opname}_{s}x{s}"
            if not want(name):
                continue
            n = int(a.gb * 1e9 / 2 / (s * s))
            x, y, rows = tiled_offsets(n, s, s, s, s, W)
            A, B = rand_u8(rows * W), rand_u8(rows * W)
            off = torch.from_numpy(y * W + x).to(dev)
            wide = op == SSE_PP
            out = torch.empty(n, dtype=torch.int64 if wide else torch.int32, device=dev)
            ms = timeit(lambda: prims.pixelcmp(op, 8, s, s, A, W, off, B, W, off, out))
            record(name, n * (2 * s * s + (8 if wide else 4)), ms, n, desc=16)
            del A, B, off, out
    # ---------------------------------------------------------------- sad_x4
    for s in (8, 16, 64):
        name = f"sad_x4_{s}x{s}"
        if not want(name):
            continue
        n = int(a.gb * 1e9 / 5 / (s * s))
        x, y, rows = tiled_offsets(n, s, s, s, s, W)
        F = rand_u8(rows * W)
        x4, y4, rows4 = tiled_offsets(4 * n, s, s, s, s, W)
        R = rand_u8(rows4 * W)
        foff = torch.from_numpy(y * W + x).to(dev)
        roff = torch.from_numpy(y4 * W + x4).to(dev)
        out = torch.empty(4 * n, dtype=torch.int32, device=dev)
        ms = timeit(lambda: prims.sad_multi(4, 8, s, s, F, W, foff, R, W, roff, out))
        record(name, n * (5 * s * s + 16), ms, n, desc=40)
        del F, R, foff, roff, out
    # ---------------------------------------------------------------- luma interp
    for op, opname in ((HPP, "luma_hpp"), (VPP, "luma_vpp"), (HVPP, "luma_hvpp")):
        for s in (8, 16, 64):
            name = f"{opname}_{s}x{s}"
            if not want(name):
                continue
            ext_w = 7 if op in (HPP, HVPP) else 0
            ext_h = 7 if op in (VPP, HVPP) else 0
            n = int(a.gb * 1e9 / ((s + ext_w) * (s + ext_h) + s * s))
            # windows tiled densely and disjointly: (s + 7) x s for hpp, s x (s + 7) for vpp, (s + 7)^2 for hvpp
            # (a pitch of s + 8 in a direction with no filter extension would leave unread gaps in every line)
            x, y, rows = tiled_offsets(n, s, s, s + (8 if ext_w else 0), s + (8 if ext_h else 0), W, margin=8)
            S = rand_u8(rows * W)
            soff = torch.from_numpy(y * W + x).to(dev)
            D = torch.empty(n * s * s, dtype=torch.uint8, device=dev)
            doff = torch.arange(n, dtype=torch.int64, device=dev) * (s * s)
            coeff = torch.randint(1, 4, (n,), dtype=torch.uint8, device=dev)
            if op == HVPP:
                coeff = coeff | (torch.randint(1, 4, (n,), dtype=torch.uint8, device=dev) << 4)
            ms = timeit(lambda: prims.interp(op, 8, 8, s, s, S, W, soff, D, s, doff, coeff))
            record(name, n * ((s + ext_w) * (s + ext_h) + s * s), ms, n, desc=17)
            del S, soff, D, doff, coeff
    # ---------------------------------------------------------------- block ops
    # sources tiled in planes (as frame blocks), destinations in compact slots
    # (as the bench's per-job output slots); (name, op, a int16?, b operand: None / "p" / "s", dst int16?)
    for bname, op, a16, bkind, d16 in (("copy_pp", 4, False, None, False), ("pixelavg", 3, False, "p", False),
                                       ("sub_ps", 0, False, "p", True), ("add_ps", 1, False, "s", False),
                                       ("addavg", 2, True, "s", False)):
        for s in (8, 16, 64):
            name = f"{bname}_{s}x{s}"
            if not want(name):
                continue
            esz_a, esz_d = (2 if a16 else 1), (2 if d16 else 1)
            esz_b = 0 if bkind is None else (2 if bkind == "s" else 1)
            n = int(a.gb * 1e9 / ((esz_a + esz_b + esz_d) * s * s))
            x, y, rows = tiled_offsets(n, s, s, s, s, W)
            mk = (lambda k: torch.randint(-2000, 2000, (k,), dtype=torch.int16, device=dev)) if a16 else rand_u8
            A = mk(rows * W)
            off = torch.from_numpy(y * W + x).to(dev)
            B = None
            if bkind == "p":
                B = rand_u8(rows * W)
            elif bkind == "s":
                B = torch.randint(-2000, 2000, (rows * W,), dtype=torch.int16, device=dev)
            D = torch.empty(n * s * s, dtype=torch.int16 if d16 else torch.uint8, device=dev)
            doff = torch.arange(n, dtype=torch.int64, device=dev) * (s * s)
            ms = timeit(lambda: prims.blockop(op, 8, s, s, D, s, doff, A, W, off, B, W, off if B is not None else None))
            record(name, n * (esz_a + esz_b + esz_d) * s * s, ms, n, desc=16 if B is None else 24)
            del A, B, D, off, doff
    # ---------------------------------------------------------------- transforms
    for kind, kname in ((DCT, "dct"), (IDCT, "idct")):
        for s in (4, 8, 16, 32):
            name = f"{kname}_{s}x{s}"
            if not want(name):
                continue
            n = int(a.gb * 1e9 / (4 * s * s))
            Sr = torch.randint(-255, 256, (n * s * s,), dtype=torch.int16, device=dev)
            Dr = torch.empty(n * s * s, dtype=torch.int16, device=dev)
            offs = torch.arange(n, dtype=torch.int64, device=dev) * (s * s)
            ms = timeit(lambda: prims.transform(kind, 8, s, Sr, s, offs, Dr, s, offs))
            record(name, n * 4 * s * s, ms, n, desc=16)
            if s >= 16:
                # matrix-core path (csrc/transform.hip k_tr16/32_mfma): two stages, each an
                # N x N x N product issued twice (hi / lo f16 halves of every int16 operand)
                flops = n * 2 * 2 * 2 * s ** 3
                results[-1]["mfma_TFLOPs"] = round(flops / (ms * 1e-3) / 1e12, 2)
                results[-1]["mfma_frac_of_2500TF_f16_dense"] = round(flops / (ms * 1e-3) / 2.5e15, 4)
                print(json.dumps({"kernel": name, "mfma_TFLOPs": results[-1]["mfma_TFLOPs"]}), flush=True)
            del Sr, Dr, offs
    # ---------------------------------------------------------------- quant
    for s in (4, 8, 16, 32):
        name = f"quant_{s}x{s}"
        if not want(name):
            continue
        num = s * s
        n = int(a.gb * 1e9 / (8 * num))
        C = torch.randint(-255, 256, (n * num,), dtype=torch.int16, device=dev)
        Q = torch.full((num,), 16384 * 16, dtype=torch.int32, device=dev)
        offs = torch.arange(n, dtype=torch.int64, device=dev) * num
        qo = torch.zeros(n, dtype=torch.int64, device=dev)
        DL = torch.empty(n * num, dtype=torch.int32, device=dev)
        O = torch.empty(n * num, dtype=torch.int16, device=dev)
        qb = torch.full((n,), 20, dtype=torch.int32, device=dev)
        ad = torch.full((n,), 85 << 11, dtype=torch.int32, device=dev)
        sig = torch.empty(n, dtype=torch.int32, device=dev)
        ms = timeit(lambda: prims.quant(num, C, offs, Q, qo, DL, offs, O, offs, qb, ad, sig))
        record(name, n * (8 * num + 4), ms, n, desc=40)
        if want(f"copy_cnt_{s}x{s}"):
            # copy_cnt: the residual block (in a plane) -> compact coefficients + count
            x, y, rows = tiled_offsets(n, s, s, s, s, W)
            R = torch.randint(-3, 4, (rows * W,), dtype=torch.int16, device=dev)
            roff = torch.from_numpy(y * W + x).to(dev)
            ms = timeit(lambda: prims.count_nonzero(s, O, offs, R, W, roff, sig))
            record(f"copy_cnt_{s}x{s}", n * (4 * num + 4), ms, n, desc=16)
            del R, roff
        if want(f"dequant_{s}x{s}"):
            dsc = torch.full((n,), 40 * 4, dtype=torch.int32, device=dev)
            dsh = torch.full((n,), 3, dtype=torch.int32, device=dev)
            ms = timeit(lambda: prims.dequant_normal(num, C, offs, O, offs, dsc, dsh))
            record(f"dequant_{s}x{s}", n * 4 * num, ms, n, desc=24)
            del dsc, dsh
        del C, offs, qo, DL, O, qb, ad, sig
    # ---------------------------------------------------------------- intra
    for s in (4, 8, 16, 32):
        name = f"intra_ang_{s}x{s}"
        if not want(name):
            continue
        m = 4 * s + 1
        n = int(a.gb * 1e9 / (m + s * s))
        NB = rand_u8(n * m)
        nbo = torch.arange(n, dtype=torch.int64, device=dev) * m
        D = torch.empty(n * s * s, dtype=torch.uint8, device=dev)
        doff = torch.arange(n, dtype=torch.int64, device=dev) * (s * s)
        mode = torch.from_numpy(np.sort(np.random.default_rng(1).integers(2, 35, n)).astype(np.uint8)).to(dev)
        bf = torch.ones(n, dtype=torch.uint8, device=dev)
        ms = timeit(lambda: prims.intra_pred(8, s, D, s, doff, NB, nbo, mode, bf))
        record(name, n * (m + s * s), ms, n, desc=18)
        del NB, nbo, D, doff, mode, bf
    # ---------------------------------------------------------------- f3 fused TU pipeline
    # TUs tiled through disjoint fenc / pred / recon / residual planes; pred = fenc + noise in
    # [-12, 12] and qp uniform in [22, 37] per TU: a mix of uncoded TUs, DC-only TUs and TUs
    # through the full inverse path, with sign hiding live.  Compared with the same TUs through
    # the 6 unfused table calls the reference makes (calcresidual, dct/dst, quant,
    # dequant_normal, idct/idst, add_ps; sign hiding has no table entry, so the unfused chain
    # does strictly less work).
    for log2 in (2, 3, 4, 5):
        s_ = 1 << log2
        name = f"tu_pipeline_{s_}x{s_}"
        if not want(name):
            continue
        num = s_ * s_
        per_tu = 3 * num + 2 * num + 2 * num + 4 + 2
        n = int(a.gb * 1e9 / per_tu)
        x, y, rows = tiled_offsets(n, s_, s_, s_, s_, W)
        g = torch.Generator(device=dev).manual_seed(log2)
        F = torch.randint(0, 256, (rows * W,), dtype=torch.int16, device=dev, generator=g)
        P = (F + torch.randint(-12, 13, F.shape, dtype=torch.int16, device=dev, generator=g)).clamp(0, 255)
        F, P = F.to(torch.uint8), P.to(torch.uint8)
        off = torch.from_numpy(y * W + x).to(dev)
        R = torch.empty(rows * W, dtype=torch.int16, device=dev)
        RC = torch.empty(rows * W, dtype=torch.uint8, device=dev)
        CO = torch.empty(n * num, dtype=torch.int16, device=dev)
        coff = torch.arange(n, dtype=torch.int64, device=dev) * num
        SIG = torch.empty(n, dtype=torch.int32, device=dev)
        QP = torch.randint(22, 38, (n,), dtype=torch.uint8, device=dev, generator=g)
        SC = torch.randint(0, 3 if log2 <= 3 else 1, (n,), dtype=torch.uint8, device=dev, generator=g)
        ms = timeit(lambda: prims.tu_pipeline(8, log2, 1, 1, 0, 1, F, W, off, P, W, off, R, W, off, CO, coff, RC, W,
                                              off, SIG, QP, SC))
        sig = SIG.cpu()
        record(name, n * per_tu, ms, n)
        results[-1]["numsig_share"] = {"0": round(float((sig == 0).float().mean()), 3),
                                       "1": round(float((sig == 1).float().mean()), 3),
                                       ">=2": round(float((sig >= 2).float().mean()), 3)}
        # the unfused chain on the same TUs (8-bit: transformShift = 7 - log2)
        DC = torch.empty(n * num, dtype=torch.int16, device=dev)
        DQ = torch.empty(n * num, dtype=torch.int16, device=dev)
        DL = torch.empty(n * num, dtype=torch.int32, device=dev)
        qps = QP.to(torch.int32)
        per, rem = qps // 6, qps % 6
        QT = torch.tensor([26214, 23302, 20560, 18396, 16384, 14564], dtype=torch.int32, device=dev)
        QT = QT.repeat_interleave(num)
        qo = rem.to(torch.int64) * num
        tsh = 15 - 8 - log2
        qb = (14 + per + tsh).to(torch.int32)
        ad = (85 * torch.pow(2, qb - 9)).to(torch.int32)
        iq = torch.tensor([40, 45, 51, 57, 64, 72], dtype=torch.int32, device=dev)
        dsc = (iq[rem.long()] * torch.pow(2, per)).to(torch.int32)
        dsh = torch.full((n,), 6 - tsh, dtype=torch.int32, device=dev)
        k_fwd = 2 if log2 == 2 else DCT      # DST for luma intra 4x4
        k_inv = 3 if log2 == 2 else IDCT

        def chain():
            prims.blockop(0, 8, s_, s_, R, W, off, F, W, off, P, W, off)              # calcresidual / sub_ps
            prims.transform(k_fwd, 8, s_, R, W, off, DC, s_, coff)
            prims.quant(num, DC, coff, QT, qo, DL, coff, CO, coff, qb, ad, SIG)
            prims.dequant_normal(num, CO, coff, DQ, coff, dsc, dsh)
            prims.transform(k_inv, 8, s_, DQ, s_, coff, R, W, off)
            prims.blockop(1, 8, s_, s_, RC, W, off, P, W, off, R, W, off)             # add_ps
        ms_u = timeit(chain)
        # sub_ps 4N^2, dct 4N^2, quant 8N^2 + 4, dequant 4N^2, idct 4N^2, add_ps 4N^2
        unf = n * (28 * num + 4)
        r = {"kernel": f"tu_unfused_chain_{s_}x{s_}", "jobs": n, "bytes_per_launch": int(unf), "ms": round(ms_u, 4),
             "achieved_GBps": round(unf / (ms_u * 1e-3) / 1e9, 1),
             "frac_of_8TBps": round(unf / (ms_u * 1e-3) / 1e9 / HBM, 3), "fused_speedup": round(ms_u / ms, 2)}
        results.append(r)
        print(json.dumps(r), flush=True)
        del F, P, off, R, RC, CO, coff, SIG, QP, SC, DC, DQ, DL, QT, qo, qb, ad, dsc, dsh
    # ---------------------------------------------------------------- f1 lookahead lowres
    # 8 frames per call.  lowres_init is HBM-bound: algorithmic bytes = the source rows it reads
    # (2 lines + 1 rows of 2 width + 1 pixels) + the four padded planes it writes.  lowres_intra is
    # compute-bound (12 predictions + 8x8 SATDs per 8x8 CU): reported as CUs/s and frames/s, with
    # the reference's own lowresIntraEstimate (oracle/_ref) timed on one host core beside it.
    for (Wf, Hf) in ((1920, 1080), (3840, 2160)):
        name = f"lowres_{Hf}p"
        if not want(name):
            continue
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from cases import lowres_geometry
        g = lowres_geometry(Wf, Hf)
        nf = 8
        ss = 2 * g["width"] + 32
        fsize = ss * (2 * g["lines"] + 4)
        SRC = rand_u8(nf * fsize)
        so = torch.arange(nf, dtype=torch.int64, device=dev) * fsize + 16
        psize = g["ls"] * (g["lines"] + 2 * g["my"])
        PL = torch.empty(4 * nf * psize, dtype=torch.uint8, device=dev)
        org = g["my"] * g["ls"] + g["mx"]
        po = torch.arange(4 * nf, dtype=torch.int64, device=dev) * psize + org
        ncu = g["wcu"] * g["hcu"]
        IC = torch.empty(nf * ncu, dtype=torch.int32, device=dev)
        IM = torch.empty(nf * ncu, dtype=torch.uint8, device=dev)
        LC = torch.empty(nf * ncu, dtype=torch.int16, device=dev)
        RS = torch.empty(nf * g["hcu"], dtype=torch.int32, device=dev)
        CE = torch.empty(2 * nf, dtype=torch.int64, device=dev)
        IQ = torch.randint(128, 384, (nf * ncu,), dtype=torch.int32, device=dev)
        ms_init = timeit(lambda: prims.lowres_init(8, nf, g["width"], g["lines"], g["mx"], g["my"], SRC, ss, so, PL,
                                                   g["ls"], po))
        init_bytes = nf * ((2 * g["lines"] + 1) * (2 * g["width"] + 1) + 4 * psize)
        record(f"lowres_init_{Hf}p_x8", init_bytes, ms_init, nf)
        p0 = po[0::4].contiguous()
        ms_intra = timeit(lambda: prims.lowres_intra(8, nf, g["wcu"], g["hcu"], PL, g["ls"], p0, IQ, IC, IM, LC, RS,
                                                     CE))
        r = {"kernel": f"lowres_intra_{Hf}p_x8", "jobs": nf * ncu, "ms": round(ms_intra, 4),
             "cu_per_s": round(nf * ncu / (ms_intra * 1e-3), 1), "frames_per_s": round(nf / (ms_intra * 1e-3), 1),
             "bound": "valu (12 predictions + 8x8 SATD per CU)"}
        try:
            import time as _t

            import numpy as _np
            from pyoracle import CpuOracle, available
            if available("ref", 8):
                ref = CpuOracle("ref", 8)
                pl = PL[:psize].cpu().numpy()
                ic, im = _np.empty(ncu, _np.int32), _np.empty(ncu, _np.uint8)
                lc, rs_, ce = _np.empty(ncu, _np.uint16), _np.empty(g["hcu"], _np.int32), _np.empty(2, _np.int64)
                import ctypes as _C
                lib = _C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libx265ref8.so"))
                t0 = _t.perf_counter()
                lib.xo_lowres_intra(g["wcu"], g["hcu"], _C.c_void_p(pl.ctypes.data + org), _C.c_ssize_t(g["ls"]),
                                    None, _C.c_void_p(ic.ctypes.data), _C.c_void_p(im.ctypes.data),
                                    _C.c_void_p(lc.ctypes.data), _C.c_void_p(rs_.ctypes.data),
                                    _C.c_void_p(ce.ctypes.data))
                dt = _t.perf_counter() - t0
                r["cpu_reference_1core_frames_per_s"] = round(1.0 / dt, 2)
        except Exception as ex:  # the CPU leg is informational
            r["cpu_reference_error"] = str(ex)
        results.append(r)
        print(json.dumps(r), flush=True)
        # P estimates of frame f+1 against frame f for the 8 frames' planes (7 estimates), coop slices as
        # Lookahead::create sets them for --lookahead-slices 8 (medium), and the whole-frame variant
        from cases import MVCOST_RANGE, mvcost_table
        TAB = torch.from_numpy(mvcost_table(8)).to(dev)
        ne = nf - 1
        fo = po[4::4].contiguous()
        ro = po[:4 * ne].contiguous()
        rps = max(g["hcu"] // 8, 10)
        ns = g["hcu"] // rps
        MVS = torch.empty(2 * ne * ncu, dtype=torch.int16, device=dev)
        MC = torch.empty(ne * ncu, dtype=torch.int32, device=dev)
        PLC = torch.empty(ne * ncu, dtype=torch.int16, device=dev)
        PRS = torch.empty(ne * g["hcu"], dtype=torch.int32, device=dev)
        PCE = torch.empty(2 * ne, dtype=torch.int64, device=dev)
        MB = torch.empty(ne, dtype=torch.int32, device=dev)
        for (rr, nn, tag) in ((rps, ns, f"slices{ns}"), (0, 0, "whole")):
            ms_p = timeit(lambda: prims.lowres_pcost(8, ne, g["wcu"], g["hcu"], rr, nn, PL, g["ls"], fo, ro,
                                                     IC[:ne * ncu], IQ[:ne * ncu], TAB.data_ptr() + 2 * MVCOST_RANGE,
                                                     MVS, MC, PLC, PRS, PCE, MB))
            r = {"kernel": f"lowres_pcost_{Hf}p_x{ne}_{tag}", "jobs": ne * ncu, "ms": round(ms_p, 4),
                 "estimates_per_s": round(ne / (ms_p * 1e-3), 1),
                 "bound": "latency (serial CU wavefront per slice; one workgroup per slice, a 4-lane quad per CU row)"}
            try:
                import ctypes as _C
                import time as _t

                import numpy as _np
                lib = _C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libx265ref8.so"))
                plh = PL[:8 * psize].cpu().numpy()
                ich = IC[:ncu].cpu().numpy()
                o = [_np.empty(2 * ncu, _np.int16), _np.empty(ncu, _np.int32), _np.empty(ncu, _np.uint16),
                     _np.empty(g["hcu"], _np.int32), _np.empty(2, _np.int64), _np.empty(1, _np.int32)]
                vp = lambda arr, off=0: _C.c_void_p(arr.ctypes.data + off * arr.itemsize)
                t0 = _t.perf_counter()
                lib.xo_lowres_pcost(g["wcu"], g["hcu"], rr, nn, vp(plh, 4 * psize + org),
                                    *[vp(plh, k * psize + org) for k in range(4)], _C.c_ssize_t(g["ls"]), vp(ich),
                                    None, None, *[vp(x) for x in o])
                r["cpu_reference_1core_estimates_per_s"] = round(1.0 / (_t.perf_counter() - t0), 2)
            except Exception as ex:
                r["cpu_reference_error"] = str(ex)
            results.append(r)
            print(json.dumps(r), flush=True)
        # throughput with a lookahead-sized batch: 56 estimates (each frame against each of the 7 others)
        pairs = [(b_, p_) for b_ in range(nf) for p_ in range(nf) if p_ != b_]
        nb = len(pairs)
        fo56 = torch.tensor([4 * b_ * psize + org for b_, _ in pairs], dtype=torch.int64, device=dev)
        ro56 = torch.tensor([(4 * p_ + k) * psize + org for _, p_ in pairs for k in range(4)], dtype=torch.int64,
                            device=dev)
        IC56 = IC[:ncu].repeat(nb)
        MVS = torch.empty(2 * nb * ncu, dtype=torch.int16, device=dev)
        MC = torch.empty(nb * ncu, dtype=torch.int32, device=dev)
        PLC = torch.empty(nb * ncu, dtype=torch.int16, device=dev)
        PRS = torch.empty(nb * g["hcu"], dtype=torch.int32, device=dev)
        PCE = torch.empty(2 * nb, dtype=torch.int64, device=dev)
        MB = torch.empty(nb, dtype=torch.int32, device=dev)
        ms_p = timeit(lambda: prims.lowres_pcost(8, nb, g["wcu"], g["hcu"], rps, ns, PL, g["ls"], fo56, ro56, IC56, None,
                                                 TAB.data_ptr() + 2 * MVCOST_RANGE, MVS, MC, PLC, PRS, PCE, MB))
        r = {"kernel": f"lowres_pcost_{Hf}p_x{nb}_slices{ns}", "jobs": nb * ncu, "ms": round(ms_p, 4),
             "estimates_per_s": round(nb / (ms_p * 1e-3), 1),
             "bound": "latency (serial CU wavefront per slice; one workgroup per slice, a 4-lane quad per CU row)"}
        results.append(r)
        print(json.dumps(r), flush=True)
        # B estimates (p0, b, p1) = (f, f+1, f+2), both lists searched: 6 per call, and a b-adapt-2
        # sized batch of 48 (every b between two frames up to 4 apart, repeated)
        for nbb in (6, 48):
            trip = [(f, f + 1, f + 2) for f in range(nf - 2)]
            trip = (trip * ((nbb + len(trip) - 1) // len(trip)))[:nbb]
            fob = torch.tensor([4 * b_ * psize + org for _, b_, _ in trip], dtype=torch.int64, device=dev)
            r0b = torch.tensor([(4 * p_ + k) * psize + org for p_, _, _ in trip for k in range(4)], dtype=torch.int64,
                               device=dev)
            r1b = torch.tensor([(4 * p_ + k) * psize + org for _, _, p_ in trip for k in range(4)], dtype=torch.int64,
                               device=dev)
            DS = torch.ones(2 * nbb, dtype=torch.uint8, device=dev)
            BM0 = torch.empty(2 * nbb * ncu, dtype=torch.int16, device=dev)
            BM1 = torch.empty_like(BM0)
            BC0 = torch.empty(nbb * ncu, dtype=torch.int32, device=dev)
            BC1 = torch.empty_like(BC0)
            BLC = torch.empty(nbb * ncu, dtype=torch.int16, device=dev)
            BRS = torch.empty(nbb * g["hcu"], dtype=torch.int32, device=dev)
            BCE = torch.empty(2 * nbb, dtype=torch.int64, device=dev)
            ms_b = timeit(lambda: prims.lowres_bcost(8, nbb, g["wcu"], g["hcu"], rps, ns, PL, g["ls"], fob, r0b, r1b, DS,
                                                     None, TAB.data_ptr() + 2 * MVCOST_RANGE, BM0, BC0, BM1, BC1, BLC,
                                                     BRS, BCE))
            r = {"kernel": f"lowres_bcost_{Hf}p_x{nbb}_slices{ns}", "jobs": nbb * ncu, "ms": round(ms_b, 4),
                 "estimates_per_s": round(nbb / (ms_b * 1e-3), 1),
                 "bound": "latency (serial CU wavefront per slice; two quads per CU search the two lists concurrently)"}
            if nbb == 6:
                try:
                    import time as _t
                    sys.path.insert(0, os.path.join(ROOT, "oracle"))
                    import pyoracle as _po
                    RB = _po.LowresB("ref", 8)
                    plh = PL[:12 * psize].cpu().numpy()
                    tabh = TAB.cpu().numpy()
                    z = lambda k, dt: np.zeros(k, dt)
                    t0 = _t.perf_counter()
                    RB.bcost(g["wcu"], g["hcu"], rps, ns, plh, g["ls"], 4 * psize + org,
                             [k * psize + org for k in range(4)], [(8 + k) * psize + org for k in range(4)], None,
                             tabh.ctypes.data + 2 * MVCOST_RANGE, 1, 1, z(2 * ncu, np.int16), z(ncu, np.int32),
                             z(2 * ncu, np.int16), z(ncu, np.int32), z(ncu, np.uint16), z(g["hcu"], np.int32),
                             z(2, np.int64))
                    r["cpu_reference_1core_estimates_per_s"] = round(1.0 / (_t.perf_counter() - t0), 2)
                except Exception as ex:
                    r["cpu_reference_error"] = str(ex)
            results.append(r)
            print(json.dumps(r), flush=True)
        del SRC, PL, IC, IM, LC, RS, CE, IQ, MVS, MC, PLC, PRS, PCE, MB
    # ---------------------------------------------------------------- f2 motion search
    # HEX + subme 2 + merange 57 (--preset medium) on the synthetic 1080p pair (pan +2/+1, object, noise):
    # every 2Nx2N PU of the frame at 8 / 16 / 32 / 64 (one batch per size), MVP = true pan +- jitter,
    # 2 candidates, QP 32.  Search-bound (serial dependent SAD rounds per PU); reported as PUs/s with
    # the reference's MotionEstimate::motionEstimate timed on one host core on the same jobs.
    for s_ in (8, 16, 32, 64):
        name = f"me_hex_{s_}x{s_}"
        if not want(name):
            continue
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from cases import ME_TAB_RANGE, me_tables
        from src.x265_amd.synth import SyntheticSource
        Wf, Hf, M = 1920, 1080, 96
        syn = SyntheticSource(Wf, Hf, 2, 8)
        padf = lambda y: np.pad(y, M, mode="edge").reshape(-1)
        f1, f0 = padf(syn.frame(1)[0]), padf(syn.frame(0)[0])
        st = Wf + 2 * M
        xs, ys = np.meshgrid(np.arange(0, Wf - s_ + 1, s_), np.arange(0, Hf - s_ + 1, s_))
        xs, ys = xs.reshape(-1), ys.reshape(-1)
        n = xs.size
        rng_ = np.random.default_rng(s_)
        fo_h = ((ys + M) * st + xs + M).astype(np.int64)
        mvp_xy = np.stack([-8 + rng_.integers(-4, 5, n), -4 + rng_.integers(-4, 5, n)], 1)
        mvp_h = mvp_xy.astype(np.int16).reshape(-1)
        # Search::setSearchRange: MVP +- merange (57) in full-pel, clipped to the picture + 40 px of padding
        rng_h = np.stack([np.maximum(-xs - 40, (mvp_xy[:, 0] >> 2) - 57), np.maximum(-ys - 40, (mvp_xy[:, 1] >> 2) - 57),
                          np.minimum(Wf - xs - s_ + 40, (mvp_xy[:, 0] >> 2) + 57),
                          np.minimum(Hf - ys - s_ + 40, (mvp_xy[:, 1] >> 2) + 57)], 1).astype(np.int16).reshape(-1)
        mvc_h = rng_.integers(-16, 17, 2 * 2 * n).astype(np.int16)
        numc_h = np.full(n, 2, np.uint8)
        tabs = me_tables(8)
        toff_h = np.full(n, 2 * (2 * ME_TAB_RANGE + 1) + ME_TAB_RANGE, np.int64)   # ME_QPS[2] = 32
        T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
        F1, F0, FO, RG, MP, MC2, NC, TB, TO = (T(f1), T(f0), T(fo_h), T(rng_h), T(mvp_h), T(mvc_h), T(numc_h),
                                               T(tabs), T(toff_h))
        OM = torch.empty(2 * n, dtype=torch.int16, device=dev)
        OC = torch.empty(n, dtype=torch.int32, device=dev)
        ms_me = timeit(lambda: prims.motion_search(8, s_, s_, 1, 2, 57, 2, F1, st, FO, F0, st, FO, RG, MP, MC2, NC, TB,
                                                   TO, OM, OC))
        r = {"kernel": name, "jobs": n, "ms": round(ms_me, 4), "pu_per_s": round(n / (ms_me * 1e-3), 1),
             "bound": "latency (serial SAD rounds per PU)"}
        try:
            from pyoracle import CpuOracle, available
            if available("ref", 8):
                import time as _t
                ref = CpuOracle("ref", 8)
                k = min(n, 2000)
                om, oc = np.empty(2 * k, np.int16), np.empty(k, np.int32)
                t0 = _t.perf_counter()
                ref.motion_search(s_, s_, 1, 2, 57, 2, f1, st, fo_h[:k], f0, st, fo_h[:k], rng_h[:4 * k], mvp_h[:2 * k],
                                  mvc_h[:4 * k], numc_h[:k], tabs, toff_h[:k], np.full(k, 32, np.uint8), om, oc)
                r["cpu_reference_1core_pu_per_s"] = round(k / (_t.perf_counter() - t0), 1)
                r["gpu_matches_reference_on_sample"] = bool(np.array_equal(om, OM[:2 * k].cpu().numpy()) and
                                                            np.array_equal(oc, OC[:k].cpu().numpy()))
        except Exception as ex:
            r["cpu_reference_error"] = str(ex)
        results.append(r)
        print(json.dumps(r), flush=True)
        # --preset slow: STAR search, subme 3 with the 4:2:0 chroma SATD
        MCp = M // 2
        padc = lambda y: np.pad(y, MCp, mode="edge").reshape(-1)
        fr1, fr0 = syn.frame(1), syn.frame(0)
        cst = Wf // 2 + 2 * MCp
        co_h = ((ys // 2 + MCp) * cst + xs // 2 + MCp).astype(np.int64)
        FCB, FCR, RCB, RCR, CO = T(padc(fr1[1])), T(padc(fr1[2])), T(padc(fr0[1])), T(padc(fr0[2])), T(co_h)
        ms_st = timeit(lambda: prims.motion_search(8, s_, s_, 2, 3, 57, 2, F1, st, FO, F0, st, FO, RG, MP, MC2, NC, TB,
                                                   TO, OM, OC, FCB, FCR, cst, CO, RCB, RCR, cst, CO))
        r = {"kernel": f"me_star_subme3_{s_}x{s_}", "jobs": n, "ms": round(ms_st, 4),
             "pu_per_s": round(n / (ms_st * 1e-3), 1), "bound": "latency (serial SAD rounds per PU)"}
        try:
            from pyoracle import CpuOracle, available
            if available("ref", 8):
                import time as _t
                ref = CpuOracle("ref", 8)
                k = min(n, 1000)
                om, oc = np.empty(2 * k, np.int16), np.empty(k, np.int32)
                t0 = _t.perf_counter()
                ref.motion_search(s_, s_, 2, 3, 57, 2, f1, st, fo_h[:k], f0, st, fo_h[:k], rng_h[:4 * k], mvp_h[:2 * k],
                                  mvc_h[:4 * k], numc_h[:k], tabs, toff_h[:k], np.full(k, 32, np.uint8), om, oc,
                                  padc(fr1[1]), padc(fr1[2]), cst, co_h[:k], padc(fr0[1]), padc(fr0[2]), cst, co_h[:k])
                r["cpu_reference_1core_pu_per_s"] = round(k / (_t.perf_counter() - t0), 1)
                r["gpu_matches_reference_on_sample"] = bool(np.array_equal(om, OM[:2 * k].cpu().numpy()) and
                                                            np.array_equal(oc, OC[:k].cpu().numpy()))
        except Exception as ex:
            r["cpu_reference_error"] = str(ex)
        results.append(r)
        print(json.dumps(r), flush=True)
        # batched: R independent (current, reference) frame pairs in ONE launch (the searches of several
        # reference frames / lists or of several frames whose references are final): the latency-bound
        # search needs many PUs in flight to fill 256 CUs
        R = 8
        synR = SyntheticSource(Wf, Hf, R + 1, 8)
        curs = np.concatenate([padf(synR.frame(q + 1)[0]) for q in range(R)])
        refs = np.concatenate([padf(synR.frame(q)[0]) for q in range(R)])
        psz = f1.size
        foR = (fo_h[None, :] + psz * np.arange(R)[:, None]).reshape(-1)
        tile = lambda x, per: np.tile(x.reshape(n, per), (R, 1)).reshape(-1)
        FR, RR, FOR = T(curs), T(refs), T(foR)
        RGR, MPR, MCR, NCR, TOR = (T(tile(rng_h, 4)), T(tile(mvp_h, 2)), T(tile(mvc_h, 4)), T(tile(numc_h, 1)),
                                   T(tile(toff_h, 1)))
        OMR = torch.empty(2 * n * R, dtype=torch.int16, device=dev)
        OCR = torch.empty(n * R, dtype=torch.int32, device=dev)
        for meth, sub, tag in ((1, 2, "hex"), (2, 3, "star_subme3")):
            if meth == 2:
                cR = np.concatenate([padc(synR.frame(q + 1)[1]) for q in range(R)])
                crR = np.concatenate([padc(synR.frame(q + 1)[2]) for q in range(R)])
                rR = np.concatenate([padc(synR.frame(q)[1]) for q in range(R)])
                rrR = np.concatenate([padc(synR.frame(q)[2]) for q in range(R)])
                coR = T((co_h[None, :] + padc(fr1[1]).size * np.arange(R)[:, None]).reshape(-1))
                chroma = (T(cR), T(crR), cst, coR, T(rR), T(rrR), cst, coR)
            else:
                chroma = ()
            ms_b = timeit(lambda: prims.motion_search(8, s_, s_, meth, sub, 57, 2, FR, st, FOR, RR, st, FOR, RGR, MPR,
                                                      MCR, NCR, TB, TOR, OMR, OCR, *chroma))
            r = {"kernel": f"me_{tag}_{s_}x{s_}_x{R}", "jobs": n * R, "ms": round(ms_b, 4),
                 "pu_per_s": round(n * R / (ms_b * 1e-3), 1),
                 "note": f"{R} (current, reference) frame pairs of 1080p PUs in one launch"}
            results.append(r)
            print(json.dumps(r), flush=True)
        # --me umh and --me full (subme 2) on the single-frame batch; FULL is the one data-parallel
        # integer search: its unit of work is one pixel of one candidate (w h per MV, (2 merange + 1)^2
        # MVs per PU when the range is not clipped), bounded by v_sad throughput, not HBM
        for meth, tag, kcpu in ((3, "umh", 1000), (4, "full", max(2, 4096 // (s_ * s_) * 4))):
            ms_x = timeit(lambda: prims.motion_search(8, s_, s_, meth, 2, 57, 2, F1, st, FO, F0, st, FO, RG, MP, MC2,
                                                      NC, TB, TO, OM, OC))
            r = {"kernel": f"me_{tag}_{s_}x{s_}", "jobs": n, "ms": round(ms_x, 4),
                 "pu_per_s": round(n / (ms_x * 1e-3), 1)}
            if meth == 4:
                rg4 = rng_h.reshape(-1, 4).astype(np.int64)
                pxc = float(((rg4[:, 2] - rg4[:, 0] + 1) * (rg4[:, 3] - rg4[:, 1] + 1)).sum() * s_ * s_)
                r["pixel_candidates_per_s"] = round(pxc / (ms_x * 1e-3), 1)
                r["bound"] = "valu (v_sad_u8: 4 pixel-candidates per lane op)"
            try:
                from pyoracle import CpuOracle, available
                if available("ref", 8):
                    import time as _t
                    ref = CpuOracle("ref", 8)
                    k = min(n, kcpu)
                    om, oc = np.empty(2 * k, np.int16), np.empty(k, np.int32)
                    t0 = _t.perf_counter()
                    ref.motion_search(s_, s_, meth, 2, 57, 2, f1, st, fo_h[:k], f0, st, fo_h[:k], rng_h[:4 * k],
                                      mvp_h[:2 * k], mvc_h[:4 * k], numc_h[:k], tabs, toff_h[:k],
                                      np.full(k, 32, np.uint8), om, oc)
                    r["cpu_reference_1core_pu_per_s"] = round(k / (_t.perf_counter() - t0), 2)
                    r["gpu_matches_reference_on_sample"] = bool(np.array_equal(om, OM[:2 * k].cpu().numpy()) and
                                                                np.array_equal(oc, OC[:k].cpu().numpy()))
            except Exception as ex:
                r["cpu_reference_error"] = str(ex)
            results.append(r)
            print(json.dumps(r), flush=True)
    # ---------------------------------------------------------------- f4 loop filters
    # Whole frames, >= --gb of distinct frame buffers per call (8 frames per launch).  Algorithmic
    # bytes per frame: deblock = the picture read once and written once + its 16-byte CU units
    # (a fused one-pass lower bound; the kernel makes two passes, V then H); sao_apply = the
    # deblocked picture read + the output written; sao_stats = source + deblocked pictures read;
    # extend_border = the margin area written.  CPU: the reference's own Deblock / SAO / extendPicBorder
    # (oracle/_ref via ref_shim, one core, frame setup included).
    for Hf in (1080, 2160):
        if not want(f"f4_{Hf}p"):
            continue
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import f4cases as F4
        from src.x265_amd.native import BorderPlane, DeblockFrame, SaoFrame, SaoStatsFrame
        import pyoracle as po4
        Wf = 3840 if Hf == 2160 else 1920
        M = F4.MARGIN
        rng = np.random.default_rng(Hf)
        pl = F4.frame_planes(Wf, Hf, 8, rng)
        U = F4.deblock_units(Wf, Hf, 6, 8, rng, "B")
        dp = F4.deblock_params(rng, "B", 0)
        prm = F4.sao_params(Wf, Hf, 6, 8, rng)
        fbytes = Wf * Hf * 3 // 2
        nfr = max(8, int(a.gb * 1e9 / (2 * sum(p.nbytes for p in pl) + U.nbytes)))
        nfr = (nfr + 7) // 8 * 8
        src = [torch.from_numpy(p).cuda().unsqueeze(0).repeat(nfr, 1, 1).contiguous() for p in pl]
        dst = [torch.empty_like(s) for s in src]
        du = torch.from_numpy(U.view(np.uint8).reshape(U.shape[0], -1)).cuda().unsqueeze(0).repeat(nfr, 1, 1).contiguous()
        dprm = torch.from_numpy(prm.view(np.uint8)).cuda()

        def org(t, i):
            return t[i].data_ptr() + (M * t.shape[2] + M) * t.element_size()

        dbk, sao, sst, bor = [], [], [], []
        nctu = ((Wf + 63) // 64) * ((Hf + 63) // 64)
        stats = torch.empty(nfr * nctu * 3 * 5 * 33, dtype=torch.int32, device=dev)
        count = torch.empty_like(stats)
        for i in range(nfr):
            fr = DeblockFrame()
            fr.width, fr.height = Wf, Hf
            for p in range(3):
                fr.plane[p] = org(dst[p], i)
            fr.stride, fr.cstride = src[0].shape[2], src[1].shape[2]
            fr.units, fr.unit_stride = du[i].data_ptr(), U.shape[1]
            fr.is_p, fr.beta_offset_div2, fr.tc_offset_div2 = 0, dp.beta_offset_div2, dp.tc_offset_div2
            fr.cb_qp_offset, fr.cr_qp_offset = dp.cb_qp_offset, dp.cr_qp_offset
            for lst in range(2):
                for k in range(16):
                    fr.ref_poc[lst][k] = dp.ref_poc[lst][k]
            dbk.append(fr)
            sf = SaoFrame()
            sf.width, sf.height, sf.ctu_log2, sf.luma_on, sf.chroma_on = Wf, Hf, 6, 1, 1
            for p in range(3):
                sf.src[p], sf.dst[p] = org(src[p], i), org(dst[p], i)
            sf.stride, sf.cstride, sf.params = src[0].shape[2], src[1].shape[2], dprm.data_ptr()
            sao.append(sf)
            tf = SaoStatsFrame()
            tf.width, tf.height, tf.ctu_log2, tf.non_deblocked = Wf, Hf, 6, 0
            for p in range(3):
                tf.fenc[p], tf.rec[p] = org(src[p], i), org(dst[p], i)
            tf.fenc_stride, tf.fenc_cstride, tf.rec_stride, tf.rec_cstride = (src[0].shape[2], src[1].shape[2],
                                                                              src[0].shape[2], src[1].shape[2])
            tf.stats = stats.data_ptr() + i * nctu * 3 * 5 * 33 * 4
            tf.count = count.data_ptr() + i * nctu * 3 * 5 * 33 * 4
            sst.append(tf)
            for p in range(3):
                bp = BorderPlane()
                bp.plane = org(dst[p], i) + 0
                w_, h_ = (Wf, Hf) if p == 0 else (Wf // 2, Hf // 2)
                bp.stride, bp.width, bp.height, bp.margin_x, bp.margin_y = src[p].shape[2], w_, h_, M, M
                bor.append(bp)
        for d_, s_ in zip(dst, src):
            d_.copy_(s_)
        # one call per filter over all frames, captured once into a hipGraph and replayed, so the
        # events time the GPU work rather than the host enqueueing ~nfr/8 launches
        def graphed(fn):
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with capture_graph(g):
                fn()
            return timeit(g.replay)

        ms_d = graphed(lambda: prims.deblock(8, dbk))
        ms_a = graphed(lambda: prims.sao_apply(8, sao))
        ms_s = graphed(lambda: prims.sao_stats(8, sst))
        ms_b = graphed(lambda: prims.extend_border(8, bor))
        border_bytes = sum((s.shape[2] * s.shape[1] - (w_ * h_)) for s, (w_, h_) in
                           zip(src, ((Wf, Hf), (Wf // 2, Hf // 2), (Wf // 2, Hf // 2))))
        cpu = {}
        try:
            if po4.available("ref", 8):
                import time as _t
                R = po4.FrameFilters("ref", 8)
                reps = 2 if Hf == 1080 else 1
                for nm, fn in (("deblock", lambda q: R.deblock(Wf, Hf, 6, q, M, U, dp)),
                               ("sao_apply", lambda q: R.sao_apply(Wf, Hf, 6, q, M, prm)),
                               ("sao_stats", lambda q: R.sao_stats(Wf, Hf, 6, pl, q, M, 0))):
                    q = F4.copy_planes(pl)
                    t0 = _t.perf_counter()
                    for _ in range(reps):
                        fn(q)
                    cpu[nm] = round(reps / (_t.perf_counter() - t0), 2)
        except Exception as ex:
            cpu["error"] = str(ex)
        for nm, ms, nbytes in (("deblock", ms_d, nfr * (2 * fbytes + U.nbytes)), ("sao_apply", ms_a, nfr * 2 * fbytes),
                               ("sao_stats", ms_s, nfr * 2 * fbytes), ("extend_border", ms_b, nfr * border_bytes)):
            gbs = nbytes / (ms * 1e-3) / 1e9
            r = {"kernel": f"f4_{nm}_{Hf}p_x{nfr}", "jobs": nfr, "bytes_per_launch": int(nbytes), "ms": round(ms, 4),
                 "frames_per_s": round(nfr / (ms * 1e-3), 1), "achieved_GBps": round(gbs, 1),
                 "frac_of_8TBps": round(gbs / HBM, 3)}
            if nm in cpu:
                r["cpu_reference_1core_frames_per_s"] = cpu[nm]
            results.append(r)
            print(json.dumps(r), flush=True)
        del src, dst, du, stats, count
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"hbm_peak_GBps": HBM, "working_set_GB": a.gb, "results": results}, f, indent=1)


if __name__ == "__main__":
    main()
