"""f4 loop filters: SAO apply, SAO statistics, deblocking, border extension.

CPU tests pin the restatement (oracle/x265_oracle.c) to the reference's own SAO / Deblock classes
run by oracle/ref_shim.cpp on the same frames; GPU tests hold the gfx950 kernels to the oracle,
bit-exact.
"""
from __future__ import annotations

import numpy as np
import pytest

import f4cases as F
import pyoracle as po

SIZES = [(200, 136, 6), (128, 64, 5), (96, 48, 4), (256, 128, 6)]
DEPTHS = [8, 10]


def _libs(depth):
    if not po.available("ref", depth):
        pytest.skip("reference library not built (make -C oracle ref)")
    return po.FrameFilters("oracle", depth), po.FrameFilters("ref", depth)


@pytest.mark.parametrize("depth", DEPTHS)
@pytest.mark.parametrize("size", SIZES)
def test_sao_apply_oracle_vs_reference(oracle_libs, depth, size):
    W, H, cl = size
    O, R = _libs(depth)
    rng = np.random.default_rng(W + H + depth + cl)
    pl = F.frame_planes(W, H, depth, rng)
    prm = F.sao_params(W, H, cl, depth, rng)
    for on in ((1, 1), (1, 0), (0, 1)):
        a, b = F.copy_planes(pl), F.copy_planes(pl)
        O.sao_apply(W, H, cl, a, F.MARGIN, prm, *on)
        R.sao_apply(W, H, cl, b, F.MARGIN, prm, *on)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    assert sum(int((x != y).sum()) for x, y in zip(b, pl)) > 0


@pytest.mark.parametrize("depth", DEPTHS)
@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("non_deblocked", [0, 1])
def test_sao_stats_oracle_vs_reference(oracle_libs, depth, size, non_deblocked):
    W, H, cl = size
    O, R = _libs(depth)
    rng = np.random.default_rng(7 * W + H + depth + cl)
    rec = F.frame_planes(W, H, depth, rng)
    fenc = F.frame_planes(W, H, depth, rng)
    s1, c1 = O.sao_stats(W, H, cl, fenc, rec, F.MARGIN, non_deblocked)
    s2, c2 = R.sao_stats(W, H, cl, fenc, rec, F.MARGIN, non_deblocked)
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(s1, s2)


@pytest.mark.parametrize("depth", DEPTHS)
@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("slice_type", ["I", "P", "B"])
@pytest.mark.parametrize("tq", [0, 1])
def test_deblock_oracle_vs_reference(oracle_libs, depth, size, slice_type, tq):
    W, H, cl = size
    O, R = _libs(depth)
    rng = np.random.default_rng(13 * W + H + depth + cl + ord(slice_type) + tq)
    pl = F.frame_planes(W, H, depth, rng)
    U = F.deblock_units(W, H, cl, depth, rng, slice_type, 0.2 if tq else 0.0)
    dp = F.deblock_params(rng, slice_type, tq)
    a, b = F.copy_planes(pl), F.copy_planes(pl)
    O.deblock(W, H, cl, a, F.MARGIN, U, dp)
    R.deblock(W, H, cl, b, F.MARGIN, U, dp)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert int((b[0] != pl[0]).sum()) > 0


@pytest.mark.parametrize("depth", DEPTHS)
def test_extend_border_oracle_vs_reference(oracle_libs, depth):
    O, R = _libs(depth)
    rng = np.random.default_rng(depth)
    W, H, mx, my = 200, 136, 96, 80
    dt = np.uint8 if depth == 8 else np.uint16
    p = rng.integers(0, 1 << depth, size=(H + 2 * my, W + 2 * mx)).astype(dt)
    a, b = p.copy(), p.copy()
    O.extend_border(a, mx, my, W, H)
    R.extend_border(b, mx, my, W, H)
    np.testing.assert_array_equal(a, b)


# 4:2:2 / 4:4:4 (SAO chroma CTUs (ctu >> hshift) x (ctu >> vshift), deblocking on the chroma
# plane's 8x8 grid with QP clamped instead of g_chromaScale, deblock.cpp:104-113, 443-521)
CSPS = [2, 3]


@pytest.mark.parametrize("csp", CSPS)
@pytest.mark.parametrize("depth", DEPTHS)
@pytest.mark.parametrize("size", SIZES)
def test_f4_chroma_formats_oracle_vs_reference(oracle_libs, csp, depth, size):
    W, H, cl = size
    O, R = _libs(depth)
    rng = np.random.default_rng(31 * W + H + depth + cl + csp)
    pl = F.frame_planes(W, H, depth, rng, csp=csp)
    prm = F.sao_params(W, H, cl, depth, rng)
    a, b = F.copy_planes(pl), F.copy_planes(pl)
    O.sao_apply(W, H, cl, a, F.MARGIN, prm, 1, 1, csp=csp)
    R.sao_apply(W, H, cl, b, F.MARGIN, prm, 1, 1, csp=csp)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    fenc = F.frame_planes(W, H, depth, rng, csp=csp)
    for nd in (0, 1):
        s1, c1 = O.sao_stats(W, H, cl, fenc, pl, F.MARGIN, nd, csp=csp)
        s2, c2 = R.sao_stats(W, H, cl, fenc, pl, F.MARGIN, nd, csp=csp)
        np.testing.assert_array_equal(c1, c2)
        np.testing.assert_array_equal(s1, s2)
    for st in ("I", "P", "B"):
        U = F.deblock_units(W, H, cl, depth, rng, st, 0.2 if st == "B" else 0.0)
        dp = F.deblock_params(rng, st, int(st == "B"))
        a, b = F.copy_planes(pl), F.copy_planes(pl)
        O.deblock(W, H, cl, a, F.MARGIN, U, dp, csp=csp)
        R.deblock(W, H, cl, b, F.MARGIN, U, dp, csp=csp)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
        assert int((b[1] != pl[1]).sum()) > 0


# ---------------------------------------------------------------- GPU: gfx950 kernels vs the oracle
GPU_SIZES = [(200, 136, 6), (128, 64, 5), (96, 48, 4), (1920, 1080, 6)]


def _dev(planes):
    import torch

    return tuple(torch.from_numpy(p.view(np.int16) if p.dtype == np.uint16 else p).cuda() for p in planes)


def _host(t, dtype):
    a = t.cpu().numpy()
    return a.view(np.uint16) if dtype == np.uint16 else a


def _org(t, margin=F.MARGIN):
    return t.data_ptr() + (margin * t.shape[1] + margin) * t.element_size()


@pytest.mark.gpu
@pytest.mark.parametrize("depth", DEPTHS)
def test_gpu_deblock(gpu_prims, depth):
    import torch
    from src.x265_amd.native import DeblockFrame

    O = po.FrameFilters("oracle", depth)
    frames, keep, expect = [], [], []
    for i, (W, H, cl) in enumerate(GPU_SIZES):
        for st in ("I", "P", "B"):
            tq = int(st == "B" and i == 0)
            rng = np.random.default_rng(100 * i + ord(st) + depth)
            pl = F.frame_planes(W, H, depth, rng)
            U = F.deblock_units(W, H, cl, depth, rng, st, 0.2 if tq else 0.0)
            dp = F.deblock_params(rng, st, tq)
            ref = F.copy_planes(pl)
            O.deblock(W, H, cl, ref, F.MARGIN, U, dp)
            d = _dev(pl)
            du = torch.from_numpy(U.view(np.uint8).reshape(U.shape[0], -1)).cuda()
            fr = DeblockFrame()
            fr.width, fr.height = W, H
            for p in range(3):
                fr.plane[p] = _org(d[p])
            fr.stride, fr.cstride = d[0].shape[1], d[1].shape[1]
            fr.units, fr.unit_stride = du.data_ptr(), U.shape[1]
            fr.is_p, fr.beta_offset_div2, fr.tc_offset_div2 = dp.is_p, dp.beta_offset_div2, dp.tc_offset_div2
            fr.cb_qp_offset, fr.cr_qp_offset, fr.tq_bypass_enabled = dp.cb_qp_offset, dp.cr_qp_offset, tq
            for lst in range(2):
                for k in range(16):
                    fr.ref_poc[lst][k] = dp.ref_poc[lst][k]
            frames.append(fr)
            keep.append((d, du))
            expect.append((ref, pl))
    gpu_prims.deblock(depth, frames)          # 12 frames of four sizes: two launches per direction
    torch.cuda.synchronize()
    for (d, _), (ref, pl) in zip(keep, expect):
        for p in range(3):
            np.testing.assert_array_equal(_host(d[p], pl[p].dtype), ref[p])


@pytest.mark.gpu
@pytest.mark.parametrize("depth", DEPTHS)
def test_gpu_sao_apply(gpu_prims, depth):
    import torch
    from src.x265_amd.native import SaoFrame

    O = po.FrameFilters("oracle", depth)
    frames, keep = [], []
    for i, (W, H, cl) in enumerate(GPU_SIZES):
        for on in ((1, 1), (1, 0), (0, 1)):
            rng = np.random.default_rng(10 * i + depth + on[0])
            pl = F.frame_planes(W, H, depth, rng)
            prm = F.sao_params(W, H, cl, depth, rng)
            ref = F.copy_planes(pl)
            O.sao_apply(W, H, cl, ref, F.MARGIN, prm, *on)
            src, dst = _dev(pl), _dev(tuple(np.zeros_like(p) for p in pl))
            dprm = torch.from_numpy(prm.view(np.uint8)).cuda()
            fr = SaoFrame()
            fr.width, fr.height, fr.ctu_log2, fr.luma_on, fr.chroma_on = W, H, cl, on[0], on[1]
            for p in range(3):
                fr.src[p], fr.dst[p] = _org(src[p]), _org(dst[p])
            fr.stride, fr.cstride = src[0].shape[1], src[1].shape[1]
            fr.params = dprm.data_ptr()
            frames.append(fr)
            keep.append((src, dst, dprm, ref, pl))
    gpu_prims.sao_apply(depth, frames)
    torch.cuda.synchronize()
    M = F.MARGIN
    for (src, dst, _, ref, pl) in keep:
        for p in range(3):
            got = _host(dst[p], pl[p].dtype)[M:-M, M:-M]
            np.testing.assert_array_equal(got, ref[p][M:-M, M:-M])


@pytest.mark.gpu
@pytest.mark.parametrize("depth", DEPTHS)
def test_gpu_sao_stats(gpu_prims, depth):
    import torch
    from src.x265_amd.native import SaoStatsFrame

    O = po.FrameFilters("oracle", depth)
    frames, keep = [], []
    for i, (W, H, cl) in enumerate(GPU_SIZES):
        for nd in (0, 1):
            rng = np.random.default_rng(31 * i + depth + nd)
            rec = F.frame_planes(W, H, depth, rng)
            fenc = F.frame_planes(W, H, depth, rng)
            s_ref, c_ref = O.sao_stats(W, H, cl, fenc, rec, F.MARGIN, nd)
            dr, df = _dev(rec), _dev(fenc)
            st = torch.full(s_ref.shape, -7, dtype=torch.int32, device="cuda")
            ct = torch.full(c_ref.shape, -7, dtype=torch.int32, device="cuda")
            fr = SaoStatsFrame()
            fr.width, fr.height, fr.ctu_log2, fr.non_deblocked = W, H, cl, nd
            for p in range(3):
                fr.fenc[p], fr.rec[p] = _org(df[p]), _org(dr[p])
            fr.fenc_stride, fr.fenc_cstride = df[0].shape[1], df[1].shape[1]
            fr.rec_stride, fr.rec_cstride = dr[0].shape[1], dr[1].shape[1]
            fr.stats, fr.count = st.data_ptr(), ct.data_ptr()
            frames.append(fr)
            keep.append((dr, df, st, ct, s_ref, c_ref))
    gpu_prims.sao_stats(depth, frames)
    torch.cuda.synchronize()
    for (_, _, st, ct, s_ref, c_ref) in keep:
        np.testing.assert_array_equal(ct.cpu().numpy(), c_ref)
        np.testing.assert_array_equal(st.cpu().numpy(), s_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", DEPTHS)
def test_gpu_extend_border(gpu_prims, depth):
    import torch
    from src.x265_amd.native import BorderPlane

    O = po.FrameFilters("oracle", depth)
    dt = np.uint8 if depth == 8 else np.uint16
    planes, keep = [], []
    # recon PicYuv geometry (picyuv.cpp:62-80) at CTU 64: luma 96 / 80, chroma 96 / 40
    for i, (W, H, mx, my) in enumerate([(1920, 1080, 96, 80), (960, 540, 96, 40), (200, 136, 96, 80),
                                        (100, 68, 96, 40), (64, 8, 3, 5)]):
        rng = np.random.default_rng(i + depth)
        stride = ((W + 63) // 64) * 64 + 2 * mx
        p = rng.integers(0, 1 << depth, size=(H + 2 * my, stride)).astype(dt)
        ref = p.copy()
        O.extend_border(ref, mx, my, W, H)
        d = torch.from_numpy(p.view(np.int16) if dt == np.uint16 else p).cuda()
        bp = BorderPlane()
        bp.plane = d.data_ptr() + (my * stride + mx) * d.element_size()
        bp.stride, bp.width, bp.height, bp.margin_x, bp.margin_y = stride, W, H, mx, my
        planes.append(bp)
        keep.append((d, ref))
    gpu_prims.extend_border(depth, planes)
    torch.cuda.synchronize()
    for d, ref in keep:
        np.testing.assert_array_equal(_host(d, dt), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", DEPTHS)
def test_gpu_loop_filter_row_bands_equal_whole_frame(gpu_prims, depth):
    """The CTU-row pipeline the frame-parallel shard publishes rows from: deblock
    band b, then SAO + border extension of band b - 1, top to bottom (x265amd_*_rows), equals
    the whole-frame deblock -> SAO -> border of the oracle bit-exactly, margins included."""
    import torch
    from src.x265_amd.native import BorderPlane, DeblockFrame, SaoFrame

    O = po.FrameFilters("oracle", depth)
    M = F.MARGIN
    for i, (W, H, cl) in enumerate(GPU_SIZES):
        rng = np.random.default_rng(700 + i + depth)
        pl = F.frame_planes(W, H, depth, rng)
        U = F.deblock_units(W, H, cl, depth, rng, "P")
        dp = F.deblock_params(rng, "P", 0)
        prm = F.sao_params(W, H, cl, depth, rng)
        # oracle: whole frame
        dbk = F.copy_planes(pl)
        O.deblock(W, H, cl, dbk, M, U, dp)
        ref = F.copy_planes(dbk)
        O.sao_apply(W, H, cl, ref, M, prm, 1, 1)
        for p in range(3):
            O.extend_border(ref[p], M, M, W if p == 0 else W // 2, H if p == 0 else H // 2)
        # GPU: row bands
        d = _dev(pl)
        out = _dev(tuple(np.zeros_like(p) for p in pl))
        du = torch.from_numpy(U.view(np.uint8).reshape(U.shape[0], -1)).cuda()
        dprm = torch.from_numpy(prm.view(np.uint8)).cuda()
        fr = DeblockFrame()
        fr.width, fr.height = W, H
        for p in range(3):
            fr.plane[p] = _org(d[p])
        fr.stride, fr.cstride = d[0].shape[1], d[1].shape[1]
        fr.units, fr.unit_stride = du.data_ptr(), U.shape[1]
        fr.is_p, fr.beta_offset_div2, fr.tc_offset_div2 = dp.is_p, dp.beta_offset_div2, dp.tc_offset_div2
        fr.cb_qp_offset, fr.cr_qp_offset = dp.cb_qp_offset, dp.cr_qp_offset
        for lst in range(2):
            for k in range(16):
                fr.ref_poc[lst][k] = dp.ref_poc[lst][k]
        sf = SaoFrame()
        sf.width, sf.height, sf.ctu_log2, sf.luma_on, sf.chroma_on = W, H, cl, 1, 1
        for p in range(3):
            sf.src[p], sf.dst[p] = _org(d[p]), _org(out[p])
        sf.stride, sf.cstride, sf.params = d[0].shape[1], d[1].shape[1], dprm.data_ptr()
        bps = []
        for p in range(3):
            bp = BorderPlane()
            bp.plane, bp.stride = _org(out[p]), out[p].shape[1]
            bp.width, bp.height = (W, H) if p == 0 else (W // 2, H // 2)
            bp.margin_x = bp.margin_y = M
            bps.append(bp)
        ctu = 1 << cl
        rows = (H + ctu - 1) // ctu

        def finish(b):
            gpu_prims.sao_apply_rows(depth, [sf], [b, b + 1])
            y0, y1 = b * ctu, min((b + 1) * ctu, H)
            gpu_prims.extend_border_rows(depth, bps, [y0, y1, b == 0, b == rows - 1] +
                                         [y0 // 2, y1 // 2, b == 0, b == rows - 1] * 2)

        for b in range(rows):
            gpu_prims.deblock_rows(depth, [fr], [b * ctu, min((b + 1) * ctu, H)])
            if b:
                finish(b - 1)
        finish(rows - 1)
        torch.cuda.synchronize()
        for p in range(3):
            np.testing.assert_array_equal(_host(out[p], pl[p].dtype), ref[p], err_msg=f"{W}x{H} plane {p}")


@pytest.mark.gpu
@pytest.mark.parametrize("csp", [2, 3])
@pytest.mark.parametrize("depth", DEPTHS)
def test_gpu_f4_chroma_formats(gpu_prims, csp, depth):
    """4:2:2 / 4:4:4 (chroma_format 2 / 3): deblocking, SAO apply and SAO statistics of the
    gfx950 kernels equal the oracle (itself equal to the reference's classes on the CPU)."""
    import torch
    from src.x265_amd.native import DeblockFrame, SaoFrame, SaoStatsFrame

    O = po.FrameFilters("oracle", depth)
    for i, (W, H, cl) in enumerate(GPU_SIZES):
        rng = np.random.default_rng(500 + 10 * i + depth + csp)
        pl = F.frame_planes(W, H, depth, rng, csp=csp)
        # deblocking (B slice, lossless CUs on)
        U = F.deblock_units(W, H, cl, depth, rng, "B", 0.2)
        dp = F.deblock_params(rng, "B", 1)
        ref = F.copy_planes(pl)
        O.deblock(W, H, cl, ref, F.MARGIN, U, dp, csp=csp)
        d = _dev(pl)
        du = torch.from_numpy(U.view(np.uint8).reshape(U.shape[0], -1)).cuda()
        fr = DeblockFrame()
        fr.width, fr.height, fr.chroma_format = W, H, csp
        for p in range(3):
            fr.plane[p] = _org(d[p])
        fr.stride, fr.cstride = d[0].shape[1], d[1].shape[1]
        fr.units, fr.unit_stride = du.data_ptr(), U.shape[1]
        fr.is_p, fr.beta_offset_div2, fr.tc_offset_div2 = dp.is_p, dp.beta_offset_div2, dp.tc_offset_div2
        fr.cb_qp_offset, fr.cr_qp_offset, fr.tq_bypass_enabled = dp.cb_qp_offset, dp.cr_qp_offset, 1
        for lst in range(2):
            for k in range(16):
                fr.ref_poc[lst][k] = dp.ref_poc[lst][k]
        gpu_prims.deblock(depth, [fr])
        # SAO apply on the deblocked picture
        prm = F.sao_params(W, H, cl, depth, rng)
        sref = F.copy_planes(ref)
        O.sao_apply(W, H, cl, sref, F.MARGIN, prm, 1, 1, csp=csp)
        out = _dev(tuple(np.zeros_like(p) for p in pl))
        dprm = torch.from_numpy(prm.view(np.uint8)).cuda()
        sf = SaoFrame()
        sf.width, sf.height, sf.ctu_log2, sf.luma_on, sf.chroma_on, sf.chroma_format = W, H, cl, 1, 1, csp
        for p in range(3):
            sf.src[p], sf.dst[p] = _org(d[p]), _org(out[p])
        sf.stride, sf.cstride, sf.params = d[0].shape[1], d[1].shape[1], dprm.data_ptr()
        gpu_prims.sao_apply(depth, [sf])
        # SAO statistics of a source against the deblocked picture
        fenc = F.frame_planes(W, H, depth, rng, csp=csp)
        s_ref, c_ref = O.sao_stats(W, H, cl, fenc, ref, F.MARGIN, 0, csp=csp)
        df = _dev(fenc)
        st = torch.full(s_ref.shape, -7, dtype=torch.int32, device="cuda")
        ct = torch.full(c_ref.shape, -7, dtype=torch.int32, device="cuda")
        tf = SaoStatsFrame()
        tf.width, tf.height, tf.ctu_log2, tf.non_deblocked, tf.chroma_format = W, H, cl, 0, csp
        for p in range(3):
            tf.fenc[p], tf.rec[p] = _org(df[p]), _org(d[p])
        tf.fenc_stride, tf.fenc_cstride = df[0].shape[1], df[1].shape[1]
        tf.rec_stride, tf.rec_cstride = d[0].shape[1], d[1].shape[1]
        tf.stats, tf.count = st.data_ptr(), ct.data_ptr()
        gpu_prims.sao_stats(depth, [tf])
        torch.cuda.synchronize()
        M = F.MARGIN
        for p in range(3):
            np.testing.assert_array_equal(_host(d[p], pl[p].dtype), ref[p], err_msg=f"deblock {W}x{H} p{p}")
            np.testing.assert_array_equal(_host(out[p], pl[p].dtype)[M:-M, M:-M], sref[p][M:-M, M:-M],
                                          err_msg=f"sao {W}x{H} p{p}")
        np.testing.assert_array_equal(ct.cpu().numpy(), c_ref)
        np.testing.assert_array_equal(st.cpu().numpy(), s_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_loop_filters_luma_only_i400(gpu_prims, depth):
    """X265AMD_CSP_I400 (x265's X265_CSP_I400 pictures: deblock.cpp:443 and sao.cpp skip chroma): the
    chroma planes may be NULL and are never touched; the luma result equals the 4:2:0 run's luma"""
    import torch
    from src.x265_amd.native import DeblockFrame, SaoFrame

    W, H, cl = GPU_SIZES[0]
    rng = np.random.default_rng(7 + depth)
    pl = F.frame_planes(W, H, depth, rng)
    U = F.deblock_units(W, H, cl, depth, rng, "P", 0.0)
    dp = F.deblock_params(rng, "P", 0)
    du = torch.from_numpy(U.view(np.uint8).reshape(U.shape[0], -1)).cuda()
    outs = []
    for csp in (1, 4):
        d = _dev(F.copy_planes(pl))
        fr = DeblockFrame()
        fr.width, fr.height, fr.chroma_format = W, H, csp
        fr.plane[0] = _org(d[0])
        if csp != 4:
            fr.plane[1], fr.plane[2] = _org(d[1]), _org(d[2])
        fr.stride, fr.cstride = d[0].shape[1], d[1].shape[1]
        fr.units, fr.unit_stride = du.data_ptr(), U.shape[1]
        fr.is_p, fr.beta_offset_div2, fr.tc_offset_div2 = dp.is_p, dp.beta_offset_div2, dp.tc_offset_div2
        gpu_prims.deblock(depth, [fr])
        torch.cuda.synchronize()
        outs.append([t.cpu().numpy() for t in d])
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[1][1], _dev(pl)[1].cpu().numpy())     # chroma untouched
    # SAO apply, luma only, NULL chroma planes: luma equals the 4:2:0 run's luma
    prm = F.sao_params(W, H, cl, depth, rng)
    dprm = torch.from_numpy(np.ascontiguousarray(prm).view(np.uint8).reshape(-1).copy()).cuda()
    res = []
    for csp in (1, 4):
        src, dst = _dev(F.copy_planes(pl)), _dev(F.copy_planes(pl))
        sf = SaoFrame()
        sf.width, sf.height, sf.ctu_log2, sf.luma_on, sf.chroma_on, sf.chroma_format = W, H, cl, 1, 1, csp
        sf.src[0], sf.dst[0] = _org(src[0]), _org(dst[0])
        if csp != 4:
            sf.src[1], sf.dst[1], sf.src[2], sf.dst[2] = _org(src[1]), _org(dst[1]), _org(src[2]), _org(dst[2])
        sf.stride, sf.cstride, sf.params = src[0].shape[1], src[1].shape[1], dprm.data_ptr()
        gpu_prims.sao_apply(depth, [sf])
        torch.cuda.synchronize()
        res.append(dst[0].cpu().numpy())
    np.testing.assert_array_equal(res[0], res[1])
