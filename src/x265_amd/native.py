"""ctypes binding of libx265amd.so (include/x265_amd.h) for torch device tensors.

This is host plumbing only: torch provides device memory and the stream; all
arithmetic runs in the hand-written gfx950 kernels of csrc/.  There is no CPU
fallback — if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("X265AMD_LIB") or os.path.join(HERE, "libx265amd.so")   # override: A/B tuning builds

_vp, _ip, _int = C.c_void_p, C.c_ssize_t, C.c_int


class X265AmdError(RuntimeError):
    pass


# descriptors of the grouped entry points (include/x265_amd.h)
class CmpBatch(C.Structure):
    _fields_ = [("w", _int), ("h", _int), ("n", _int), ("a", _vp), ("a_stride", _ip), ("a_off", _vp),
                ("b", _vp), ("b_stride", _ip), ("b_off", _vp), ("out", _vp)]


class BlockBatch(C.Structure):
    _fields_ = [("w", _int), ("h", _int), ("n", _int), ("param", _int), ("dst", _vp), ("dst_stride", _ip),
                ("dst_off", _vp), ("a", _vp), ("a_stride", _ip), ("a_off", _vp), ("b", _vp), ("b_stride", _ip),
                ("b_off", _vp)]


class InterpBatch(C.Structure):
    _fields_ = [("w", _int), ("h", _int), ("n", _int), ("is_row_ext", _int), ("src", _vp), ("src_stride", _ip),
                ("src_off", _vp), ("dst", _vp), ("dst_stride", _ip), ("dst_off", _vp), ("coeff", _vp)]


class TuBatch(C.Structure):
    _fields_ = [("log2_size", _int), ("n", _int), ("is_luma", _int), ("is_intra", _int), ("i_slice", _int),
                ("sign_hide", _int), ("fenc", _vp), ("fenc_stride", _ip), ("fenc_off", _vp), ("pred", _vp),
                ("pred_stride", _ip), ("pred_off", _vp), ("resi", _vp), ("resi_stride", _ip), ("resi_off", _vp),
                ("coeff", _vp), ("coeff_off", _vp), ("recon", _vp), ("recon_stride", _ip), ("recon_off", _vp),
                ("num_sig", _vp), ("qp", _vp), ("scan", _vp)]


class LowresBatch(C.Structure):
    _fields_ = [("n", _int), ("width", _int), ("lines", _int), ("margin_x", _int), ("margin_y", _int),
                ("src", _vp), ("src_stride", _ip), ("src_off", _vp), ("planes", _vp), ("lowres_stride", _ip),
                ("plane_off", _vp)]


class LowresIntraBatch(C.Structure):
    _fields_ = [("n", _int), ("width_cu", _int), ("height_cu", _int), ("planes", _vp), ("lowres_stride", _ip),
                ("plane_off", _vp), ("inv_qscale", _vp), ("intra_cost", _vp), ("intra_mode", _vp),
                ("lowres_cost", _vp), ("row_satd", _vp), ("cost_est", _vp)]


class LowresPcostBatch(C.Structure):
    _fields_ = [("n", _int), ("width_cu", _int), ("height_cu", _int), ("rows_per_slice", _int), ("num_slices", _int),
                ("planes", _vp), ("lowres_stride", _ip), ("fenc_off", _vp), ("ref_off", _vp), ("intra_cost", _vp),
                ("inv_qscale", _vp), ("mvcost", _vp), ("mvs", _vp), ("mv_costs", _vp), ("lowres_costs", _vp),
                ("row_satd", _vp), ("cost_est", _vp), ("intra_mbs", _vp)]


class LowresBcostBatch(C.Structure):
    _fields_ = [("n", _int), ("width_cu", _int), ("height_cu", _int), ("rows_per_slice", _int), ("num_slices", _int),
                ("planes", _vp), ("lowres_stride", _ip), ("fenc_off", _vp), ("ref0_off", _vp), ("ref1_off", _vp),
                ("do_search", _vp), ("inv_qscale", _vp), ("mvcost", _vp), ("mvs0", _vp), ("mv_costs0", _vp),
                ("mvs1", _vp), ("mv_costs1", _vp), ("lowres_costs", _vp), ("row_satd", _vp), ("cost_est", _vp)]


class MeBatch(C.Structure):
    _fields_ = [("w", _int), ("h", _int), ("n", _int), ("method", _int), ("subme", _int), ("merange", _int),
                ("max_cand", _int), ("fenc", _vp), ("fenc_stride", _ip), ("fenc_off", _vp), ("ref", _vp),
                ("ref_stride", _ip), ("ref_off", _vp), ("mv_range", _vp), ("mvp", _vp), ("mvc", _vp), ("num_cand", _vp),
                ("mvcost", _vp), ("mvcost_off", _vp), ("out_mv", _vp), ("out_cost", _vp), ("fenc_cb", _vp),
                ("fenc_cr", _vp), ("fenc_cstride", _ip), ("fenc_coff", _vp), ("ref_cb", _vp), ("ref_cr", _vp),
                ("ref_cstride", _ip), ("ref_coff", _vp), ("eval_count", _vp)]


# f4 frame descriptors (include/x265_amd.h): device addresses of the plane origins
_i64 = C.c_int64


class SaoFrame(C.Structure):
    _fields_ = [("width", _int), ("height", _int), ("ctu_log2", _int), ("luma_on", _int), ("chroma_on", _int),
                ("src", _vp * 3), ("dst", _vp * 3), ("stride", _i64), ("cstride", _i64), ("params", _vp),
                ("chroma_format", _int)]


class SaoStatsFrame(C.Structure):
    _fields_ = [("width", _int), ("height", _int), ("ctu_log2", _int), ("non_deblocked", _int), ("fenc", _vp * 3),
                ("fenc_stride", _i64), ("fenc_cstride", _i64), ("rec", _vp * 3), ("rec_stride", _i64),
                ("rec_cstride", _i64), ("stats", _vp), ("count", _vp), ("chroma_format", _int)]


class DeblockFrame(C.Structure):
    _fields_ = [("width", _int), ("height", _int), ("plane", _vp * 3), ("stride", _i64), ("cstride", _i64),
                ("units", _vp), ("unit_stride", _i64), ("is_p", _int), ("beta_offset_div2", _int),
                ("tc_offset_div2", _int), ("cb_qp_offset", _int), ("cr_qp_offset", _int), ("tq_bypass_enabled", _int),
                ("ref_poc", (C.c_int32 * 16) * 2), ("chroma_format", _int)]


class PropagateBatch(C.Structure):
    _fields_ = [("width_cu", _int), ("height_cu", _int), ("propagate_in", _vp), ("intra_cost", _vp),
                ("lowres_costs", _vp), ("inv_qscale", _vp), ("mvs", _vp * 2), ("fps_factor", C.c_double),
                ("bipred_weight", _int * 2), ("ref_costs", _vp * 2), ("scratch", _vp)]


class WeightsBatch(C.Structure):
    _fields_ = [("width", _int), ("lines", _int), ("stride", _i64), ("padded_lines", _int), ("pad_offset", _i64),
                ("fenc_plane", _vp), ("ref_buf", _vp * 4), ("intra_cost", _vp), ("wbuf", _vp * 4),
                ("scratch", _vp), ("fenc_ssd", C.c_uint64), ("ref_ssd", C.c_uint64), ("fenc_sum", C.c_uint64),
                ("ref_sum", C.c_uint64), ("weighted", _int), ("scale", _int), ("denom", _int), ("offset", _int),
                ("cost_delta", C.c_double)]


class BorderPlane(C.Structure):
    _fields_ = [("plane", _vp), ("stride", _i64), ("width", _int), ("height", _int), ("margin_x", _int),
                ("margin_y", _int)]



class capture_graph:
    """torch.cuda.graph(g) with Python's cyclic GC held off for the capture.

    A dead reference cycle that owns CUDA graphs or tensors (e.g. a discarded
    GpuFramePipeline, whose lambdas reference itself) must not be collected while a
    stream is capturing: freeing a graph's private pool there calls hipFree inside
    the capture and aborts the process.  Collect first, then capture with GC off."""

    def __init__(self, g, pool=None):
        import torch

        # pool: another graph's pool() (or torch.cuda.graph_pool_handle()), so graphs that hand tensors to
        # each other allocate from ONE private pool and none of them can release memory another still reads
        self._ctx = torch.cuda.graph(g, pool=pool)

    def __enter__(self):
        import gc

        gc.collect()
        self._was = gc.isenabled()
        gc.disable()
        return self._ctx.__enter__()

    def __exit__(self, *exc):
        import gc

        try:
            return self._ctx.__exit__(*exc)
        finally:
            if self._was:
                gc.enable()

def _addr(t):
    return None if t is None else t.data_ptr()


def cmp_batches(items):
    """items: (w, h, a, sa, aoff, b, sb, boff, out) with torch tensors -> CmpBatch array"""
    arr = (CmpBatch * len(items))()
    for i, (w, h, a, sa, aoff, b, sb, boff, out) in enumerate(items):
        arr[i] = CmpBatch(w, h, aoff.numel(), _addr(a), sa, _addr(aoff), _addr(b), sb, _addr(boff), _addr(out))
    return arr


def block_batches(items):
    """items: (w, h, param, d, ds, doff, a, sa, aoff, b, sb, boff) -> BlockBatch array"""
    arr = (BlockBatch * len(items))()
    for i, (w, h, param, d, ds, doff, a, sa, aoff, b, sb, boff) in enumerate(items):
        arr[i] = BlockBatch(w, h, doff.numel(), int(param), _addr(d), ds, _addr(doff), _addr(a), sa, _addr(aoff),
                            _addr(b), sb, _addr(boff))
    return arr


def interp_batches(items):
    """items: (w, h, rowext, s, ss, soff, d, ds, doff, coeff) -> InterpBatch array"""
    arr = (InterpBatch * len(items))()
    for i, (w, h, rowext, s, ss, soff, d, ds, doff, coeff) in enumerate(items):
        arr[i] = InterpBatch(w, h, soff.numel(), int(rowext), _addr(s), ss, _addr(soff), _addr(d), ds, _addr(doff),
                             _addr(coeff))
    return arr


def _ptr(t):
    if t is None:
        return None
    return _vp(t.data_ptr())


def _stream():
    import torch

    return _vp(torch.cuda.current_stream().cuda_stream)


class Primitives:
    """Batched primitive calls on torch tensors (all tensors on the current device)."""

    _lib = None

    def __init__(self, device: int | None = None):
        if Primitives._lib is None:
            if not os.path.exists(LIB_PATH):
                raise X265AmdError(f"{LIB_PATH} not built: run __graft_entry__.build()")
            lib = C.CDLL(LIB_PATH)
            lib.x265amd_strerror.restype = C.c_char_p
            lib.x265amd_target.restype = C.c_char_p
            Primitives._lib = lib
        self.lib = Primitives._lib
        if device is not None:
            self._check(self.lib.x265amd_set_device(int(device)), "set_device")

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise X265AmdError(f"x265amd_{what}: {self.lib.x265amd_strerror(rc).decode()} (status {rc})")

    # -- a4 a6 a7 a8 a15
    def pixelcmp(self, op, depth, w, h, a, sa, aoff, b, sb, boff, out, stream=None):
        n = aoff.numel()
        self._check(self.lib.x265amd_pixelcmp(op, depth, w, h, n, _ptr(a), _ip(sa), _ptr(aoff), _ptr(b), _ip(sb),
                                              _ptr(boff), _ptr(out), stream or _stream()), "pixelcmp")

    # -- a5
    def sad_multi(self, nref, depth, w, h, f, fs, foff, r, rs, roff, out, stream=None):
        n = foff.numel()
        self._check(self.lib.x265amd_sad_multi(nref, depth, w, h, n, _ptr(f), _ip(fs), _ptr(foff), _ptr(r), _ip(rs),
                                               _ptr(roff), _ptr(out), stream or _stream()), "sad_multi")

    # -- a9
    def interp(self, op, taps, depth, w, h, s, ss, soff, d, ds, doff, coeff, rowext=0, stream=None):
        n = soff.numel()
        self._check(self.lib.x265amd_interp(op, taps, depth, w, h, n, _ptr(s), _ip(ss), _ptr(soff), _ptr(d), _ip(ds),
                                            _ptr(doff), _ptr(coeff), rowext, stream or _stream()), "interp")

    # -- a10 a11
    def transform(self, kind, depth, size, s, ss, soff, d, ds, doff, stream=None):
        n = soff.numel()
        self._check(self.lib.x265amd_transform(kind, depth, size, n, _ptr(s), _ip(ss), _ptr(soff), _ptr(d), _ip(ds),
                                               _ptr(doff), stream or _stream()), "transform")

    # -- a12 a13
    def quant(self, num, c, co, q, qo, dl, dlo, o, oo, qb, ad, sig, stream=None):
        n = co.numel()
        self._check(self.lib.x265amd_quant(n, num, _ptr(c), _ptr(co), _ptr(q), _ptr(qo), _ptr(dl), _ptr(dlo), _ptr(o),
                                           _ptr(oo), _ptr(qb), _ptr(ad), _ptr(sig), stream or _stream()), "quant")

    def dequant_normal(self, num, q, qo, o, oo, scale, shift, stream=None):
        n = qo.numel()
        self._check(self.lib.x265amd_dequant_normal(n, num, _ptr(q), _ptr(qo), _ptr(o), _ptr(oo), _ptr(scale),
                                                    _ptr(shift), stream or _stream()), "dequant_normal")

    def dequant_scaling(self, num, q, qo, dq, dqo, o, oo, per, shift, stream=None):
        n = qo.numel()
        self._check(self.lib.x265amd_dequant_scaling(n, num, _ptr(q), _ptr(qo), _ptr(dq), _ptr(dqo), _ptr(o),
                                                     _ptr(oo), _ptr(per), _ptr(shift), stream or _stream()),
                    "dequant_scaling")

    # -- a14
    def intra_filter(self, depth, size, s, soff, d, doff, stream=None):
        self._check(self.lib.x265amd_intra_filter(depth, size, soff.numel(), _ptr(s), _ptr(soff), _ptr(d), _ptr(doff),
                                                  stream or _stream()), "intra_filter")

    def intra_pred(self, depth, size, d, ds, doff, nb, nboff, mode, bfilter, stream=None):
        self._check(self.lib.x265amd_intra_pred(depth, size, doff.numel(), _ptr(d), _ip(ds), _ptr(doff), _ptr(nb),
                                                _ptr(nboff), _ptr(mode), _ptr(bfilter), stream or _stream()),
                    "intra_pred")

    def intra_allangs(self, depth, size, d, doff, ref, roff, filt, foff, bluma, stream=None):
        self._check(self.lib.x265amd_intra_allangs(depth, size, doff.numel(), _ptr(d), _ptr(doff), _ptr(ref),
                                                   _ptr(roff), _ptr(filt), _ptr(foff), _ptr(bluma),
                                                   stream or _stream()), "intra_allangs")

    # -- a15
    def blockop(self, op, depth, w, h, d, ds, doff, a, sa, aoff, b, sb, boff, param=0, stream=None):
        self._check(self.lib.x265amd_blockop(op, depth, w, h, doff.numel(), _ptr(d), _ip(ds), _ptr(doff), _ptr(a),
                                             _ip(sa), _ptr(aoff), _ptr(b), _ip(sb), _ptr(boff), int(param),
                                             stream or _stream()), "blockop")

    # -- grouped forms: `arr` from cmp_batches / block_batches / interp_batches
    def pixelcmp_grouped(self, op, depth, arr, stream=None):
        self._check(self.lib.x265amd_pixelcmp_grouped(op, depth, len(arr), arr, stream or _stream()),
                    "pixelcmp_grouped")

    def sad_multi_grouped(self, nref, depth, arr, stream=None):
        self._check(self.lib.x265amd_sad_multi_grouped(nref, depth, len(arr), arr, stream or _stream()),
                    "sad_multi_grouped")

    def blockop_grouped(self, op, depth, arr, stream=None):
        self._check(self.lib.x265amd_blockop_grouped(op, depth, len(arr), arr, stream or _stream()),
                    "blockop_grouped")

    def interp_grouped(self, op, taps, depth, arr, stream=None):
        self._check(self.lib.x265amd_interp_grouped(op, taps, depth, len(arr), arr, stream or _stream()),
                    "interp_grouped")

    def denoise_dct(self, num, c, co, rsum, offset, stream=None):
        self._check(self.lib.x265amd_denoise_dct(co.numel(), num, _ptr(c), _ptr(co), _ptr(rsum), _ptr(offset),
                                                 stream or _stream()), "denoise_dct")

    def count_nonzero(self, size, c, co, r, rs, ro, cnt, stream=None):
        self._check(self.lib.x265amd_count_nonzero(size, co.numel(), _ptr(c), _ptr(co), _ptr(r), _ip(rs), _ptr(ro),
                                                   _ptr(cnt), stream or _stream()), "count_nonzero")

    # -- f3 fused TU pipeline: one TuBatch per call (or an array from tu_batches)
    def tu_pipeline(self, depth, log2, luma, intra, islice, sh, f, fs, fo, p, ps, po, r, rs, ro, c, co, rc, rcs, rco,
                    sig, qp, scan, stream=None):
        arr = (TuBatch * 1)()
        arr[0] = TuBatch(log2, fo.numel(), int(luma), int(intra), int(islice), int(sh), _addr(f), fs, _addr(fo),
                         _addr(p), ps, _addr(po), _addr(r), rs, _addr(ro), _addr(c), _addr(co), _addr(rc), rcs,
                         _addr(rco), _addr(sig), _addr(qp), _addr(scan))
        self.tu_pipeline_grouped(depth, arr, stream)

    def tu_pipeline_grouped(self, depth, arr, stream=None):
        self._check(self.lib.x265amd_tu_pipeline(depth, len(arr), arr, stream or _stream()), "tu_pipeline")

    # -- f1 lookahead lowres pipeline
    def lowres_init(self, depth, n, width, lines, mx, my, src, ss, so, planes, ls, po, stream=None):
        b = LowresBatch(n, width, lines, mx, my, _addr(src), ss, _addr(so), _addr(planes), ls, _addr(po))
        self._check(self.lib.x265amd_lowres_init(depth, C.byref(b), stream or _stream()), "lowres_init")

    def lowres_intra(self, depth, n, wcu, hcu, planes, ls, p0, inv_q, ic, im, lc, rs, ce, stream=None):
        b = LowresIntraBatch(n, wcu, hcu, _addr(planes), ls, _addr(p0), _addr(inv_q), _addr(ic), _addr(im), _addr(lc),
                             _addr(rs), _addr(ce))
        self._check(self.lib.x265amd_lowres_intra(depth, C.byref(b), stream or _stream()), "lowres_intra")

    def lowres_pcost(self, depth, n, wcu, hcu, rps, ns, planes, ls, fo, ro, ic, iq, tab_centre_ptr, mvs, mc, lc, rs, ce,
                     mbs, stream=None):
        b = LowresPcostBatch(n, wcu, hcu, rps, ns, _addr(planes), ls, _addr(fo), _addr(ro), _addr(ic), _addr(iq),
                             tab_centre_ptr, _addr(mvs), _addr(mc), _addr(lc), _addr(rs), _addr(ce), _addr(mbs))
        self._check(self.lib.x265amd_lowres_pcost(depth, C.byref(b), stream or _stream()), "lowres_pcost")

    def lowres_bcost(self, depth, n, wcu, hcu, rps, ns, planes, ls, fo, r0o, r1o, ds, iq, tab_centre_ptr, mvs0, mc0,
                     mvs1, mc1, lc, rs, ce, stream=None):
        b = LowresBcostBatch(n, wcu, hcu, rps, ns, _addr(planes), ls, _addr(fo), _addr(r0o), _addr(r1o), _addr(ds),
                             _addr(iq), tab_centre_ptr, _addr(mvs0), _addr(mc0), _addr(mvs1), _addr(mc1), _addr(lc),
                             _addr(rs), _addr(ce))
        self._check(self.lib.x265amd_lowres_bcost(depth, C.byref(b), stream or _stream()), "lowres_bcost")

    # -- f2 full-resolution motion search
    def motion_search(self, depth, w, h, method, subme, merange, max_cand, f, fs, fo, r, rs, ro, rng, mvp, mvc, numc,
                      tab, tab_off, out_mv, out_cost, fcb=None, fcr=None, fcs=0, fco=None, rcb=None, rcr=None, rcs=0,
                      rco=None, stream=None):
        arr = (MeBatch * 1)()
        arr[0] = MeBatch(w, h, fo.numel(), method, subme, merange, max_cand, _addr(f), fs, _addr(fo), _addr(r), rs,
                         _addr(ro), _addr(rng), _addr(mvp), _addr(mvc), _addr(numc), _addr(tab), _addr(tab_off),
                         _addr(out_mv), _addr(out_cost), _addr(fcb), _addr(fcr), fcs, _addr(fco), _addr(rcb),
                         _addr(rcr), rcs, _addr(rco))
        self._check(self.lib.x265amd_motion_search(depth, 1, arr, stream or _stream()), "motion_search")

    def motion_search_multi(self, depth, jobs, stream=None):
        """several batches (one per PU size) in ONE call: they run concurrently on the library's
        internal streams, joined back into `stream`.  jobs: dicts of motion_search's arguments."""
        arr = (MeBatch * len(jobs))()
        for i, j in enumerate(jobs):
            arr[i] = MeBatch(j["w"], j["h"], j["fo"].numel(), j["method"], j["subme"], j["merange"], j["max_cand"],
                             _addr(j["f"]), j["fs"], _addr(j["fo"]), _addr(j["r"]), j["rs"], _addr(j["ro"]),
                             _addr(j["rng"]), _addr(j["mvp"]), _addr(j["mvc"]), _addr(j["numc"]), _addr(j["tab"]),
                             _addr(j["tab_off"]), _addr(j["out_mv"]), _addr(j["out_cost"]), None, None, 0, None, None,
                             None, 0, None)
        self._check(self.lib.x265amd_motion_search(depth, len(jobs), arr, stream or _stream()), "motion_search")

    # -- f4 loop filters and border extension (frame descriptors: SaoFrame, SaoStatsFrame,
    #    DeblockFrame, BorderPlane with device addresses)
    def _frames(self, entry, what, depth, frames, stream):
        arr = (type(frames[0]) * len(frames))(*frames)
        self._check(getattr(self.lib, entry)(depth, len(frames), arr, stream or _stream()), what)

    def sao_apply(self, depth, frames, stream=None):
        self._frames("x265amd_sao_apply", "sao_apply", depth, frames, stream)

    def sao_stats(self, depth, frames, stream=None):
        self._frames("x265amd_sao_stats", "sao_stats", depth, frames, stream)

    def deblock(self, depth, frames, stream=None):
        self._frames("x265amd_deblock", "deblock", depth, frames, stream)

    def extend_border(self, depth, planes, stream=None):
        self._frames("x265amd_extend_border", "extend_border", depth, planes, stream)

    # -- f1 cuTree propagation (x265amd_cutree_propagate): one estimateCUPropagate per dict, in order
    def cutree_propagate(self, jobs, stream=None):
        arr = (PropagateBatch * len(jobs))()
        for i, j in enumerate(jobs):
            b = arr[i]
            b.width_cu, b.height_cu = j["wcu"], j["hcu"]
            b.propagate_in, b.intra_cost = _addr(j["prop"]), _addr(j["intra"])
            b.lowres_costs, b.inv_qscale = _addr(j["lowres"]), _addr(j["invq"])
            b.mvs[0], b.mvs[1] = _addr(j["mvs"][0]), _addr(j["mvs"][1])
            b.fps_factor = float(j["fps_factor"])
            b.bipred_weight[0], b.bipred_weight[1] = int(j["weights"][0]), int(j["weights"][1])
            b.ref_costs[0], b.ref_costs[1] = _addr(j["refs"][0]), _addr(j["refs"][1])
            b.scratch = _addr(j["scratch"])
        self._check(self.lib.x265amd_cutree_propagate(len(jobs), arr, stream or _stream()), "cutree_propagate")

    # -- f1 weightp (x265amd_weights_analyse): synchronous on the stream
    def weights_analyse(self, depth, width, lines, stride, padded_lines, pad_offset, fenc_buf, ref_buf, intra, wbuf,
                        fenc_ssd, ref_ssd, fenc_sum, ref_sum, stream=None):
        """fenc_buf / ref_buf / wbuf: device tensors holding 4 contiguous padded lowres planes
        (Lowres::create); returns the decision dict"""
        import torch

        b = WeightsBatch()
        b.width, b.lines, b.stride, b.padded_lines, b.pad_offset = width, lines, stride, padded_lines, pad_offset
        es = ref_buf.element_size()
        ps = stride * padded_lines
        b.fenc_plane = fenc_buf.data_ptr() + pad_offset * es
        for i in range(4):
            b.ref_buf[i] = ref_buf.data_ptr() + i * ps * es
            b.wbuf[i] = wbuf.data_ptr() + i * ps * es
        b.intra_cost = intra.data_ptr()
        scratch = torch.zeros(1, dtype=torch.int32, device=ref_buf.device)
        b.scratch = scratch.data_ptr()
        b.fenc_ssd, b.ref_ssd, b.fenc_sum, b.ref_sum = int(fenc_ssd), int(ref_ssd), int(fenc_sum), int(ref_sum)
        self._check(self.lib.x265amd_weights_analyse(depth, C.byref(b), stream or _stream()), "weights_analyse")
        return {"weighted": b.weighted, "scale": b.scale, "denom": b.denom, "offset": b.offset,
                "cost_delta": b.cost_delta}

    # row-band forms (the frame-parallel pipeline): rows is a flat list of ints per frame / plane
    def _rows(self, entry, what, depth, frames, rows, per, stream):
        if len(rows) != per * len(frames):
            raise ValueError(f"{what}: {per} row values per frame expected")
        arr = (type(frames[0]) * len(frames))(*frames)
        r = (C.c_int32 * len(rows))(*rows)
        self._check(getattr(self.lib, entry)(depth, len(frames), arr, r, stream or _stream()), what)

    def deblock_rows(self, depth, frames, rows, stream=None):
        self._rows("x265amd_deblock_rows", "deblock_rows", depth, frames, rows, 2, stream)

    def sao_apply_rows(self, depth, frames, ctu_rows, stream=None):
        self._rows("x265amd_sao_apply_rows", "sao_apply_rows", depth, frames, ctu_rows, 2, stream)

    def extend_border_rows(self, depth, planes, rows, stream=None):
        self._rows("x265amd_extend_border_rows", "extend_border_rows", depth, planes, rows, 4, stream)
