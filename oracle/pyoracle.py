"""ctypes front-end of oracle/_build/libcpubatch.so — TEST INFRASTRUCTURE ONLY.

Runs the batch descriptors of the GPU C ABI (include/x265_amd.h) on the CPU
through one of the per-call oracle libraries:

    CpuOracle("oracle", depth)  -> oracle/_build/liboracle{8,10}.so  (restatement)
    CpuOracle("ref", depth)     -> oracle/_ref/libx265ref{8,10}.so   (reference C)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# X265AMD_ORACLE_DIR=_build_asan selects the ASan/UBSan build (oracle/Makefile asan)
BUILD = os.environ.get("X265AMD_ORACLE_DIR", "_build")

_vp, _i64, _ip = C.c_void_p, C.c_int64, C.c_ssize_t


def lib_path(kind: str, depth: int) -> str:
    d = 8 if depth == 8 else 10
    if kind == "oracle":
        return os.path.join(HERE, BUILD, f"liboracle{d}.so")
    if kind == "ref":
        return os.path.join(HERE, "_ref", f"libx265ref{d}.so")
    raise ValueError(kind)


def available(kind: str, depth: int = 8) -> bool:
    return os.path.exists(lib_path(kind, depth)) and os.path.exists(os.path.join(HERE, BUILD, "libcpubatch.so"))


def _p(a):
    return None if a is None else a.ctypes.data_as(_vp)


class CpuOracle:
    _cb = None

    def __init__(self, kind: str, depth: int):
        if CpuOracle._cb is None:
            cb = C.CDLL(os.path.join(HERE, BUILD, "libcpubatch.so"))
            cb.cb_open.restype = _vp
            cb.cb_open.argtypes = [C.c_char_p]
            CpuOracle._cb = cb
        self.kind, self.depth = kind, depth
        self.h = CpuOracle._cb.cb_open(lib_path(kind, depth).encode())
        if not self.h:
            raise RuntimeError(f"cannot open oracle library {lib_path(kind, depth)}")
        self.nthreads = 1

    @property
    def cb(self):
        return CpuOracle._cb

    # every wrapper takes numpy arrays and int64 offset arrays (element units)
    def pixelcmp(self, op, w, h, a, sa, aoff, b, sb, boff, out):
        self.cb.cb_pixelcmp(_vp(self.h), op, w, h, _i64(len(aoff)), _p(a), _ip(sa), _p(aoff), _p(b), _ip(sb),
                            _p(boff), _p(out), self.nthreads)

    def sad_multi(self, nref, w, h, f, fs, foff, r, rs, roff, out):
        rc = self.cb.cb_sad_multi(_vp(self.h), nref, w, h, _i64(len(foff)), _p(f), _ip(fs), _p(foff), _p(r), _ip(rs),
                                  _p(roff), _p(out), self.nthreads)
        if rc:
            raise ValueError("sad_multi oracle: block larger than 64x64")

    def interp(self, op, taps, w, h, s, ss, soff, d, ds, doff, coeff, rowext):
        self.cb.cb_interp(_vp(self.h), op, taps, w, h, _i64(len(soff)), _p(s), _ip(ss), _p(soff), _p(d), _ip(ds),
                          _p(doff), _p(coeff), rowext, self.nthreads)

    def transform(self, kind, size, s, ss, soff, d, ds, doff):
        self.cb.cb_transform(_vp(self.h), kind, size, _i64(len(soff)), _p(s), _ip(ss), _p(soff), _p(d), _ip(ds),
                             _p(doff), self.nthreads)

    def quant(self, num, c, co, q, qo, dl, dlo, o, oo, qb, ad, sig):
        self.cb.cb_quant(_vp(self.h), _i64(len(co)), num, _p(c), _p(co), _p(q), _p(qo), _p(dl), _p(dlo), _p(o),
                         _p(oo), _p(qb), _p(ad), _p(sig), self.nthreads)

    def dequant(self, scaling, num, q, qo, dq, dqo, o, oo, p0, p1):
        self.cb.cb_dequant(_vp(self.h), int(scaling), _i64(len(qo)), num, _p(q), _p(qo), _p(dq), _p(dqo), _p(o),
                           _p(oo), _p(p0), _p(p1), self.nthreads)

    def intra(self, kind, size, d, ds, doff, nb, nboff, f, foff, mode, bf):
        self.cb.cb_intra(_vp(self.h), kind, size, _i64(len(doff)), _p(d), _ip(ds), _p(doff), _p(nb), _p(nboff),
                         _p(f), _p(foff), _p(mode), _p(bf), self.nthreads)

    def blockop(self, op, w, h, d, ds, doff, a, sa, aoff, b, sb, boff, param):
        self.cb.cb_blockop(_vp(self.h), op, w, h, _i64(len(doff)), _p(d), _ip(ds), _p(doff), _p(a), _ip(sa),
                           _p(aoff), _p(b), _ip(sb), _p(boff), param, self.nthreads)

    def count_nonzero(self, size, c, co, r, rs, ro, cnt):
        self.cb.cb_count_nonzero(_vp(self.h), size, _i64(len(co)), _p(c), _p(co), _p(r), _ip(rs), _p(ro),
                                 _p(cnt), self.nthreads)

    def denoise(self, num, c, co, rsum, offset):
        self.cb.cb_denoise(_vp(self.h), _i64(len(co)), num, _p(c), _p(co), _p(rsum), _p(offset))


    def tu(self, log2, luma, intra, islice, sh, f, fs, fo, p, ps, po, r, rs, ro, c, co, rc, rcs, rco, sig, qp, scan):
        self.cb.cb_tu(_vp(self.h), _i64(len(fo)), log2, luma, intra, islice, sh, _p(f), _ip(fs), _p(fo), _p(p), _ip(ps),
                      _p(po), _p(r), _ip(rs), _p(ro), _p(c), _p(co), _p(rc), _ip(rcs), _p(rco), _p(sig), _p(qp),
                      _p(scan), self.nthreads)

    def lowres(self, n, width, lines, mx, my, src, ss, so, planes, ls, po, wcu, hcu, inv_q, ic, im, lc, rs, ce):
        self.cb.cb_lowres(_vp(self.h), n, width, lines, mx, my, _p(src), _ip(ss), _p(so), _p(planes), _ip(ls), _p(po),
                          wcu, hcu, _p(inv_q), _p(ic), _p(im), _p(lc), _p(rs), _p(ce))

    def lowres_pcost(self, n, wcu, hcu, rps, ns, planes, ls, fo, ro, ic, iq, tab_centre_ptr, mvs, mc, lc, rs, ce, mbs):
        self.cb.cb_lowres_pcost(_vp(self.h), n, wcu, hcu, rps, ns, _p(planes), _ip(ls), _p(fo), _p(ro), _p(ic), _p(iq),
                                _vp(tab_centre_ptr), _p(mvs), _p(mc), _p(lc), _p(rs), _p(ce), _p(mbs))

    def mvcost_table(self, rng):
        out = np.zeros(2 * rng + 1, np.uint16)
        self.cb.cb_mvcost_table(_vp(self.h), rng, _p(out))
        return out

    def motion_search(self, w, h, method, subme, merange, max_cand, f, fs, fo, r, rs, ro, rng, mvp, mvc, numc, tab,
                      tab_off, qp, out_mv, out_cost, fcb=None, fcr=None, fcs=0, fco=None, rcb=None, rcr=None, rcs=0,
                      rco=None):
        self.cb.cb_motion_search(_vp(self.h), _i64(len(fo)), w, h, method, subme, merange, max_cand, _p(f), _ip(fs),
                                 _p(fo), _p(r), _ip(rs), _p(ro), _p(rng), _p(mvp), _p(mvc), _p(numc), _p(tab),
                                 _p(tab_off), _p(qp), _p(out_mv), _p(out_cost), _p(fcb), _p(fcr), _ip(fcs), _p(fco),
                                 _p(rcb), _p(rcr), _ip(rcs), _p(rco))

    def scan_table(self, typ, log2):
        out = np.zeros(1 << (2 * log2), np.uint16)
        self.cb.cb_scan_table(_vp(self.h), typ, log2, _p(out))
        return out


class CpuPrims:
    """The GPU `Primitives` call surface (src/x265_amd/native.py) executed on the
    CPU through a CpuOracle, on torch CPU tensors.  Used for bench.py's
    cpu_baseline leg (the same batch descriptors, timed on host cores) and for
    CPU-only tests of the workload plumbing.  Never a fallback for the product."""

    def __init__(self, kind: str, depth: int, nthreads: int = 1):
        self.orc = CpuOracle(kind, depth)
        self.orc.nthreads = nthreads

    @staticmethod
    def _n(t):
        return None if t is None else t.numpy()

    def pixelcmp(self, op, depth, w, h, a, sa, aoff, b, sb, boff, out, stream=None):
        n = self._n
        self.orc.pixelcmp(op, w, h, n(a), sa, n(aoff), n(b), sb, n(boff), n(out))

    def sad_multi(self, nref, depth, w, h, f, fs, foff, r, rs, roff, out, stream=None):
        n = self._n
        # cpubatch stages each fenc block into a FENC_STRIDE buffer like setSourcePU
        self.orc.sad_multi(nref, w, h, n(f), fs, n(foff), n(r), rs, n(roff), n(out))

    def interp(self, op, taps, depth, w, h, s, ss, soff, d, ds, doff, coeff, rowext=0, stream=None):
        n = self._n
        self.orc.interp(op, taps, w, h, n(s), ss, n(soff), n(d), ds, n(doff), n(coeff), rowext)

    def transform(self, kind, depth, size, s, ss, soff, d, ds, doff, stream=None):
        n = self._n
        self.orc.transform(kind, size, n(s), ss, n(soff), n(d), ds, n(doff))

    def quant(self, num, c, co, q, qo, dl, dlo, o, oo, qb, ad, sig, stream=None):
        n = self._n
        self.orc.quant(num, n(c), n(co), n(q), n(qo), n(dl), n(dlo), n(o), n(oo), n(qb), n(ad), n(sig))

    def dequant_normal(self, num, q, qo, o, oo, scale, shift, stream=None):
        n = self._n
        self.orc.dequant(0, num, n(q), n(qo), None, None, n(o), n(oo), n(scale), n(shift))

    def dequant_scaling(self, num, q, qo, dq, dqo, o, oo, per, shift, stream=None):
        n = self._n
        self.orc.dequant(1, num, n(q), n(qo), n(dq), n(dqo), n(o), n(oo), n(per), n(shift))

    def intra_filter(self, depth, size, s, soff, d, doff, stream=None):
        n = self._n
        self.orc.intra(0, size, n(d), 0, n(doff), n(s), n(soff), None, None, None, None)

    def intra_pred(self, depth, size, d, ds, doff, nb, nboff, mode, bfilter, stream=None):
        n = self._n
        self.orc.intra(1, size, n(d), ds, n(doff), n(nb), n(nboff), None, None, n(mode), n(bfilter))

    def intra_allangs(self, depth, size, d, doff, ref, roff, filt, foff, bluma, stream=None):
        n = self._n
        self.orc.intra(2, size, n(d), 0, n(doff), n(ref), n(roff), n(filt), n(foff), None, n(bluma))

    def blockop(self, op, depth, w, h, d, ds, doff, a, sa, aoff, b, sb, boff, param=0, stream=None):
        n = self._n
        self.orc.blockop(op, w, h, n(d), ds, n(doff), n(a), sa, n(aoff), n(b), sb, n(boff), param)

    def count_nonzero(self, size, c, co, r, rs, ro, cnt, stream=None):
        n = self._n
        self.orc.count_nonzero(size, n(c), n(co), n(r), rs, n(ro), n(cnt))

    def tu_pipeline(self, depth, log2, luma, intra, islice, sh, f, fs, fo, p, ps, po, r, rs, ro, c, co, rc, rcs, rco,
                    sig, qp, scan, stream=None):
        n = self._n
        self.orc.tu(log2, luma, intra, islice, sh, n(f), fs, n(fo), n(p), ps, n(po), n(r), rs, n(ro), n(c), n(co),
                    n(rc), rcs, n(rco), n(sig), n(qp), n(scan))


# ---------------------------------------------------------------- f4 loop filters (frame level)
# numpy layouts of xo_sao_param / xo_deblock_unit (x265_oracle.h) == x265amd_sao_param /
# x265amd_deblock_unit (include/x265_amd.h)
SAO_PARAM = np.dtype([("type", np.int8), ("band", np.uint8), ("offset", np.int8, 4)])
DEBLOCK_UNIT = np.dtype([("cu_log2", np.uint8), ("tu_log2", np.uint8), ("part", np.uint8), ("flags", np.uint8),
                         ("qp", np.int8), ("ref_idx", np.int8, 2), ("pad", np.uint8), ("mv", np.int16, (2, 2))])
assert SAO_PARAM.itemsize == 6 and DEBLOCK_UNIT.itemsize == 16


class DeblockParams(C.Structure):
    _fields_ = [("is_p", C.c_int), ("beta_offset_div2", C.c_int), ("tc_offset_div2", C.c_int),
                ("cb_qp_offset", C.c_int), ("cr_qp_offset", C.c_int), ("tq_bypass_enabled", C.c_int),
                ("ref_poc", (C.c_int32 * 16) * 2)]


class FrameFilters:
    """xo_sao_apply / xo_sao_stats / xo_deblock / xo_extend_border of one oracle library."""

    def __init__(self, kind: str, depth: int):
        self.depth = depth
        self.lib = C.CDLL(lib_path(kind, depth))
        L = self.lib
        L.xo_sao_apply.argtypes = [C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _ip, _ip, _vp, C.c_int, C.c_int]
        L.xo_sao_stats.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _ip, _ip, _vp, _vp, _vp, _ip,
                                   _ip, _vp, _vp]
        L.xo_deblock.argtypes = [C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _ip, _ip, _vp, _ip, C.POINTER(DeblockParams)]
        L.xo_extend_border.argtypes = [_vp, _ip, C.c_int, C.c_int, C.c_int, C.c_int]
        L.xo_sao_apply_csp.argtypes = L.xo_sao_apply.argtypes + [C.c_int]
        L.xo_sao_stats_csp.argtypes = L.xo_sao_stats.argtypes + [C.c_int]
        L.xo_deblock_csp.argtypes = L.xo_deblock.argtypes + [C.c_int]

    @staticmethod
    def _org(buf, margin, stride):
        return buf.ctypes.data + (margin * stride + margin) * buf.itemsize

    def sao_apply(self, width, height, ctu_log2, planes, margin, params, luma_on=1, chroma_on=1, csp=1):
        """planes: (Y, Cb, Cr) padded 2-D arrays with `margin` pixels on every side; in place.
        csp: 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4"""
        y, cb, cr = planes
        self.lib.xo_sao_apply_csp(width, height, ctu_log2, self._org(y, margin, y.shape[1]),
                                  self._org(cb, margin, cb.shape[1]), self._org(cr, margin, cr.shape[1]), y.shape[1],
                                  cb.shape[1], params.ctypes.data, luma_on, chroma_on, csp)

    def sao_stats(self, width, height, ctu_log2, fenc, rec, margin, non_deblocked=0, csp=1):
        ctu = 1 << ctu_log2
        nctu = ((width + ctu - 1) // ctu) * ((height + ctu - 1) // ctu)
        stats = np.zeros((nctu, 3, 5, 33), np.int32)
        count = np.zeros((nctu, 3, 5, 33), np.int32)
        f = [self._org(p, margin, p.shape[1]) for p in fenc]
        r = [self._org(p, margin, p.shape[1]) for p in rec]
        self.lib.xo_sao_stats_csp(width, height, ctu_log2, non_deblocked, f[0], f[1], f[2], fenc[0].shape[1],
                                  fenc[1].shape[1], r[0], r[1], r[2], rec[0].shape[1], rec[1].shape[1],
                                  stats.ctypes.data, count.ctypes.data, csp)
        return stats, count

    def deblock(self, width, height, ctu_log2, planes, margin, units, prm: DeblockParams, csp=1):
        y, cb, cr = planes
        self.lib.xo_deblock_csp(width, height, ctu_log2, self._org(y, margin, y.shape[1]),
                                self._org(cb, margin, cb.shape[1]), self._org(cr, margin, cr.shape[1]), y.shape[1],
                                cb.shape[1], units.ctypes.data, units.shape[1], C.byref(prm), csp)

    def extend_border(self, plane, margin_x, margin_y, width, height):
        self.lib.xo_extend_border(plane.ctypes.data + (margin_y * plane.shape[1] + margin_x) * plane.itemsize,
                                  plane.shape[1], width, height, margin_x, margin_y)


class LowresB:
    """xo_lowres_bcost of one oracle library (one B estimate per call)."""

    def __init__(self, kind: str, depth: int):
        self.lib = C.CDLL(lib_path(kind, depth))
        self.lib.xo_lowres_bcost.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _vp, C.POINTER(_vp), C.POINTER(_vp),
                                             _ip, _vp, _vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp]

    def bcost(self, wcu, hcu, rps, ns, planes, ls, fo, r0o, r1o, iq, tab_centre_ptr, ds0, ds1, mvs0, mc0, mvs1, mc1, lc,
              rs, ce):
        """planes: the frames' lowres planes (numpy); fo / r0o[4] / r1o[4]: element offsets"""
        base, esz = planes.ctypes.data, planes.itemsize
        r0 = (_vp * 4)(*[base + int(o) * esz for o in r0o])
        r1 = (_vp * 4)(*[base + int(o) * esz for o in r1o])
        self.lib.xo_lowres_bcost(wcu, hcu, rps, ns, base + int(fo) * esz, r0, r1, ls, _p(iq), tab_centre_ptr, ds0, ds1,
                                 _p(mvs0), _p(mc0), _p(mvs1), _p(mc1), _p(lc), _p(rs), _p(ce))


class CuTree:
    """xo_cutree_propagate of one library: Lookahead::estimateCUPropagate (slicetype.cpp:1738-1836)."""

    def __init__(self, kind: str, depth: int = 8):
        self.lib = C.CDLL(lib_path(kind, depth))
        self.lib.xo_cutree_propagate.argtypes = [C.c_int] * 8 + [C.c_double] + [_vp] * 8

    def propagate(self, wcu, hcu, b_p0, p1_b, referenced, weighted_bipred, fps_num, fps_den, avg_duration,
                  prop_b, intra, lowres_costs, inv_q, mvs0, mvs1, ref0, ref1):
        """in place on prop_b (first row zeroed when not referenced), ref0, ref1 (numpy arrays)"""
        self.lib.xo_cutree_propagate(wcu, hcu, b_p0, p1_b, referenced, weighted_bipred, fps_num, fps_den,
                                     avg_duration, _p(prop_b), _p(intra), _p(lowres_costs), _p(inv_q), _p(mvs0),
                                     _p(mvs1), _p(ref0), _p(ref1))


class Weights:
    """xo_weights_analyse of one library: LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495)."""

    def __init__(self, kind: str, depth: int = 8):
        self.lib = C.CDLL(lib_path(kind, depth))
        self.lib.xo_weights_analyse.argtypes = [C.c_int, C.c_int, _ip, C.c_int, _ip, _vp, C.POINTER(_vp), _vp,
                                                C.POINTER(_vp), C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _vp,
                                                C.POINTER(C.c_double)]

    def analyse(self, width, lines, stride, padded_lines, pad_offset, fenc_buf, ref_buf, intra, wbuf, fssd, rssd,
                fsum, rsum):
        """fenc_buf / ref_buf / wbuf: contiguous (4, planesize) numpy arrays; returns (out[4], cost_delta)"""
        ps = ref_buf.shape[1]
        es = ref_buf.itemsize
        rb = (_vp * 4)(*[ref_buf.ctypes.data + i * ps * es for i in range(4)])
        wb = (_vp * 4)(*[wbuf.ctypes.data + i * ps * es for i in range(4)])
        out = np.zeros(4, np.int32)
        delta = C.c_double(-1.0)
        self.lib.xo_weights_analyse(width, lines, stride, padded_lines, pad_offset,
                                    fenc_buf.ctypes.data + pad_offset * es, rb, _p(intra), wb, int(fssd), int(rssd),
                                    int(fsum), int(rsum), _p(out), C.byref(delta))
        return out, delta.value
