"""Census-driven primitive workload over HBM-resident frames (bench + full-size tests).

One bench *step* replays, for F synthetic frames at once, every primitive call
the reference encoder makes per frame (x265 1.9, --preset medium, 1080p:
tests/golden/census_1080p_medium.json, produced by oracle/run_census.py), as
one batched C-ABI launch per (table entry, block shape).  Operands live in
HBM in x265's own picture layout (PicYuv, picyuv.cpp:54-80: luma margins
64+32 / 64+16, chroma margins 96 / 40, CTU-aligned planes):

  * fenc blocks at CU/PU-aligned positions of frame f, reference blocks in
    frame f-1 displaced by a motion vector within +-48 px (medium's
    searchRange is 57, param.cpp:159);
  * residual/coefficient int16 planes and pools for transforms and quant;
  * intra neighbour pools (4N+1 samples) gathered from the frame;
  * disjoint per-job output slots for block outputs.

Entries that stay on the CPU in this design (CABAC-estimate helpers, SAO,
lowres init, propagateCost, weighting, plane copies — SURVEY.md §8(a) "not on
the ★ list") are skipped and reported.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

from .synth import SyntheticSource

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CENSUS_1080P = os.path.join(ROOT, "tests", "golden", "census_1080p_medium.json")

# C-ABI codes (include/x265_amd.h)
SAD, SATD, SA8D, SSE_PP, SSE_SS, PSY, SSD_S, VAR = range(8)
HPP, HPS, VPP, VPS, VSP, VSS, HVPP, P2S = range(8)
DCT, IDCT, DST, IDST = range(4)
(SUB_PS, ADD_PS, ADDAVG, PIXELAVG, COPY_PP, COPY_SP, COPY_PS, COPY_SS, BLOCKFILL,
 CPY2D1D_SHL, CPY2D1D_SHR, CPY1D2D_SHL, CPY1D2D_SHR, TRANSPOSE) = range(14)

PIXELCMP_OPS = {"sad": SAD, "satd": SATD, "sa8d": SA8D, "sse_pp": SSE_PP, "sse_ss": SSE_SS, "psy_cost_pp": PSY,
                "ssd_s": SSD_S, "var": VAR}
INTERP_OPS = {"luma_hpp": HPP, "luma_hps": HPS, "luma_vpp": VPP, "luma_vps": VPS, "luma_vsp": VSP,
              "luma_vss": VSS, "luma_hvpp": HVPP, "convert_p2s": P2S, "p2s": P2S, "filter_hpp": HPP,
              "filter_hps": HPS, "filter_vpp": VPP, "filter_vps": VPS, "filter_vsp": VSP, "filter_vss": VSS}
BLOCK_OPS = {"sub_ps": SUB_PS, "calcresidual": SUB_PS, "add_ps": ADD_PS, "addAvg": ADDAVG,
             "pixelavg_pp": PIXELAVG, "copy_pp": COPY_PP, "copy_sp": COPY_SP, "copy_ps": COPY_PS,
             "copy_ss": COPY_SS, "blockfill_s": BLOCKFILL, "cpy2Dto1D_shl": CPY2D1D_SHL,
             "cpy2Dto1D_shr": CPY2D1D_SHR, "cpy1Dto2D_shl": CPY1D2D_SHL, "cpy1Dto2D_shr": CPY1D2D_SHR,
             "transpose": TRANSPOSE}

MV_RANGE = 48


def load_census(path: str = CENSUS_1080P) -> dict:
    with open(path) as f:
        return json.load(f)["per_frame"]


class FrameSet:
    """F padded frames (luma + 4:2:0 chroma) plus int16 residual planes, on one device."""

    def __init__(self, width: int, height: int, nframes: int, depth: int = 8, device: str = "cuda", ctu: int = 64,
                 first_frame: int = 0, frame_ids: list | None = None, store_ids: list | None = None,
                 ref_slots: list | None = None):
        import torch

        self.w, self.h, self.F, self.depth, self.device = width, height, nframes, depth, device
        self.pw = (width + ctu - 1) // ctu * ctu
        self.ph = (height + ctu - 1) // ctu * ctu
        self.mx, self.my = ctu + 32, ctu + 16               # picyuv.cpp:62-63
        self.stride = self.pw + 2 * self.mx
        self.rows = self.ph + 2 * self.my
        self.cmx, self.cmy = self.mx, self.my // 2          # picyuv.cpp:71-73 (4:2:0)
        self.cstride = self.pw // 2 + 2 * self.cmx
        self.crows = self.ph // 2 + 2 * self.cmy
        # Default: stored frames 0..F-1 are the chunk being encoded (synthetic frames
        # first+1 .. first+F); stored frame F is the REFERENCE SLOT holding the
        # picture before the chunk (synthetic frame `first`), which frame 0
        # predicts from; frame f > 0 predicts from stored frame f - 1.
        # Frame-parallel pipeline (pipeline.py): stored frames 0..F-1 are this rank's frames
        # (synthetic frames frame_ids), stored frames F.. its REFERENCE STORE (synthetic frames
        # store_ids until the exchange overwrites them with the producers' reconstructions);
        # ref_slots[k] lists the stored indices of local frame k's references (L0 then L1; empty
        # for an I frame, whose inter-shaped census jobs then read its own picture).
        self.ref_slots = ref_slots
        if ref_slots is not None:
            assert frame_ids is not None and len(frame_ids) == nframes and len(ref_slots) == nframes
            ids = list(frame_ids) + list(store_ids or [])
        else:
            ids = [first_frame + i + 1 for i in range(nframes)] + [first_frame]
        src = SyntheticSource(width, height, max(ids) + 1, depth)
        dt = np.uint8 if depth == 8 else np.uint16
        S = len(ids)
        self.stored = S
        Y = np.zeros((S, self.rows, self.stride), dt)
        U = np.zeros((S, self.crows, self.cstride), dt)
        V = np.zeros((S, self.crows, self.cstride), dt)
        for i in range(S):
            y, u, v = src.frame(ids[i])
            Y[i] = self._pad(y, self.mx, self.my, self.rows, self.stride)
            U[i] = self._pad(u, self.cmx, self.cmy, self.crows, self.cstride)
            V[i] = self._pad(v, self.cmx, self.cmy, self.crows, self.cstride)
        # residual planes: frame f minus its (first) reference (int16), same layout as luma
        ref_idx = [self.ref_of(f) if f < nframes else f for f in range(S)]
        R = (Y.astype(np.int32) - Y[ref_idx].astype(np.int32)).astype(np.int16)
        self.host = dict(Y=Y.reshape(-1), U=U.reshape(-1), V=V.reshape(-1), R=R.reshape(-1))
        t = lambda a: torch.from_numpy(a).to(device)
        self.luma, self.cb, self.cr, self.resid = t(self.host["Y"]), t(self.host["U"]), t(self.host["V"]), t(self.host["R"])
        self.plane_size = self.rows * self.stride
        self.cplane_size = self.crows * self.cstride

    def ref_of(self, f, sel=None):
        """stored index of the reference a job of stored frame f reads: the previous frame (or the
        reference slot for frame 0); with reference stores, entry sel mod n of f's reference list"""
        if self.ref_slots is not None:
            if getattr(self, "_ref_tab", None) is None:
                # [frame, k] = k-th reference slot (an I frame: itself), and the list lengths
                n = max(1, max(len(r) for r in self.ref_slots))
                self._ref_tab = np.zeros((len(self.ref_slots), n), np.int64)
                self._ref_len = np.array([len(r) for r in self.ref_slots], np.int64)
                for i, rs in enumerate(self.ref_slots):
                    self._ref_tab[i, :max(1, len(rs))] = rs if rs else i
            fa = np.atleast_1d(np.asarray(f, np.int64))
            sa = np.zeros_like(fa) if sel is None else np.broadcast_to(np.asarray(sel, np.int64), fa.shape)
            ln = self._ref_len[fa]
            out = np.where(ln > 0, self._ref_tab[fa, sa % np.maximum(ln, 1)], fa)
            return out if not np.isscalar(f) else int(out[0])
        return np.where(np.asarray(f) == 0, self.F, np.asarray(f) - 1) if not np.isscalar(f) else (self.F if f == 0 else f - 1)

    def planes(self, f: int):
        """flat views (luma, cb, cr) of stored frame f"""
        return (self.luma[f * self.plane_size:(f + 1) * self.plane_size],
                self.cb[f * self.cplane_size:(f + 1) * self.cplane_size],
                self.cr[f * self.cplane_size:(f + 1) * self.cplane_size])

    @staticmethod
    def _pad(p, mx, my, rows, stride):
        """x265 extendPicBorder (pixel.cpp:908-922): replicate edges into the margins."""
        h, w = p.shape
        out = np.empty((rows, stride), p.dtype)
        core = np.pad(p, ((my, rows - h - my), (mx, stride - w - mx)), mode="edge")
        out[:] = core
        return out

    # ---- offsets (element units, into the concatenated [F, rows, stride] tensors)
    def luma_off(self, f, x, y):
        return f * self.plane_size + (self.my + y) * self.stride + (self.mx + x)

    def chroma_off(self, f, x, y):
        return f * self.cplane_size + (self.cmy + y) * self.cstride + (self.cmx + x)


@dataclass
class Batch:
    name: str
    kind: str
    op: int
    w: int
    h: int
    n: int
    depth: int
    taps: int = 8
    params: dict = field(default_factory=dict)     # ints (strides, flags)
    dev: dict = field(default_factory=dict)        # device tensors
    host_src: dict = field(default_factory=dict)   # name -> host array key for inputs shared with the FrameSet
    outs: dict = field(default_factory=dict)       # out name -> ("scalar", per_job) | ("slot", elems_per_job)
    bytes: float = 0.0                             # algorithmic bytes per launch
    pos: tuple | None = None                       # (stored frame, luma row) of each job's coded block, if any

    def run(self, prims, stream=None):
        d, p = self.dev, self.params
        k = self.kind
        if k == "pixelcmp":
            prims.pixelcmp(self.op, self.depth, self.w, self.h, d["a"], p["sa"], d["aoff"], d.get("b"), p.get("sb", 0),
                           d.get("boff", d["aoff"]), d["out"], stream)
        elif k == "sad_multi":
            prims.sad_multi(self.op, self.depth, self.w, self.h, d["f"], p["fs"], d["foff"], d["r"], p["rs"], d["roff"],
                            d["out"], stream)
        elif k == "interp":
            prims.interp(self.op, self.taps, self.depth, self.w, self.h, d["s"], p["ss"], d["soff"], d["d"], p["ds"],
                         d["doff"], d["coeff"], p.get("rowext", 0), stream)
        elif k == "transform":
            prims.transform(self.op, self.depth, self.w, d["s"], p["ss"], d["soff"], d["d"], p["ds"], d["doff"], stream)
        elif k == "quant":
            prims.quant(self.w * self.w, d["c"], d["co"], d["q"], d["qo"], d.get("dl"), d.get("dlo"), d["o"], d["oo"],
                        d["qb"], d["ad"], d["sig"], stream)
        elif k == "dequant":
            prims.dequant_normal(self.w * self.w, d["q"], d["qo"], d["o"], d["oo"], d["p0"], d["p1"], stream)
        elif k == "intra":
            prims.intra_pred(self.depth, self.w, d["d"], p["ds"], d["doff"], d["nb"], d["nbo"], d["mode"], d["bf"],
                             stream)
        elif k == "intra_filter":
            prims.intra_filter(self.depth, self.w, d["nb"], d["nbo"], d["d"], d["doff"], stream)
        elif k == "blockop":
            prims.blockop(self.op, self.depth, self.w, self.h, d["d"], p["ds"], d["doff"], d.get("a"), p.get("sa", 0),
                          d.get("aoff"), d.get("b"), p.get("sb", 0), d.get("boff"), p.get("param", 0), stream)
        elif k == "count":
            prims.count_nonzero(self.w, d["c"], d["co"], d.get("r"), p.get("rs", 0), d.get("ro"), d["cnt"], stream)
        else:
            raise ValueError(k)

    # ---- sampled CPU verification -------------------------------------------------
    def sample(self, k: int, seed: int = 7) -> np.ndarray:
        rng = np.random.default_rng(seed + self.n)
        return np.sort(rng.choice(self.n, size=min(k, self.n), replace=False))

    def verify_sample(self, orc, host: dict, idx: np.ndarray) -> list:
        """Recompute the sampled jobs with a CPU oracle; return names of mismatching outputs."""
        import sys

        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from cases import Case, run_cpu

        bufs = {}
        for k, v in self.params.items():
            bufs[k] = v
        for k, t in self.dev.items():
            if k in self.outs:
                continue
            arr = host[self.host_src[k]] if k in self.host_src else t.cpu().numpy()
            if k.endswith("off") or k in ("co", "qo", "oo", "dlo", "nbo", "ro", "qb", "ad", "p0", "p1", "coeff", "mode", "bf"):
                per = len(arr) // self.n
                arr = arr.reshape(self.n, per)[idx].reshape(-1) if per > 1 else arr[idx]
            bufs[k] = arr
        gpu_outs = {}
        for k, (typ, per) in self.outs.items():
            full = self.dev[k].cpu().numpy()
            if typ == "scalar":
                bufs[k] = np.zeros(len(idx) * per, full.dtype)
                gpu_outs[k] = full.reshape(self.n, per)[idx].reshape(-1)
            else:
                bufs[k] = np.zeros_like(full)
                gpu_outs[k] = full
        fam = {"intra_filter": "intra", "dequant": "dequant"}.get(self.kind, self.kind)
        params = dict(self.params, op=self.op, w=self.w, h=self.h, depth=self.depth, taps=self.taps, nref=self.op,
                      kind=self.op if self.kind == "transform" else (0 if self.kind == "intra_filter" else 1),
                      size=self.w, scaling=0, rowext=self.params.get("rowext", 0))
        for k in ("b", "boff", "dl", "dlo", "dq", "dqo", "f", "fo", "mode", "bf", "r", "ro", "coeff"):
            bufs.setdefault(k, None)
        bufs.setdefault("rs", 0)
        bufs.setdefault("sb", 0)
        case = Case(fam, params, bufs, list(self.outs))
        cpu = run_cpu(case, orc)
        bad = []
        for k, (typ, per) in self.outs.items():
            if typ == "scalar":
                if not np.array_equal(cpu[k], gpu_outs[k]):
                    bad.append(k)
            else:
                # a job's slot is where its own output offset points (jobs may have been reordered)
                okey = {"d": "doff", "o": "oo", "dl": "dlo"}.get(k)
                rows = idx
                if okey in self.dev:
                    rows = self.dev[okey].cpu().numpy().astype(np.int64)[idx] // per
                g, c = gpu_outs[k].reshape(-1, per), cpu[k].reshape(-1, per)
                if not np.array_equal(g[rows], c[rows]):
                    bad.append(k)
        return bad


MAX_SUB = 16   # sub-batches per grouped launch (csrc/common.h kMaxSub)


def launch_class(b: Batch):
    """Kernel instantiation a batch runs in (mirrors cmp_class / blockop_class /
    interp_class in csrc/): batches with equal keys share one grouped launch.
    None for kinds that are not grouped."""
    w, h = b.w, b.h
    if b.kind == "pixelcmp":
        uwd = 4 if w % 8 else 8
        if b.op == SA8D:
            cls = (16, 16) if w % 16 == 0 and h % 16 == 0 else (8, 8) if w % 8 == 0 and h % 8 == 0 else ("satd", uwd)
        elif b.op == PSY:
            cls = 4 if w == 4 else 8
        else:
            cls = uwd
        return ("pixelcmp", b.op, b.depth, cls)
    if b.kind == "sad_multi":
        return ("sad_multi", b.op, b.depth, 4 if w % 8 else 8)
    if b.kind == "blockop":
        # csrc/blockops.hip blockop_class: ~32 loaded bytes per lane
        p = 1 if b.depth == 8 else 2
        a_b = {SUB_PS: (p, p), ADD_PS: (p, 2), ADDAVG: (2, 2), PIXELAVG: (p, p), COPY_SP: (2, 0), COPY_SS: (2, 0),
               BLOCKFILL: (2, 0), CPY2D1D_SHL: (2, 0), CPY2D1D_SHR: (2, 0), CPY1D2D_SHL: (2, 0),
               CPY1D2D_SHR: (2, 0)}.get(b.op, (p, 0))
        uw = 8 if w % 8 == 0 else 4 if w % 4 == 0 else 2
        want = max(1, 32 // (uw * sum(a_b)))
        uh = 4 if want >= 4 and h % 4 == 0 else 2 if want >= 2 and h % 2 == 0 else 1
        return ("blockop", b.op, b.depth, uw, uh)
    if b.kind == "interp":
        taps = 4 if b.op == P2S else b.taps
        rows = h + taps - 1 if b.op == HPS and b.params.get("rowext", 0) else h
        if b.op == HVPP:
            rows = h
        pk8 = b.op in (VPP, VPS) and b.depth == 8     # csrc/interp.hip: packed 8-bit vertical path
        uh = 16 if pk8 and rows % 16 == 0 and w % 4 == 0 else 4 if rows % 4 == 0 else 1
        if b.op == HVPP and h <= 16 and h % 2 == 0:
            uh = 2                                      # csrc/interp.hip interp_class: 2-row hv units
        return ("interp", b.op, taps, b.depth, 8 if w % 8 == 0 else 4 if w % 4 == 0 else 2, uh)
    return None


class LaunchGroup:
    """Up to MAX_SUB batches of one kernel class issued as ONE grouped launch
    (x265amd_*_grouped).  Each member keeps its own operands and outputs, so
    verification stays per member batch."""

    def __init__(self, members: list):
        self.members = members
        b0 = members[0]
        self.kind, self.op, self.depth, self.taps = b0.kind, b0.op, b0.depth, b0.taps
        self.n = sum(b.n for b in members)
        self.bytes = sum(b.bytes for b in members)
        self.name = "grp[" + "+".join(b.name for b in members) + "]" if len(members) > 1 else b0.name
        self._arr = None

    def _descriptors(self):
        from . import native as nv

        items = []
        for b in self.members:
            d, p = b.dev, b.params
            if self.kind == "pixelcmp":
                items.append((b.w, b.h, d["a"], p["sa"], d["aoff"], d.get("b"), p.get("sb", 0),
                              d.get("boff", d["aoff"]), d["out"]))
            elif self.kind == "sad_multi":
                items.append((b.w, b.h, d["f"], p["fs"], d["foff"], d["r"], p["rs"], d["roff"], d["out"]))
            elif self.kind == "blockop":
                items.append((b.w, b.h, p.get("param", 0), d["d"], p["ds"], d["doff"], d.get("a"), p.get("sa", 0),
                              d.get("aoff"), d.get("b"), p.get("sb", 0), d.get("boff")))
            else:
                items.append((b.w, b.h, p.get("rowext", 0), d["s"], p["ss"], d["soff"], d["d"], p["ds"], d["doff"],
                              d.get("coeff")))
        make = {"pixelcmp": nv.cmp_batches, "sad_multi": nv.cmp_batches, "blockop": nv.block_batches,
                "interp": nv.interp_batches}[self.kind]
        return make(items)

    def run(self, prims, stream=None):
        if len(self.members) == 1:
            return self.members[0].run(prims, stream)
        if self._arr is None:
            self._arr = self._descriptors()   # device addresses are fixed for the life of the batches
            # the table holds raw addresses: keep the tensors they point into alive with it (a batch
            # whose per-job tensors are later replaced, e.g. reordered, must not leave it dangling)
            self._keep = [dict(b.dev) for b in self.members]
        if self.kind == "pixelcmp":
            prims.pixelcmp_grouped(self.op, self.depth, self._arr, stream)
        elif self.kind == "sad_multi":
            prims.sad_multi_grouped(self.op, self.depth, self._arr, stream)
        elif self.kind == "blockop":
            prims.blockop_grouped(self.op, self.depth, self._arr, stream)
        else:
            prims.interp_grouped(self.op, self.taps, self.depth, self._arr, stream)


def group_launches(batches: list, max_sub: int = MAX_SUB) -> list:
    """Pack batches of one kernel class into LaunchGroups of at most max_sub
    members (largest first inside a class); other batches become groups of one.
    Result is ordered by bytes, largest first."""
    classes, out = {}, []
    for b in batches:
        key = launch_class(b)
        if key is None:
            out.append(LaunchGroup([b]))
        else:
            classes.setdefault(key, []).append(b)
    for key, bs in classes.items():
        bs = sorted(bs, key=lambda b: -b.bytes)
        for i in range(0, len(bs), max_sub):
            out.append(LaunchGroup(bs[i:i + max_sub]))
    out.sort(key=lambda g: -g.bytes)
    return out


def _aligned(rng, lo, hi, align, n):
    return (rng.integers(lo // align, hi // align + 1, n) * align).astype(np.int64)


class WorkloadBuilder:
    """Turns census entries into device batches over a FrameSet."""

    def __init__(self, fs: FrameSet, seed: int = 1):
        self.fs = fs
        self.rng = np.random.default_rng(seed)
        self.skipped = {}
        self._pools = {}
        self._pos = None

    # ---- shared pools ------------------------------------------------------------
    def pool(self, name, make):
        if name not in self._pools:
            self._pools[name] = make()
        return self._pools[name]

    def _t(self, a):
        import torch

        return torch.from_numpy(np.ascontiguousarray(a)).to(self.fs.device)

    def _positions(self, n, w, h, chroma=False):
        """Job block positions the way an encoder visits them: frame by frame,
        blocks in raster (CTU-row) order; when a frame needs more calls than it
        has blocks of this shape, each block is evaluated several times in a
        row (motion-search candidates).  Returns frame, x, y, candidate index."""
        fs, rng = self.fs, self.rng
        pw, ph = (fs.pw // 2, fs.ph // 2) if chroma else (fs.pw, fs.ph)
        bx, by = max(1, pw // w), max(1, ph // h)
        nblk = bx * by
        per = -(-n // fs.F)
        if per <= nblk:
            # fewer calls than blocks: whole CTUs of blocks, the way CU analysis visits a CTU's blocks at
            # each depth (analysis.cpp compressInterCU_rd*) — a run of consecutive CTUs (raster order,
            # from a random start) and the blocks of a CTU in raster order inside it, so neighbouring
            # jobs share the CTU's rows and cache lines, and so do neighbouring CTUs
            ctu = 32 if chroma else 64
            cw, ch = max(1, ctu // w), max(1, ctu // h)          # blocks per CTU across / down
            ncx, ncy = -(-bx // cw), -(-by // ch)
            k = min(-(-per // (cw * ch)), ncx * ncy)
            ctus = np.sort((int(rng.integers(0, ncx * ncy)) + np.arange(k)) % (ncx * ncy))
            ix = (ctus % ncx)[:, None] * cw + (np.arange(cw * ch) % cw)[None, :]
            iy = (ctus // ncx)[:, None] * ch + (np.arange(cw * ch) // cw)[None, :]
            ok = (ix < bx) & (iy < by)
            blk = (iy * bx + ix)[ok][:per]
            if len(blk) < per:                                 # partial CTUs at the picture edge
                rest = np.setdiff1d(np.arange(nblk), blk)
                blk = np.concatenate([blk, np.sort(rng.choice(rest, size=per - len(blk), replace=False))])
            cand = np.zeros(per, np.int64)
        else:
            reps = -(-per // nblk)
            blk = np.repeat(np.arange(nblk), reps)[:per]
            cand = np.tile(np.arange(reps), nblk)[:per]
        f = np.repeat(np.arange(fs.F, dtype=np.int64), per)[:n]
        blk = np.tile(blk, fs.F)[:n]
        cand = np.tile(cand, fs.F)[:n]
        x = (blk % bx) * w
        y = (blk // bx) * h
        return f, x.astype(np.int64), y.astype(np.int64), cand.astype(np.int64)

    def _mv(self, f, x, y, cand, chroma=False):
        """Smooth motion field: the source pans (+2,+1)/frame, so the match in
        frame f-1 sits near (-2,-1); each 64x64 CTU adds a stable +-6 px local
        motion and each search candidate a +-2 px step around it (clamped to
        the +-MV_RANGE search window)."""
        cx, cy = x // (32 if chroma else 64), y // (32 if chroma else 64)
        lx = ((cx * 7 + cy * 13 + f * 3) % 13) - 6
        ly = ((cx * 11 + cy * 5 + f * 7) % 13) - 6
        jx, jy = (cand % 5) - 2, ((cand // 5) % 5) - 2
        mx = np.clip(-2 + lx + jx, -MV_RANGE, MV_RANGE)
        my = np.clip(-1 + ly + jy, -MV_RANGE, MV_RANGE)
        if chroma:
            mx, my = mx // 2, my // 2
        return mx.astype(np.int64), my.astype(np.int64)

    def _fenc_ref_offsets(self, n, w, h, chroma=False, nref=1):
        fs = self.fs
        f, x, y, cand = self._positions(n, w, h, chroma)
        if self._pos is None:                  # the batch's jobs: frame and luma row of the block coded
            self._pos = (f, y * (2 if chroma else 1))
        # the reference a job reads: one entry of its frame's list (a PU's candidates search one picture)
        r = fs.ref_of(f, (x // max(w, 1)) * 7 + (y // max(h, 1)) * 13 + cand // 5)
        off = fs.chroma_off if chroma else fs.luma_off
        a = off(f, x, y)
        refs = []
        for k in range(nref):
            mx, my = self._mv(f, x, y, cand + 7 * k, chroma)
            refs.append(off(r, x + mx, y + my))
        return a, refs

    def _slots(self, n, w, h, dtype, stride=None):
        """disjoint per-job output slots of `h` rows x `stride` elements; by
        default compact (stride = w), the layout a batched caller collects
        predictions / residuals / coefficients in"""
        import torch

        stride = max(stride or w, w)
        slot = stride * h
        buf = torch.zeros(n * slot, dtype=dtype, device=self.fs.device)
        offs = self._t(np.arange(n, dtype=np.int64) * slot)
        return buf, stride, offs, slot

    # ---- batch factories ----------------------------------------------------------
    def batch(self, key: str, count: float):
        self._pos = None
        b = self._batch(key, count)
        if b is not None:
            b.pos = self._pos
        return b

    def _batch(self, key: str, count: float):
        import torch

        fs = self.fs
        pdt = torch.uint8 if fs.depth == 8 else torch.uint16
        b = fs.depth > 8 and 2 or 1
        parts = key.split(".")
        chroma = parts[0] == "chroma"
        if chroma:
            csp, table, entry, dims = parts[1], parts[2], parts[3], parts[4]
            if csp != "i420":
                self.skipped[key] = count
                return None
        else:
            table, entry, dims = parts[0], parts[1], parts[-1]
        n = int(round(count))
        if n <= 0:
            return None
        if key.startswith("cu.intra_pred."):
            size = int(parts[2].split("x")[0])
            mode = int(parts[3][4:])
            return self._intra(key, n, size, mode)
        if table == "scalar":
            return self._scalar(key, entry, n)
        if "x" not in dims:
            self.skipped[key] = count
            return None
        w, h = (int(v) for v in dims.split("x"))
        plane, pstride = (fs.cb, fs.cstride) if chroma else (fs.luma, fs.stride)
        hsrc = "U" if chroma else "Y"

        if entry in PIXELCMP_OPS:
            op = PIXELCMP_OPS[entry]
            if table == "cu" and entry == "sa8d" and w == 4:
                op = SATD
            wide = op in (SSE_PP, SSE_SS, SSD_S, VAR)
            out = torch.zeros(n, dtype=torch.int64 if wide else torch.int32, device=fs.device)
            if op in (SSE_SS, SSD_S):
                a, (r,) = self._fenc_ref_offsets(n, w, h)
                bt = Batch(key, "pixelcmp", op, w, h, n, fs.depth, params=dict(sa=fs.stride, sb=fs.stride),
                           dev=dict(a=fs.resid, aoff=self._t(a), b=fs.resid, boff=self._t(r), out=out),
                           host_src=dict(a="R", b="R"), outs=dict(out=("scalar", 1)))
                bt.bytes = n * ((4 if op == SSE_SS else 2) * w * h + 8)
                return bt
            a, (r,) = self._fenc_ref_offsets(n, w, h, chroma)
            bt = Batch(key, "pixelcmp", op, w, h, n, fs.depth, params=dict(sa=pstride, sb=pstride),
                       dev=dict(a=plane, aoff=self._t(a), b=plane, boff=self._t(r), out=out),
                       host_src=dict(a=hsrc, b=hsrc), outs=dict(out=("scalar", 1)))
            single = op == VAR
            bt.bytes = n * ((1 if single else 2) * w * h * b + (8 if wide else 4))
            return bt
        if entry in ("sad_x3", "sad_x4"):
            nref = 3 if entry == "sad_x3" else 4
            a, refs = self._fenc_ref_offsets(n, w, h, nref=1)
            base = refs[0]
            pattern = [(0, -2), (-2, 0), (2, 0), (0, 2)][:nref]
            ro = np.stack([base + dy * fs.stride + dx for dx, dy in pattern], axis=1).reshape(-1)
            out = torch.zeros(n * nref, dtype=torch.int32, device=fs.device)
            bt = Batch(key, "sad_multi", nref, w, h, n, fs.depth, params=dict(fs=fs.stride, rs=fs.stride),
                       dev=dict(f=fs.luma, foff=self._t(a), r=fs.luma, roff=self._t(ro), out=out),
                       host_src=dict(f="Y", r="Y"), outs=dict(out=("scalar", nref)))
            bt.bytes = n * ((nref + 1) * w * h * b + 4 * nref)
            return bt
        if entry in INTERP_OPS:
            op = INTERP_OPS[entry]
            taps = 4 if (chroma or entry.startswith("filter_")) else 8
            src16 = op in (VSP, VSS)
            dst16 = op in (HPS, VPS, VSS, P2S)
            _, (r,) = self._fenc_ref_offsets(n, w, h, chroma)
            if src16:
                _, (r,) = self._fenc_ref_offsets(n, w, h, False)
                s, ss, hs = fs.resid, fs.stride, "R"
            else:
                s, ss, hs = plane, pstride, hsrc
            d, ds, doff, slot = self._slots(n, w, h, torch.int16 if dst16 else pdt)
            nidx = 4 if taps == 8 else 8
            cx = self.rng.integers(1, nidx, n)
            coeff = (cx | (self.rng.integers(1, nidx, n) << 4)) if op == HVPP else cx
            bt = Batch(key, "interp", op, w, h, n, fs.depth, taps=taps, params=dict(ss=ss, ds=ds, rowext=0),
                       dev=dict(s=s, soff=self._t(r), d=d, doff=doff, coeff=self._t(coeff.astype(np.uint8))),
                       host_src=dict(s=hs), outs=dict(d=("slot", slot)))
            sb_ = 2 if src16 else b
            db_ = 2 if dst16 else b
            ext = taps - 1
            if op in (HPP, HPS):
                inb = (w + ext) * h
            elif op in (VPP, VPS, VSP, VSS):
                inb = w * (h + ext)
            elif op == HVPP:
                inb = (w + ext) * (h + ext)
            else:
                inb = w * h
            bt.bytes = n * (inb * sb_ + w * h * db_ + 1)
            return bt
        if entry in ("dct", "idct"):
            return self._transform(key, DCT if entry == "dct" else IDCT, w, n)
        if entry == "count_nonzero":
            c, co = self._coef_pool(w, n)
            cnt = torch.zeros(n, dtype=torch.int32, device=fs.device)
            bt = Batch(key, "count", 0, w, w, n, fs.depth, dev=dict(c=c, co=co, cnt=cnt), outs=dict(cnt=("scalar", 1)))
            bt.bytes = n * (2 * w * w + 4)
            return bt
        if entry == "intra_filter":
            nb, nbo = self._nb_pool(w, n)
            d, ds, doff, slot = self._slots(n, 4 * w + 1, 1, pdt, stride=4 * w + 1)
            bt = Batch(key, "intra_filter", 0, w, w, n, fs.depth, dev=dict(nb=nb, nbo=nbo, d=d, doff=doff),
                       params=dict(ds=ds), outs=dict(d=("slot", slot)))
            bt.bytes = n * 2 * (4 * w + 1) * b
            return bt
        if entry in BLOCK_OPS:
            return self._blockop(key, BLOCK_OPS[entry], w, h, n, chroma)
        self.skipped[key] = count
        return None

    def _coef_pool(self, size, n):
        import torch

        num = size * size
        pool = self.pool(("coef", size), lambda: self._t(
            (self.rng.integers(-64, 65, 4096 * num) * (self.rng.integers(0, 3, 4096 * num) == 0)).astype(np.int16)))
        co = self._t(self.rng.integers(0, 4096, n).astype(np.int64) * num)
        return pool, co

    def _nb_pool(self, size, n):
        fs = self.fs
        m = 4 * size + 1
        host = fs.host["Y"]

        def make():
            f, x, y, _ = self._positions(8192, 2 * size, 1)
            offs = fs.luma_off(f, x, y)
            return self._t(np.stack([host[o:o + m] for o in offs]).reshape(-1))

        pool = self.pool(("nb", size), make)
        nbo = self._t(self.rng.integers(0, 8192, n).astype(np.int64) * m)
        return pool, nbo

    def _transform(self, key, kind, size, n):
        import torch

        fs = self.fs
        if kind in (DCT, DST):
            a, _ = self._fenc_ref_offsets(n, size, size)
            d, ds, doff, slot = self._slots(n, size, size, torch.int16, stride=size)
            bt = Batch(key, "transform", kind, size, size, n, fs.depth, params=dict(ss=fs.stride, ds=ds),
                       dev=dict(s=fs.resid, soff=self._t(a), d=d, doff=doff), host_src=dict(s="R"),
                       outs=dict(d=("slot", slot)))
        else:
            c, co = self._coef_pool(size, n)
            d, ds, doff, slot = self._slots(n, size, size, torch.int16, stride=size)
            bt = Batch(key, "transform", kind, size, size, n, fs.depth, params=dict(ss=size, ds=ds),
                       dev=dict(s=c, soff=co, d=d, doff=doff), outs=dict(d=("slot", slot)))
        bt.bytes = n * 4 * size * size
        return bt

    def _intra(self, key, n, size, mode):
        return self.intra_merged(key, size, {mode: n})

    def intra_merged(self, key, size, mode_counts: dict):
        """One launch for every (TU, mode) evaluation of one TU size; jobs are
        grouped by mode (wave-uniform prediction direction), as a batched
        mode search would issue them."""
        import torch

        fs = self.fs
        pdt = torch.uint8 if fs.depth == 8 else torch.uint16
        modes = np.concatenate([np.full(int(round(c)), m, np.uint8) for m, c in sorted(mode_counts.items())])
        n = len(modes)
        if n == 0:
            return None
        nb, nbo = self._nb_pool(size, n)
        d, ds, doff, slot = self._slots(n, size, size, pdt)
        bf = np.full(n, 1 if size <= 16 else 0, np.uint8)
        bt = Batch(key, "intra", 0, size, size, n, fs.depth, params=dict(ds=ds),
                   dev=dict(d=d, doff=doff, nb=nb, nbo=nbo, mode=self._t(modes),
                            bf=self._t(bf)), outs=dict(d=("slot", slot)))
        bt.bytes = n * ((4 * size + 1) + size * size) * (2 if fs.depth > 8 else 1)
        return bt

    def _scalar(self, key, entry, n):
        """quant / nquant / dequant / dst / idst: TU size distributed like the dct / idct census."""
        return None   # expanded by census_batches, which knows the size distribution

    def _blockop(self, key, op, w, h, n, chroma):
        import torch

        fs = self.fs
        pdt = torch.uint8 if fs.depth == 8 else torch.uint16
        b = 2 if fs.depth > 8 else 1
        plane, pstride, hsrc = (fs.cb, fs.cstride, "U") if chroma else (fs.luma, fs.stride, "Y")
        a, (r,) = self._fenc_ref_offsets(n, w, h, chroma)
        p = dict(sa=pstride, sb=pstride, param=0)
        dev = dict(a=plane, aoff=self._t(a), b=plane, boff=self._t(r))
        hs = dict(a=hsrc, b=hsrc)
        d16 = op in (SUB_PS, COPY_PS, COPY_SS, BLOCKFILL, CPY2D1D_SHL, CPY2D1D_SHR, CPY1D2D_SHL, CPY1D2D_SHR)
        if op in (ADDAVG, COPY_SP, COPY_SS, CPY2D1D_SHL, CPY2D1D_SHR, CPY1D2D_SHL, CPY1D2D_SHR):
            a16, (r16,) = self._fenc_ref_offsets(n, w, h)
            dev = dict(a=fs.resid, aoff=self._t(a16), b=fs.resid, boff=self._t(r16))
            hs = dict(a="R", b="R")
            p = dict(sa=fs.stride, sb=fs.stride, param=0)
        if op == ADD_PS:
            _, (r16,) = self._fenc_ref_offsets(n, w, h)
            dev["b"], dev["boff"], hs["b"], p["sb"] = fs.resid, self._t(r16), "R", fs.stride
        if op in (CPY2D1D_SHL, CPY2D1D_SHR, CPY1D2D_SHL, CPY1D2D_SHR):
            p["param"] = 2 if op in (CPY2D1D_SHL, CPY1D2D_SHL) else 1
        if op == BLOCKFILL:
            p["param"] = 5
        d, ds, doff, slot = self._slots(n, w, h, torch.int16 if d16 else pdt)
        p["ds"] = ds
        dev.update(d=d, doff=doff)
        bt = Batch(key, "blockop", op, w, h, n, fs.depth, params=p, dev=dev, host_src=hs, outs=dict(d=("slot", slot)))
        ins = {SUB_PS: 2 * b, ADD_PS: b + 2, ADDAVG: 4, PIXELAVG: 2 * b, COPY_PP: b, COPY_SP: 2, COPY_PS: b,
               COPY_SS: 2, BLOCKFILL: 0, TRANSPOSE: b}.get(op, 2)
        outb = 2 if d16 else b
        bt.bytes = n * w * h * (ins + outb)
        return bt

    def quant_batches(self, census: dict, frames: int, scale: float):
        """quant / nquant / dequant_normal / dst4 / idst4 from the scalar census entries."""
        import torch

        fs = self.fs
        out = []
        fwd = {n: census.get(f"cu.dct.{n}x{n}", 0) for n in (4, 8, 16, 32)}
        fwd[4] += census.get("scalar.dst4x4", 0)
        inv = {n: census.get(f"cu.idct.{n}x{n}", 0) for n in (4, 8, 16, 32)}
        inv[4] += census.get("scalar.idst4x4", 0)
        for kind, key in ((DST, "scalar.dst4x4"), (IDST, "scalar.idst4x4")):
            n = int(round(census.get(key, 0) * frames * scale))
            if n:
                out.append(self._transform(key, kind, 4, n))
        for key, dist in (("scalar.quant", fwd), ("scalar.nquant", fwd), ("scalar.dequant_normal", inv)):
            total = census.get(key, 0)
            tot_w = sum(dist.values()) or 1
            for size, wgt in dist.items():
                n = int(round(total * wgt / tot_w * frames * scale))
                if n <= 0:
                    continue
                num = size * size
                c, co = self._coef_pool(size, n)
                if key == "scalar.dequant_normal":
                    o, _, oo, slot = self._slots(n, num, 1, torch.int16, stride=num)
                    per = self.rng.integers(2, 7, n)
                    inv_s = np.array([40, 45, 51, 57, 64, 72])[self.rng.integers(0, 6, n)]
                    tshift = 15 - fs.depth - int(math.log2(size))
                    bt = Batch(f"{key}.{size}x{size}", "dequant", 0, size, size, n, fs.depth,
                               dev=dict(q=c, qo=co, o=o, oo=oo, p0=self._t((inv_s << per).astype(np.int32)),
                                        p1=self._t(np.full(n, 20 - 14 - tshift, np.int32))),
                               outs=dict(o=("slot", slot)))
                    bt.bytes = n * 4 * num
                else:
                    qtab = self.pool(("qtab", size), lambda: self._t(
                        np.repeat(np.array([26214, 23302, 20560, 18396, 16384, 14564], np.int32) * 16, num)))
                    rem = self.rng.integers(0, 6, n)
                    qo = self._t(rem.astype(np.int64) * num)
                    o, _, oo, slot = self._slots(n, num, 1, torch.int16, stride=num)
                    per = self.rng.integers(2, 7, n)
                    tshift = 15 - fs.depth - int(math.log2(size))
                    qb = (14 + per + tshift).astype(np.int32)
                    ad = ((85 << (qb - 9))).astype(np.int32)
                    sig = torch.zeros(n, dtype=torch.int32, device=fs.device)
                    dev = dict(c=c, co=co, q=qtab, qo=qo, o=o, oo=oo, qb=self._t(qb), ad=self._t(ad), sig=sig)
                    outs = dict(o=("slot", slot), sig=("scalar", 1))
                    if key == "scalar.quant":
                        dl, _, dlo, dslot = self._slots(n, num, 1, torch.int32, stride=num)
                        dev.update(dl=dl, dlo=dlo)
                        outs["dl"] = ("slot", dslot)
                        bt = Batch(f"{key}.{size}x{size}", "quant", 0, size, size, n, fs.depth, dev=dev, outs=outs)
                        bt.bytes = n * (2 * num + 4 * num + 2 * num + 4)
                    else:
                        bt = Batch(f"{key}.{size}x{size}", "quant", 1, size, size, n, fs.depth, dev=dev, outs=outs)
                        bt.bytes = n * (2 * num + 2 * num + 4)
                out.append(bt)
        return out


def census_batches(fs: FrameSet, frames: int, scale: float = 1.0, families=None, census: dict | None = None,
                   builder: WorkloadBuilder | None = None):
    """All GPU batches for `frames` frames of the census (x `scale`), largest first."""
    census = census or load_census()
    wb = builder or WorkloadBuilder(fs)
    out = []
    intra = {}
    for key, per_frame in census.items():
        if families is not None and not any(("." + f + ".") in ("." + key + ".") for f in families):
            continue
        if key.startswith("scalar."):
            continue
        if key.startswith("cu.intra_pred."):
            p = key.split(".")
            intra.setdefault(int(p[2].split("x")[0]), {})[int(p[3][4:])] = per_frame * frames * scale
            continue
        b = wb.batch(key, per_frame * frames * scale)
        if b is not None:
            out.append(b)
    for size, mc in sorted(intra.items()):
        b = wb.intra_merged(f"cu.intra_pred.{size}x{size}.all_modes", size, mc)
        if b is not None:
            out.append(b)
    if families is None or any(f in ("quant", "dequant_normal", "dst4x4", "nquant") for f in families):
        out += wb.quant_batches(census, frames, scale)
    for key, v in census.items():
        if key.startswith("scalar.") and key not in ("scalar.quant", "scalar.nquant", "scalar.dequant_normal",
                                                      "scalar.dst4x4", "scalar.idst4x4"):
            wb.skipped[key] = v * frames * scale
    out.sort(key=lambda b: -b.bytes)
    return out, wb
