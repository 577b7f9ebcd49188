"""The frame-parallel GPU step (bench.py --mode pipeline).

Per rank: the frames j with j mod G == rank of a G * F frame sequence (closed segments of the
--preset medium GOP, pipeline.Schedule), each encoded band by band of CTU rows in the steps the
schedule gives: a band runs once every reference it reads has published the rows it needs;
after it the band is deblocked and the bands that became final are SAO-filtered,
border-extended and sent to the reference stores of every rank that owns a frame referencing
them (RCCL P2P; a local copy for the rank's own consumers).

The per-band work is the recorded x265 primitive census of the frame (census_batches), its jobs
split by the (frame, band) they belong to and regrouped per STEP: every census batch contributes
one slice per step (all frames and bands the step holds), so a step is one set of grouped
launches whatever the number of frames in it, followed by the f4 loop filters of the step
(x265amd_deblock_rows / _sao_apply_rows / _extend_border_rows, one call per kernel for all its
bands).  Census jobs of a frame read its references (L0 and L1) from the rank's reference store;
`check_reference_reach` verifies that no job reads a reference row beyond refLagRows.

On one rank the whole sequence (steps + local reference copies) is ONE hipGraph; with several
ranks (or the native exchange) each step is a graph replay followed by the step's exchange:
torch.distributed P2P batches, or one x265amd_exchange call (csrc/exchange.cpp, RCCL groups
enqueued on the stream) with exchange="rccl".

The reconstruction a real encoder writes (prediction + residual) is stood in for by the band's
source pixels, copied into the recon buffer before the loop filters.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .native import capture_graph
from .pipeline import BandPlan, RefExchange, Schedule
from .workload import CENSUS_1080P, FrameSet, WorkloadBuilder, census_batches, group_launches, load_census

# per-job device tensors of a Batch (everything else — planes, pools, slot buffers — is shared)
PER_JOB = {"aoff", "boff", "foff", "roff", "soff", "doff", "coeff", "co", "qo", "oo", "dlo", "nbo", "mode", "bf",
           "qb", "ad", "p0", "p1", "out", "sig", "cnt", "ro"}


def job_rows(b, fs: FrameSet):
    """(stored frame, luma picture row) of every job of batch b: the block the job codes (recorded
    by the workload builder); jobs of pool-based batches (coefficients, intra neighbours) are
    spread evenly over the frames and rows in job order"""
    if b.pos is not None:
        f, y = b.pos
        return np.asarray(f, np.int64), np.clip(np.asarray(y, np.int64), 0, fs.ph - 1)
    j = np.arange(b.n, dtype=np.int64)
    frame = j * fs.F // b.n
    start = (frame * b.n + fs.F - 1) // fs.F
    cnt = np.bincount(frame, minlength=fs.F)[frame]
    return frame, (j - start) * fs.ph // np.maximum(cnt, 1)


def _take(b, idx=None, lo=None, hi=None):
    """copy of batch b restricted to jobs idx (a permutation) or [lo, hi)"""
    from dataclasses import replace

    dev = {}
    for k, t in b.dev.items():
        if k in PER_JOB and t is not None and t.numel() % b.n == 0:
            per = t.numel() // b.n
            v = t.view(b.n, per)
            if idx is not None:
                import torch

                v = v[torch.as_tensor(idx, device=t.device)]
            else:
                v = v[lo:hi]
            dev[k] = v.reshape(-1).contiguous() if idx is not None else v.reshape(-1)
        else:
            dev[k] = t
    n = b.n if idx is not None else hi - lo
    pos = None
    if b.pos is not None:
        pos = tuple(np.asarray(a)[idx] if idx is not None else np.asarray(a)[lo:hi] for a in b.pos)
    out = replace(b, n=n, dev=dev, pos=pos)
    out.bytes = b.bytes * n / b.n
    return out


def reads_store(b, fs: FrameSet) -> np.ndarray:
    """per job of batch b: does it read a reference picture (the rank's reference store)?"""
    out = np.zeros(b.n, bool)
    for key, plane_key in (("aoff", "a"), ("boff", "b"), ("roff", "r"), ("soff", "s"), ("foff", "f")):
        t, pl = b.dev.get(key), b.dev.get(plane_key)
        if t is None or pl is None or not (pl is fs.luma or pl is fs.cb or pl is fs.cr):
            continue
        psize = fs.plane_size if pl is fs.luma else fs.cplane_size
        off = t.cpu().numpy().astype(np.int64)
        per = len(off) // b.n
        out |= (off.reshape(b.n, per) // psize >= fs.F).any(axis=1)
    return out


def store_slots(b, fs: FrameSet) -> np.ndarray:
    """per job of batch b and per read entry: the reference-store slot it reads (-1: not the store);
    shape (n, entries)"""
    cols = []
    for key, plane_key in (("aoff", "a"), ("boff", "b"), ("roff", "r"), ("soff", "s"), ("foff", "f")):
        t, pl = b.dev.get(key), b.dev.get(plane_key)
        if t is None or pl is None or not (pl is fs.luma or pl is fs.cb or pl is fs.cr):
            continue
        psize = fs.plane_size if pl is fs.luma else fs.cplane_size
        slot = t.cpu().numpy().astype(np.int64) // psize
        slot = slot.reshape(b.n, -1)
        cols.append(np.where(slot >= fs.F, slot, -1))
    return np.concatenate(cols, axis=1) if cols else np.full((b.n, 1), -1, np.int64)


def keyed_slices(batches, fs: FrameSet, key_of, nkeys: int, ctu: int, plan: BandPlan):
    """{key: [batch slices]}: every job of every batch in exactly one slice; key_of(batch, frame, band)
    (numpy arrays per job) gives the job's key"""
    out = {}
    for b in batches:
        frame, y = job_rows(b, fs)
        band = np.minimum(y // ctu, plan.ctu_rows - 1) // plan.band_rows
        key = key_of(b, frame, band)
        if np.any(np.diff(key) < 0):
            # reorder the batch's own jobs (descriptors AND per-job outputs), so the slices below are
            # views of it and their results land in the batch's outputs, where verification reads them
            order = np.argsort(key, kind="stable")
            p = _take(b, idx=order)
            b.dev, b.pos = p.dev, p.pos
            key = key[order]
        bounds = np.searchsorted(key, np.arange(nkeys + 1))
        for kk in range(nkeys):
            lo, hi = int(bounds[kk]), int(bounds[kk + 1])
            if hi > lo:
                out.setdefault(kk, []).append(_take(b, lo=lo, hi=hi))
    return out


def check_reference_reach(slices_by_fb, fs: FrameSet, plan: BandPlan, ctu: int = 64, taps: int = 8):
    """every reference read of band b's jobs lies in CTU rows < rows(b)[1] - 1 + lag, i.e. within
    the rows frameencoder.cpp:526-527 lets row r1 - 1 see; reads of the rank's own pictures (an I
    frame's jobs) are not reference reads and are skipped entry by entry"""
    bad = []
    for (k, band), bs in slices_by_fb.items():
        limit = plan.reach_rows(band) * ctu                    # first luma row not yet published
        for b in bs:
            for key, plane_key in (("boff", "b"), ("roff", "r"), ("soff", "s")):
                t = b.dev.get(key)
                pl = b.dev.get(plane_key)
                if t is None or pl is None or not (pl is fs.luma or pl is fs.cb or pl is fs.cr):
                    continue
                off = t.cpu().numpy().astype(np.int64)
                chroma = pl is not fs.luma
                psize, stride, my = (fs.cplane_size, fs.cstride, fs.cmy) if chroma else (fs.plane_size, fs.stride, fs.my)
                stored = off // psize
                sel = stored >= fs.F                               # entries that read the reference store
                if not sel.any():
                    continue
                last = (off[sel] % psize) // stride - my + b.h + taps // 2   # last row the block (+ filter taps) reads
                if chroma:
                    last = 2 * last + 1
                if last.max() >= limit:
                    bad.append((b.name, k, band, int(last.max()), limit))
    return bad


class GpuFramePipeline:
    def __init__(self, prims, width, height, depth, frames_local, world, rank, census=None, band_rows=None,
                 segment_frames=None, streams=8, device="cuda", seed=11, early_independent=True, exchange="torch",
                 inplace_store=True, job_wait="band", background=False, recon="tu"):
        """exchange: "torch" (torch.distributed P2P batches; local copies on the stream) or "rccl" (the
        native communicator, x265amd_exchange; with inplace_store=False a rank's own reference pictures
        are finished in their own buffers and reach its store as loop-back transfers — the one-GPU check
        of the native path).
        job_wait: "band" — a job that reads a reference waits for its band's step (x265: a CTU row waits
        until every reference has published its rows, frameencoder.cpp:516-531); "reference" — it waits
        only for the band of the ONE reference picture it reads (the data it actually depends on).
        background (one rank, whole sequence in one graph): the jobs that read no reference run on
        background streams from the start, in step order, and a step's loop filters wait only for the
        background work of THAT step's pictures — instead of all reference-free work joining step 0.
        recon: "tu" — every band's reconstruction is coded by the fused TU pipeline (f3,
        x265amd_tu_pipeline: residual -> DCT -> quant -> dequant -> iDCT -> prediction + residual) from
        a motion-compensated prediction out of the picture's first reference as the reference store
        holds it (the producer's final, filtered band), so each picture's reconstruction depends on its
        references' published bands; "source" — the source pixels stand in for it (rounds 1-3)."""
        import torch

        self.early_independent = early_independent
        self.exchange_kind, self.inplace_store, self.job_wait = exchange, inplace_store, job_wait
        self.background = background
        self.prims, self.world, self.rank, self.depth = prims, world, rank, depth
        self.F = frames_local
        self.total = frames_local * world
        ctu = 64
        ph = (height + ctu - 1) // ctu * ctu
        self.plan = plan = BandPlan(ctu_rows=ph // ctu, band_rows=band_rows or ph // ctu)
        self.segment_frames = segment_frames or frames_local
        self.sched = s = Schedule(self.total, world, plan, segment_frames=self.segment_frames)
        self.local = s.local_frames(rank)
        assert len(self.local) == frames_local
        self.kof = {j: k for k, j in enumerate(self.local)}
        # the reference store: every picture this rank's frames reference, plus this rank's own reference
        # pictures, whose final reconstruction is written straight into their store slot (local users
        # then read it in place: no copy)
        self.store = sorted(set(s.store_frames(rank)) | {j for j in self.local if s.is_ref[j]})
        self.sof = {r: frames_local + i for i, r in enumerate(self.store)}
        self.fs = fs = FrameSet(width, height, frames_local, depth, device=device,
                                frame_ids=[s.poc[j] for j in self.local], store_ids=[s.poc[r] for r in self.store],
                                ref_slots=[[self.sof[r] for r in s.refs[j]] for j in self.local])
        census = census or load_census(CENSUS_1080P)
        self.batches, self.wb = census_batches(fs, frames=frames_local, census=census,
                                               builder=WorkloadBuilder(fs, seed=seed + rank))
        nb = plan.nbands
        self.slices = {divmod(kk, nb): v for kk, v in
                       keyed_slices(self.batches, fs, lambda bt, f, b: f * nb + b, frames_local * nb, ctu,
                                    plan).items()}
        bad = check_reference_reach(self.slices, fs, plan, ctu)
        if bad:
            raise RuntimeError(f"census jobs read reference rows beyond refLagRows: {bad[:4]}")
        # recon buffers: work (deblocked in place) and final (SAO output, border-extended), per local frame
        mk = lambda ref: torch.empty_like(ref[:frames_local * (ref.numel() // fs.stored)])
        self.work = [mk(fs.luma), mk(fs.cb), mk(fs.cr)]
        self.final = [mk(fs.luma), mk(fs.cb), mk(fs.cr)]
        for t in self.work + self.final:
            t.zero_()
        sizes = [fs.plane_size, fs.cplane_size, fs.cplane_size]
        self._sizes = sizes

        def frame_planes(bufs, k):
            return [bufs[p][k * sizes[p]:(k + 1) * sizes[p]] for p in range(3)]

        self.frame_planes = frame_planes
        self.src_planes = src_planes = [fs.luma, fs.cb, fs.cr]
        regions = []
        for p in range(3):
            rows, stride, my = (fs.rows, fs.stride, fs.my) if p == 0 else (fs.crows, fs.cstride, fs.cmy)
            regions.append(lambda b, p=p, rows=rows, stride=stride, my=my: tuple(
                stride * r for r in self.plan.region(b, ctu, my, rows, shift=int(p > 0))))
        self.regions = regions

        def planes_of(kind, j):
            return self.final_planes(self.kof[j]) if kind == "final" else frame_planes(src_planes, self.sof[j])

        if exchange == "rccl":
            from .pipeline import Comm, RcclExchange

            self.comm = Comm(world, rank)
            self.ex = RcclExchange(s, rank, planes_of, regions, self.comm, loopback=not inplace_store)
        elif exchange == "torch":
            self.ex = RefExchange(s, rank, planes_of, regions)
        else:
            raise ValueError(f"exchange {exchange!r}")
        self._f4_setup(width, height, device)
        self.recon = recon
        if recon == "tu":
            self.tu = self.tu_setup(lambda k, p: self._store_pred(k, p), self.work)
        elif recon != "source":
            raise ValueError(f"recon {recon!r}")
        self.streams = [torch.cuda.Stream() for _ in range(max(1, streams))] if streams > 1 else []
        self.bg_streams = []
        self._bgroups, self._bg_events, self.bg = {}, {}, False
        self.graphs = {}
        self._pool = None
        self.comm = getattr(self, "comm", None)

    # ---------------------------------------------------------------- teardown
    def _drop_graphs(self):
        """reset every captured graph after the device has drained (a graph's replay may still run on a
        background stream); graphs go before the buffers they read, never in reference-cycle order"""
        import torch

        if self.graphs:
            torch.cuda.synchronize()
            for g in self.graphs.values():
                g.reset()
        self.graphs = {}
        self._pool = None

    def close(self):
        """explicit teardown: drain every stream, reset the graphs (which releases their shared pool only
        now that nothing can replay them), close the communicator, then drop the descriptor tables and
        buffers the graphs pointed into.  The pipeline's lambdas reference the pipeline, so without this
        it dies as a reference cycle, in whatever order and at whatever later moment the cyclic GC picks."""
        import torch

        if getattr(self, "_closed", False):
            return
        self._closed = True
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        self._drop_graphs()
        if self.comm is not None:
            self.comm.close()
        for name in ("_sgroups", "_bgroups", "step_slices", "slices", "tu", "_bg_events"):
            if hasattr(self, name):
                setattr(self, name, {})
        for name in ("batches", "_tu_keep", "dbk", "sao", "bor", "work", "final", "streams", "bg_streams"):
            if hasattr(self, name):
                setattr(self, name, [])
        self.regions = self.frame_planes = self.ex = None
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def final_planes(self, k, final=None):
        """where local frame k's final reconstruction lives: its store slot for a reference picture,
        else the frame's own final buffer"""
        j = self.local[k]
        if final is None and self.inplace_store and j in self.sof:
            return self.frame_planes(self.src_planes, self.sof[j])
        return self.frame_planes(self.final if final is None else final, k)

    # ---------------------------------------------------------------- f3 reconstruction
    TU_QP = 30

    def mv_of(self, k):
        """integer luma displacement of local picture k's prediction from its first reference: the
        synthetic source pans (+2, +1) pixels per picture (synth.py), so a block at (x, y) of POC p was at
        (x + 2 d, y + d) in POC p - d"""
        j = self.local[k]
        refs = self.sched.refs[j]
        if not refs:
            return None
        d = self.sched.poc[j] - self.sched.poc[refs[0]]
        return 2 * d, d

    def _store_pred(self, k, p):
        """(base tensor, element offset of the picture) of local picture k's prediction source for plane p:
        its first reference as this rank's reference store holds it, or the flat plane (I picture)"""
        refs = self.sched.refs[self.local[k]]
        if not refs:
            return self._flat[p], 0
        return self.src_planes[p], self.sof[refs[0]] * self._sizes[p]

    def tu_setup(self, pred_of, recon_planes):
        """TU descriptors of every (local picture, band): 8x8 luma and 4x4 chroma TUs tiling the band,
        fenc = the picture's source, pred = pred_of(k, plane) displaced by mv_of(k) (a flat mid-grey plane
        for an I picture), recon = the picture's slot of recon_planes; one TuBatch per (picture, band,
        plane), each with its own coefficient scratch"""
        import torch

        from .native import TuBatch

        fs, dev = self.fs, self.fs.luma.device
        if not hasattr(self, "_flat"):
            mid = 1 << (self.depth - 1)
            self._flat = [torch.full((self._sizes[p],), mid, dtype=fs.luma.dtype, device=dev) for p in range(3)]
        geo = [(fs.stride, fs.mx, fs.my, self.W, self.H, 3), (fs.cstride, fs.cmx, fs.cmy, self.W // 2, self.H // 2, 2),
               (fs.cstride, fs.cmx, fs.cmy, self.W // 2, self.H // 2, 2)]
        keep, out = [], {}
        nb = self.plan.nbands
        i64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.int64)).to(dev)
        for k in range(self.F):
            j = self.local[k]
            intra = not self.sched.refs[j]
            mv = self.mv_of(k) or (0, 0)
            for b in range(nb):
                y0, y1 = self._rows_px(b)
                arr = (TuBatch * 3)()
                for p, (stride, mx, my, w, h, lg) in enumerate(geo):
                    n_ = 1 << lg
                    ys = np.arange((y0 >> (p > 0)), (y1 >> (p > 0)), n_)
                    xs = np.arange(0, w, n_)
                    yy, xx = np.meshgrid(ys, xs, indexing="ij")
                    yy, xx = yy.reshape(-1), xx.reshape(-1)
                    org = (my + yy) * stride + mx + xx
                    dx, dy = (mv[0], mv[1]) if p == 0 else (mv[0] // 2, mv[1] // 2)
                    pbase, poff = pred_of(k, p)
                    fo = i64(k * self._sizes[p] + org)
                    po = i64(poff + org + dy * stride + dx)
                    ro = i64(k * self._sizes[p] + org)
                    m = len(org)
                    co = i64(np.arange(m) * n_ * n_)
                    coef = torch.empty(m * n_ * n_, dtype=torch.int16, device=dev)
                    sig = torch.empty(m, dtype=torch.int32, device=dev)
                    qp = torch.full((m,), self.TU_QP, dtype=torch.uint8, device=dev)
                    keep += [fo, po, ro, co, coef, sig, qp]
                    arr[p] = TuBatch(lg, m, int(p == 0), int(intra), int(intra), 1, self.src_planes[p].data_ptr(), stride,
                                     fo.data_ptr(), pbase.data_ptr(), stride, po.data_ptr(), None, 0, None,
                                     coef.data_ptr(), co.data_ptr(), recon_planes[p].data_ptr(), stride, ro.data_ptr(),
                                     sig.data_ptr(), qp.data_ptr(), None)
                out[(k, b)] = arr
        self._tu_keep = getattr(self, "_tu_keep", []) + keep
        return out

    # ---------------------------------------------------------------- f4 descriptors
    def _f4_setup(self, width, height, device, work=None, final=None):
        """loop-filter descriptors of every local frame: deblock in place in `work`, SAO into the final
        planes (final_planes, or `final` for every frame when given), border extension there"""
        import torch

        from .caller_bench import _SAO, _UNIT
        from .native import BorderPlane, DeblockFrame, SaoFrame

        fs = self.fs
        rng = np.random.default_rng(9)
        hu, wu = height // 4, width // 4
        U = np.zeros((hu, wu), _UNIT)
        cu = rng.random((hu // 4 + 1, wu // 4 + 1)) < 0.25
        U["cu_log2"], U["tu_log2"], U["qp"] = 4, 3, 32
        U["flags"] = np.repeat(np.repeat(cu, 4, 0), 4, 1)[:hu, :wu].astype(np.uint8) | (rng.random((hu, wu)) < 0.5) * 2
        U["ref_idx"][..., 0], U["ref_idx"][..., 1] = 0, -1
        mv = np.repeat(np.repeat(rng.integers(-6, 7, (hu // 4 + 1, wu // 4 + 1, 2)), 4, 0), 4, 1)[:hu, :wu]
        U["mv"][..., 0, :] = mv
        nctu = (fs.pw // 64) * (fs.ph // 64)
        prm = np.zeros(3 * nctu, _SAO)
        prm["type"] = rng.integers(-1, 5, 3 * nctu)
        prm["type"][2 * nctu:] = prm["type"][nctu:2 * nctu]
        prm["band"] = rng.integers(0, 32, 3 * nctu)
        prm["offset"] = rng.integers(-3, 4, (3 * nctu, 4))
        self.units = torch.from_numpy(U.view(np.uint8).reshape(hu, -1).copy()).to(device)
        self.sao_prm = torch.from_numpy(prm.view(np.uint8).copy()).to(device)
        es = self.fs.luma.element_size()

        def org(t, p):
            stride, mx, my = (fs.stride, fs.mx, fs.my) if p == 0 else (fs.cstride, fs.cmx, fs.cmy)
            return t.data_ptr() + (my * stride + mx) * es

        self.dbk, self.sao, self.bor = [], [], []
        for k in range(self.F):
            wk, fin = self.frame_planes(work if work is not None else self.work, k), self.final_planes(k, final)
            d = DeblockFrame()
            d.width, d.height, d.is_p = width, height, 1
            for p in range(3):
                d.plane[p] = org(wk[p], p)
            d.stride, d.cstride, d.units, d.unit_stride = fs.stride, fs.cstride, self.units.data_ptr(), wu
            self.dbk.append(d)
            a = SaoFrame()
            a.width, a.height, a.ctu_log2, a.luma_on, a.chroma_on = width, height, 6, 1, 1
            for p in range(3):
                a.src[p], a.dst[p] = org(wk[p], p), org(fin[p], p)
            a.stride, a.cstride, a.params = fs.stride, fs.cstride, self.sao_prm.data_ptr()
            self.sao.append(a)
            bps = []
            for p in range(3):
                bp = BorderPlane()
                bp.plane = org(fin[p], p)
                bp.stride = fs.stride if p == 0 else fs.cstride
                bp.width, bp.height = (width, height) if p == 0 else (width // 2, height // 2)
                bp.margin_x, bp.margin_y = (fs.mx, fs.my) if p == 0 else (fs.cmx, fs.cmy)
                bps.append(bp)
            self.bor.append(bps)
        self.W, self.H = width, height

    # ---------------------------------------------------------------- steps
    def _rows_px(self, b):
        r0, r1 = self.plan.rows(b)
        return r0 * 64, min(r1 * 64, self.H)

    def build(self, graphs=True):
        """regroup the census slices per step (one slice per census batch per step, grouped launches),
        and capture the work: one graph for the whole sequence on one rank, one per step otherwise"""
        import torch

        s, nb = self.sched, self.plan.nbands
        step_of = np.array([[s.step[j, b] for b in range(nb)] for j in self.local], np.int64)
        # a job waits for its band's step only if it reads a reference picture: x265's frame threads wait
        # on reference rows and on nothing else (frameencoder.cpp:516-531); the census jobs that read no
        # reference (transforms, quant, intra, residual and current-picture block ops, an I picture's
        # jobs) carry no cross-frame dependency and go out with the first step
        one_graph = self.world == 1 and self.exchange_kind == "torch"
        self.bg = self.background and self.job_wait == "band" and graphs
        if self.bg:
            # reference-reading jobs keyed by their band's step (the step lanes), the others by
            # nsteps + their band's step (the background streams)
            key_of = lambda bt, f, b: np.where(reads_store(bt, self.fs), step_of[f, b], s.nsteps + step_of[f, b])
            sl = keyed_slices(self.batches, self.fs, key_of, 2 * s.nsteps, 64, self.plan)
            self.step_slices = {k: v for k, v in sl.items() if k < s.nsteps}
            self._bgroups = {k - s.nsteps: group_launches(v) for k, v in sl.items() if k >= s.nsteps}
            self.bg_streams = [torch.cuda.Stream() for _ in range(max(1, len(self.streams) // 2))]
        elif self.job_wait == "reference":
            # the step after the reference band the job reads was published (for band b: the band holding
            # row r1 - 2 + lag of that reference, BandPlan.need)
            need = np.array([self.plan.need(b) for b in range(nb)], np.int64)
            pub = np.array([[s.pub_step(r, c) for c in range(nb)] for r in self.store], np.int64)
            F = self.fs.F

            def key_of(bt, f, b):
                slots = store_slots(bt, self.fs)
                k = np.where(slots >= 0, pub[np.clip(slots - F, 0, None), need[b][:, None]] + 1, 0).max(axis=1)
                return np.minimum(k, step_of[f, b])
        elif self.early_independent:
            key_of = lambda bt, f, b: np.where(reads_store(bt, self.fs), step_of[f, b], 0)
        else:
            key_of = lambda bt, f, b: step_of[f, b]
        if not self.bg:
            self.step_slices = keyed_slices(self.batches, self.fs, key_of, s.nsteps, 64, self.plan)
        self._sgroups = {st: group_launches(bs) for st, bs in self.step_slices.items()}
        for gs in list(self._sgroups.values()) + list(self._bgroups.values()):
            for g in gs:
                g.run(self.prims)       # build grouped descriptor tables outside any capture
        torch.cuda.synchronize()
        self._drop_graphs()
        if not graphs:
            return
        # every graph of this pipeline allocates from one private pool: a tensor first allocated inside one
        # capture and read by another graph (or a background replay) lives as long as the pool, which is
        # released only after ALL the pipeline's graphs are reset (close())
        self._pool = torch.cuda.graph_pool_handle()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):                        # warm-up pass (allocations, descriptor uploads)
            self._run_all(exchange=self.world == 1 and self.exchange_kind == "torch")
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if self.world == 1 and self.exchange_kind == "torch":
            g = torch.cuda.CUDAGraph()
            with capture_graph(g, pool=self._pool):
                self._run_all(exchange=True)                 # exchange = local copies: capturable
            self.graphs["all"] = g
        elif not self.bg:
            for st in range(s.nsteps):
                g = torch.cuda.CUDAGraph()
                with capture_graph(g, pool=self._pool):
                    self._step_work(st)
                self.graphs[st] = g
        else:
            # per step: the step's reference-reading work, its loop filters, and its background work as
            # three graphs; step() replays the background graphs on their own stream and joins each into
            # the main stream right before that step's filters
            for st in range(s.nsteps):
                for kind, fn, need in (("c", self._census_work, bool(self._sgroups.get(st))),
                                       ("f", self._filter_work, st == 0 or bool(s.items(self.rank, st))
                                        or bool(s.finals(self.rank, st))),
                                       ("b", self._bg_graph_work, bool(self._bgroups.get(st)))):
                    if need:
                        g = torch.cuda.CUDAGraph()
                        with capture_graph(g, pool=self._pool):
                            fn(st)
                        self.graphs[(kind, st)] = g
            self._bg_main = torch.cuda.Stream()
            self._bg_step_events = [torch.cuda.Event() for _ in range(s.nsteps)]
        torch.cuda.synchronize()

    def _run_all(self, exchange):
        import torch

        cur = torch.cuda.current_stream()
        self._bg_events = {}
        if self.bg:
            # every step's background work, in step order, spread over the background streams (balanced by
            # bytes); one event per (step, stream) for the step's loop filters to wait on
            load = [0.0] * len(self.bg_streams)
            for s_ in self.bg_streams:
                s_.wait_stream(cur)
            for st in range(self.sched.nsteps):
                used = set()
                for g in self._bgroups.get(st, []):
                    i = min(range(len(self.bg_streams)), key=lambda j: load[j])
                    g.run(self.prims, ctypes.c_void_p(self.bg_streams[i].cuda_stream))
                    load[i] += g.bytes
                    used.add(i)
                evs = []
                for i in sorted(used):
                    ev = torch.cuda.Event()
                    ev.record(self.bg_streams[i])
                    evs.append(ev)
                self._bg_events[st] = evs
        for st in range(self.sched.nsteps):
            self._step_work(st)
            if exchange:
                self.ex.exchange(st)
        for s_ in self.bg_streams:
            cur.wait_stream(s_)

    def _bg_graph_work(self, st):
        """step st's background work forked over the background streams and joined back into the current
        stream (the body of one background graph)"""
        import torch

        cur = torch.cuda.current_stream()
        load = [0.0] * len(self.bg_streams)
        used = set()
        for g in self._bgroups.get(st, []):
            i = min(range(len(self.bg_streams)), key=lambda j: load[j])
            if i not in used:
                self.bg_streams[i].wait_stream(cur)
                used.add(i)
            g.run(self.prims, ctypes.c_void_p(self.bg_streams[i].cuda_stream))
            load[i] += g.bytes
        for i in used:
            cur.wait_stream(self.bg_streams[i])

    def _step_work(self, st):
        """launch the whole work of step st on the current stream (graph-capturable)"""
        import torch

        self._census_work(st)
        cur = torch.cuda.current_stream()
        for ev in self._bg_events.get(st, []) if self.bg else []:
            cur.wait_event(ev)
        self._filter_work(st)

    def _census_work(self, st):
        """step st's census slices forked over the step lanes and joined into the current stream"""
        import torch

        cur = torch.cuda.current_stream()
        groups = self._sgroups.get(st, [])
        if self.streams:
            lanes = [[] for _ in self.streams]
            load = [0.0] * len(self.streams)
            for g in groups:
                i = min(range(len(self.streams)), key=lambda j: load[j])
                lanes[i].append(g)
                load[i] += g.bytes
            for s_, lst in zip(self.streams, lanes):
                if not lst:
                    continue
                s_.wait_stream(cur)
                h = ctypes.c_void_p(s_.cuda_stream)
                for g in lst:
                    g.run(self.prims, h)
            for s_, lst in zip(self.streams, lanes):
                if lst:
                    cur.wait_stream(s_)
        else:
            for g in groups:
                g.run(self.prims)

    def _filter_work(self, st):
        """step st's loop filters on the current stream: deblocking of the step's bands, SAO and border
        extension of the bands that became final"""
        import torch

        s, plan = self.sched, self.plan
        items = s.items(self.rank, st)
        cur = torch.cuda.current_stream()
        if self.recon == "source" and st == 0:
            # the reconstruction of every band (stand-in: the source pixels), written before any band is
            # deblocked: one copy per plane for all local frames
            for p in range(3):
                n = self.F * self._sizes[p]
                self.work[p][:n].copy_(self.src_planes[p][:n])
        if self.recon == "tu" and items:
            # the step's bands coded: prediction from the reference store (final bands published in
            # earlier steps), residual through the fused TU pipeline, reconstruction into `work`
            from .native import TuBatch

            arrs = [self.tu[(self.kof[j], b)] for j, b in items]
            grp = (TuBatch * (3 * len(arrs)))(*[x for a in arrs for x in a])
            self.prims.tu_pipeline_grouped(self.depth, grp, ctypes.c_void_p(cur.cuda_stream))
        h = ctypes.c_void_p(cur.cuda_stream)
        if items:
            rows = []
            for j, b in items:
                rows += list(self._rows_px(b))
            self.prims.deblock_rows(self.depth, [self.dbk[self.kof[j]] for j, _ in items], rows, h)
        done = s.finals(self.rank, st)           # bands that became final in this step
        if done:
            self.prims.sao_apply_rows(self.depth, [self.sao[self.kof[j]] for j, _ in done],
                                      [r for _, c in done for r in plan.rows(c)], h)
            planes, brows = [], []
            nb = plan.nbands
            for j, c in done:
                y0, y1 = self._rows_px(c)
                first, last = int(c == 0), int(c == nb - 1)
                planes += self.bor[self.kof[j]]
                brows += [y0, y1, first, last] + [y0 // 2, y1 // 2, first, last] * 2
            self.prims.extend_border_rows(self.depth, planes, brows, h)

    def reset_stores(self):
        """put the reference stores back to the unfiltered source pictures they start with (tests: a
        job that reads a reference before its publication then sees different pixels)"""
        import torch

        fs = self.fs
        for dev, key, size in ((fs.luma, "Y", fs.plane_size), (fs.cb, "U", fs.cplane_size), (fs.cr, "V", fs.cplane_size)):
            lo = self.F * size
            dev[lo:].copy_(torch.from_numpy(fs.host[key][lo:]).to(dev.device))
        torch.cuda.synchronize()

    def step(self):
        """one sequence: this rank's frames in the schedule's steps, with the reference exchange"""
        if "all" in self.graphs:
            self.graphs["all"].replay()
            return
        if self.bg and self.graphs:
            import torch

            cur, bgs = torch.cuda.current_stream(), self._bg_main
            bgs.wait_stream(cur)
            with torch.cuda.stream(bgs):
                for st in range(self.sched.nsteps):
                    g = self.graphs.get(("b", st))
                    if g is not None:
                        g.replay()
                    self._bg_step_events[st].record(bgs)
            for st in range(self.sched.nsteps):
                for kind in ("c", "f"):
                    if kind == "f":
                        cur.wait_event(self._bg_step_events[st])
                    g = self.graphs.get((kind, st))
                    if g is not None:
                        g.replay()
                self.ex.exchange(st)
            cur.wait_stream(bgs)
            return
        for st in range(self.sched.nsteps):
            g = self.graphs.get(st)
            if g is not None:
                g.replay()
            else:
                self._step_work(st)
            self.ex.exchange(st)

    @property
    def launches_per_step(self):
        s = self.sched
        filt = sum((1 if s.items(self.rank, st) else 0) + 2 * (1 if s.finals(self.rank, st) else 0)
                   for st in range(s.nsteps))
        return sum(len(v) for v in self._sgroups.values()) + sum(len(v) for v in self._bgroups.values()) + filt

    @property
    def calls(self):
        return sum(b.n for b in self.batches)

    @property
    def bytes(self):
        return sum(b.bytes for b in self.batches)
