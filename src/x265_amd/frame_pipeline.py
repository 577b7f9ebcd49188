"""The frame-parallel GPU step (bench.py --mode pipeline).

Per rank: the frames i = k * G + rank (k < F) of a G * F frame sequence, each
encoded band by band of CTU rows with the row dependencies of x265's frame
threads (pipeline.py): band b of frame i runs once the reference (frame i - 1,
encoded by rank (i - 1) mod G) has published the rows band b's motion search
reads; after it, band b is deblocked and band b - 1 SAO-filtered,
border-extended and published to the owner of frame i + 1 over RCCL.

The per-band work is the recorded x265 primitive census of the frame
(census_batches), its jobs split by the CTU row they belong to (`band_slices`),
followed by the f4 loop filters on the band (x265amd_deblock_rows /
_sao_apply_rows / _extend_border_rows).  Each (frame, band) is one captured
hipGraph (its launches spread over several streams); the exchange runs between
graph replays (an RCCL receive is a stream wait, not a host block).

The census jobs of band b read the reference slot of their frame only inside
rows <= r1 - 1 + refLagRows (CTU rows): the motion vectors of the census
workload stay within +-MV_RANGE (48) + 2 px plus the 8-tap window, less than the
57 + 7 px that refLagRows = 2 covers (frameencoder.cpp:114-119);
`check_reference_reach` verifies it on the built batches.

The reconstruction a real encoder writes (prediction + residual) is stood in for
by the band's source pixels, copied into the recon buffer before the loop filters.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .native import capture_graph
from .pipeline import BandPlan, RowExchange, run_frames
from .workload import (CENSUS_1080P, FrameSet, WorkloadBuilder, census_batches, group_launches, load_census)

# per-job device tensors of a Batch (everything else — planes, pools, slot buffers — is shared)
PER_JOB = {"aoff", "boff", "foff", "roff", "soff", "doff", "coeff", "co", "qo", "oo", "dlo", "nbo", "mode", "bf",
           "qb", "ad", "p0", "p1", "out", "sig", "cnt", "ro"}


def job_rows(b, fs: FrameSet):
    """(stored frame, luma picture row) of every job of batch b, from the offset of its
    block in a frame plane; jobs of pool-based batches (coefficients, intra
    neighbours) are spread evenly over the frames and rows in job order."""
    d = b.dev
    key = {"pixelcmp": ("a", "aoff"), "sad_multi": ("f", "foff"), "interp": ("s", "soff"),
           "blockop": ("a", "aoff"), "transform": ("s", "soff")}.get(b.kind)
    plane = d.get(key[0]) if key else None
    if plane is not None and (plane is fs.luma or plane is fs.resid or plane is fs.cb or plane is fs.cr):
        off = d[key[1]].cpu().numpy().astype(np.int64)
        per = len(off) // b.n
        off = off.reshape(b.n, per)[:, 0]
        chroma = plane is fs.cb or plane is fs.cr
        psize, stride, my = (fs.cplane_size, fs.cstride, fs.cmy) if chroma else (fs.plane_size, fs.stride, fs.my)
        frame = (off // psize) % fs.F
        y = (off % psize) // stride - my
        return frame, np.clip(y * (2 if chroma else 1), 0, fs.ph - 1)
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
    out = replace(b, n=n, dev=dev)
    out.bytes = b.bytes * n / b.n
    return out


def band_slices(batches, fs: FrameSet, plan: BandPlan, ctu: int = 64):
    """{(frame, band): [batch slices]} — every job of every batch in exactly one slice"""
    out = {}
    for b in batches:
        frame, y = job_rows(b, fs)
        band = np.minimum(y // ctu, plan.ctu_rows - 1) // plan.band_rows
        key = frame * plan.nbands + band
        if np.any(np.diff(key) < 0):
            order = np.argsort(key, kind="stable")
            b = _take(b, idx=order)
            key = key[order]
        bounds = np.searchsorted(key, np.arange(fs.F * plan.nbands + 1))
        for kk in range(fs.F * plan.nbands):
            lo, hi = int(bounds[kk]), int(bounds[kk + 1])
            if hi > lo:
                out.setdefault(divmod(kk, plan.nbands), []).append(_take(b, lo=lo, hi=hi))
    return out


def wave_delay(plan: BandPlan) -> int:
    """bands by which frame k + 1 trails frame k in the single-rank wavefront: its band b needs
    reference band need(b), which frame k publishes in the step of band need(b) + 1 (after that
    band's deblocking) or, for the last band, in its own step; the publication must come from an
    earlier step, so d > need(b) + 1 - b for every b"""
    return max(min(plan.need(b) + 1, plan.nbands - 1) + 1 - b for b in range(plan.nbands))


def step_slices(batches, fs: FrameSet, plan: BandPlan, d: int, ctu: int = 64):
    """{step: [batch slices]} of the wavefront schedule, step = frame * d + band: the (frame, band)
    pairs of one step are independent, so each census batch contributes ONE slice per step"""
    out = {}
    nsteps = (fs.F - 1) * d + plan.nbands
    for b in batches:
        frame, y = job_rows(b, fs)
        band = np.minimum(y // ctu, plan.ctu_rows - 1) // plan.band_rows
        key = frame * d + band
        if np.any(np.diff(key) < 0):
            order = np.argsort(key, kind="stable")
            b = _take(b, idx=order)
            key = key[order]
        bounds = np.searchsorted(key, np.arange(nsteps + 1))
        for st in range(nsteps):
            lo, hi = int(bounds[st]), int(bounds[st + 1])
            if hi > lo:
                out.setdefault(st, []).append(_take(b, lo=lo, hi=hi))
    return out


def check_reference_reach(slices, fs: FrameSet, plan: BandPlan, ctu: int = 64, taps: int = 8):
    """every reference read of band b's jobs lies in CTU rows <= rows(b)[1] - 1 + lag"""
    bad = []
    for (k, band), bs in slices.items():
        limit = (plan.rows(band)[1] + plan.lag) * ctu          # first luma row that is not yet published
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
                if not np.all(stored >= fs.F):
                    continue                                       # not a reference-slot read
                last = (off % psize) // stride - my + b.h + taps // 2   # last row the block (+ filter taps) reads
                if chroma:
                    last = 2 * last + 1
                if last.max() >= limit:
                    bad.append((b.name, k, band, int(last.max()), limit))
    return bad


class GpuFramePipeline:
    def __init__(self, prims, width, height, depth, frames_local, world, rank, census=None, band_rows=1,
                 streams=8, device="cuda", seed=11):
        import torch

        self.prims, self.world, self.rank, self.depth = prims, world, rank, depth
        self.F = frames_local
        self.total = frames_local * world
        ids = [k * world + rank for k in range(frames_local)]
        self.fs = fs = FrameSet(width, height, frames_local, depth, device=device, frame_ids=ids)
        ctu = 64
        self.plan = plan = BandPlan(ctu_rows=fs.ph // ctu, band_rows=band_rows)
        census = census or load_census(CENSUS_1080P)
        self.batches, self.wb = census_batches(fs, frames=frames_local, census=census,
                                               builder=WorkloadBuilder(fs, seed=seed + rank))
        self.slices = band_slices(self.batches, fs, plan, ctu)
        bad = check_reference_reach(self.slices, fs, plan, ctu)
        if bad:
            raise RuntimeError(f"census jobs read reference rows beyond refLagRows: {bad[:4]}")
        # recon buffers: work (deblocked in place) and final (SAO output, border-extended), per local frame
        mk = lambda ref: torch.empty_like(ref)
        self.work = [mk(fs.luma), mk(fs.cb), mk(fs.cr)]
        self.final = [mk(fs.luma), mk(fs.cb), mk(fs.cr)]
        for t in self.work + self.final:
            t.zero_()
        sizes = [fs.plane_size, fs.cplane_size, fs.cplane_size]
        self._sizes = sizes

        def frame_planes(bufs, k):
            return [bufs[p][k * sizes[p]:(k + 1) * sizes[p]] for p in range(3)]

        self.frame_planes = frame_planes
        src_planes = [fs.luma, fs.cb, fs.cr]
        regions = []
        for p in range(3):
            rows, stride, my = (fs.rows, fs.stride, fs.my) if p == 0 else (fs.crows, fs.cstride, fs.cmy)
            regions.append(lambda b, p=p, rows=rows, stride=stride, my=my: tuple(
                stride * r for r in self.plan.region(b, ctu, my, rows, shift=int(p > 0))))
        self.regions = regions

        def planes_of(kind, k):
            return frame_planes(self.final, k) if kind == "final" else frame_planes(src_planes, self.F + k)

        self._planes_of = planes_of
        self.ex = RowExchange(world, rank, plan, planes_of, regions, self.total)
        self._f4_setup(width, height, device)
        self.streams = [torch.cuda.Stream() for _ in range(max(1, streams))] if streams > 1 else []
        self.graphs = {}
        self.src_planes = src_planes

    # ---------------------------------------------------------------- f4 descriptors
    def _f4_setup(self, width, height, device):
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
            wk, fin = self.frame_planes(self.work, k), self.frame_planes(self.final, k)
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

    # ---------------------------------------------------------------- per-band work
    def _rows_px(self, b):
        r0, r1 = self.plan.rows(b)
        return r0 * 64, min(r1 * 64, self.H)

    def _finish(self, k, b, stream):
        y0, y1 = self._rows_px(b)
        last = b == self.plan.nbands - 1
        self.prims.sao_apply_rows(self.depth, [self.sao[k]], [self.plan.rows(b)[0], self.plan.rows(b)[1]], stream)
        self.prims.extend_border_rows(self.depth, self.bor[k], [y0, y1, b == 0, last] +
                                      [y0 // 2, y1 // 2, b == 0, last] * 2, stream)

    def band_work(self, k, b):
        """launch the whole work of (frame k, band b) on the current stream (graph-capturable)"""
        import torch

        cur = torch.cuda.current_stream()
        groups = self._groups.get((k, b), [])
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
        # the reconstruction of the band (stand-in: its source pixels) into the recon buffer
        y0, y1 = self._rows_px(b)
        fs = self.fs
        for p in range(3):
            stride, my, sh = (fs.stride, fs.my, 0) if p == 0 else (fs.cstride, fs.cmy, 1)
            s, e = (my + (y0 >> sh)) * stride, (my + (y1 >> sh)) * stride
            src = self.src_planes[p][k * self._sizes[p]:(k + 1) * self._sizes[p]]
            self.frame_planes(self.work, k)[p][s:e].copy_(src[s:e])
        h = ctypes.c_void_p(cur.cuda_stream)
        self.prims.deblock_rows(self.depth, [self.dbk[k]], [y0, y1], h)
        if b:
            self._finish(k, b - 1, h)
        if b == self.plan.nbands - 1:
            self._finish(k, b, h)

    def set_band_rows(self, band_rows: int):
        """re-slice the same census batches into bands of another height (single rank);
        call build() again afterwards"""
        assert self.world == 1
        self.plan = BandPlan(ctu_rows=self.fs.ph // 64, band_rows=band_rows)
        self.slices = band_slices(self.batches, self.fs, self.plan, 64)
        self.ex = RowExchange(1, 0, self.plan, self._planes_of, self.regions, self.total)
        self.graphs = {}

    def build(self, graphs=True, one_graph=False):
        """group each (frame, band)'s slices into launches and capture one hipGraph per band
        (one_graph, single rank only: the whole step — every band and the local row
        publications — as ONE graph)"""
        import torch

        self._groups = {kb: group_launches(bs) for kb, bs in self.slices.items()}
        for kb, gs in self._groups.items():
            for g in gs:
                g.run(self.prims)       # build grouped descriptor tables outside any capture
        torch.cuda.synchronize()
        if not graphs:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k in range(self.F):
                for b in range(self.plan.nbands):
                    self.band_work(k, b)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if one_graph and self.world == 1:
            g = torch.cuda.CUDAGraph()
            with capture_graph(g):
                self._eager_step()
            self.graphs["step"] = g
            torch.cuda.synchronize()
            return
        for k in range(self.F):
            for b in range(self.plan.nbands):
                g = torch.cuda.CUDAGraph()
                with capture_graph(g):
                    self.band_work(k, b)
                self.graphs[(k, b)] = g
        torch.cuda.synchronize()

    def _eager_step(self):
        run_frames(self.ex, self.F, self.band_work, lambda k, b: None, lambda k, b: None)

    # ---------------------------------------------------------------- single-rank wavefront
    def build_wave(self):
        """Single rank: schedule (frame k, band b) at step k * d + b (d = wave_delay) — the bands of
        consecutive frames that x265's frame threads run concurrently — so one step's census work
        of every frame goes out as one set of grouped launches and its loop filters as one call per
        kernel, and capture the whole sequence as ONE hipGraph.  Same results as step()."""
        import torch

        assert self.world == 1
        self.d = wave_delay(self.plan)
        self.nsteps = (self.F - 1) * self.d + self.plan.nbands
        self.wslices = step_slices(self.batches, self.fs, self.plan, self.d)
        self._wgroups = {st: group_launches(bs) for st, bs in self.wslices.items()}
        for gs in self._wgroups.values():
            for g in gs:
                g.run(self.prims)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._wave_all()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with capture_graph(g):
            self._wave_all()
        self.graphs = {"wave": g}
        torch.cuda.synchronize()

    def _wave_all(self):
        for st in range(self.nsteps):
            self._wave_step(st)

    def _wave_step(self, st):
        import torch

        plan, nb = self.plan, self.plan.nbands
        pairs = [(k, st - k * self.d) for k in range(self.F) if 0 <= st - k * self.d < nb]
        cur = torch.cuda.current_stream()
        groups = self._wgroups.get(st, [])
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
        fs = self.fs
        for k, b in pairs:                       # the bands' reconstruction (stand-in: source pixels)
            y0, y1 = self._rows_px(b)
            for p in range(3):
                stride, my, sh = (fs.stride, fs.my, 0) if p == 0 else (fs.cstride, fs.cmy, 1)
                s0, e0 = (my + (y0 >> sh)) * stride, (my + (y1 >> sh)) * stride
                src = self.src_planes[p][k * self._sizes[p]:(k + 1) * self._sizes[p]]
                self.frame_planes(self.work, k)[p][s0:e0].copy_(src[s0:e0])
        h = ctypes.c_void_p(cur.cuda_stream)
        rows = []
        for k, b in pairs:
            rows += list(self._rows_px(b))
        self.prims.deblock_rows(self.depth, [self.dbk[k] for k, _ in pairs], rows, h)
        # bands finished in this step: b - 1 of every pair, and b itself when it is the last band
        done = [(k, b - 1) for k, b in pairs if b] + [(k, b) for k, b in pairs if b == nb - 1]
        if done:
            self.prims.sao_apply_rows(self.depth, [self.sao[k] for k, _ in done],
                                      [r for _, c in done for r in plan.rows(c)], h)
            planes, brows = [], []
            for k, c in done:
                y0, y1 = self._rows_px(c)
                first, last = int(c == 0), int(c == nb - 1)
                planes += self.bor[k]
                brows += [y0, y1, first, last] + [y0 // 2, y1 // 2, first, last] * 2
            self.prims.extend_border_rows(self.depth, planes, brows, h)
            for k, c in done:
                self.ex.publish(k, c)

    def wave_launches_per_step(self):
        return sum(len(v) for v in self._wgroups.values()) + 3 * self.nsteps

    def step(self):
        """one sequence of G * F frames: this rank's F frames with the row exchange"""
        if "wave" in self.graphs:
            self.graphs["wave"].replay()
            return
        if "step" in self.graphs:
            self.graphs["step"].replay()
            return

        def encode(k, b):
            g = self.graphs.get((k, b))
            if g is not None:
                g.replay()
            else:
                self.band_work(k, b)
        run_frames(self.ex, self.F, encode, lambda k, b: None, lambda k, b: None)

    @property
    def launches_per_step(self):
        return sum(len(v) for v in self._groups.values()) + self.F * (2 * self.plan.nbands + 2 * self.plan.nbands)

    @property
    def calls(self):
        return sum(b.n for b in self.batches)

    @property
    def bytes(self):
        return sum(b.bytes for b in self.batches)
