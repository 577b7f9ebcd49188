"""Frame-parallel shard with reconstructed-row exchange (src/x265_amd/pipeline.py), on CPU.

Multi-process gloo runs at world 1, 2 and 4 of the same pipeline bench.py drives
over RCCL, with a CPU stand-in for the per-band work that has the encoder's row
dependencies:

  encode(k, b)  reads reference rows up to r1 - 1 + refLagRows CTU rows (ME window);
  deblock(k, b) rewrites the 3 rows on each side of the band's top edge;
  finish(k, b)  reads one row of band b + 1 (SAO), then extends the borders.

Checked: every rank's reference slots hold, byte for byte, the producer's final
frames (margins included); no band is encoded before the reference rows it reads
are in place (reference slots start poisoned with -1, and the encoder asserts it
never sees one); and every frame's output equals a one-rank run.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from src.x265_amd.pipeline import BandPlan, RowExchange, owned_frames, owner, run_frames

CTU, W, H, M = 16, 96, 88, 8            # 6 CTU rows (the last one partial), margins 8 / 4
TOTAL = 8


def _geom(p):
    w, h, m = (W, H, M) if p == 0 else (W // 2, H // 2, M // 2)
    pw = -(-w // (CTU >> (p > 0))) * (CTU >> (p > 0))
    ph = -(-h // (CTU >> (p > 0))) * (CTU >> (p > 0))
    return w, h, m, pw + 2 * m, ph + 2 * m      # width, height, margin, stride, rows


def _source(i):
    rng = np.random.default_rng(1000 + i)
    out = []
    for p in range(3):
        w, h, m, stride, rows = _geom(p)
        a = np.full((rows, stride), 0, np.int16)
        a[m:m + h, m:m + w] = rng.integers(0, 256, (h, w))
        out.append(a.reshape(-1))
    return out


class StandIn:
    """Per-rank buffers and the CPU stand-in band work."""

    def __init__(self, world, rank, band_rows):
        self.world, self.rank = world, rank
        self.frames = [i for i in owned_frames(TOTAL, rank, world)]
        self.plan = BandPlan(ctu_rows=-(-H // CTU), band_rows=band_rows)
        n = len(self.frames)
        self.src = [[torch.from_numpy(a) for a in _source(i)] for i in self.frames]
        self.ref = [[torch.full_like(t, -1) for t in s] for s in self.src]
        self.work = [[torch.zeros_like(t) for t in s] for s in self.src]
        self.final = [[torch.zeros_like(t) for t in s] for s in self.src]
        self.planes = {"ref": self.ref, "final": self.final}
        regions = []
        for p in range(3):
            _, _, m, stride, rows = _geom(p)
            regions.append(lambda b, p=p, m=m, stride=stride, rows=rows: tuple(
                stride * r for r in self.plan.region(b, CTU, m, rows, shift=int(p > 0))))
        self.ex = RowExchange(world, rank, self.plan, lambda kind, k: self.planes[kind][k], regions, TOTAL)
        assert n == len(self.src)

    def view(self, bufs, k, p):
        w, h, m, stride, rows = _geom(p)
        return bufs[k][p].view(rows, stride)

    def band_px(self, b, p):
        r0, r1 = self.plan.rows(b)
        c = CTU >> (p > 0)
        h = _geom(p)[1]
        return r0 * c, min(r1 * c, h)

    def encode(self, k, b):
        i = self.frames[k]
        assert self.ex.avail[k] >= self.plan.need(b), "band encoded before its reference rows were published"
        for p in range(3):
            w, h, m, _, _ = _geom(p)
            y0, y1 = self.band_px(b, p)
            src, wk = self.view(self.src, k, p), self.view(self.work, k, p)
            if i == 0:
                wk[m + y0:m + y1, m:m + w] = src[m + y0:m + y1, m:m + w]
                continue
            ref = self.view(self.ref, k, p)
            lag = self.plan.lag * (CTU >> (p > 0))
            ys = torch.arange(y0, y1)
            far = ref[m + torch.clamp(ys + lag, max=h - 1), m - 2:m + w + 2]   # motion window: +lag rows, 2 px
            near = ref[m + ys, m:m + w]
            assert int(far.min()) >= 0 and int(near.min()) >= 0, "read a reference row before it was published"
            wk[m + y0:m + y1, m:m + w] = (src[m + y0:m + y1, m:m + w] + 3 * far[:, 2:-2] + (near >> 1)
                                         + far[:, :-4] - far[:, 4:]) & 255

    def deblock(self, k, b):
        for p in range(3):
            w, h, m, _, _ = _geom(p)
            y0, _ = self.band_px(b, p)
            if y0 == 0:
                continue
            wk = self.view(self.work, k, p)
            a = wk[m + y0 - 3:m + y0 + 3, m:m + w].clone()
            wk[m + y0 - 3:m + y0 + 3, m:m + w] = (a + a.flip(0) + 1) >> 1

    def finish(self, k, b):
        for p in range(3):
            w, h, m, stride, rows = _geom(p)
            y0, y1 = self.band_px(b, p)
            wk, fin = self.view(self.work, k, p), self.view(self.final, k, p)
            ys = torch.arange(y0, y1)
            up, dn = m + torch.clamp(ys - 1, min=0), m + torch.clamp(ys + 1, max=h - 1)
            fin[m + y0:m + y1, m:m + w] = (wk[up, m:m + w] + 2 * wk[m + ys, m:m + w] + wk[dn, m:m + w] + 2) >> 2
            fin[m + y0:m + y1, :m] = fin[m + y0:m + y1, m:m + 1]
            fin[m + y0:m + y1, m + w:] = fin[m + y0:m + y1, m + w - 1:m + w]
            if b == 0:
                fin[:m] = fin[m:m + 1]
            if b == self.plan.nbands - 1:
                fin[m + h:] = fin[m + h - 1:m + h]

    def run(self):
        run_frames(self.ex, len(self.frames), self.encode, self.deblock, self.finish)
        return ({i: [t.numpy().copy() for t in self.final[k]] for k, i in enumerate(self.frames)},
                {i: [t.numpy().copy() for t in self.ref[k]] for k, i in enumerate(self.frames)})


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, band_rows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank,) + StandIn(world, rank, band_rows).run())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, band_rows):
    if world == 1:
        return StandIn(1, 0, band_rows).run()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_rows, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    finals, refs = {}, {}
    for _, f, r in res:
        finals.update(f)
        refs.update(r)
    return finals, refs


def test_band_plan_matches_ref_lag():
    plan = BandPlan(ctu_rows=17, band_rows=1, lag=2)          # 1080p, --preset medium
    assert plan.nbands == 17 and [plan.need(b) for b in (0, 1, 14, 15, 16)] == [2, 3, 16, 16, 16]
    plan = BandPlan(ctu_rows=17, band_rows=4, lag=2)
    assert plan.nbands == 5 and [plan.need(b) for b in range(5)] == [1, 2, 3, 4, 4]
    assert plan.region(0, 64, 80, 1240) == (0, 80 + 4 * 64) and plan.region(4, 64, 80, 1240) == (80 + 16 * 64, 1240)
    assert [owner(i, 4) for i in range(6)] == [0, 1, 2, 3, 0, 1] and owned_frames(8, 1, 4) == [1, 5]


@pytest.mark.parametrize("world,band_rows", [(2, 1), (4, 1), (2, 2), (4, 3)])
def test_frame_parallel_rows_gloo(world, band_rows):
    ref_finals, ref_refs = _run(1, band_rows)
    finals, refs = _run(world, band_rows)
    assert sorted(finals) == list(range(TOTAL))
    for i in range(TOTAL):
        for p in range(3):
            # output identical to the one-rank run
            np.testing.assert_array_equal(finals[i][p], ref_finals[i][p], err_msg=f"frame {i} plane {p}")
            if i:
                # the reference slot holds the producer's final frame i - 1, byte for byte (margins too)
                np.testing.assert_array_equal(refs[i][p], finals[i - 1][p], err_msg=f"ref of frame {i} plane {p}")
                assert refs[i][p].min() >= 0


@pytest.mark.parametrize("ctu_rows", [4, 17, 34])
@pytest.mark.parametrize("band_rows", [1, 2, 3, 4, 17])
def test_wavefront_schedule_respects_row_dependencies(ctu_rows, band_rows):
    """The single-rank wavefront (frame_pipeline.wave_delay): frame k's band b runs at step k*d + b.
    Every (frame, band) runs exactly once, and every reference band a band needs (BandPlan.need) was
    published in an EARLIER step by the previous frame — band c is published in the step of band
    c + 1 (its SAO needs the next band's deblocking), the last band in its own step."""
    from src.x265_amd.frame_pipeline import wave_delay

    plan = BandPlan(ctu_rows=ctu_rows, band_rows=band_rows)
    nb, d, F = plan.nbands, wave_delay(plan), 6
    step = {(k, b): k * d + b for k in range(F) for b in range(nb)}
    pub = {(k, c): step[(k, min(c + 1, nb - 1))] for k in range(F) for c in range(nb)}
    assert len(set(step.items())) == F * nb
    for k in range(1, F):
        for b in range(nb):
            assert pub[(k - 1, plan.need(b))] < step[(k, b)], (k, b, d)
    # and d is the smallest such delay
    if d > 1:
        d2 = d - 1
        assert any(k * d2 + b <= (k - 1) * d2 + min(plan.need(b) + 1, nb - 1)
                   for k in range(1, F) for b in range(nb))
