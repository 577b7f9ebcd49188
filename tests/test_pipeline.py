"""Frame-parallel GOP shard with reconstructed-reference exchange (src/x265_amd/pipeline.py,
csrc/schedule.cpp), on CPU.

The schedule (x265amd_schedule, the C ABI every rank computes the plan with) is checked against
the mini-GOP and reference-list rules of x265 1.9 --preset medium, and the row dependencies of
frameencoder.cpp:516-531.  Then multi-process gloo runs at world 1, 2 and 4 of the same pipeline
bench.py drives over RCCL, with a CPU stand-in for the per-band work that has the encoder's row
dependencies:

  encode(j, b)  reads every reference of frame j (L0 and L1) up to refLagRows rows below the
                band (the motion-search window), 2 px beyond the sides;
  deblock(j, b) rewrites the 3 rows on each side of the band's top edge;
  finish(j, c)  reads one row of band c + 1 (SAO), then extends the borders.

Checked: every rank's reference store holds, byte for byte, the producer's final pictures
(margins included) for every reference its frames use; no band is encoded before the reference
rows it reads are in place (stores start poisoned with -1, the encoder asserts it never sees one);
non-reference b pictures are never sent; and every picture equals the one-rank run.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from src.x265_amd.pipeline import FRAME_B, FRAME_BREF, FRAME_I, FRAME_P, BandPlan, RefExchange, Schedule, run_steps

CTU, W, H, M = 16, 96, 88, 8            # 6 CTU rows (the last one partial), margins 8 / 4


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

    def __init__(self, world, rank, band_rows, total, segment):
        self.world, self.rank = world, rank
        self.plan = BandPlan(ctu_rows=-(-H // CTU), band_rows=band_rows)
        self.s = Schedule(total, world, self.plan, segment_frames=segment)
        self.frames = self.s.local_frames(rank)
        self.src = {j: [torch.from_numpy(a) for a in _source(j)] for j in self.frames}
        self.store = {j: [torch.full_like(t, -1) for t in self.src[self.frames[0]]] for j in self.s.store_frames(rank)}
        self.work = {j: [torch.zeros_like(t) for t in self.src[j]] for j in self.frames}
        self.final = {j: [torch.zeros_like(t) for t in self.src[j]] for j in self.frames}
        regions = []
        for p in range(3):
            _, _, m, stride, rows = _geom(p)
            regions.append(lambda b, p=p, m=m, stride=stride, rows=rows: tuple(
                stride * r for r in self.plan.region(b, CTU, m, rows, shift=int(p > 0))))
        self.ex = RefExchange(self.s, rank, lambda kind, j: (self.final if kind == "final" else self.store)[j],
                              regions)
        self.received = set()

    def view(self, bufs, j, p):
        w, h, m, stride, rows = _geom(p)
        return bufs[j][p].view(rows, stride)

    def band_px(self, b, p):
        r0, r1 = self.plan.rows(b)
        c = CTU >> (p > 0)
        h = _geom(p)[1]
        return r0 * c, min(r1 * c, h)

    def encode(self, j, b):
        for p in range(3):
            w, h, m, _, _ = _geom(p)
            y0, y1 = self.band_px(b, p)
            src, wk = self.view(self.src, j, p), self.view(self.work, j, p)
            acc = src[m + y0:m + y1, m:m + w].clone()
            ys = torch.arange(y0, y1)
            # rows r of the band may read reference rows < (r // CTU + lag) * CTU (frameencoder.cpp:526)
            reach = torch.clamp(((ys // (CTU >> (p > 0))) + self.plan.lag) * (CTU >> (p > 0)) - 1, max=h - 1)
            for k, r in enumerate(self.s.refs[j]):
                ref = self.view(self.store, r, p)
                far = ref[m + reach, m - 2:m + w + 2]                  # motion window: lag rows below, 2 px out
                near = ref[m + ys, m:m + w]
                assert int(far.min()) >= 0 and int(near.min()) >= 0, \
                    f"frame {j} band {b} read reference {r} before it was published"
                acc += (k + 1) * far[:, 2:-2] + (near >> 1) + far[:, :-4] - far[:, 4:]
            wk[m + y0:m + y1, m:m + w] = acc & 255

    def deblock(self, j, b):
        for p in range(3):
            w, h, m, _, _ = _geom(p)
            y0, _ = self.band_px(b, p)
            if y0 == 0:
                continue
            wk = self.view(self.work, j, p)
            a = wk[m + y0 - 3:m + y0 + 3, m:m + w].clone()
            wk[m + y0 - 3:m + y0 + 3, m:m + w] = (a + a.flip(0) + 1) >> 1

    def finish(self, j, b):
        for p in range(3):
            w, h, m, stride, rows = _geom(p)
            y0, y1 = self.band_px(b, p)
            wk, fin = self.view(self.work, j, p), self.view(self.final, j, p)
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
        run_steps(self.s, self.rank, self.ex, self.encode, self.deblock, self.finish)
        return ({j: [t.numpy().copy() for t in self.final[j]] for j in self.frames},
                {j: [t.numpy().copy() for t in self.store[j]] for j in self.store})


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank,) + StandIn(world, rank, *args).run())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, band_rows, total, segment):
    if world == 1:
        return StandIn(1, 0, band_rows, total, segment).run()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, (band_rows, total, segment), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    finals, stores = {}, []
    for _, f, s in res:
        finals.update(f)
        stores.append(s)
    return finals, stores


# ---------------------------------------------------------------- the schedule
def test_band_plan_matches_ref_lag():
    """row r waits for reference rows 0 .. r + lag - 1 (frameencoder.cpp:526-527)"""
    plan = BandPlan(ctu_rows=17, band_rows=1, lag=2)          # 1080p, --preset medium
    assert plan.nbands == 17 and [plan.need(b) for b in (0, 1, 14, 15, 16)] == [1, 2, 15, 16, 16]
    plan = BandPlan(ctu_rows=17, band_rows=4, lag=2)
    assert plan.nbands == 5 and [plan.need(b) for b in range(5)] == [1, 2, 3, 4, 4]
    plan = BandPlan(ctu_rows=17, band_rows=17, lag=2)
    assert plan.nbands == 1 and plan.need(0) == 0
    assert plan.region(0, 64, 80, 1240) == (0, 1240)


def test_medium_gop_structure_and_references():
    """mini-GOP of --preset medium: encode order P, B-ref, b, b, b (slicetype.cpp:993-996,
    1050-1078); L0 = the 3 nearest earlier-coded reference pictures before it, L1 (B only) = the
    2 nearest after it (dpb.cpp:149-150, 188-207, dpb.h:57-58)"""
    s = Schedule(11, 1, BandPlan(ctu_rows=4, band_rows=4))
    assert s.poc == [0, 5, 3, 1, 2, 4, 10, 8, 6, 7, 9]
    T = {FRAME_I: "I", FRAME_P: "P", FRAME_BREF: "Bref", FRAME_B: "b"}
    assert [T[t] for t in s.type] == ["I", "P", "Bref", "b", "b", "b", "P", "Bref", "b", "b", "b"]
    assert s.refs == [[], [0], [0, 1], [0, 2, 1], [0, 2, 1], [2, 0, 1], [1, 2, 0], [1, 2, 0, 6], [1, 2, 0, 7, 6],
                      [1, 2, 0, 7, 6], [7, 1, 2, 6]]
    assert [s.is_ref[j] for j in range(11)] == [True, True, True] + [False] * 3 + [True, True] + [False] * 3
    # segments are closed: each starts with an I picture and references nothing before it
    s2 = Schedule(20, 2, BandPlan(ctu_rows=4, band_rows=4), segment_frames=10)
    assert s2.type[10] == FRAME_I and all(r >= 10 for j in range(10, 20) for r in s2.refs[j])
    assert s2.rank == [j % 2 for j in range(20)]


@pytest.mark.parametrize("ctu_rows", [4, 17, 34])
@pytest.mark.parametrize("band_rows", [1, 2, 4, 17])
def test_schedule_respects_row_dependencies(ctu_rows, band_rows):
    """every (frame, band) runs after its previous band and after every reference band it needs
    was published in an EARLIER step; and at the earliest such step"""
    plan = BandPlan(ctu_rows=ctu_rows, band_rows=band_rows)
    s = Schedule(24, 4, plan, segment_frames=12)
    s.check()
    for j in range(24):
        for b in range(plan.nbands):
            lo = s.step[j, b - 1] + 1 if b else 0
            for r in s.refs[j]:
                lo = max(lo, s.pub_step(r, plan.need(b)) + 1)
            assert s.step[j, b] == lo
    # the non-reference b pictures' bands are never sent; reference pictures reach every user's rank
    sent = {(j, d) for st in range(s.nsteps) for (j, c, src, d) in s.transfers(st)}
    assert all(s.is_ref[j] for j, _ in sent)
    for j in range(24):
        for u in s.users[j]:
            assert (j, s.rank[u]) in sent


def test_schedule_overlaps_frames():
    """whole-frame bands: the next mini-GOP's P runs beside the previous mini-GOP's b pictures (the
    critical path is P -> B-ref -> next P, two steps per mini-GOP: a P references the previous
    B-ref), so a 32-frame segment needs far fewer steps than frames"""
    s = Schedule(32, 1, BandPlan(ctu_rows=17, band_rows=17))
    assert s.nsteps <= 2 * (32 // 5) + 3
    assert max(len(s.items(0, st)) for st in range(s.nsteps)) >= 4


# ---------------------------------------------------------------- the exchange
@pytest.mark.parametrize("world,band_rows,total,segment", [(2, 1, 11, 11), (4, 2, 16, 8), (2, 6, 12, 6),
                                                           (4, 3, 12, 12)])
def test_frame_parallel_exchange_gloo(world, band_rows, total, segment):
    ref_finals, ref_stores = _run(1, band_rows, total, segment)
    finals, stores = _run(world, band_rows, total, segment)
    assert sorted(finals) == list(range(total))
    s = Schedule(total, world, BandPlan(ctu_rows=-(-H // CTU), band_rows=band_rows), segment_frames=segment)
    fanout = max(len(s.dest_ranks(j)) for j in range(total))
    if world == 4:
        assert fanout >= 2, "no reference picture was sent to more than one rank"
    for j in range(total):
        for p in range(3):
            # output identical to the one-rank run
            np.testing.assert_array_equal(finals[j][p], ref_finals[j][p], err_msg=f"frame {j} plane {p}")
    # every store slot holds the producer's final picture, byte for byte (margins too)
    for st in stores:
        for r, planes in st.items():
            for p in range(3):
                np.testing.assert_array_equal(planes[p], finals[r][p], err_msg=f"store copy of frame {r} plane {p}")
                assert planes[p].min() >= 0


class _LockstepComm:
    """CPU stand-in of the native communicator (x265amd_exchange): records each rank's transfer table
    of the step; `deliver` then matches them the way RCCL's point-to-point does (per ordered pair of
    ranks, the k-th send to a peer with the peer's k-th receive from this rank, equal sizes)"""

    def __init__(self):
        self.pending = {}

    def bind(self, rank):
        comm = self

        class _R:
            def exchange(self, tab, stream):
                comm.pending[rank] = list(tab)
        return _R()

    def deliver(self):
        import ctypes

        sends, recvs = {}, {}
        for rank, tab in self.pending.items():
            for t in tab:
                (sends if t.send else recvs).setdefault((rank, t.peer) if t.send else (t.peer, rank), []).append(t)
        assert sends.keys() == recvs.keys()
        n = 0
        for key in sends:
            assert [t.bytes for t in sends[key]] == [t.bytes for t in recvs[key]], f"unmatched transfers {key}"
            for s_, r_ in zip(sends[key], recvs[key]):
                ctypes.memmove(r_.buf, s_.buf, s_.bytes)
                n += 1
        self.pending.clear()
        return n


@pytest.mark.parametrize("world,band_rows,total,segment", [(2, 1, 11, 11), (4, 2, 16, 8)])
def test_native_exchange_tables_match_pairwise(world, band_rows, total, segment):
    """the native exchange path (RcclExchange -> x265amd_exchange): every rank's per-step transfer table,
    delivered with RCCL's pairing rule, reproduces the one-rank pictures and the producer-identical stores"""
    from src.x265_amd.pipeline import RcclExchange

    ref_finals, _ = _run(1, band_rows, total, segment)
    lock = _LockstepComm()
    ranks = [StandIn(world, r, band_rows, total, segment) for r in range(world)]
    for r, st in enumerate(ranks):
        st.ex = RcclExchange(st.s, r, st.ex.planes_of, st.ex.regions, lock.bind(r))
    moved = 0
    for step in range(ranks[0].s.nsteps):
        for r, st in enumerate(ranks):
            run_steps(st.s, r, st.ex, st.encode, st.deblock, st.finish, steps=[step])
        moved += lock.deliver()
    assert moved > 0
    for st in ranks:
        for j in st.frames:
            for p in range(3):
                np.testing.assert_array_equal(st.final[j][p].numpy(), ref_finals[j][p], err_msg=f"frame {j} plane {p}")
        for r, planes in st.store.items():
            owner = ranks[st.s.rank[r]]
            for p in range(3):
                np.testing.assert_array_equal(planes[p].numpy(), owner.final[r][p].numpy(), err_msg=f"store {r}")


def test_native_exchange_argument_checks():
    """x265amd_exchange / x265amd_comm_create reject bad arguments before touching RCCL or a device"""
    import ctypes

    from src.x265_amd.pipeline import _lib

    lib = _lib()
    assert lib.x265amd_exchange(None, None, 0, None) == 1000
    h = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(128)
    assert lib.x265amd_comm_create(ctypes.byref(h), uid, 0, 0) == 1000
    assert lib.x265amd_comm_create(ctypes.byref(h), uid, 2, 2) == 1000
    assert lib.x265amd_comm_destroy(None) == 0


def test_cpp_frame_shard_host_built_and_needs_a_device(tmp_path):
    """the C++ host of the frame-parallel shard is built by build() and, without a GPU, exits with
    status 3 instead of running on anything else"""
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_bin",
                       "frame_shard_host")
    if not os.path.exists(exe):
        pytest.skip("not built (run __graft_entry__.build())")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = subprocess.run([exe, "416", "240", "8", "1", "1", "0", str(tmp_path / "id")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 3 and "no device" in r.stderr
