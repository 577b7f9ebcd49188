"""Frame-parallel GOP shard with reconstructed-reference exchange (BASELINE config 4).

x265 runs frames in parallel on FrameEncoders assigned round robin (encoder.cpp:649-650).
Frames share nothing but reconstructed reference rows: FrameFilter publishes a CTU row once it
is deblocked, SAO-filtered and border-extended (m_reconRowCount, framefilter.cpp:520), and a
frame encoding CTU row r waits until EACH of its references has published r + refLagRows rows
(frameencoder.cpp:516-531; refLagRows = 2 at --preset medium, frameencoder.cpp:114-119).
Across GPUs the same structure is:

  * the GOP of --preset medium (bframes 4, b-pyramid, 3 references; x265amd_schedule in
    csrc/schedule.cpp restates the mini-GOP and reference-list rules) over closed segments;
    frame j (encode order) is encoded by rank j mod G;
  * a frame is processed in bands of CTU rows; the schedule gives every (frame, band) the
    earliest STEP after its previous band and after each reference published the band that
    holds row r1 - 2 + refLagRows (BandPlan.need);
  * FrameFilter's row order: deblocking band b changes the last rows of band b - 1, so band
    b - 1 becomes final (SAO, border extension) in band b's step, the last band in its own;
  * a final band of a REFERENCE picture goes to every rank that owns a frame referencing it
    (fan-out up to the pictures' L0 + L1 users; non-reference b pictures publish nothing),
    point to point over RCCL / xGMI on the GPU (torch.distributed P2P; gloo in the CPU tests),
    into that rank's reference store; a rank's own consumers get a local copy.

Each rank runs the steps in order: its (frame, band) work of the step, then the step's
exchange (one batch of sends and receives, identical order on both sides of every link).
The pipeline is generic over the per-band work (`encode`, `deblock`, `finish` callbacks);
bench.py plugs in the census primitive workload and the f4 loop-filter kernels
(frame_pipeline.py), tests/test_pipeline.py a CPU stand-in with the same row dependencies.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

REF_LAG_ROWS_MEDIUM = 2   # frameencoder.cpp:114-119 with merange 57
FRAME_I, FRAME_P, FRAME_BREF, FRAME_B = range(4)


@dataclass
class BandPlan:
    """CTU-row bands of a picture and the reference rows each band needs."""
    ctu_rows: int          # CTU rows in the picture
    band_rows: int = 1     # CTU rows per band
    lag: int = REF_LAG_ROWS_MEDIUM

    @property
    def nbands(self) -> int:
        return -(-self.ctu_rows // self.band_rows)

    def rows(self, b: int):
        """CTU rows [r0, r1) of band b"""
        return b * self.band_rows, min((b + 1) * self.band_rows, self.ctu_rows)

    def band_of(self, row: int) -> int:
        return min(row, self.ctu_rows - 1) // self.band_rows

    def need(self, b: int) -> int:
        """last reference band that must be published before band b is encoded: row r of the band
        waits for rows 0 .. r + lag - 1 (frameencoder.cpp:526-527), so the last row r1 - 1 needs
        the band holding row r1 - 2 + lag"""
        return self.band_of(self.rows(b)[1] - 2 + self.lag)

    def reach_rows(self, b: int) -> int:
        """CTU rows of every reference that band b may read: rows 0 .. r1 - 2 + lag"""
        return self.rows(b)[1] - 1 + self.lag

    def region(self, b: int, ctu: int, margin_rows: int, rows_total: int, shift: int = 0):
        """buffer rows [start, end) of band b in a padded plane (full stride): the
        picture rows of the band, plus the margin rows above band 0 / below the last
        band.  shift = 1 for 4:2:0 chroma."""
        r0, r1 = self.rows(b)
        c = ctu >> shift
        start = 0 if b == 0 else margin_rows + r0 * c
        end = rows_total if b == self.nbands - 1 else margin_rows + r1 * c
        return start, end


class _SchedConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("frames", "segment_frames", "bframes", "b_pyramid", "max_refs",
                                            "max_refs_l1", "ctu_rows", "band_rows", "lag", "world")]


class _SchedFrame(ctypes.Structure):
    _fields_ = [("poc", ctypes.c_int), ("type", ctypes.c_int), ("is_ref", ctypes.c_int), ("rank", ctypes.c_int),
                ("nrefs", ctypes.c_int), ("nrefs_l0", ctypes.c_int), ("refs", ctypes.c_int * 6)]


def _lib():
    from .native import LIB_PATH

    lib = ctypes.CDLL(LIB_PATH)
    lib.x265amd_schedule.restype = ctypes.c_int
    return lib


class Schedule:
    """The plan every rank computes identically (x265amd_schedule, csrc/schedule.cpp): per frame its
    type, references and rank; per (frame, band) its step; per step the bands published and where
    they go."""

    def __init__(self, frames: int, world: int, plan: BandPlan, segment_frames: int | None = None, bframes: int = 4,
                 b_pyramid: bool = True, max_refs: int = 3, max_refs_l1: int = 2):
        self.frames, self.world, self.plan = frames, world, plan
        self.segment_frames = segment_frames or frames
        cfg = _SchedConfig(frames, self.segment_frames, bframes, int(b_pyramid), max_refs,
                           max_refs_l1 if b_pyramid else 1, plan.ctu_rows, plan.band_rows, plan.lag, world)
        fr = (_SchedFrame * frames)()
        nb = plan.nbands
        step = (ctypes.c_int * (frames * nb))()
        nsteps = ctypes.c_int()
        rc = _lib().x265amd_schedule(ctypes.byref(cfg), fr, step, ctypes.byref(nsteps))
        if rc:
            raise ValueError(f"x265amd_schedule: status {rc}")
        self.nsteps = nsteps.value
        self.type = [f.type for f in fr]
        self.poc = [f.poc for f in fr]
        self.is_ref = [bool(f.is_ref) for f in fr]
        self.rank = [f.rank for f in fr]
        self.refs = [list(f.refs[:f.nrefs]) for f in fr]
        self.nrefs_l0 = [f.nrefs_l0 for f in fr]
        self.step = np.frombuffer(step, dtype=np.int32).reshape(frames, nb).copy()
        self.users = [[] for _ in range(frames)]              # frames that reference frame j
        for j, rs in enumerate(self.refs):
            for r in rs:
                self.users[r].append(j)

    # ---- derived plans
    def pub_step(self, j: int, c: int) -> int:
        """step in which band c of frame j becomes final"""
        nb = self.plan.nbands
        return int(self.step[j, min(c + 1, nb - 1)])

    def local_frames(self, rank: int) -> list:
        return [j for j in range(self.frames) if self.rank[j] == rank]

    def store_frames(self, rank: int) -> list:
        """reference pictures rank keeps a copy of: every reference of its frames"""
        return sorted({r for j in self.local_frames(rank) for r in self.refs[j]})

    def dest_ranks(self, j: int) -> list:
        """ranks that receive the reference picture j (owners of its users)"""
        return sorted({self.rank[u] for u in self.users[j]})

    def items(self, rank: int, step: int) -> list:
        """(frame, band) pairs rank encodes in step, frames in encode order"""
        nb = self.plan.nbands
        return [(j, b) for j in self.local_frames(rank) for b in range(nb) if self.step[j, b] == step]

    def finals(self, rank: int, step: int) -> list:
        """(frame, band) pairs of rank's frames that become final in step (SAO + border)"""
        nb = self.plan.nbands
        out = []
        for j in self.local_frames(rank):
            for c in range(nb):
                if self.pub_step(j, c) == step:
                    out.append((j, c))
        return out

    def transfers(self, step: int) -> list:
        """(frame j, band c, src rank, dst rank) of every band published in step, canonical order"""
        nb = self.plan.nbands
        out = []
        for j in range(self.frames):
            if not self.is_ref[j] or not self.users[j]:
                continue
            for c in range(nb):
                if self.pub_step(j, c) == step:
                    for d in self.dest_ranks(j):
                        out.append((j, c, self.rank[j], d))
        return out

    def check(self):
        """every band needed from every reference is published strictly before it is used"""
        plan = self.plan
        for j in range(self.frames):
            for b in range(plan.nbands):
                for r in self.refs[j]:
                    assert self.pub_step(r, plan.need(b)) < self.step[j, b], (j, b, r)
                if b:
                    assert self.step[j, b - 1] < self.step[j, b]


class RefExchange:
    """Moves final bands of reference pictures into the reference stores of the ranks that read them.

    planes_of(kind, idx) -> list of flat per-plane tensors: kind "final" with a frame index owned by
    this rank (its finished reconstruction), kind "store" with a reference frame index in this rank's
    store; regions[p](b) -> (start, end) element range of band b in plane p."""

    def __init__(self, sched: Schedule, rank: int, planes_of, regions):
        self.s, self.rank, self.planes_of, self.regions = sched, rank, planes_of, regions
        self.world = sched.world
        self.store = set(sched.store_frames(rank))
        self.plans = [[t for t in sched.transfers(st) if rank in (t[2], t[3])] for st in range(sched.nsteps)]

    def _band(self, kind, j, c):
        out = []
        for p, t in enumerate(self.planes_of(kind, j)):
            s, e = self.regions[p](c)
            out.append(t[s:e])
        return out

    def exchange(self, step: int):
        """after step's work: local copies, then this rank's sends and receives of the step (NCCL:
        enqueued on the communicator's stream and waited on by the current stream; gloo: host waits)"""
        ops = []
        for j, c, src, dst in self.plans[step]:
            if src == dst == self.rank:
                for s_, d_ in zip(self._band("final", j, c), self._band("store", j, c)):
                    if s_.data_ptr() != d_.data_ptr():         # a final written in place in the store: nothing to do
                        d_.copy_(s_)
            elif src == self.rank:
                ops += [("send", t, dst) for t in self._band("final", j, c)]
            else:
                ops += [("recv", t, src) for t in self._band("store", j, c)]
        if not ops:
            return
        import torch.distributed as dist

        p2p = [dist.P2POp(dist.isend if k == "send" else dist.irecv, t, peer) for k, t, peer in ops]
        for w in dist.batch_isend_irecv(p2p):
            w.wait()


class _Transfer(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("bytes", ctypes.c_size_t), ("peer", ctypes.c_int), ("send", ctypes.c_int)]


class Comm:
    """A native RCCL communicator (x265amd_comm_*, csrc/exchange.cpp) on the current HIP device.  Rank 0
    makes the 128-byte id; with world > 1 it reaches the other ranks over the torch.distributed group
    (any channel would do: the id is plain bytes)."""

    def __init__(self, world: int, rank: int):
        self.lib = lib = _lib()
        lib.x265amd_comm_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_int,
                                            ctypes.c_int]
        lib.x265amd_comm_destroy.argtypes = [ctypes.c_void_p]
        lib.x265amd_exchange.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            rc = lib.x265amd_comm_unique_id(uid)
            if rc:
                raise RuntimeError(f"x265amd_comm_unique_id: status {rc} (librccl not loadable?)")
        if world > 1:
            import torch.distributed as dist

            obj = [uid.raw if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            uid = ctypes.create_string_buffer(obj[0], 128)
        self.handle = ctypes.c_void_p()
        rc = lib.x265amd_comm_create(ctypes.byref(self.handle), uid, world, rank)
        if rc:
            raise RuntimeError(f"x265amd_comm_create: status {rc}")
        self.world, self.rank = world, rank
        lib.x265amd_comm_backend.restype = ctypes.c_char_p
        b = lib.x265amd_comm_backend()
        self.backend = b.decode() if b else None    # which RCCL the C ABI bound (recorded by bench.py)

    def exchange(self, xfers, stream):
        """xfers: a ctypes array of _Transfer; stream: a HIP stream handle (int)"""
        rc = self.lib.x265amd_exchange(self.handle, ctypes.cast(xfers, ctypes.c_void_p), len(xfers),
                                       ctypes.c_void_p(stream))
        if rc:
            raise RuntimeError(f"x265amd_exchange: status {rc}")

    def close(self):
        if self.handle:
            self.lib.x265amd_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class RcclExchange(RefExchange):
    """RefExchange through the native communicator: every step's sends and receives (and, with
    loopback, the rank's local band copies as send / receive pairs to itself) are one
    x265amd_exchange call enqueued on the current stream.  The transfer tables are built once: the
    frame buffers never move."""

    def __init__(self, sched: Schedule, rank: int, planes_of, regions, comm: Comm, loopback: bool = False):
        super().__init__(sched, rank, planes_of, regions)
        self.comm, self.loop_local = comm, loopback
        self.tables = []
        for st in range(sched.nsteps):
            rows = []
            for j, c, src, dst in self.plans[st]:
                if src == dst == self.rank:
                    if not loopback:
                        continue
                    pairs = list(zip(self._band("final", j, c), self._band("store", j, c)))
                    if all(s_.data_ptr() == d_.data_ptr() for s_, d_ in pairs):
                        continue
                    for s_, d_ in pairs:
                        rows += [(s_, self.rank, 1), (d_, self.rank, 0)]
                elif src == self.rank:
                    rows += [(t, dst, 1) for t in self._band("final", j, c)]
                else:
                    rows += [(t, src, 0) for t in self._band("store", j, c)]
            tab = (_Transfer * len(rows))()
            for i, (t, peer, send) in enumerate(rows):
                tab[i] = _Transfer(t.data_ptr(), t.numel() * t.element_size(), peer, send)
            self.tables.append(tab)

    def exchange(self, step: int):
        import torch

        if not self.loop_local:
            for j, c, src, dst in self.plans[step]:
                if src == dst == self.rank:
                    for s_, d_ in zip(self._band("final", j, c), self._band("store", j, c)):
                        if s_.data_ptr() != d_.data_ptr():
                            d_.copy_(s_)
        if len(self.tables[step]):
            stream = torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else 0
            self.comm.exchange(self.tables[step], stream)


def run_steps(sched: Schedule, rank: int, ex: RefExchange, encode, deblock, finish, steps=None):
    """This rank's share of the schedule, step by step: each (frame, band) of the step is encoded and
    deblocked (encode order), then the bands that became final are SAO-filtered / border-extended
    (finish), then the step's exchange runs.

    encode(j, b): the band's encoder work (reads reference rows < reach_rows(b) CTU rows)
    deblock(j, b): deblocking of band b (changes the last rows of band b - 1)
    finish(j, c): SAO + border extension of band c (reads one row of band c + 1)
    """
    for st in (range(sched.nsteps) if steps is None else steps):
        for j, b in sched.items(rank, st):
            encode(j, b)
            deblock(j, b)
        for j, c in sched.finals(rank, st):
            finish(j, c)
        ex.exchange(st)
