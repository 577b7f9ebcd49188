"""Frame-parallel shard with reconstructed-row exchange (BASELINE config 4).

x265 runs frames in parallel on FrameEncoders assigned round robin
(encoder.cpp:649-650).  Frames share nothing but reconstructed reference rows:
FrameFilter publishes a CTU row once it is deblocked, SAO-filtered and
border-extended (m_reconRowCount, framefilter.cpp:520), and a frame encoding CTU
row r waits until its reference has published r + refLagRows rows
(frameencoder.cpp:516-531; refLagRows = 1 + ceil((merange + 1 + 4 + 2) / 64) = 2 at
--preset medium, frameencoder.cpp:114-119).  Across GPUs the same structure is:

  * frame i is encoded by rank i mod G (`owner`);
  * a frame is processed in bands of CTU rows; band b is encoded once the
    reference frame has published the bands covering rows up to
    r1 - 1 + refLagRows (`BandPlan.need`);
  * FrameFilter's row order: deblocking band b changes the last rows of band
    b - 1 (a horizontal edge filter writes 3 rows on each side), so band b - 1
    is SAO-filtered, border-extended and published after band b is deblocked
    (the last band right after its own deblocking);
  * a published band (full-stride rows, plus the margin rows above band 0 and
    below the last band) goes to the owner of frame i + 1 — point-to-point over
    RCCL / xGMI on the GPU (gloo in the CPU tests), on one 2-rank communicator
    per ring link so that every communicator carries traffic in one direction
    only (a rank's sends can never queue behind its own receives).  With G = 1
    the band is copied into the local reference slot.

Nothing else crosses ranks.  The pipeline is generic over the per-band work
(`encode`, `deblock`, `finish` callbacks); bench.py plugs in the census
primitive workload and the f4 loop-filter kernels, tests/test_pipeline.py a
CPU stand-in with the same row dependencies.
"""
from __future__ import annotations

from dataclasses import dataclass

REF_LAG_ROWS_MEDIUM = 2   # frameencoder.cpp:114-119 with merange 57


def owner(i: int, world: int) -> int:
    """Rank that encodes frame i (encoder.cpp:649-650 round robin over FrameEncoders)."""
    return i % world


def owned_frames(total: int, rank: int, world: int) -> list:
    return list(range(rank, total, world))


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
        """last reference band that must be published before band b is encoded:
        the band holding CTU row r1 - 1 + lag (frameencoder.cpp:516-531)"""
        return self.band_of(self.rows(b)[1] - 1 + self.lag)

    def region(self, b: int, ctu: int, margin_rows: int, rows_total: int, shift: int = 0):
        """buffer rows [start, end) of band b in a padded plane (full stride): the
        picture rows of the band, plus the margin rows above band 0 / below the last
        band.  shift = 1 for 4:2:0 chroma."""
        r0, r1 = self.rows(b)
        c = ctu >> shift
        start = 0 if b == 0 else margin_rows + r0 * c
        end = rows_total if b == self.nbands - 1 else margin_rows + r1 * c
        return start, end


class RowExchange:
    """Publishes bands of final reconstructed frames to the owner of the next frame.

    planes_of(kind, k) -> list of flat per-plane tensors of local frame k, kind in
    {"final", "ref"}; regions[p](b) -> (start, end) element range of band b in plane p.
    """

    def __init__(self, world: int, rank: int, plan: BandPlan, planes_of, regions, total_frames: int):
        self.world, self.rank, self.plan = world, rank, plan
        self.planes_of, self.regions, self.total = planes_of, regions, total_frames
        self.recv_works = {}
        self.send_works = []
        self.avail = {}           # local frame k -> last reference band known to be in place
        self.g_out = self.g_in = None
        if world > 1:
            import torch.distributed as dist

            # one communicator per ring link j -> j+1: rank r sends only on link r, receives only on link r-1
            groups = [dist.new_group([j, (j + 1) % world]) for j in range(world)]
            self.g_out, self.g_in = groups[rank], groups[(rank - 1) % world]

    def _band(self, kind, k, b):
        out = []
        for p, t in enumerate(self.planes_of(kind, k)):
            s, e = self.regions[p](b)
            out.append(t[s:e])
        return out

    def frame_index(self, k: int) -> int:
        return k * self.world + self.rank

    def start_frame(self, k: int):
        """post the receives of every band of frame i - 1 into local frame k's reference slot"""
        i = self.frame_index(k)
        self.avail[k] = -1
        if i == 0:
            self.avail[k] = self.plan.nbands - 1      # first frame of the sequence: no reference
            return
        if self.world == 1:
            return                                     # filled by the local publication of frame k - 1
        import torch.distributed as dist

        src = owner(i - 1, self.world)
        self.recv_works[k] = [[dist.irecv(t, src=src, group=self.g_in) for t in self._band("ref", k, b)]
                              for b in range(self.plan.nbands)]

    def wait(self, k: int, band: int):
        """make the work issued next wait until reference bands 0..band of local frame k are in place
        (NCCL: a stream wait, no host block; gloo: a host wait)"""
        if self.avail[k] >= band:
            return
        if self.world == 1:          # published by frame k - 1, which the stream has already ordered
            self.avail[k] = band
            return
        for b in range(self.avail[k] + 1, band + 1):
            for w in self.recv_works[k][b]:
                w.wait()
        self.avail[k] = band

    def publish(self, k: int, b: int):
        """band b of local frame k is final: send it to the owner of frame i + 1"""
        i = self.frame_index(k)
        if i + 1 >= self.total:
            return
        if self.world == 1:
            for s, d in zip(self._band("final", k, b), self._band("ref", k + 1, b)):
                d.copy_(s)
            return
        import torch.distributed as dist

        dst = owner(i + 1, self.world)
        self.send_works += [dist.isend(t, dst=dst, group=self.g_out) for t in self._band("final", k, b)]

    def finish_frame(self, k: int):
        self.recv_works.pop(k, None)

    def drain(self):
        """wait for every outstanding send (its buffer may be rewritten afterwards)"""
        for w in self.send_works:
            w.wait()
        self.send_works = []


def run_frames(ex: RowExchange, nlocal: int, encode, deblock, finish):
    """Encode this rank's frames in order, band by band, with FrameFilter's row order.

    encode(k, b): the band's encoder work (reads reference rows <= rows(b)[1] - 1 + lag)
    deblock(k, b): deblocking of band b (changes the last rows of band b - 1)
    finish(k, b): SAO + border extension of band b (reads one row of band b + 1)
    """
    plan = ex.plan
    nb = plan.nbands
    for k in range(nlocal):
        if ex.frame_index(k) >= ex.total:
            break
        ex.start_frame(k)
        for b in range(nb):
            ex.wait(k, plan.need(b))
            encode(k, b)
            deblock(k, b)
            if b:
                finish(k, b - 1)
                ex.publish(k, b - 1)
        finish(k, nb - 1)
        ex.publish(k, nb - 1)
        ex.finish_frame(k)
    ex.drain()
