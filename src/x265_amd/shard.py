"""Frame-parallel sharding across GPUs (BASELINE config 4).

x265 already runs frames in parallel (round-robin FrameEncoders,
encoder.cpp:649-650) and the only cross-frame data dependency is the
reconstructed reference picture, published row by row through
m_reconRowCount (framefilter.cpp:520, waited on at frameencoder.cpp:516-531).
Across GPUs the same structure becomes:

  * every rank owns a contiguous GOP chunk of frames (gop_shard);
  * the first frame of rank r's chunk references the last frame of rank
    r-1's chunk, so each step ships exactly one reference picture around a
    ring (RefRing) — point-to-point send/recv over RCCL/xGMI on the GPU, gloo
    in the CPU tests — and nothing else crosses ranks (no data-path
    all-reduce; timing uses one MAX all-reduce outside the timed region).
"""
from __future__ import annotations


def gop_shard(total_frames: int, rank: int, world: int) -> range:
    """Contiguous frame range owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(total_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


class RefRing:
    """Pass one reference picture per step from rank r to rank r+1 (mod world).

    `send` is this rank's last frame of the chunk (luma + chroma planes as one
    flat tensor), `recv` the slot its first frame predicts from.  Uses
    batch_isend_irecv so the pair of transfers is one grouped call.
    """

    def __init__(self, world: int, rank: int):
        self.world, self.rank = world, rank

    def exchange(self, send, recv):
        """send / recv: tensors or equal-length lists of tensors (one per plane)."""
        send = send if isinstance(send, (list, tuple)) else [send]
        recv = recv if isinstance(recv, (list, tuple)) else [recv]
        if self.world == 1:
            for s, r in zip(send, recv):
                r.copy_(s)
            return
        import torch.distributed as dist

        nxt, prv = (self.rank + 1) % self.world, (self.rank - 1) % self.world
        ops = []
        for s, r in zip(send, recv):
            ops += [dist.P2POp(dist.isend, s, nxt), dist.P2POp(dist.irecv, r, prv)]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
