"""Multi-process (gloo, world_size 2, CPU) coverage of the frame-parallel path:
GOP sharding and the reference-picture ring that bench.py runs over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from src.x265_amd.shard import RefRing, gop_shard


def test_gop_shard_partitions_every_frame():
    for total in (1, 7, 64, 65):
        for world in (1, 2, 3, 8):
            got = [f for r in range(world) for f in gop_shard(total, r, world)]
            assert got == list(range(total))
            sizes = [len(gop_shard(total, r, world)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ring_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.x265_amd.workload import FrameSet

        F = 2
        fs = FrameSet(256, 128, F, 8, device="cpu", first_frame=rank * F)
        ring = RefRing(world, rank)
        ring.exchange(list(fs.planes(F - 1)), list(fs.planes(F)))
        # what the previous rank sent = its last frame = synthetic frame (prev*F + F)
        prev = (rank - 1) % world
        ref = FrameSet(256, 128, F, 8, device="cpu", first_frame=prev * F)
        ok = all(torch.equal(a, b) for a, b in zip(fs.planes(F), ref.planes(F - 1)))
        # timing reduction used by bench.py: MAX over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, ok, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_reference_ring_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ring_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, tmax in res:
        assert ok, f"rank {rank} received the wrong reference picture"
        assert tmax == float(world)
