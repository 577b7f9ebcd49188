"""The frame-parallel GPU step (src/x265_amd/frame_pipeline.py) on one GPU.

The pictures of a --preset medium GOP (pipeline.Schedule: I, P, B-ref and b pictures with their
L0 / L1 references) are encoded step by step (census primitive work per band + the f4 row-band
loop filters) and every final band of a reference picture is copied into the reference store.
Every band's reconstruction is coded by the fused TU pipeline (f3) from a motion-compensated
prediction out of the picture's first reference as the rank's reference store holds it, so a
picture's reconstruction depends on the bands its references published.  Checked: every picture's
final reconstruction equals a whole-frame chain run picture by picture in encode order (TU coding
from the chain's own final references -> x265amd_deblock / _sao_apply / _extend_border, themselves
bit-exact vs the reference's Deblock / SAO classes in test_f4.py); every store slot holds its producer's
final reconstruction, margins included; and every census batch still matches the oracle on
sampled jobs read against the FINAL stores — the stores start out holding the unfiltered source,
so a job that read a reference before its rows were published would not match.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_gpu_native_exchange_loopback():
    """x265amd_exchange (csrc/exchange.cpp) on one GPU: a group of send / receive pairs to the own rank
    moves every byte, in the group's order, on the given stream"""
    import torch

    from src.x265_amd.pipeline import Comm, _Transfer

    comm = Comm(1, 0)
    try:
        # torch has RCCL loaded already: the C ABI must bind that copy, not load a second runtime
        assert comm.backend and comm.backend.startswith("already loaded"), comm.backend
        g = torch.Generator(device="cuda").manual_seed(3)
        src = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g) for n in (1, 4097, 1 << 20)]
        dst = [torch.zeros_like(t) for t in src]
        tab = (_Transfer * 6)()
        for i, (a, b) in enumerate(zip(src, dst)):
            tab[2 * i] = _Transfer(a.data_ptr(), a.numel(), 0, 1)
            tab[2 * i + 1] = _Transfer(b.data_ptr(), b.numel(), 0, 0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        comm.exchange(tab, s.cuda_stream)
        s.synchronize()
        for a, b in zip(src, dst):
            assert torch.equal(a, b)
    finally:
        comm.close()


@pytest.mark.parametrize("band_rows,frames,exchange,job_wait,background", [
    (1, 8, "torch", "band", False), (2, 6, "torch", "band", False), (None, 11, "torch", "band", False),
    (2, 8, "rccl", "band", False), (None, 11, "torch", "reference", False), (2, 8, "torch", "reference", False),
    (None, 11, "torch", "band", True), (2, 8, "rccl", "band", True)])
def test_gpu_pipeline_gop_equals_whole_frame_chain(request, gpu_prims, oracle_libs, band_rows, frames, exchange,
                                                   job_wait, background):
    """exchange "rccl": the rank's own reference pictures are finished in their own buffers and reach the
    store through the native communicator (loop-back transfers, x265amd_exchange); job_wait "reference":
    a job waits only for the reference picture it reads; background: reference-free jobs on background
    streams / graphs joined before each step's filters (one graph, or per-step graphs with "rccl")"""
    import torch

    from pyoracle import CpuOracle
    from src.x265_amd.frame_pipeline import GpuFramePipeline

    W, H = 416, 240
    pipe = GpuFramePipeline(gpu_prims, W, H, 8, frames, 1, 0, band_rows=band_rows, streams=4, device="cuda",
                            exchange=exchange, inplace_store=exchange == "torch", job_wait=job_wait,
                            background=background)
    request.addfinalizer(pipe.close)     # graphs reset after a device drain, before the buffers they read
    pipe.build(graphs=True)
    pipe.reset_stores()                  # the build's warm-up pass already filled them
    pipe.step()
    torch.cuda.synchronize()
    fs, F = pipe.fs, pipe.F
    # the whole-frame chain in encode order, independent of the pipeline's bands, steps and stores: each
    # picture coded by the fused TU pipeline from its first reference's CHAIN-final planes (a flat plane
    # for an I picture), then deblock -> SAO -> border extension of the whole picture
    work = [torch.zeros_like(t) for t in pipe.work]
    final = [torch.zeros_like(t) for t in pipe.work]
    saved = (pipe.dbk, pipe.sao, pipe.bor)
    pipe._f4_setup(W, H, "cuda", work=work, final=final)

    def chain_pred(k, p):
        refs = pipe.sched.refs[pipe.local[k]]
        if not refs:
            return pipe._flat[p], 0
        return final[p], pipe.kof[refs[0]] * pipe._sizes[p]

    tu = pipe.tu_setup(chain_pred, work)
    from src.x265_amd.native import TuBatch
    for k in sorted(range(F), key=lambda k: pipe.local[k]):          # encode order
        arrs = [tu[(k, b)] for b in range(pipe.plan.nbands)]
        gpu_prims.tu_pipeline_grouped(8, (TuBatch * (3 * len(arrs)))(*[x for a in arrs for x in a]))
        gpu_prims.deblock(8, [pipe.dbk[k]])
        gpu_prims.sao_apply(8, [pipe.sao[k]])
        gpu_prims.extend_border(8, pipe.bor[k])
    torch.cuda.synchronize()
    pipe.dbk, pipe.sao, pipe.bor = saved
    # the reconstruction is a real coding of the source (not a copy of it): P / B pictures differ from
    # their source but stay close to it
    k0 = next(k for k in range(F) if pipe.sched.refs[pipe.local[k]])
    src_k = pipe.frame_planes([fs.luma, fs.cb, fs.cr], k0)[0].view(-1, fs.stride)[fs.my:fs.my + H, fs.mx:fs.mx + W].float()
    rec_k = pipe.frame_planes(final, k0)[0].view(-1, fs.stride)[fs.my:fs.my + H, fs.mx:fs.mx + W].float()
    err = (src_k - rec_k).abs()
    assert err.max() > 0 and err.mean() < 8, f"reconstruction error {err.mean():.2f}"
    # the area the chain defines: the picture and its margins (rows below the CTU-aligned plane's bottom
    # margin and columns right of the right margin are never written or read)
    geo = [(fs.stride, 2 * fs.my + H, 2 * fs.mx + W)] + [(fs.cstride, 2 * fs.cmy + H // 2, 2 * fs.cmx + W // 2)] * 2

    def area(t, p):
        stride, rows, cols = geo[p]
        return t[:rows * stride].view(rows, stride)[:, :cols]

    for k in range(F):
        got, want = pipe.final_planes(k), pipe.frame_planes(final, k)
        for p in range(3):
            assert torch.equal(area(got[p], p), area(want[p], p)), \
                f"picture {k} plane {p}: band pipeline != whole-frame chain"
    for r, slot in pipe.sof.items():
        st = pipe.frame_planes([fs.luma, fs.cb, fs.cr], slot)
        fin = pipe.final_planes(pipe.kof[r]) if r in pipe.kof else None
        if fin is None:
            continue
        for p in range(3):
            assert torch.equal(st[p], fin[p]), f"reference store of picture {r} plane {p}"
    assert len(pipe.store) >= 2 and any(len(pipe.sched.refs[j]) >= 3 for j in pipe.local)
    orc = CpuOracle("oracle", 8)
    orc.nthreads = 8
    bad = []
    host = {"Y": fs.luma.cpu().numpy(), "U": fs.cb.cpu().numpy(), "V": fs.cr.cpu().numpy(),
            "R": fs.resid.cpu().numpy()}
    for b in pipe.batches:
        m = b.verify_sample(orc, host, b.sample(16))
        if m:
            bad.append((b.name, m))
    assert not bad, bad[:5]
    if exchange == "rccl":
        assert sum(len(t) for t in pipe.ex.tables) > 0


@pytest.mark.parametrize("band_rows,frames,segment", [(1, 11, 11), (2, 16, 8)])
def test_cpp_frame_shard_host_one_rank(tmp_path, band_rows, frames, segment):
    """integration/frame_shard_host (C++ only: x265amd_schedule, the row-band loop filters and
    x265amd_exchange loop-back transfers into the rank's reference stores): every picture equals the
    whole-frame deblock -> SAO -> border chain and every store slot its producer's picture"""
    import json
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_bin",
                       "frame_shard_host")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    r = subprocess.run([exe, "416", "240", str(frames), str(band_rows), "1", "0", str(tmp_path / "id"), str(segment),
                        "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["mismatches"] == 0 and out["transfers"] > 0 and out["stores"] >= 2, out
