"""The frame-parallel GPU step (src/x265_amd/frame_pipeline.py) on one GPU.

Frames are encoded band by band (census primitive work per band + the f4 row-band
loop filters) and published into the next frame's reference slot.  Checked: every
frame's final reconstruction equals the whole-frame deblock -> SAO -> border chain
(x265amd_deblock / _sao_apply / _extend_border, themselves bit-exact vs the
reference's Deblock / SAO classes in test_f4.py) on the same picture; every
reference slot holds the previous frame's final reconstruction, margins included;
and every census batch still matches the oracle on sampled jobs after the band split
(a job that read a reference row before it was published would not).  Both schedules:
frame by frame, and the single-rank wavefront.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("band_rows,wave", [(1, False), (3, False), (1, True), (4, True)])
def test_gpu_pipeline_rows_equal_whole_frame(gpu_prims, oracle_libs, band_rows, wave):
    """wave=True: the single-rank wavefront schedule (frame k's band b at step k * d + b, one set
    of grouped launches per step, the whole sequence one hipGraph) must give the same frames"""
    import torch

    from pyoracle import CpuOracle
    from src.x265_amd.frame_pipeline import GpuFramePipeline

    W, H, F = 416, 240, 4
    pipe = GpuFramePipeline(gpu_prims, W, H, 8, F, 1, 0, band_rows=band_rows, streams=4, device="cuda")
    if wave:
        pipe.build_wave()
    else:
        pipe.build(graphs=True)
    pipe.step()
    torch.cuda.synchronize()
    fs = pipe.fs
    # whole-frame f4 chain on a copy of each frame's source (the pipeline's stand-in reconstruction)
    work = [t.clone() for t in (fs.luma, fs.cb, fs.cr)]
    final = [torch.zeros_like(t) for t in work]
    saved = (pipe.work, pipe.final)
    pipe.work, pipe.final = work, final
    pipe._f4_setup(W, H, "cuda")
    gpu_prims.deblock(8, pipe.dbk)
    gpu_prims.sao_apply(8, pipe.sao)
    gpu_prims.extend_border(8, [bp for bps in pipe.bor for bp in bps])
    torch.cuda.synchronize()
    pipe.work, pipe.final = saved
    for k in range(F):
        got, want = pipe.frame_planes(pipe.final, k), pipe.frame_planes(final, k)
        for p in range(3):
            assert torch.equal(got[p], want[p]), f"frame {k} plane {p}: band pipeline != whole-frame chain"
        if k + 1 < F:
            ref = pipe.frame_planes([fs.luma, fs.cb, fs.cr], F + k + 1)
            for p in range(3):
                assert torch.equal(ref[p], got[p]), f"reference slot of frame {k + 1} plane {p}"
    orc = CpuOracle("oracle", 8)
    orc.nthreads = 8
    bad = []
    for b in pipe.batches:
        m = b.verify_sample(orc, {"Y": fs.luma.cpu().numpy(), "U": fs.cb.cpu().numpy(), "V": fs.cr.cpu().numpy(),
                                  "R": fs.resid.cpu().numpy()}, b.sample(16))
        if m:
            bad.append((b.name, m))
    assert not bad, bad[:5]
