"""CPU coverage of the bench workload plumbing (no GPU): the census batches
are built over a 1080p FrameSet, executed through the CPU call surface
(oracle restatement) and a sample of every batch is re-checked against the
reference x265 C primitives.  The GPU version of this check is
test_gpu_parity.py::test_gpu_fullsize_frame_batch."""
import pytest

from pyoracle import CpuOracle, CpuPrims, available


@pytest.mark.skipif(not available("ref", 8), reason="reference library oracle/_ref not built")
def test_census_batches_cpu_roundtrip(oracle_libs):
    from src.x265_amd.workload import FrameSet, census_batches, load_census

    census = load_census()
    assert sum(census.values()) > 1e6            # per-frame calls of a 1080p medium encode
    fs = FrameSet(1920, 1080, 2, 8, device="cpu")
    batches, wb = census_batches(fs, frames=2, scale=0.01, census=census)
    assert len(batches) > 100
    assert "scalar.costCoeffNxN" in wb.skipped      # CABAC estimation stays on the CPU
    prims = CpuPrims("oracle", 8, nthreads=4)
    ref = CpuOracle("ref", 8)
    bad = []
    for b in batches:
        b.run(prims)
        m = b.verify_sample(ref, fs.host, b.sample(8))
        if m:
            bad.append((b.name, m))
    assert not bad, bad[:5]


def test_frame_layout_matches_picyuv():
    from src.x265_amd.workload import FrameSet

    fs = FrameSet(1920, 1080, 1, 8, device="cpu")
    # picyuv.cpp:62-80 for a 64x64 CTU: luma stride 2112, chroma stride 1152
    assert (fs.stride, fs.cstride) == (2112, 1152)
    assert (fs.mx, fs.my, fs.cmy) == (96, 80, 40)
    assert fs.ref_of(0) == 1 and fs.ref_of(1) == 0
