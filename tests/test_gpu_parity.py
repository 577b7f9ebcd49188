"""GPU parity of the gfx950 kernels (through the C ABI) — bit-exact.

1. every case of cases.all_cases() against the golden hashes from the
   reference x265 1.9 C primitives (both bit depths);
2. larger random batches against the CPU oracle;
3. full-size (bench) batches over HBM-resident 1080p planes: a 1/64 sample
   of the jobs is recomputed on the CPU oracle and must match exactly, and
   size-independent properties are checked on the whole batch.
"""
import json
import os

import numpy as np
import pytest

from cases import (DCT, HPP, HVPP, IDCT, LUMA_PU, SA8D, SAD, SATD, VPP, all_cases, case_interp, case_pixelcmp,
                   case_sad_multi, case_transform, run_cpu, run_gpu, seed_of)
from pyoracle import CpuOracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def prims(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a gfx950 device"
    from src.x265_amd import Primitives

    return Primitives(device=0)


@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_matches_reference_golden(prims, depth):
    with open(os.path.join(GOLDEN, f"golden_d{depth}.json")) as f:
        g = json.load(f)
    bad = []
    for c, e in zip(all_cases(depth), g["cases"]):
        outs = run_gpu(c, prims)
        if c.output_hashes(outs) != e["sha256"]:
            detail = ""
            if "values" in e:
                k = next(iter(e["values"]))
                detail = f" gpu={outs[k].tolist()[:8]} ref={e['values'][k][:8]}"
            bad.append(c.key() + detail)
    assert not bad, f"{len(bad)}/{len(g['cases'])} mismatches:\n" + "\n".join(bad[:20])


@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_matches_oracle_random(prims, oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    orc.nthreads = 8
    cases = []
    for (w, h) in LUMA_PU:
        for op in (SAD, SATD):
            cases.append(case_pixelcmp(op, w, h, depth, 512, seed_of("g", op, depth, w, h)))
        cases.append(case_sad_multi(4, w, h, depth, 256, seed_of("gx4", depth, w, h)))
        for op in (HPP, VPP, HVPP):
            cases.append(case_interp(op, 8, w, h, depth, 128, seed_of("gi", op, depth, w, h)))
    for n in (8, 16, 32, 64):
        cases.append(case_pixelcmp(SA8D, n, n, depth, 512, seed_of("gs", depth, n)))
    for n in (4, 8, 16, 32):
        cases.append(case_transform(DCT, n, depth, 512, seed_of("gd", depth, n)))
        cases.append(case_transform(IDCT, n, depth, 512, seed_of("gid", depth, n)))
    bad = []
    for c in cases:
        a, b = run_gpu(c, prims), run_cpu(c, orc)
        for k in c.outs:
            if not np.array_equal(a[k], b[k]):
                bad.append(c.key())
    assert not bad, bad[:10]


@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_interp_compact_destinations(prims, oracle_libs, depth):
    """every interp op into census-style compact slots (stride = width): the 8-bit LDS-staged
    write-back (interp.hip k_interp / k_hvpp_stream STG) for power-of-two shapes, the direct
    stores otherwise;
    77 jobs leave a partial last wavefront, the slot order is shuffled and five slots stay
    untouched"""
    orc = CpuOracle("oracle", depth)
    bad = []
    from cases import HPS, P2S, VPS, VSP, VSS
    for op in (HPP, HPS, VPP, VPS, VSP, VSS, P2S, HVPP):
        for taps in ((8,) if op == HVPP else (4,) if op == P2S else (4, 8)):
            for (w, h) in ((4, 4), (8, 4), (4, 8), (8, 8), (16, 16), (32, 32), (64, 64), (16, 8), (8, 32), (32, 16),
                           (16, 64), (64, 16), (12, 16), (24, 32), (16, 4)):
                c = case_interp(op, taps, w, h, depth, 77, seed_of("gc", op, taps, depth, w, h), compact=True)
                a, b = run_gpu(c, prims), run_cpu(c, orc)
                if not np.array_equal(a["d"], b["d"]):
                    bad.append(c.key())
    assert not bad, bad[:10]


@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_blockop_compact_destinations(prims, oracle_libs, depth):
    """every block op into compact, shuffled stride-w slots: the LDS-staged write-back
    (blockops.hip k_blockop STG) for power-of-two shapes, direct stores otherwise; 77 jobs
    leave a partial last wavefront and partial two-job lane groups"""
    from cases import (ADD_PS, ADDAVG, BLOCKFILL, COPY_PP, COPY_PS, COPY_SP, COPY_SS, CPY1D2D_SHL, CPY2D1D_SHR,
                       PIXELAVG, SUB_PS, TRANSPOSE, case_blockop)
    orc = CpuOracle("oracle", depth)
    bad = []
    for op in (SUB_PS, ADD_PS, ADDAVG, PIXELAVG, COPY_PP, COPY_SP, COPY_PS, COPY_SS, BLOCKFILL, CPY2D1D_SHR,
               CPY1D2D_SHL, TRANSPOSE):
        for (w, h) in ((4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (16, 8), (8, 32), (12, 16), (16, 4), (8, 2)):
            if op in (TRANSPOSE, CPY2D1D_SHR, CPY1D2D_SHL, BLOCKFILL) and w != h:
                continue
            c = case_blockop(op, w, h, depth, 77, seed_of("gbc", op, depth, w, h), compact=True)
            a, b = run_gpu(c, prims), run_cpu(c, orc)
            if not np.array_equal(a["d"], b["d"]):
                bad.append(c.key())
    assert not bad, bad[:10]


CENSUSES = [("census_1080p_medium.json", 1920, 1080, 8), ("census_2160p_medium.json", 3840, 2160, 8),
            ("census_2160p_slow.json", 3840, 2160, 8), ("census_2160p_medium_main10.json", 3840, 2160, 10)]


@pytest.mark.parametrize("census_file,width,height,depth", CENSUSES, ids=[c[0][7:-5] for c in CENSUSES])
def test_gpu_fullsize_frame_batch(prims, oracle_libs, census_file, width, height, depth):
    """Every batch of a recorded census (BASELINE configs 2, 3 and 5: 1080p medium, 2160p
    medium, 2160p slow with rect PUs / nquant, 2160p Main10) on full-size planes, issued
    through the bench's grouped launches: sampled exact parity of every batch against the
    oracle + properties."""
    import torch

    from src.x265_amd.workload import FrameSet, census_batches, group_launches, load_census

    census = load_census(os.path.join(os.path.dirname(__file__), "golden", census_file))
    fs = FrameSet(width, height, nframes=2, depth=depth, device="cuda")
    orc = CpuOracle("oracle", depth)
    orc.nthreads = 8
    batches, wb = census_batches(fs, frames=2, census=census)
    assert len(batches) > 100
    for g in group_launches(batches):
        g.run(prims)
    torch.cuda.synchronize()
    bad = []
    for b in batches:
        mism = b.verify_sample(orc, fs.host, b.sample(48))
        if mism:
            bad.append((b.name, mism))
        if b.kind == "pixelcmp" and b.op in (SAD, SATD, SA8D):
            assert int(b.dev["out"].min()) >= 0, b.name
    assert not bad, bad[:10]


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_gpu_writes_stay_inside_outputs(prims, depth):
    """every golden case again with each output buffer inside 64 Ki canary elements on both sides: no kernel
    writes outside the outputs it is given (a stray write corrupts other allocations silently and surfaces
    later, in another kernel, as wrong data or an illegal address)"""
    bad = []
    for c in all_cases(depth):
        guard = {}
        run_gpu(c, prims, guard=guard)
        bad += [f"{c.key()}:{k}" for k, ok in guard.items() if not ok]
    assert not bad, f"{len(bad)} outputs with writes outside them:\n" + "\n".join(bad[:20])
