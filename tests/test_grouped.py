"""Grouped multi-shape launches (x265amd_*_grouped, csrc/common.h BatchGroup).

CPU: the Python launch grouping (workload.group_launches) packs only batches
of one kernel class, at most 16 per launch, and keeps every batch exactly once.
GPU: one grouped call over every shape of a family (more than 16 per class, so
the library splits launches itself) matches the CPU oracle bit-exactly, and the
census workload gives identical outputs grouped and one launch per batch.
"""
import numpy as np
import pytest

from cases import (ADDAVG, CHROMA420_PU, COPY_PP, CPY2D1D_SHR, HPP, HPS, HVPP, LUMA_PU, P2S, PSY, SA8D, SA8D_SIZES,
                   SAD, SATD, SATD_SIZES, SSE_PP, SSE_PP_SIZES, SUB_PS, VAR, VPP, VSP, case_blockop, case_interp,
                   case_pixelcmp, case_sad_multi, run_cpu, seed_of)
from pyoracle import CpuOracle


# ------------------------------------------------------------------ CPU side
class _B:
    def __init__(self, kind, op, w, h, depth=8, taps=8, rowext=0, nbytes=1.0):
        self.kind, self.op, self.w, self.h, self.depth, self.taps = kind, op, w, h, depth, taps
        self.params = {"rowext": rowext}
        self.bytes, self.n, self.name = nbytes, 1, f"{kind}.{op}.{w}x{h}.{taps}.{rowext}"


def test_group_launches_one_class_per_launch():
    from src.x265_amd.workload import MAX_SUB, group_launches, launch_class

    bs = [_B("pixelcmp", op, w, h) for op in (SAD, SATD) for (w, h) in LUMA_PU]
    bs += [_B("pixelcmp", SA8D, w, h) for (w, h) in SA8D_SIZES]
    bs += [_B("interp", op, w, h, taps=t, rowext=r) for op in (HPP, HPS, VPP) for t in (4, 8) for r in (0, 1)
           for (w, h) in LUMA_PU]
    bs += [_B("blockop", COPY_PP, w, h) for (w, h) in CHROMA420_PU]
    bs += [_B("transform", 0, 8, 8)]
    groups = group_launches(bs)
    seen = [id(b) for g in groups for b in g.members]
    assert sorted(seen) == sorted(id(b) for b in bs)
    for g in groups:
        assert 1 <= len(g.members) <= MAX_SUB
        assert len({launch_class(b) for b in g.members}) == 1
    # SA8D: 16x16-multiple, 8x8-multiple and satd-aliased shapes are three classes
    assert len({launch_class(b) for b in bs if b.op == SA8D and b.kind == "pixelcmp"}) == 3
    # fewer launches than batches
    assert len(groups) < len(bs) / 4


# ------------------------------------------------------------------ GPU side
def _dev(v):
    import torch

    return torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) else v


def _run_grouped(family, op, cases, prims, taps=8, nref=4):
    """All `cases` (one family/op, any shapes) in ONE grouped C-ABI call."""
    import torch

    from src.x265_amd import native as nv

    bufs = [{k: _dev(v) for k, v in c.bufs.items()} for c in cases]
    depth = cases[0].params["depth"]
    if family == "pixelcmp":
        arr = nv.cmp_batches([(c.params["w"], c.params["h"], b["a"], b["sa"], b["aoff"], b["b"], b["sb"], b["boff"],
                               b["out"]) for c, b in zip(cases, bufs)])
        prims.pixelcmp_grouped(op, depth, arr)
    elif family == "sad_multi":
        arr = nv.cmp_batches([(c.params["w"], c.params["h"], b["f"], b["fs"], b["foff"], b["r"], b["rs"], b["roff"],
                               b["out"]) for c, b in zip(cases, bufs)])
        prims.sad_multi_grouped(nref, depth, arr)
    elif family == "interp":
        arr = nv.interp_batches([(c.params["w"], c.params["h"], c.params["rowext"], b["s"], b["ss"], b["soff"], b["d"],
                                  b["ds"], b["doff"], b["coeff"]) for c, b in zip(cases, bufs)])
        prims.interp_grouped(op, taps, depth, arr)
    else:
        arr = nv.block_batches([(c.params["w"], c.params["h"], b["param"], b["d"], b["ds"], b["doff"], b["a"], b["sa"],
                                 b["aoff"], b["b"], b["sb"], b["boff"]) for c, b in zip(cases, bufs)])
        prims.blockop_grouped(op, depth, arr)
    torch.cuda.synchronize()
    return [{k: b[k].cpu().numpy() for k in c.outs} for c, b in zip(cases, bufs)]


@pytest.fixture(scope="module")
def prims(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a gfx950 device"
    from src.x265_amd import Primitives

    return Primitives(device=0)


def _families(depth):
    n = 96
    fam = []
    for op, sizes in ((SAD, LUMA_PU), (SATD, SATD_SIZES), (SA8D, SA8D_SIZES), (SSE_PP, SSE_PP_SIZES),
                      (PSY, [(s, s) for s in (4, 8, 16, 32, 64)]), (VAR, [(s, s) for s in (8, 16, 32, 64)])):
        fam.append(("pixelcmp", op, 8, [case_pixelcmp(op, w, h, depth, n, seed_of("gp", op, depth, w, h))
                                        for (w, h) in sizes]))
    fam.append(("sad_multi", 4, 8, [case_sad_multi(4, w, h, depth, n, seed_of("gx", depth, w, h)) for (w, h) in LUMA_PU]))
    for op, taps, rowext in ((HPP, 8, 0), (HPS, 8, 1), (VPP, 8, 0), (VSP, 4, 0), (HVPP, 8, 0), (P2S, 4, 0),
                             (HPP, 4, 0)):
        sizes = LUMA_PU if taps == 8 else [s for s in CHROMA420_PU if s != (2, 2)]
        fam.append(("interp", op, taps, [case_interp(op, taps, w, h, depth, 48, seed_of("gi", op, taps, depth, w, h),
                                                     rowext) for (w, h) in sizes]))
    for op in (SUB_PS, ADDAVG, COPY_PP, CPY2D1D_SHR):
        sizes = [(s, s) for s in (4, 8, 16, 32)] if op == CPY2D1D_SHR else LUMA_PU + CHROMA420_PU
        fam.append(("blockop", op, 8, [case_blockop(op, w, h, depth, 48, seed_of("gb", op, depth, w, h))
                                       for (w, h) in sizes if w % 2 == 0]))
    return fam


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_grouped_call_matches_oracle(prims, oracle_libs, depth):
    orc = CpuOracle("oracle", depth)
    orc.nthreads = 8
    bad = []
    for family, op, taps, cases in _families(depth):
        outs = _run_grouped(family, op, cases, prims, taps=taps, nref=op)
        for c, o in zip(cases, outs):
            ref = run_cpu(c, orc)
            for k in c.outs:
                if not np.array_equal(o[k], ref[k]):
                    bad.append(f"{family}:{op}:{c.key()}")
    assert not bad, bad[:12]


@pytest.mark.gpu
def test_grouped_census_equals_single_launches(prims):
    """Bench workload: grouped launches write exactly what per-batch launches write."""
    import torch

    from src.x265_amd.workload import FrameSet, census_batches, group_launches

    fs = FrameSet(1920, 1080, nframes=2, depth=8, device="cuda")
    batches, _ = census_batches(fs, frames=2, scale=0.25)
    groups = group_launches(batches)
    assert len(groups) < len(batches)
    outs = lambda: {(b.name, k): b.dev[k].clone() for b in batches for k in b.outs}
    for b in batches:
        b.run(prims)
    torch.cuda.synchronize()
    single = outs()
    for b in batches:
        for k in b.outs:
            b.dev[k].fill_(0x5A if b.dev[k].dtype == torch.uint8 else 77)
    for g in groups:
        g.run(prims)
    torch.cuda.synchronize()
    grouped = outs()
    diff = [key for key in single if not torch.equal(single[key], grouped[key])]
    assert not diff, diff[:10]
