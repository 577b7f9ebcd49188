#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes (HBM traffic per bench launch).

Runs the bench step (same FrameSet, seed and grouped launches as bench.py,
eager launches so every dispatch is its own counter row) `--steps` times, then
two calibration kernels with known byte counts on disjoint, cache-cold tiles
(SAD 64x64: reads only; copy_pp 64x64: reads + writes), and writes the launch
order to --order so tools/pmc_parse.py can attribute the dispatch rows.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
        python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json
    (again with --pmc WRITE_SIZE into gpurun_out/pmc_write)
    python3 tools/pmc_parse.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_order.json \
        --out profiles/pmc_traffic.json
Other configurations (--width / --height / --depth / --preset, as bench.py) go to
profiles/pmc_traffic_<height>p_<preset>_<depth>bit.json, which bench.py reads for them.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--order", required=True)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--preset", default="medium")
    a = ap.parse_args()

    import torch

    from src.x265_amd import Primitives
    from src.x265_amd.workload import FrameSet, WorkloadBuilder, census_batches, group_launches, load_census

    prims = Primitives(device=0)
    from src.x265_amd import replay_bench

    census, _ = replay_bench.pick_census(a)            # the census bench.py uses for this configuration
    fs = FrameSet(a.width, a.height, a.frames, a.depth, device="cuda:0")
    batches, _ = census_batches(fs, frames=a.frames, census=census, builder=WorkloadBuilder(fs, seed=11))
    launches = group_launches(batches)
    # a one-element fill after every launch marks its end (a launch may dispatch several kernels,
    # tools/pmc_segments.py)
    mark = torch.zeros(1, device="cuda")
    for _ in range(a.steps):
        for g in launches:
            g.run(prims)
            mark.fill_(1.0)
    torch.cuda.synchronize()

    # calibration: disjoint 64x64 tiles through >= 1.5 GB (cache-cold)
    W, s = 8192, 64
    n = int(1.5e9 / 2 / (s * s))
    import numpy as np

    j = np.arange(n, dtype=np.int64)
    off = torch.from_numpy((j // (W // s)) * s * W + (j % (W // s)) * s).cuda()
    rows = (n // (W // s) + 1) * s
    A = torch.randint(0, 256, (rows * W,), dtype=torch.uint8, device="cuda")
    B = torch.randint(0, 256, (rows * W,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    prims.pixelcmp(0, 8, s, s, A, W, off, B, W, off, out)
    D = torch.empty(n * s * s, dtype=torch.uint8, device="cuda")
    doff = torch.arange(n, dtype=torch.int64, device="cuda") * (s * s)
    prims.blockop(4, 8, s, s, D, s, doff, A, W, off, None, 0, None)
    torch.cuda.synchronize()

    order = {"steps": a.steps, "marker": True, "launches": [{"name": g.name, "kind": g.kind, "bytes": g.bytes, "jobs": g.n}
                                            for g in launches],
             # known bytes: blocks + int64 job offsets (one offset array for both operands of the SAD)
             "calibration": [{"name": "cal_sad_64x64", "kind": "pixelcmp", "read_bytes": 2 * n * s * s + 8 * n,
                              "write_bytes": 4 * n},
                             {"name": "cal_copy_pp_64x64", "kind": "blockop", "read_bytes": n * s * s + 16 * n,
                              "write_bytes": n * s * s}]}
    with open(a.order, "w") as f:
        json.dump(order, f, indent=1)
    print(f"[pmc_workload] {len(launches)} launches x {a.steps} steps + 2 calibration kernels")


if __name__ == "__main__":
    main()
