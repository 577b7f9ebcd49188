#!/usr/bin/env python3
"""SQ (shader sequencer) counters per bench launch from one rocprofv3 PMC pass
over tools/pmc_workload.py.  CPU only.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/pmc_workload.py --order ...
    python3 tools/pmc_sq.py gpurun_out/pmc_sq gpurun_out/pmc_order.json --out profiles/r02/pmc_sq.json

Per launch (last step): the raw counters (summed over the dispatch's XCDs /
SEs as rocprofv3 reports them) and
  valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
      (share of resident-wave time spent issuing VALU; both count quad-cycles,
       MI355X_MICROARCH.md constants table),
  valu_insts_per_wave = SQ_INSTS_VALU / SQ_WAVES.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

COUNTERS = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq_dir")
    ap.add_argument("order")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    order = json.load(open(a.order))
    L, steps = order["launches"], order["steps"]
    from pmc_segments import launch_groups

    groups, _ = launch_groups(a.sq_dir, order)
    out = {"_counters": COUNTERS, "_derived": "valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES "
                                              "(counters summed over a launch's dispatches)"}
    for g, (name, nd, c) in zip(L, groups):
        e = {"kernel": name.split("(")[0].replace("void ", ""), "dispatches": nd, **{k: c.get(k) for k in COUNTERS}}
        if c.get("SQ_WAVE_CYCLES"):
            e["valu_active_frac"] = round(c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_WAVES"):
            e["valu_insts_per_wave"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"], 1)
        out[g["name"]] = e
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    print(f"{len(L)} launches written to {a.out}")


if __name__ == "__main__":
    main()
