#!/usr/bin/env python3
"""Mean PMC counters per kernel name from rocprofv3 --pmc CSV output (CPU only).

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... --output-format csv -d gpurun_out/pmc_k -o run -- \
        python3 tools/kernel_roofline.py --only luma_ --reps 2
    python3 tools/pmc_kernels.py gpurun_out/pmc_k [--out profiles/r02/pmc_kernels.json]

Derived (when the counters are present; SQ cycle counters are quad-cycles, MI355X_MICROARCH.md):
  valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  lds_active_frac  = SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  wait_inst_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (waiting on an outstanding memory result)
  wait_any_frac    = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  waves_resident   = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES     (mean resident waves over the busy time, chip-wide)
  fetch_bytes      = FETCH_SIZE * 1024 * 2 (gfx950 wide-load correction), write_bytes = WRITE_SIZE * 1024
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))
            with open(path) as f:
                for r in csv.DictReader(f):
                    key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"])
                    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            for (_, name), cs in per.items():
                for c, v in cs.items():
                    acc[name][c].append(v)
    out = {}
    for name, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dict(m)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for k, c in (("valu_active_frac", "SQ_ACTIVE_INST_VALU"), ("lds_active_frac", "SQ_ACTIVE_INST_LDS"),
                         ("wait_inst_frac", "SQ_WAIT_INST_ANY"), ("wait_any_frac", "SQ_WAIT_ANY")):
                if c in m:
                    d[k] = round(m[c] / wc, 3)
            if m.get("SQ_BUSY_CYCLES"):
                d["waves_resident"] = round(wc / m["SQ_BUSY_CYCLES"], 1)
        if "FETCH_SIZE" in m:
            d["fetch_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            d["write_bytes"] = m["WRITE_SIZE"] * 1024
        short = name.split("(")[0][:90]
        out[short] = d
        print(short, json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
