#!/usr/bin/env python3
"""Sum a rocprofv3 --pmc counter_collection.csv per kernel name: dispatches and the total of each
counter (rocprofv3 writes one row per dispatch and counter).  Prints JSON {kernel: {"dispatches": n,
counter: total, ...}} sorted by dispatch count; the raw CSV of a long encode is tens of MB.

    python tools/pmc_by_kernel.py <rocprofv3 output dir>
"""
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    agg = {}
    seen = set()
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "?")
                a = agg.setdefault(name, {"dispatches": 0})
                disp = (f, row.get("Dispatch_Id"))
                if disp not in seen:
                    seen.add(disp)
                    a["dispatches"] += 1
                ctr = row.get("Counter_Name")
                if ctr:
                    a[ctr] = a.get(ctr, 0.0) + float(row.get("Counter_Value") or 0)
    out = dict(sorted(agg.items(), key=lambda kv: -kv[1]["dispatches"]))
    json.dump({"files": len(files), "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
