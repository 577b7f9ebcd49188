#!/usr/bin/env python3
"""MFMA utilisation of the matrix-core transforms from one rocprofv3 PMC pass over
tools/kernel_roofline.py (SQ_VALU_MFMA_BUSY_CYCLES, SQ_WAIT_ANY, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE).  CPU only.

    python3 tools/mfma_util.py gpurun_out/pmc_tr > profiles/r03/pmc_transform_split/mfma_utilisation.json

mfma_busy_frac_of_1024_simds = MFMA busy cycles / (kernel GPU cycles x 1024 SIMDs), counters
summed over a kernel's dispatches; kernel GPU cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 reports the
sum over the 8 XCDs, MI355X_MICROARCH.md "DVFS give-back").
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    sums = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0]
                if "_mfma" in k:
                    sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, c in sums.items():
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        out[k] = {"mfma_busy_cycles": c["SQ_VALU_MFMA_BUSY_CYCLES"], "kernel_cycles": cyc,
                  "mfma_busy_frac_of_1024_simds": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, cyc * 1024), 4),
                  "wait_any_frac": round(c["SQ_WAIT_ANY"] / max(1.0, c["SQ_WAVE_CYCLES"]), 3),
                  "valu_active_frac": round(c["SQ_ACTIVE_INST_VALU"] / max(1.0, c["SQ_WAVE_CYCLES"]), 3)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
