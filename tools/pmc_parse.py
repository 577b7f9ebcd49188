#!/usr/bin/env python3
"""HBM traffic per bench launch from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE) over tools/pmc_workload.py.  CPU only.

Units and gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md
§7): both counters are KiB; FETCH_SIZE under-reports wide streaming reads (up
to 2x) and other access widths are uncalibrated, so each counter is scaled by
the factor measured on a calibration kernel of KNOWN bytes run in the same
process on disjoint, cache-cold tiles with the same 8-byte-per-lane loads the
primitive kernels use (SAD 64x64 for reads, copy_pp 64x64 for writes).

    python3 tools/pmc_parse.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_order.json \
        --out profiles/pmc_traffic.json
"""
from __future__ import annotations

import argparse
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("order")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    order = json.load(open(a.order))
    L, steps = order["launches"], order["steps"]
    from pmc_segments import launch_groups

    fe, cf = launch_groups(a.fetch_dir, order)
    wr, cw = launch_groups(a.write_dir, order)
    kind_kernel = {"pixelcmp": "k_pixelcmp", "sad_multi": "k_sad_multi", "interp": ("k_interp", "k_hvpp"),
                   "blockop": "k_blockop", "transform": ("k_tr", "k_dst"), "quant": "k_quant",
                   "dequant": "k_dequant", "intra": "k_intra", "intra_filter": "k_intra_filter", "count": "k_count"}
    cal = order["calibration"]
    read_corr = cal[0]["read_bytes"] / (cf[0][2]["FETCH_SIZE"] * 1024)
    write_corr = cal[1]["write_bytes"] / (cw[1][2]["WRITE_SIZE"] * 1024)
    out = {"_units": "bytes per launch; hbm_bytes = FETCH_SIZE*1024*read_corr + WRITE_SIZE*1024*write_corr "
                     "(summed over a launch's dispatches)",
           "_calibration": {"read_corr": round(read_corr, 4), "write_corr": round(write_corr, 4),
                            "copy_read_corr_crosscheck": round(cal[1]["read_bytes"] / (cf[1][2]["FETCH_SIZE"] * 1024), 4),
                            "kernels": [c["name"] for c in cal]}}
    for g, f, w in zip(L, fe, wr):
        kk = kind_kernel.get(g["kind"], "")
        kk = kk if isinstance(kk, tuple) else (kk,)
        assert any(k in f[0] for k in kk), (g["name"], f[0])
        fk, wk = f[2]["FETCH_SIZE"], w[2]["WRITE_SIZE"]
        hbm = fk * 1024 * read_corr + wk * 1024 * write_corr
        out[g["name"]] = {"kernel": f[0].split("(")[0].replace("void ", ""), "dispatches": f[1], "fetch_kib": fk,
                          "write_kib": wk, "hbm_bytes": int(hbm), "algorithmic_bytes": int(g["bytes"]),
                          "hbm_over_algorithmic": round(hbm / max(1.0, g["bytes"]), 3)}
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    tot_h = sum(v["hbm_bytes"] for k, v in out.items() if not k.startswith("_"))
    tot_a = sum(v["algorithmic_bytes"] for k, v in out.items() if not k.startswith("_"))
    print(f"{len(L)} launches: HBM {tot_h / 1e9:.3f} GB vs algorithmic {tot_a / 1e9:.3f} GB per step; "
          f"read_corr {read_corr:.3f} write_corr {write_corr:.3f}")


if __name__ == "__main__":
    main()
