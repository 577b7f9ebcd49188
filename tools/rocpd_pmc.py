#!/usr/bin/env python3
"""Per-kernel PMC totals from a rocprofv3 results database (rocpd sqlite).

    python tools/rocpd_pmc.py gpurun_out/pmc/x/run_results.db [kernel-substring]

Prints, per kernel symbol: dispatches, mean duration, each counter summed over
its dispatches, and the SQ wave-cycle breakdown (WAIT_ANY / WAIT_INST_ANY /
ACTIVE_INST_*) as fractions of SQ_WAVE_CYCLES when those were collected."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cur = sqlite3.connect(db).cursor()
    q = ("select s.kernel_name, i.name, sum(e.value) from rocpd_pmc_event e "
         "join rocpd_info_pmc i on e.pmc_id = i.id "
         "join rocpd_kernel_dispatch d on d.event_id = e.event_id "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name, i.name")
    per = {}
    for k, name, v in cur.execute(q):
        per.setdefault(k, {})[name] = v
    q2 = ("select s.kernel_name, count(*), avg(d.end - d.start) from rocpd_kernel_dispatch d "
          "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name")
    for k, cnt, dur in cur.execute(q2):
        if filt and filt not in k:
            continue
        d = per.get(k, {})
        print(f"{k[:90]}  dispatches={cnt} mean_us={dur / 1e3:.1f}")
        for name, v in sorted(d.items()):
            print(f"    {name:24s} {v:.4g}")
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            print("    wave-cycle shares:", {n: round(d[n] / wc, 3) for n in
                                             ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                              "SQ_ACTIVE_INST_VALU") if n in d})


if __name__ == "__main__":
    main()
