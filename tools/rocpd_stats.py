#!/usr/bin/env python3
"""rocprofv3 --kernel-trace --stats summary from its results database (rocpd sqlite),
in the columns of rocprofv3's kernel_stats.csv.  CPU only.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/r02/rocprof_kernel_stats.csv
"""
import sqlite3
import sys


def main():
    cur = sqlite3.connect(sys.argv[1]).cursor()
    q = ("select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
         "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by sum(d.end - d.start) desc")
    rows = list(cur.execute(q))
    total = sum(r[2] for r in rows) or 1
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for name, n, tot, avg, mn, mx in rows:
        print(f'"{name}",{n},{tot},{avg:.1f},{100.0 * tot / total:.3f},{mn},{mx}')


if __name__ == "__main__":
    main()
