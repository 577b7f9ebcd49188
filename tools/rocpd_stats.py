#!/usr/bin/env python3
"""rocprofv3 --kernel-trace --stats summary from its results database (rocpd sqlite),
in the columns of rocprofv3's kernel_stats.csv.  CPU only.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/r02/rocprof_kernel_stats.csv
    python tools/rocpd_stats.py gpurun_out/prof/run_results.db --by-grid > profiles/r02/rocprof_kernel_grid_stats.csv

--by-grid splits each kernel by its grid size, so one bench launch (a grouped launch has
one grid size per step) can be compared with bench.py's own kernel_ms.
"""
import sqlite3
import sys


def main():
    cur = sqlite3.connect(sys.argv[1]).cursor()
    by_grid = "--by-grid" in sys.argv[2:]
    grid = ", d.grid_size_x" if by_grid else ""
    q = (f"select s.kernel_name{grid}, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
         "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         f"group by s.kernel_name{grid} order by sum(d.end - d.start) desc")
    rows = list(cur.execute(q))
    total = sum(r[-4] for r in rows) or 1
    print('"Name",' + ('"GridX",' if by_grid else "") + '"Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for r in rows:
        name, rest = r[0], r[1:]
        g = f"{rest[0]}," if by_grid else ""
        n, tot, avg, mn, mx = rest[-5:]
        print(f'"{name}",{g}{n},{tot},{avg:.1f},{100.0 * tot / total:.3f},{mn},{mx}')


if __name__ == "__main__":
    main()
