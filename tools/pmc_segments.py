"""Group rocprofv3 PMC rows of tools/pmc_workload.py by bench launch.  CPU only.

A grouped launch dispatches one kernel per kernel class it holds (a batch group that mixes
LDS-staged and direct-store classes dispatches two), so pmc_workload.py issues a one-element
torch fill after every launch as a marker ("marker": true in the order file): the x265amd
dispatches between two markers are one launch and their counter values are summed.  Order
files without markers keep the one-dispatch-per-launch reading.
"""
from __future__ import annotations

import csv
import glob
import os
from collections import defaultdict


def read_rows(d: str):
    """{dispatch id: (kernel name, {counter: value summed over the row's instances})}"""
    vals, names = defaultdict(lambda: defaultdict(float)), {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                i = int(r["Dispatch_Id"])
                vals[i][r["Counter_Name"]] += float(r["Counter_Value"])
                names[i] = r["Kernel_Name"]
    return {i: (names[i], dict(vals[i])) for i in vals}


def launch_groups(d: str, order: dict):
    """(per-launch entries of the LAST step, calibration entries); an entry is
    (kernel name of its first dispatch, number of dispatches, {counter: summed value})"""
    rows = read_rows(d)
    ids = sorted(rows)
    L, steps, ncal = order["launches"], order["steps"], len(order["calibration"])
    own = [i for i in ids if "x265amd::" in rows[i][0]]
    cal = [(rows[i][0], 1, rows[i][1]) for i in own[-ncal:]]
    if not order.get("marker"):
        want = steps * len(L) + ncal
        assert len(own) == want, (len(own), want)
        last = own[(steps - 1) * len(L): steps * len(L)]
        return [(rows[i][0], 1, rows[i][1]) for i in last], cal
    groups, cur = [], []
    cal_ids = set(own[-ncal:])
    for i in ids:
        if i in cal_ids:
            break
        if "x265amd::" in rows[i][0]:
            cur.append(i)
        elif cur:                                   # a marker closes the launch
            groups.append(cur)
            cur = []
    if cur:
        groups.append(cur)
    assert len(groups) == steps * len(L), (len(groups), steps * len(L))
    out = []
    for g in groups[(steps - 1) * len(L):]:
        c = defaultdict(float)
        for i in g:
            for k, v in rows[i][1].items():
                c[k] += v
        out.append((rows[g[0]][0], len(g), dict(c)))
    return out, cal
