#!/usr/bin/env python3
"""Where a GPU interpolation build differs from the CPU oracle: runs a few luma / chroma hpp / vpp / hvpp
cases through the library X265AMD_LIB names (default: the tree's) and the oracle, and prints, per case, the
number of differing output pixels and the first few (job, row, col, gpu, oracle) — a debugging aid for
kernel rewrites that fail the parity suite."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    from cases import HPP, HVPP, VPP, case_interp, run_cpu, run_gpu
    from pyoracle import CpuOracle

    import torch

    from src.x265_amd import Primitives

    # torch's HIP runtime first (as the tests' fixture does): initialised after the library's, it finds no GPU
    assert torch.cuda.is_available(), "needs the MI355X"
    prims = Primitives(device=0)
    orc = CpuOracle("oracle", 8)
    for op, taps, w, h in ((HPP, 4, 8, 8), (HPP, 4, 4, 4), (HPP, 4, 16, 16), (HPP, 8, 8, 8), (HPP, 8, 16, 16),
                           (VPP, 4, 8, 8), (VPP, 8, 16, 16), (HVPP, 8, 8, 8), (HVPP, 8, 16, 16)):
        c = case_interp(op, taps, w, h, 8, 6, 1234 + w + 7 * h + taps)
        got, exp = run_gpu(c, prims)["d"], run_cpu(c, orc)["d"]
        diff = np.nonzero(got != exp)[0]
        ds = c.bufs["ds"]
        print(f"op {op} taps {taps} {w}x{h}: {len(diff)} differing of {got.size} (coeff {list(c.bufs['coeff'])})")
        for i in diff[:8]:
            off = [j for j, o in enumerate(c.bufs["doff"]) if o <= i][-1]
            rel = i - c.bufs["doff"][off]
            print(f"   job {off} row {rel // ds} col {rel % ds}: gpu {int(got[i])} oracle {int(exp[i])}")


if __name__ == "__main__":
    main()
