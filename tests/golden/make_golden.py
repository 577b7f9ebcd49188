"""Generate the golden parity fixtures from the REFERENCE x265 1.9 C primitives.

Run in the build container (where /root/reference exists):

    make -C oracle ref cpubatch
    python tests/golden/make_golden.py

For every case of tests/cases.all_cases(depth) — every primitive family x
block shape the reference table holds x the three TestBench input classes —
the reference library (oracle/_ref/libx265ref{8,10}.so, built from the
reference sources by oracle/Makefile) produces the outputs; the fixture
stores the case parameters and the SHA-256 of each whole output buffer
(inputs are regenerated bit-identically from the case seed by cases.py).
Small scalar outputs (pixel-compare results, quant counts) are stored in full
so a failing test can show the values.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from cases import all_cases, run_cpu  # noqa: E402
from pyoracle import CpuOracle, available  # noqa: E402


def main() -> None:
    import numpy as np

    from cases import MVCOST_RANGE

    for depth in (8, 10):
        if not available("ref", depth):
            raise SystemExit("reference library missing: run `make -C oracle ref cpubatch` first")
        ref = CpuOracle("ref", depth)
        # the lookahead's BitCost table (input of the lowres P-estimate cases), from the reference
        np.save(os.path.join(HERE, f"mvcost_lookahead_d{depth}.npy"), ref.mvcost_table(MVCOST_RANGE))
        # BitCost tables of the motion-search cases' QPs (lambda_tab is reference data, taken as input)
        import ctypes as C
        from cases import ME_QPS, ME_TAB_RANGE
        lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", f"libx265ref{depth}.so"))
        tabs = np.zeros((len(ME_QPS), 2 * ME_TAB_RANGE + 1), np.uint16)
        for k, qp in enumerate(ME_QPS):
            lib.xo_mvcost_table_qp(qp, ME_TAB_RANGE, C.c_void_p(tabs[k].ctypes.data))
        np.save(os.path.join(HERE, f"mvcost_qp_d{depth}.npy"), tabs)
        entries = []
        for c in all_cases(depth):
            outs = run_cpu(c, ref)
            e = {"family": c.family, "params": c.params, "sha256": c.output_hashes(outs)}
            for k, v in outs.items():
                if v.size <= 64:
                    e.setdefault("values", {})[k] = [int(x) for x in v.tolist()]
            entries.append(e)
        path = os.path.join(HERE, f"golden_d{depth}.json")
        with open(path, "w") as f:
            json.dump({"source": "x265_1.9 C primitives (oracle/_ref/libx265ref%d.so)" % depth,
                       "depth": depth, "cases": entries}, f, separators=(",", ":"))
        print(f"wrote {path}: {len(entries)} cases")


if __name__ == "__main__":
    main()
