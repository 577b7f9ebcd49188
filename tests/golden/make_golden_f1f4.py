"""Generate tests/golden/golden_f1f4.json from the REFERENCE (oracle/_ref: the reference's own
estimateCUCost, Deblock and SAO classes driven by oracle/ref_shim.cpp).  Run where
/root/reference exists, after `make -C oracle ref cpubatch`:

    python tests/golden/make_golden_f1f4.py

Stores, per case (tests/golden_f1f4.cases), the SHA-256 of every output buffer; inputs are
regenerated from seeds by tests/golden_f1f4.py.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import golden_f1f4 as G  # noqa: E402
from pyoracle import available  # noqa: E402


def main():
    out = {}
    for depth in (8, 10):
        if not available("ref", depth):
            raise SystemExit("reference library missing: make -C oracle ref cpubatch")
        for case in G.cases(depth):
            res = G.run_cpu("ref", case)
            out[G.key(*case)] = {k: G.sha(v) for k, v in sorted(res.items())}
    with open(G.GOLDEN, "w") as f:
        json.dump({"source": "x265_1.9 estimateCUCost / Deblock / SAO via oracle/_ref (ref_shim.cpp)",
                   "cases": out}, f, indent=0, sort_keys=True)
    print(f"wrote {G.GOLDEN}: {len(out)} cases")


if __name__ == "__main__":
    main()
