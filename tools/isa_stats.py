#!/usr/bin/env python3
"""Per-kernel instruction statistics of a hipcc device assembly file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only X.hip -o X.s
    python tools/isa_stats.py X.s [substring ...]

Prints static instruction counts (total / VALU / VMEM / LDS / SALU) and the
VGPR / SGPR / LDS usage from the code-object metadata.
"""
import re
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2:]
    s = open(path).read()
    heads = list(re.finditer(r"^(_Z\S+):\s*(;.*)?$", s, re.M))
    for i, m in enumerate(heads):
        name = m.group(1)
        if filt and not all(f in name for f in filt):
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        ins = [l.strip() for l in body.split("\n")]
        ins = [l for l in ins if l and not l.startswith((".", ";")) and not l.endswith(":")]
        cnt = lambda pre: sum(1 for l in ins if l.startswith(pre))
        meta = re.search(r"\.name:\s+" + re.escape(name) + r".*?(?=\n  - \.|\Z)", s, re.S)
        vg = sg = lds = "?"
        if meta:
            t = meta.group(0)
            vg = (re.search(r"\.vgpr_count:\s+(\d+)", t) or [None, "?"])[1]
            sg = (re.search(r"\.sgpr_count:\s+(\d+)", t) or [None, "?"])[1]
            lds = (re.search(r"\.group_segment_fixed_size:\s+(\d+)", t) or [None, "?"])[1]
        print(f"{name[:100]}\n    instrs {len(ins)} valu {cnt('v_')} vmem {cnt(('global_', 'buffer_'))} "
              f"lds {cnt('ds_')} salu {cnt('s_')} vgpr {vg} sgpr {sg} lds_bytes {lds}")


if __name__ == "__main__":
    main()
