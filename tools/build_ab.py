#!/usr/bin/env python3
"""Build an A/B variant of libx265amd.so: the current tree with some csrc files taken from another git
revision (e.g. the round-4 kernels that ran on the box), into src/x265_amd/ab/libx265amd_<tag>.so (travels
to the GPU box; select it with X265AMD_LIB=...).

    python tools/build_ab.py r4 fc10ce6 interp.hip intra.hip
    python tools/build_ab.py ku2 - me.hip -DX265AMD_ME_KU64=2     (rev "-": the working tree's file)

Each variant is also copied to src/x265_amd/ab/<tag>/libx265amd.so, for programs linked against the library
(the hooked reference encoders): LD_LIBRARY_PATH=src/x265_amd/ab/<tag> selects it (RUNPATH yields to it).
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    tag, rev = sys.argv[1], sys.argv[2]
    files = [a for a in sys.argv[3:] if not a.startswith("-D")]
    defines = [a for a in sys.argv[3:] if a.startswith("-D")]
    from src.x265_amd import build as B

    out_dir = os.path.join(B.HERE, "ab")
    os.makedirs(out_dir, exist_ok=True)
    # the variant sources sit beside csrc/ (same depth, so "../../../include/x265_amd.h" resolves)
    tmp = os.path.join(B.HERE, "_abtmp_" + tag)
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    try:
        for f in os.listdir(B.CSRC):
            if os.path.isfile(os.path.join(B.CSRC, f)):
                shutil.copy(os.path.join(B.CSRC, f), os.path.join(tmp, f))
        for f in files if rev != "-" else []:
            blob = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:src/x265_amd/csrc/{f}"], check=True,
                                  capture_output=True).stdout
            open(os.path.join(tmp, f), "wb").write(blob)
        objs = []
        for src, obj, extra in B.SOURCES:
            if src not in files:
                objs.append(os.path.join(B.OBJ, obj))
                continue
            o = os.path.join(tmp, obj)
            lang = ["-x", "hip"] if src.endswith(".cpp") else []
            r = subprocess.run([B.HIPCC, *B.FLAGS, *extra, *defines, *lang, "-c", os.path.join(tmp, src), "-o", o],
                               capture_output=True, text=True)
            if r.returncode != 0:
                raise SystemExit(f"hipcc failed for {src}:\n{r.stderr[-3000:]}")
            objs.append(o)
        lib = os.path.join(out_dir, f"libx265amd_{tag}.so")
        r = subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-3000:])
        os.makedirs(os.path.join(out_dir, tag), exist_ok=True)
        shutil.copy(lib, os.path.join(out_dir, tag, "libx265amd.so"))
        print(lib)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
