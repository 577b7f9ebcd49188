"""Build the gfx950 primitive library (libx265amd.so) in-tree with hipcc.

One code object per source file (compiled in parallel), linked into a single
shared library next to this file so it travels with the repository snapshot
to the GPU box.  No JIT cache, no torch extension machinery: the product is a
plain C-ABI shared library (include/x265_amd.h).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
LIB = os.path.join(HERE, "libx265amd.so")
# MFMA results in VGPRs, not AGPRs (no v_accvgpr_read per accumulator element; measured with the
# MFMA transforms, profiles/r03/tr_split_ab.txt)
MFMA_VGPR = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
# (source, object, extra flags): the EncoderPrimitives provider is built once per bit depth
SOURCES = [("pixel.hip", "pixel.o", []), ("interp.hip", "interp.o", []), ("transform.hip", "transform.o", MFMA_VGPR),
           ("intra.hip", "intra.o", []), ("blockops.hip", "blockops.o", []), ("tu.hip", "tu.o", MFMA_VGPR), ("lowres.hip", "lowres.o", []), ("me.hip", "me.o", []), ("loopfilter.hip", "loopfilter.o", []),
           ("runtime.hip", "runtime.o", []), ("lookahead.cpp", "lookahead.o", []), ("mesession.cpp", "mesession.o", []), ("rdosession.cpp", "rdosession.o", []),
           ("schedule.cpp", "schedule.o", []), ("exchange.cpp", "exchange.o", []),
           ("provider.cpp", "provider8.o", ["-DX265_DEPTH=8"]),
           ("provider.cpp", "provider10.o", ["-DX265_DEPTH=10"])]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-command-line-argument"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _headers():
    inc = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include")
    return [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + \
           [os.path.join(inc, h) for h in os.listdir(inc) if h.endswith(".h")]


def _compile(entry) -> str:
    src, obj, extra = entry
    out = os.path.join(OBJ, obj)
    deps = [os.path.join(CSRC, src)] + _headers()
    if _newer(out, deps):
        return out
    lang = ["-x", "hip"] if src.endswith(".cpp") else []
    cmd = [HIPCC, *FLAGS, *extra, *lang, "-c", os.path.join(CSRC, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return out


def build(verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    jobs = min(len(SOURCES), max(1, (os.cpu_count() or 4)), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if not _newer(LIB, objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    _build_hosts()
    if verbose:
        print(f"[x265amd] built {LIB}", file=sys.stderr)
    return LIB


# C++ host programs over the C ABI (integration/): built next to their sources, linked to the library
ROOT = os.path.dirname(os.path.dirname(HERE))
HOSTS = [("frame_shard_host.cpp", "frame_shard_host")]


def _build_hosts():
    out_dir = os.path.join(ROOT, "integration", "_bin")
    os.makedirs(out_dir, exist_ok=True)
    for src, exe in HOSTS:
        srcp, out = os.path.join(ROOT, "integration", src), os.path.join(out_dir, exe)
        if _newer(out, [srcp, LIB] + _headers()):
            continue
        cmd = [HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950", srcp, "-o", out,
               "-L" + HERE, "-lx265amd", "-Wl,-rpath,$ORIGIN/../../src/x265_amd"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")


if __name__ == "__main__":
    build()
