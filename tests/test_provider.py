"""The per-call provider boundary: include/x265_amd_primitives.h.

* (no GPU) the restated `EncoderPrimitives` has the reference's exact layout
  — every member offset and sizeof — checked by compiling oracle/layout_check.cpp
  against the reference header where /root/reference is mounted;
* (GPU) X265_NS::setupHipPrimitives fills a table whose entries, called
  through the table like x265 calls them, match the CPU oracle bit-exactly
  (tests/provider_check.cpp, TestBench-style), at 8-bit and 10-bit.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/x265_1.9/source"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources not mounted (GPU box)")
@pytest.mark.parametrize("depth", [8, 10])
def test_encoder_primitives_layout_matches_reference(tmp_path, depth):
    exe = tmp_path / f"layout{depth}"
    defs = [f"-DX265_DEPTH={depth}", f"-DHIGH_BIT_DEPTH={int(depth > 8)}", "-DEXPORT_C_API=1", "-DX265_ARCH_X86=1",
            "-DHAVE_INT_TYPES_H=1", "-D__STDC_LIMIT_MACROS=1"]
    incs = ["-I" + os.path.join(ROOT, "oracle", "_ref"), "-I" + REF, "-I" + os.path.join(REF, "common")]
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/x265_config.h"], check=True)
    subprocess.run(["g++", "-std=gnu++11", "-w", *defs, *incs, os.path.join(ROOT, "oracle", "layout_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "0 mismatches" in r.stdout and "sizeof 15008" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_hip_provider_through_the_table(native_lib, oracle_libs, tmp_path, depth):
    libdir = os.path.dirname(native_lib)
    odir = os.path.join(ROOT, "oracle", "_build")
    exe = tmp_path / f"provider_check{depth}"
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", f"-DX265_DEPTH={depth}", "-x", "hip",
           os.path.join(ROOT, "tests", "provider_check.cpp"), "-o", str(exe),
           f"-L{libdir}", "-lx265amd", f"-Wl,-rpath,{libdir}",
           "-x", "none", os.path.join(odir, f"liboracle{8 if depth == 8 else 10}.so"), f"-Wl,-rpath,{odir}"]
    subprocess.run(cmd, check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "0 failures" in r.stdout
