"""the CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer.

oracle/Makefile `asan` builds oracle/_build_asan/liboracle{8,10}.so and its
batch driver with -fsanitize=address,undefined -fno-sanitize-recover=undefined
(any out-of-bounds access or UB — e.g. a signed overflow where the reference's
int arithmetic wraps — aborts).  The golden-case parity tests then run in a
child python with the sanitizer runtimes preloaded and pyoracle pointed at that
build (X265AMD_ORACLE_DIR).  Host code only: GPU sanitizers are not available.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    r = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(not _runtime("libasan.so"), reason="gcc sanitizer runtimes not installed")
def test_oracle_golden_cases_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, capture_output=True)
    env = dict(os.environ, X265AMD_ORACLE_DIR="_build_asan",
               LD_PRELOAD=f"{_runtime('libasan.so')}:{_runtime('libubsan.so')}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle.py")],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert " passed" in out
