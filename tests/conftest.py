import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_oracle():
    """Build the CPU checker libraries (gcc only, seconds) when missing."""
    import subprocess

    need = [os.path.join(ROOT, "oracle", "_build", f) for f in ("liboracle8.so", "liboracle10.so", "libcpubatch.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle", "cpubatch"], check=True,
                       capture_output=True)


@pytest.fixture(scope="session")
def oracle_libs():
    _ensure_oracle()
    return True


@pytest.fixture(scope="session")
def native_lib():
    """The product library, built in-tree if missing (hipcc cross-compiles without a GPU)."""
    from src.x265_amd import build as b

    if not os.path.exists(b.LIB):
        b.build(verbose=False)
    return b.LIB


@pytest.fixture(scope="session")
def gpu_prims(native_lib):
    """The gfx950 library on cuda:0 (GPU tests only; fails loudly without the device)."""
    import torch

    assert torch.cuda.is_available(), "GPU test needs the MI355X"
    from src.x265_amd import Primitives

    return Primitives(device=0)


@pytest.fixture(autouse=True)
def _gpu_teardown(request):
    """After every GPU test: collect dead reference cycles (a discarded GpuFramePipeline owns CUDA graphs,
    streams and device buffers through lambdas that reference itself) and synchronise the device, inside
    the test that made them.  Without it the cycles die whenever the cyclic GC next runs — in some later
    test — and any asynchronous device error is reported by a later test's first call instead of the one
    that caused it (two full runs saw an illegal address surface at the first copy of an unrelated test)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc

    gc.collect()
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        torch.cuda.synchronize()
