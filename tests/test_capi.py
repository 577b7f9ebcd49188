"""The product C ABI: the library loads without a GPU and exports every
entry point include/x265_amd.h declares (no compute calls here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "x265_amd.h")).read()
    return sorted(set(re.findall(r"\b(x265amd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entries():
    syms = declared_symbols()
    for s in ("x265amd_pixelcmp", "x265amd_sad_multi", "x265amd_interp", "x265amd_transform", "x265amd_quant",
              "x265amd_intra_pred", "x265amd_blockop"):
        assert s in syms


def test_library_exports_every_declared_symbol(native_lib):
    lib = ctypes.CDLL(native_lib)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_library_metadata(native_lib):
    lib = ctypes.CDLL(native_lib)
    lib.x265amd_target.restype = ctypes.c_char_p
    lib.x265amd_strerror.restype = ctypes.c_char_p
    assert lib.x265amd_abi_version() == 1
    assert lib.x265amd_target() == b"gfx950"
    assert b"unsupported" in lib.x265amd_strerror(1000)


def test_invalid_shapes_rejected_without_launch(native_lib):
    """Shape validation happens on the host before any device work."""
    lib = ctypes.CDLL(native_lib)
    # n > 0 with an impossible block shape / depth must return X265AMD_EINVAL
    assert lib.x265amd_pixelcmp(0, 9, 8, 8, 1, None, 0, None, None, 0, None, None, None) == 1000
    assert lib.x265amd_pixelcmp(0, 8, 6, 8, 1, None, 0, None, None, 0, None, None, None) == 1000
    assert lib.x265amd_transform(0, 8, 64, 1, None, 0, None, None, 0, None, None) == 1000
    assert lib.x265amd_quant(1, 20, None, None, None, None, None, None, None, None, None, None, None, None) == 1000
    # n == 0 is a no-op
    assert lib.x265amd_interp(0, 8, 8, 8, 8, 0, None, 0, None, None, 0, None, None, 0, None) == 0
