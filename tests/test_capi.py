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


def test_ctypes_descriptors_match_the_library(native_lib):
    """every ctypes descriptor of src/x265_amd/native.py has the size of the C type it mirrors (a field missing
    on the Python side would let the library read past the structure)"""
    import sys

    sys.path.insert(0, ROOT)
    from src.x265_amd import native as N

    lib = ctypes.CDLL(native_lib)
    lib.x265amd_sizeof.argtypes = [ctypes.c_char_p]
    pairs = {"CmpBatch": "x265amd_cmp_batch", "BlockBatch": "x265amd_block_batch", "InterpBatch": "x265amd_interp_batch",
             "TuBatch": "x265amd_tu_batch", "LowresBatch": "x265amd_lowres_batch",
             "LowresIntraBatch": "x265amd_lowres_intra_batch", "LowresPcostBatch": "x265amd_lowres_pcost_batch",
             "LowresBcostBatch": "x265amd_lowres_bcost_batch", "MeBatch": "x265amd_me_batch",
             "SaoFrame": "x265amd_sao_frame", "SaoStatsFrame": "x265amd_sao_stats_frame",
             "DeblockFrame": "x265amd_deblock_frame", "PropagateBatch": "x265amd_propagate_batch",
             "WeightsBatch": "x265amd_weights_batch", "BorderPlane": "x265amd_border_plane"}
    bad = {}
    for py, c in pairs.items():
        want = lib.x265amd_sizeof(c.encode())
        assert want > 0, c
        got = ctypes.sizeof(getattr(N, py))
        if got != want:
            bad[py] = (got, want)
    assert not bad, bad


def test_library_metadata(native_lib):
    lib = ctypes.CDLL(native_lib)
    lib.x265amd_target.restype = ctypes.c_char_p
    lib.x265amd_strerror.restype = ctypes.c_char_p
    assert lib.x265amd_abi_version() == 2
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


def test_grouped_entries_reject_whole_call_without_launch(native_lib):
    """A grouped call with one invalid batch enqueues nothing and returns EINVAL."""
    import sys

    sys.path.insert(0, ROOT)
    from src.x265_amd.native import BlockBatch, CmpBatch, InterpBatch

    lib = ctypes.CDLL(native_lib)
    cmp = (CmpBatch * 3)(CmpBatch(8, 8, 1), CmpBatch(16, 16, 1), CmpBatch(6, 8, 1))   # 6x8: invalid
    assert lib.x265amd_pixelcmp_grouped(0, 8, 3, cmp) == 1000
    assert lib.x265amd_sad_multi_grouped(4, 8, 3, cmp) == 1000
    assert lib.x265amd_sad_multi_grouped(5, 8, 1, cmp) == 1000                           # nref
    psy = (CmpBatch * 1)(CmpBatch(8, 16, 1))                                              # psy needs w == h
    assert lib.x265amd_pixelcmp_grouped(5, 8, 1, psy) == 1000
    blk = (BlockBatch * 2)(BlockBatch(8, 8, 1), BlockBatch(3, 8, 1))                     # odd width
    assert lib.x265amd_blockop_grouped(4, 8, 2, blk) == 1000
    itp = (InterpBatch * 2)(InterpBatch(8, 8, 1), InterpBatch(2, 8, 1))                   # 2-wide luma hpp
    assert lib.x265amd_interp_grouped(0, 8, 8, 2, itp) == 1000
    assert lib.x265amd_interp_grouped(6, 8, 8, 1, (InterpBatch * 1)(InterpBatch(8, 8, 1))) == 1000  # hvpp, no coeff
    assert lib.x265amd_pixelcmp_grouped(0, 8, -1, None) == 1000
    # empty batches / empty calls are no-ops
    assert lib.x265amd_pixelcmp_grouped(0, 8, 0, None) == 0
    assert lib.x265amd_blockop_grouped(4, 8, 1, (BlockBatch * 1)(BlockBatch(3, 8, 0))) == 0
