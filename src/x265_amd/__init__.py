"""x265_amd — MI355X (gfx950) batched backend for the x265 1.9 primitive table.

The product is the C-ABI shared library libx265amd.so (include/x265_amd.h)
built from csrc/*.hip; this package only builds and binds it.
"""
from .native import LIB_PATH, Primitives, X265AmdError, capture_graph  # noqa: F401
