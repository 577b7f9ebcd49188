"""The f1 encoder session's lifetime through the public C ABI (x265amd_la_*, csrc/lookahead.cpp).

Threads that used a destroyed session keep thread_local entries the session could not reach; a
later session may be allocated at the same address.  Here: four threads run intra estimates on a
session, the session is destroyed, a new one is created, and the same threads run the same
estimates on it — each thread must get a fresh context (no use of the freed stream / scratch) and
identical results.  A second geometry gets a session of its own.
"""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class LaConfig(ctypes.Structure):
    _fields_ = [("depth", ctypes.c_int), ("width_cu", ctypes.c_int), ("height_cu", ctypes.c_int),
                ("lowres_stride", ctypes.c_ssize_t), ("planesize", ctypes.c_int64), ("padoffset", ctypes.c_int64),
                ("max_frames", ctypes.c_int), ("max_threads", ctypes.c_int),
                ("mvcost", ctypes.POINTER(ctypes.c_uint16)), ("mvcost_range", ctypes.c_int)]


def _lib():
    from src.x265_amd import Primitives

    lib = Primitives(device=0).lib
    lib.x265amd_la_create.argtypes = [ctypes.POINTER(LaConfig), ctypes.POINTER(ctypes.c_void_p)]
    lib.x265amd_la_destroy.argtypes = [ctypes.c_void_p]
    lib.x265amd_la_load.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.x265amd_la_intra.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_void_p] * 5
    return lib


class Geometry:
    def __init__(self, wcu, hcu, pad=32, seed=0):
        self.wcu, self.hcu = wcu, hcu
        self.stride = wcu * 8 + 2 * pad
        rows = hcu * 8 + 2 * pad
        self.planesize = self.stride * rows
        self.padoffset = pad * self.stride + pad
        self.range = 1 << 14
        self.tab = np.minimum(np.abs(np.arange(-self.range, self.range + 1)) * 3, 30000).astype(np.uint16)
        self.rng = np.random.default_rng(seed)

    def config(self):
        c = LaConfig()
        c.depth, c.width_cu, c.height_cu = 8, self.wcu, self.hcu
        c.lowres_stride, c.planesize, c.padoffset = self.stride, self.planesize, self.padoffset
        c.max_frames, c.max_threads = 16, 16
        c.mvcost = ctypes.cast(self.tab.ctypes.data + 2 * self.range, ctypes.POINTER(ctypes.c_uint16))
        c.mvcost_range = self.range
        return c

    def picture(self):
        return self.rng.integers(0, 256, 4 * self.planesize, dtype=np.uint8)


def _intra(lib, la, g, buf, key):
    ncu = g.wcu * g.hcu
    ic = np.zeros(ncu, np.int32)
    im = np.zeros(ncu, np.uint8)
    lc = np.zeros(ncu, np.uint16)
    rs = np.zeros(g.hcu, np.int32)
    ce = np.zeros(2, np.int64)
    assert lib.x265amd_la_load(la, key, 0, buf.ctypes.data, None) == 0
    assert lib.x265amd_la_intra(la, key, ic.ctypes.data, im.ctypes.data, lc.ctypes.data, rs.ctypes.data,
                                ce.ctypes.data) == 0
    return ic, im, lc, rs, ce


def _create(lib, g):
    la = ctypes.c_void_p()
    cfg = g.config()
    assert lib.x265amd_la_create(ctypes.byref(cfg), ctypes.byref(la)) == 0
    return la


def test_la_session_destroy_create_reuse_threads():
    import torch

    assert torch.cuda.is_available()
    lib = _lib()
    g = Geometry(12, 7, seed=5)
    pics = [g.picture() for _ in range(4)]
    keys = [ctypes.c_void_p(0x1000 + 64 * i) for i in range(4)]
    sessions = [_create(lib, g)]
    results = [[None, None] for _ in range(4)]
    errors = []
    bar = threading.Barrier(5)

    def worker(i):
        try:
            for phase in range(2):
                if phase:
                    bar.wait()            # main thread replaced the session
                results[i][phase] = _intra(lib, sessions[-1], g, pics[i], keys[i])
                bar.wait()
        except Exception as e:           # reported by the main thread
            errors.append(repr(e))
            bar.abort()

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    bar.wait()                            # phase 0 done on every thread
    first = sessions[0].value
    lib.x265amd_la_destroy(sessions[0])
    sessions.append(_create(lib, g))      # often the same address as the destroyed one
    bar.wait()
    bar.wait()                            # phase 1 done
    for t in ts:
        t.join()
    assert not errors, errors
    # the main thread used neither session yet: it must work on the new one too
    main = _intra(lib, sessions[1], g, pics[0], keys[0])
    for i in range(4):
        for a, b in zip(results[i][0], results[i][1]):
            assert np.array_equal(a, b), f"thread {i}: results differ across sessions"
    for a, b in zip(results[0][0], main):
        assert np.array_equal(a, b)
    # a second geometry in the same process: a session of its own, its own results
    g2 = Geometry(20, 9, seed=6)
    la2 = _create(lib, g2)
    pic2 = g2.picture()                   # x265amd_la_load page-locks it: it must outlive the session
    r2 = _intra(lib, la2, g2, pic2, keys[0])
    assert r2[0].shape == (180,) and int(r2[4][0]) > 0
    lib.x265amd_la_destroy(la2)
    lib.x265amd_la_destroy(sessions[1])
    del pic2, pics
    print(f"session addresses: {first:#x} -> {sessions[1].value:#x}")
