"""Random inputs of Lookahead::estimateCUPropagate (slicetype.cpp:1738-1836) shaped like a
lowres lookahead frame: intra / inter SATD costs of 8x8 lowres CUs, inverse qscales (Q8.8),
list flags in the top 2 bits of lowresCosts, quarter-pel lowres MVs (mostly small, some zero,
some pointing outside the frame), propagate costs of a referenced frame."""
import numpy as np


def cutree_case(wcu, hcu, b_p0, p1_b, referenced, seed):
    rng = np.random.default_rng(seed)
    n = wcu * hcu
    intra = rng.integers(0, 4000, n).astype(np.int32)
    intra[rng.random(n) < 0.03] = 0                                   # flat blocks
    inter = np.minimum(rng.integers(0, 5000, n), (1 << 14) - 1)
    lists = rng.integers(1, 4, n) if p1_b else np.ones(n, np.int64)   # P: list 0 only
    lists[rng.random(n) < 0.1] = 0                                   # intra-coded: no list
    lowres = (inter | (lists << 14)).astype(np.uint16)
    invq = rng.integers(180, 340, n).astype(np.int32)
    mv = rng.integers(-80, 81, (2, n, 2))
    mv[:, rng.random(n) < 0.25] = 0
    far = rng.random(n) < 0.05
    mv[0, far] = rng.integers(-600, 600, (int(far.sum()), 2))
    mvs = [((m[:, 0] & 0xffff) | ((m[:, 1] & 0xffff) << 16)).astype(np.uint32).view(np.int32) for m in mv]
    prop = rng.integers(0, 30000, n).astype(np.uint16) if referenced else rng.integers(0, 100, n).astype(np.uint16)
    ref0 = rng.integers(0, 20000, n).astype(np.uint16)
    ref1 = rng.integers(0, 20000, n).astype(np.uint16)
    ref0[rng.random(n) < 0.02] = 65000                                # near saturation
    return dict(intra=intra, lowres=lowres, invq=invq, mvs0=mvs[0], mvs1=mvs[1], prop=prop, ref0=ref0, ref1=ref1)


CASES = [  # (wcu, hcu, b - p0, p1 - b, referenced, weighted_bipred, fps_num, fps_den, average duration)
    (30, 17, 1, 0, 1, 0, 30, 1, 1 / 30),        # P frame (b = p1), referenced
    (30, 17, 2, 2, 1, 1, 30, 1, 1 / 30),        # b-pyramid middle B, weighted bipred
    (30, 17, 1, 3, 0, 0, 25, 1, 0.05),          # non-referenced B
    (17, 9, 3, 1, 0, 1, 60000, 1001, 1 / 50),   # odd size, NTSC rate
    (120, 68, 1, 1, 1, 0, 30, 1, 1 / 30),       # 1080p lowres
]
