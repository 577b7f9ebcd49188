"""Lowres frame pairs for LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495): geometry of
Lowres::create (lowres.cpp:30-60) for a W x H picture with PicYuv margins (64 + 32, 64 + 16),
the wp_sum / wp_ssd statistics of slicetype.cpp:40-56, 219-226, and content classes: a fade
(the reference scaled and offset: a weight is chosen), a near-identical pair (early exit), a
noisy mismatch (no weight helps), an offset-only change and a strong fade whose offset clips."""
import numpy as np


def geometry(W, H):
    mx, my = 64 + 32, 64 + 16
    width, lines = W // 2, H // 2
    stride = width + 2 * mx
    if stride & 31:
        stride += 32 - (stride & 31)
    wcu, hcu = (width + 7) // 8, (lines + 7) // 8
    width, lines = wcu * 8, hcu * 8
    padded = lines + 2 * my
    return dict(width=width, lines=lines, stride=stride, padded=padded, padoff=stride * my + mx, wcu=wcu, hcu=hcu,
                mx=mx, my=my)


def _planes(g, base, depth):
    """4 lowres planes (the half-pel ones shifted copies), border-extended like Lowres"""
    dt = np.uint8 if depth == 8 else np.uint16
    out = np.zeros((4, g["padded"] * g["stride"]), dt)
    for i in range(4):
        p = np.roll(base, (i >> 1, i & 1), axis=(0, 1))
        full = np.pad(p, ((g["my"], g["padded"] - g["lines"] - g["my"]),
                          (g["mx"], g["stride"] - g["width"] - g["mx"])), mode="edge")
        out[i] = full.reshape(-1)
    return out


def _stats(p, depth):
    """wp_sum / wp_ssd of the lowres luma plane (slicetype.cpp:40-56, 219-226)"""
    v = p.astype(np.int64)
    s = int(v.sum())
    ssd = int((v * v).sum())
    n = v.size
    return s, ssd - (s * s + n // 2) // n


def weights_case(kind, W, H, depth, seed):
    g = geometry(W, H)
    rng = np.random.default_rng(seed)
    pmax = (1 << depth) - 1
    k = 1 << (depth - 8)
    yy, xx = np.mgrid[0:g["lines"], 0:g["width"]]
    ref = 100 + 60 * np.sin(xx / 9.0) * np.cos(yy / 7.0) + rng.normal(0, 6, xx.shape)
    if kind == "fade":
        cur = ref * 0.78 + 12
    elif kind == "same":
        cur = ref + rng.normal(0, 0.3, ref.shape)
    elif kind == "noise":
        cur = rng.uniform(0, 255, ref.shape)
    elif kind == "offset":
        cur = ref + 9
    else:   # "clip": strong fade to black with a large mean shift
        cur = ref * 0.35 + 150
    ref = np.clip(np.rint(ref * k), 0, pmax)
    cur = np.clip(np.rint(cur * k + rng.normal(0, 1, ref.shape)), 0, pmax)
    fb, rb = _planes(g, cur, depth), _planes(g, ref, depth)
    fsum, fssd = _stats(cur, depth)
    rsum, rssd = _stats(ref, depth)
    intra = rng.integers(200, 3000, g["wcu"] * g["hcu"]).astype(np.int32)
    return g, fb, rb, intra, (fssd, rssd, fsum, rsum)


KINDS = ["fade", "same", "noise", "offset", "clip"]
