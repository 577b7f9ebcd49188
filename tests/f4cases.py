"""Synthetic frames, SAO parameters and CU trees for the f4 loop-filter tests.

Content is blocky on purpose (8x8 piecewise-flat regions plus noise and gradients) so the
deblocking decisions (no filter / weak / strong, one- or two-sided) and all SAO edge classes occur.
"""
from __future__ import annotations

import numpy as np

import pyoracle as po

MARGIN = 16


def chroma_shift(csp):
    """(hshift, vshift) of a chroma format: 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4 (x265.h CHROMA_*_SHIFT)"""
    return (0 if csp == 3 else 1), (1 if csp == 1 else 0)


def frame_planes(width, height, depth, rng, margin=MARGIN, csp=1):
    """(Y, Cb, Cr) as padded 2-D arrays (margin on every side), the margins filled too."""
    hs, vs = chroma_shift(csp)
    dt = np.uint8 if depth == 8 else np.uint16
    maxv = (1 << depth) - 1
    out = []
    for p in range(3):
        w, h = (width, height) if p == 0 else (width >> hs, height >> vs)
        yy, xx = np.mgrid[0:h + 2 * margin, 0:w + 2 * margin]
        base = rng.integers(0, maxv + 1, size=((h + 2 * margin) // 8 + 1, (w + 2 * margin) // 8 + 1))
        blocks = base[yy // 8, xx // 8].astype(np.int64)
        # mostly small steps between neighbouring blocks so the filters engage
        smooth = (maxv // 2 + (xx * 3 + yy * 2) % (maxv // 4 + 1)).astype(np.int64)
        mix = rng.random(blocks.shape) < 0.8
        v = np.where(mix, smooth + (blocks % (8 << (depth - 8))) - (4 << (depth - 8)), blocks)
        v = v + rng.integers(-2, 3, size=v.shape) * (1 << (depth - 8))
        out.append(np.clip(v, 0, maxv).astype(dt))
    return tuple(out)


def sao_params(width, height, ctu_log2, depth, rng, p_off=0.15):
    """Final per-CTU SaoCtuParam values, [plane * nctu + ctu]; Cr shares Cb's type (HEVC syntax)."""
    ctu = 1 << ctu_log2
    nctu = ((width + ctu - 1) // ctu) * ((height + ctu - 1) // ctu)
    prm = np.zeros((3, nctu), po.SAO_PARAM)
    omax = (1 << (min(depth, 10) - 5)) - 1
    for p in range(3):
        for c in range(nctu):
            if p == 2:
                t = int(prm[1, c]["type"])
            else:
                t = -1 if rng.random() < p_off else int(rng.integers(0, 5))
            prm[p, c]["type"] = t
            prm[p, c]["band"] = rng.integers(0, 32)
            if t == 4:
                prm[p, c]["offset"] = rng.integers(-omax, omax + 1, 4)
            else:   # EO: positive offsets for the valley classes, negative for the peaks
                o = rng.integers(0, omax + 1, 4)
                prm[p, c]["offset"] = [o[0], o[1], -o[2], -o[3]]
    return prm.reshape(-1)


_PU = {
    0: lambda s: [(0, 0, s, s)],
    1: lambda s: [(0, 0, s, s // 2), (0, s // 2, s, s // 2)],
    2: lambda s: [(0, 0, s // 2, s), (s // 2, 0, s // 2, s)],
    3: lambda s: [(0, 0, s // 2, s // 2), (s // 2, 0, s // 2, s // 2), (0, s // 2, s // 2, s // 2),
                  (s // 2, s // 2, s // 2, s // 2)],
    4: lambda s: [(0, 0, s, s // 4), (0, s // 4, s, 3 * s // 4)],
    5: lambda s: [(0, 0, s, 3 * s // 4), (0, 3 * s // 4, s, s // 4)],
    6: lambda s: [(0, 0, s // 4, s), (s // 4, 0, 3 * s // 4, s)],
    7: lambda s: [(0, 0, 3 * s // 4, s), (3 * s // 4, 0, s // 4, s)],
}


def deblock_units(width, height, ctu_log2, depth, rng, slice_type="B", p_bypass=0.0):
    """A random CU / PU / TU tree per CTU (CUs never cross the picture edge), as 4x4 units."""
    U = np.zeros((height // 4, width // 4), po.DEBLOCK_UNIT)
    qmin = -6 * (depth - 8)
    gmv = rng.integers(-6, 7, 2)

    def tu_split(x, y, log2, force4):
        if log2 > 5 or (force4 and log2 > 2) or (log2 > 2 and rng.random() < 0.35):
            h = 1 << (log2 - 1)
            for dy in (0, h):
                for dx in (0, h):
                    tu_split(x + dx, y + dy, log2 - 1, force4)
            return
        s = 1 << log2
        sl = U[y // 4:(y + s) // 4, x // 4:(x + s) // 4]
        sl["tu_log2"] = log2
        if rng.random() < 0.5:
            sl["flags"] |= 2

    def cu(x, y, log2):
        if x >= width or y >= height:
            return
        s = 1 << log2
        must = x + s > width or y + s > height
        if log2 > 3 and (must or rng.random() < 0.45):
            h = s // 2
            for dy in (0, h):
                for dx in (0, h):
                    cu(x + dx, y + dy, log2 - 1)
            return
        intra = slice_type == "I" or rng.random() < 0.25
        if intra:
            part = 3 if (log2 == 3 and rng.random() < 0.4) else 0
        else:
            choices = [0, 1, 2] + ([4, 5, 6, 7] if log2 >= 4 else [])
            part = int(rng.choice(choices))
        sl = U[y // 4:(y + s) // 4, x // 4:(x + s) // 4]
        sl["cu_log2"] = log2
        sl["part"] = part
        sl["flags"] = 1 if intra else 0
        if rng.random() < p_bypass:
            sl["flags"] |= 4
        sl["qp"] = rng.integers(0 if rng.random() < 0.5 else qmin, 52)
        for (px, py, pw, ph) in _PU[part](s):
            pu = U[(y + py) // 4:(y + py + ph) // 4, (x + px) // 4:(x + px + pw) // 4]
            if intra:
                pu["ref_idx"] = -1
                continue
            if slice_type == "P":
                r = [int(rng.integers(0, 3)), -1]
            else:
                k = rng.integers(0, 3)
                r = [int(rng.integers(0, 3)) if k != 1 else -1, int(rng.integers(0, 3)) if k != 0 else -1]
            pu["ref_idx"] = r
            for lst in range(2):
                mv = gmv + rng.integers(-5, 6, 2) if rng.random() < 0.7 else rng.integers(-64, 65, 2)
                pu["mv"][..., lst, :] = mv
        tu_split(x, y, log2, intra and part == 3)

    ctu = 1 << ctu_log2
    for cy in range(0, height, ctu):
        for cx in range(0, width, ctu):
            cu(cx, cy, ctu_log2)
    return U


def deblock_params(rng, slice_type="B", tq_bypass=0):
    prm = po.DeblockParams()
    prm.is_p = 1 if slice_type == "P" else 0
    prm.beta_offset_div2 = int(rng.integers(-6, 7))
    prm.tc_offset_div2 = int(rng.integers(-6, 7))
    prm.cb_qp_offset = int(rng.integers(-12, 13))
    prm.cr_qp_offset = int(rng.integers(-12, 13))
    prm.tq_bypass_enabled = tq_bypass
    l0, l1 = [8, 4, 0], [16, 8, 12]      # POC 8 sits in both lists
    for i in range(16):
        prm.ref_poc[0][i] = l0[i] if i < 3 else 100 + i
        prm.ref_poc[1][i] = l1[i] if i < 3 else 200 + i
    return prm


def copy_planes(planes):
    return tuple(p.copy() for p in planes)
