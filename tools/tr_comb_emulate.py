#!/usr/bin/env python3
"""CPU emulation of the MFMA transform recombination.

k_tr16_mfma / k_tr32_mfma (csrc/transform.hip) compute every stage of the HEVC transform
(dct.cpp:83-416) as two f16 MFMA products over an exact operand split x = 1024 * hi + lo
(split10, transform1d.h: lo in [0, 1023], hi in [-32, 31]) and recombine the two f32 tiles into
the int32 sum.  Round 3 tried to replace the two v_cvt_i32_f32 per element by the "magic add"
(f32 bits of t + 1.5 * 2^23 minus 0x4B400000 = t for integer |t| < 2^22) and got wrong outputs on
the GPU.  This script replays both recombinations in numpy float32 on the same arithmetic:

  * per tile, the float32 sum of the products in MFMA k order (each product exact in f32, one
    rounding per add: v_mfma is a k-ordered chain for these shapes), for every stage of forward
    and inverse 16 / 32 transforms, on the reference TestBench input classes (residuals,
    full-range int16 coefficients, all-min / all-max);
  * the largest |partial sum| any tile reaches, against the 2^22 bound of the magic add and the
    2^24 bound of exact f32 integers;
  * the mismatches of cvt and magic-add recombination against the exact int64 result;
  * the same for an 11-bit split (lo in [0, 2047]) — the form whose lo sums the verdict bounded
    at 32 * 90 * 2047 ~ 5.9 M > 2^22.

    python tools/tr_comb_emulate.py [--out profiles/r04/tr_comb_emulation.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dct_matrix(n: int) -> np.ndarray:
    """the HEVC integer transform matrix (constants.cpp:259-333 g_t4 .. g_t32) from the spec rule:
    row 0 is 64; T32[k][j] = +-C[m] with m = k (2j + 1) mod 128 folded into [0, 32], where C[m]
    is the scaled cos(m pi / 64) of the spec's coefficient list; the N-point matrix is every
    (32 / N)-th row of the 32-point one, first N columns"""
    c = {1: 90, 2: 90, 3: 90, 4: 89, 5: 88, 6: 87, 7: 85, 8: 83, 9: 82, 10: 80, 11: 78, 12: 75, 13: 73, 14: 70,
         15: 67, 16: 64, 17: 61, 18: 57, 19: 54, 20: 50, 21: 46, 22: 43, 23: 38, 24: 36, 25: 31, 26: 25, 27: 22,
         28: 18, 29: 13, 30: 9, 31: 4}
    t = np.zeros((32, 32), dtype=np.int64)
    for k in range(32):
        for j in range(32):
            if k == 0:
                t[k, j] = 64
                continue
            m = k * (2 * j + 1) % 128
            t[k, j] = c[m] if m < 32 else -c[64 - m] if m < 64 else -c[m - 64] if m < 96 else c[128 - m]
    assert list(t[1, :4]) == [90, 90, 88, 85] and list(t[16, :4]) == [64, -64, -64, 64] and list(t[8, :4]) == [83, 36, -36, -83]
    return t[:: 32 // n, :n]


MAGIC = np.float32(1.5 * 2 ** 23)
MAGIC_BITS = 0x4B400000


def f32_chain(coef: np.ndarray, part: np.ndarray) -> tuple[np.ndarray, int]:
    """sum_k coef[..., k] * part[..., k] as a float32 chain in k order; returns (sum, max |partial|)"""
    acc = np.zeros(np.broadcast_shapes(coef.shape, part.shape)[:-1], dtype=np.float32)
    peak = 0
    for k in range(coef.shape[-1]):
        prod = (coef[..., k] * part[..., k]).astype(np.float32)      # exact: |c * lo| < 2^17
        acc = (acc + prod).astype(np.float32)
        peak = max(peak, int(np.abs(acc).max()))
    return acc, peak


def recombine(lo: np.ndarray, hi: np.ndarray, bits: int, how: str) -> np.ndarray:
    if how == "cvt":
        return hi.astype(np.int64) * (1 << bits) + lo.astype(np.int64)
    bl = (lo + MAGIC).astype(np.float32).view(np.uint32).astype(np.int64)
    bh = (hi + MAGIC).astype(np.float32).view(np.uint32).astype(np.int64)
    v = ((bh << bits) + bl - ((MAGIC_BITS << bits) + MAGIC_BITS)) & 0xFFFFFFFF
    return np.where(v >= 1 << 31, v - (1 << 32), v)


def stage(x: np.ndarray, t: np.ndarray, bits: int, stats: dict, name: str) -> np.ndarray:
    """one transform stage y[b, i, j] = sum_k x[b, i, k] * t[j, k] through the split, every
    recombination checked against the exact product; returns the exact int64 sums"""
    exact = np.einsum("bik,jk->bij", x, t)
    lo = x & ((1 << bits) - 1)
    hi = x >> bits
    tl, pl = f32_chain(t[None, None, :, :], lo[:, :, None, :])
    th, ph = f32_chain(t[None, None, :, :], hi[:, :, None, :])
    st = stats.setdefault(name, {"max_abs_lo_partial": 0, "max_abs_hi_partial": 0, "values": 0,
                                 "f32_tiles_exact": True, "cvt_mismatches": 0, "magic_mismatches": 0})
    st["max_abs_lo_partial"] = max(st["max_abs_lo_partial"], pl)
    st["max_abs_hi_partial"] = max(st["max_abs_hi_partial"], ph)
    st["values"] += int(exact.size)
    st["f32_tiles_exact"] &= bool(np.array_equal(tl.astype(np.int64), np.einsum("bik,jk->bij", lo, t)) and
                                  np.array_equal(th.astype(np.int64), np.einsum("bik,jk->bij", hi, t)))
    st["cvt_mismatches"] += int((recombine(tl, th, bits, "cvt") != exact).sum())
    st["magic_mismatches"] += int((recombine(tl, th, bits, "magic") != exact).sum())
    return exact


def fwd_round(s, shift):
    v = (s + (1 << (shift - 1))) >> shift
    return ((v + 32768) & 0xFFFF) - 32768


def inv_round(s, shift):
    return np.clip((s + (1 << (shift - 1))) >> shift, -32768, 32767)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--batch", type=int, default=48)
    a = ap.parse_args()
    rng = np.random.default_rng(20261017)
    report = {"what": "float32 emulation of the split-operand MFMA transform recombination (tools/tr_comb_emulate.py)",
              "magic_bound": 1 << 22, "f32_exact_bound": 1 << 24, "splits": {}}
    for bits in (10, 11):
        stats: dict = {}
        for n in (16, 32):
            t = dct_matrix(n)
            for depth in (8, 10):
                pmax = (1 << depth) - 1
                # TestBench input classes (mbdstharness.cpp:56-81): residuals for the forward transform,
                # int16 coefficients for the inverse; random, all-min, all-max
                res = [rng.integers(-pmax, pmax + 1, (a.batch, n, n)), np.full((2, n, n), -pmax), np.full((2, n, n), pmax)]
                coef = [rng.integers(-32768, 32768, (a.batch, n, n)), np.full((2, n, n), -32768),
                        np.full((2, n, n), 32767)]
                sh1f, sh2f = (int(np.log2(n)) - 1 + depth - 8), int(np.log2(n)) + 6
                sh1i, sh2i = 7, 12 - (depth - 8)
                for x in res:
                    # forward: U = X T^T (rows), then Y = T U' (columns) — as two row passes
                    u = fwd_round(stage(x.astype(np.int64), t, bits, stats, f"dct{n} stage1"), sh1f)
                    stage(np.swapaxes(u, 1, 2), t, bits, stats, f"dct{n} stage2")
                for c in coef:
                    m = inv_round(stage(np.swapaxes(c, 1, 2).astype(np.int64), t.T, bits, stats, f"idct{n} stage1"),
                                  sh1i)
                    stage(np.swapaxes(m, 1, 2), t.T, bits, stats, f"idct{n} stage2")
        report["splits"][f"{bits}-bit lo"] = stats
    txt = json.dumps(report, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
