"""Deterministic synthetic YUV 4:2:0 source ("Encoder-level
synthetic inputs").

There is no network and no test sequences in the tree, so every workload in
this repository runs on this generator:

* luma: uniform noise in [0, 255] smoothed by a separable 5-tap box filter
  (seed 20261015 for 1080p, 20261016 for 2160p, anything else for other sizes),
  panned +2 px/frame horizontally and +1 px/frame vertically;
* one 128x128 textured object moving (+7, +3) px/frame;
* additive Gaussian noise sigma = 1 per frame;
* chroma: 3-tap-smoothed noise in [64, 192] panned at half rate;
* optional luma fade (`fade` > 0): frame i's luma scaled by 1 - fade * i (a fade to black, the
  case x265's weighted prediction analysis, slicetype.cpp:391-495, exists for).

10-bit output is the 8-bit picture scaled by 4 (plus the same noise scaled),
stored as little-endian uint16, as the survey's Main10 config describes.
"""
from __future__ import annotations

import numpy as np

PAN_X, PAN_Y = 2, 1
OBJ = 128
OBJ_VX, OBJ_VY = 7, 3


def _seed_for(width: int, height: int) -> int:
    if (width, height) == (1920, 1080):
        return 20261015
    if (width, height) == (3840, 2160):
        return 20261016
    return 20261000 + (width * 7 + height) % 997


def _box_fast(a: np.ndarray, taps: int) -> np.ndarray:
    """Separable box filter with wrap-around, via cumulative sums (float64)."""
    pad = taps // 2
    p = np.pad(a.astype(np.float64), pad, mode="wrap")
    c = np.cumsum(p, axis=1)
    c = np.concatenate([np.zeros((c.shape[0], 1)), c], axis=1)
    p = (c[:, taps:] - c[:, :-taps]) / taps
    c = np.cumsum(p, axis=0)
    c = np.concatenate([np.zeros((1, c.shape[1])), c], axis=0)
    return (c[taps:, :] - c[:-taps, :]) / taps


class SyntheticSource:
    """Frame generator; frame(i) returns (Y, U, V) uint8 or uint16 planes."""

    def __init__(self, width: int, height: int, nframes: int, depth: int = 8, seed: int | None = None,
                 fade: float = 0.0):
        assert width % 2 == 0 and height % 2 == 0
        self.w, self.h, self.n, self.depth = width, height, nframes, depth
        self.fade = fade
        self.seed = _seed_for(width, height) if seed is None else seed
        rng = np.random.default_rng(self.seed)
        span_x = width + PAN_X * nframes + 8
        span_y = height + PAN_Y * nframes + 8
        self.tex = _box_fast(rng.uniform(0, 255, (span_y, span_x)), 5)
        obj = _box_fast(rng.uniform(0, 255, (OBJ, OBJ)), 3)
        # give the object more contrast than the background so it is trackable
        self.obj = np.clip((obj - obj.mean()) * 2.5 + 128, 0, 255)
        cw, ch = width // 2, height // 2
        cspan_x = cw + nframes + 8
        cspan_y = ch + nframes + 8
        self.ctex = [
            64 + 128 * (_box_fast(rng.uniform(0, 1, (cspan_y, cspan_x)), 3))
            for _ in range(2)
        ]

    def frame(self, i: int):
        w, h = self.w, self.h
        ox, oy = PAN_X * i, PAN_Y * i
        y = self.tex[oy:oy + h, ox:ox + w].copy()
        px = (w // 4 + OBJ_VX * i) % max(1, w - OBJ)
        py = (h // 4 + OBJ_VY * i) % max(1, h - OBJ)
        y[py:py + OBJ, px:px + OBJ] = self.obj[: min(OBJ, h - py), : min(OBJ, w - px)]
        rng = np.random.default_rng(self.seed * 1000 + i)
        y = y + rng.normal(0.0, 1.0, y.shape)
        if self.fade:
            y = y * max(0.05, 1.0 - self.fade * i)
        cw, ch = w // 2, h // 2
        cx, cy = (PAN_X * i) // 2, (PAN_Y * i) // 2
        u = self.ctex[0][cy:cy + ch, cx:cx + cw]
        v = self.ctex[1][cy:cy + ch, cx:cx + cw]
        if self.depth == 8:
            cvt = lambda a: np.clip(np.rint(a), 0, 255).astype(np.uint8)
        else:
            scale = 1 << (self.depth - 8)
            maxv = (1 << self.depth) - 1
            cvt = lambda a: np.clip(np.rint(a * scale), 0, maxv).astype(np.uint16)
        return cvt(y), cvt(u), cvt(v)

    def write_yuv(self, path: str) -> None:
        with open(path, "wb") as f:
            for i in range(self.n):
                for plane in self.frame(i):
                    f.write(plane.astype("<u2" if self.depth > 8 else np.uint8).tobytes())


if __name__ == "__main__":  # pragma: no cover - CLI helper for census runs
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--depth", type=int, default=8)
    a = ap.parse_args()
    SyntheticSource(a.width, a.height, a.frames, a.depth).write_yuv(a.out)
