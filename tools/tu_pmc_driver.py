"""Minimal driver for PMC passes over the fused TU kernel of one size (no timing logic):
    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python tools/tu_pmc_driver.py --log2 5"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src.x265_amd import Primitives  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--log2", type=int, default=5)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--sh", type=int, default=1)
a = ap.parse_args()
prims = Primitives(device=0)
W, dev, log2 = 8192, "cuda", a.log2
s = 1 << log2
num = s * s
n = int(1.5e9 / (7 * num + 6))
per_row = W // s
j = torch.arange(n, device=dev, dtype=torch.int64)
off = (j // per_row) * s * W + (j % per_row) * s
rows = int((n // per_row + 1) * s)
g = torch.Generator(device=dev).manual_seed(1)
F = torch.randint(0, 256, (rows * W,), dtype=torch.int16, device=dev, generator=g)
P = (F + torch.randint(-12, 13, F.shape, dtype=torch.int16, device=dev, generator=g)).clamp(0, 255)
F, P = F.to(torch.uint8), P.to(torch.uint8)
R = torch.empty(rows * W, dtype=torch.int16, device=dev)
RC = torch.empty(rows * W, dtype=torch.uint8, device=dev)
CO = torch.empty(n * num, dtype=torch.int16, device=dev)
SIG = torch.empty(n, dtype=torch.int32, device=dev)
QP = torch.randint(22, 38, (n,), dtype=torch.uint8, device=dev, generator=g)
SC = torch.zeros(n, dtype=torch.uint8, device=dev)
for _ in range(a.reps):
    prims.tu_pipeline(8, log2, 1, 1, 0, a.sh, F, W, off, P, W, off, R, W, off, CO, j * num, RC, W, off, SIG, QP, SC)
torch.cuda.synchronize()
print("done", n)
