# diff pattern of a transform build against the oracle on seeded cases (diagnostic; X265AMD_LIB selects the build)
import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np
import torch
assert torch.cuda.is_available()
from cases import DCT, IDCT, case_transform, run_cpu, run_gpu
from pyoracle import CpuOracle
from src.x265_amd import Primitives
prims = Primitives(device=0); orc = CpuOracle("oracle", 8)
for kind in (DCT, IDCT):
    for seed in (232949807741904, 96453540148203, 5, 6):
        c = case_transform(kind, 32, 8, 64, seed)
        a, b = run_gpu(c, prims)["d"].astype(np.int64), run_cpu(c, orc)["d"].astype(np.int64)
        d = a - b
        nz = np.nonzero(d)[0]
        print(kind, seed, "mismatches", len(nz), "of", d.size, "diffs", np.unique(d[nz])[:10].tolist(),
              "pairs", list(zip(a[nz][:6].tolist(), b[nz][:6].tolist())))
