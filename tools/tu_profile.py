"""Fused TU pipeline sensitivity: HBM fraction per TU size at several QPs with sign hiding on/off,
plus the share of TUs with numSig 0 / 1 (inverse skipped / DC shortcut).  python tools/tu_profile.py"""
import sys, os, torch, json
sys.path.insert(0, os.getcwd())
from src.x265_amd import Primitives
prims = Primitives(device=0)
W = 8192; dev = "cuda"
def timeit(fn, reps=10):
    for _ in range(2): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); [fn() for _ in range(reps)]; e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
for log2 in (2, 3, 4, 5):
    s = 1 << log2; num = s * s; per_tu = 7 * num + 6
    n = int(1.5e9 / per_tu)
    per_row = W // s
    j = torch.arange(n, device=dev, dtype=torch.int64)
    off = (j // per_row) * s * W + (j % per_row) * s
    rows = int((n // per_row + 1) * s)
    g = torch.Generator(device=dev).manual_seed(1)
    F = torch.randint(0, 256, (rows * W,), dtype=torch.int16, device=dev, generator=g)
    P = (F + torch.randint(-6, 7, F.shape, dtype=torch.int16, device=dev, generator=g)).clamp(0, 255)
    F, P = F.to(torch.uint8), P.to(torch.uint8)
    R = torch.empty(rows * W, dtype=torch.int16, device=dev); RC = torch.empty(rows * W, dtype=torch.uint8, device=dev)
    CO = torch.empty(n * num, dtype=torch.int16, device=dev); coff = j * num
    SIG = torch.empty(n, dtype=torch.int32, device=dev)
    SC = torch.zeros(n, dtype=torch.uint8, device=dev)
    out = {}
    for qp in (0, 22, 32, 51):
        QP = torch.full((n,), qp, dtype=torch.uint8, device=dev)
        for sh in (1, 0):
            ms = timeit(lambda: prims.tu_pipeline(8, log2, 1, 0, 0, sh, F, W, off, P, W, off, R, W, off, CO, coff, RC, W, off, SIG, QP, SC))
            out[f"qp{qp}_sh{sh}"] = round(n * per_tu / ms / 1e6 / 8000, 3)
        sig = SIG.cpu()
        out[f"qp{qp}_sig0"] = round(float((sig == 0).float().mean()), 3)
        out[f"qp{qp}_sig1"] = round(float((sig == 1).float().mean()), 3)
    print(s, json.dumps(out), flush=True)
