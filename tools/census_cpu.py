"""TEST / BASELINE INFRASTRUCTURE (moved out of src/ in round 6): the census workload of
src/x265_amd/replay_bench.py run by the reference C primitives (oracle/_ref) or the oracle restatement on the host
cores — the CPU leg the round 1-4 bench reported beside the replay.  It imports oracle/pyoracle, which the product
package must not.

  python tools/census_cpu.py [--width 1920 --height 1080 --depth 8 --preset medium --seconds 10]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from src.x265_amd.replay_bench import host_cores, pick_census  # noqa: E402


def census_replay_cpu(args, census):
    """Reference C primitives over a bounded sample of the same census workload."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import CpuPrims, available

    from src.x265_amd.workload import FrameSet, WorkloadBuilder, census_batches

    kind = "reference" if available("ref", args.depth) else "port"
    threads = host_cores()
    prims = CpuPrims("ref" if kind == "reference" else "oracle", args.depth, nthreads=threads)
    frames = 2
    fs = FrameSet(args.width, args.height, frames, args.depth, device="cpu")
    # the census of `frames` frames, replayed until about args.cpu_seconds of CPU time have passed
    bs, _ = census_batches(fs, frames=frames, census=census, builder=WorkloadBuilder(fs, seed=4))
    torch.set_num_threads(1)
    reps, t0 = 0, time.perf_counter()
    while True:
        for b in bs:
            b.run(prims)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= args.seconds:
            break
    fps = frames * reps / dt
    return {"value": round(fps, 3), "unit": "fps", "cores": threads, "kind": kind,
            "sample": f"{reps} x the census workload of {frames} {args.width}x{args.height} frames ({sum(b.n for b in bs)} calls per "
                      f"pass, the same batch descriptors as the GPU path) in {dt:.1f}s on {threads} host threads "
                      f"({'x265 1.9 C primitives, oracle/_ref' if kind == 'reference' else 'oracle restatement'})",
            "mpix_per_s": round(fps * args.width * args.height / 1e6, 3)}



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--preset", default="medium")
    ap.add_argument("--seconds", type=float, default=10.0)
    args = ap.parse_args()
    census, name = pick_census(args)
    out = census_replay_cpu(args, census)
    out["census"] = name
    print(json.dumps(out))


if __name__ == "__main__":
    main()
