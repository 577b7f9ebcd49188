"""Rate of the frame-parallel pipeline step on one GPU (frame_pipeline.GpuFramePipeline) for a few
frame counts / band heights, beside the independent replay of the same frame count."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n):
    import torch

    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="8,32")
    ap.add_argument("--band-rows", default="17,4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--segments", default="0", help="comma list of pictures per closed GOP segment (0: all frames)")
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--job-wait", default="band", help="comma list of band / reference")
    ap.add_argument("--background", default="0", help="comma list of 1 / 0")
    ap.add_argument("--streams", default="8", help="comma list of stream counts for the step lanes")
    ap.add_argument("--exchange", default="torch",
                    help="comma list of torch / rccl (rccl at one rank: the multi-rank graph structure, per-step "
                         "graphs, with an empty native exchange)")
    a = ap.parse_args()
    import torch

    from src.x265_amd import Primitives
    from src.x265_amd.frame_pipeline import GpuFramePipeline
    from src.x265_amd.workload import FrameSet, WorkloadBuilder, census_batches, group_launches

    prims = Primitives(device=0)
    for F in (int(x) for x in a.frames.split(",")):
        if not a.no_replay:
            fs = FrameSet(1920, 1080, F, 8, device="cuda")
            bs, _ = census_batches(fs, frames=F, builder=WorkloadBuilder(fs, seed=11))
            ls = group_launches(bs)
            dt = timed(lambda: [b.run(prims) for b in ls], a.reps)
            print(json.dumps({"mode": "replay-eager-1stream", "frames": F, "fps": round(F / dt, 1),
                              "launches": len(ls)}), flush=True)
            del fs, bs, ls
        for br, seg, jw, bgv, ex, nst in [(int(x), int(g), w, int(v), e, int(sn)) for x in a.band_rows.split(",")
                                          for g in a.segments.split(",") for w in a.job_wait.split(",")
                                          for v in a.background.split(",") for e in a.exchange.split(",")
                                          for sn in a.streams.split(",")]:
            early = True
            t0 = time.perf_counter()
            pipe = GpuFramePipeline(prims, 1920, 1080, 8, F, 1, 0, band_rows=br, streams=nst, device="cuda",
                                    early_independent=early, segment_frames=seg or None, job_wait=jw,
                                    background=bool(bgv), exchange=ex)
            pipe.build(graphs=True)
            tb = time.perf_counter() - t0
            dt = timed(pipe.step, a.reps)
            print(json.dumps({"mode": "pipeline", "frames": F, "band_rows": br, "segment_frames": seg or F, "job_wait": jw, "background": bgv, "exchange": ex, "streams": nst, "fps": round(F / dt, 1),
                              "ms_per_step": round(dt * 1e3, 3), "steps": pipe.sched.nsteps,
                              "launches": pipe.launches_per_step, "build_s": round(tb, 1)}), flush=True)
            pipe.close()
            del pipe


if __name__ == "__main__":
    main()
