"""Primitive-workload replay (the round 1-4 bench step), kept beside the encoder headline of bench.py.

A step replays, for F synthetic frames resident in HBM, every EncoderPrimitives call the reference
encoder makes per frame at that resolution and preset (exact per-entry census:
tests/golden/census_<H>p_<preset>[_main10].json, oracle/run_census.py) as batched gfx950 launches
through the C ABI (include/x265_amd.h).  `ReplayStep` gives its rate and its dominant launch (the
grouped census SATD) with the PMC-calibrated roofline (profiles/pmc_traffic*.json); `pipeline_rates`
the frame-parallel GOP-shard forms; tools/census_cpu.py (test infrastructure, round 6: moved out of the product package) the reference C primitives over
the same descriptors on the host cores.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def progress(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_cores() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def kernel_times(batches, prims, reps=2):
    """mean device time per batch launch (HIP events on the launch stream)"""
    import torch

    st = torch.cuda.current_stream()
    out = {}
    for _ in range(reps):
        for b in batches:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            b.run(prims)
            e1.record(st)
            out.setdefault(b.name, []).append((e0, e1))
    torch.cuda.synchronize()
    return {k: sum(a.elapsed_time(c) for a, c in v) / len(v) for k, v in out.items()}


def pmc_traffic_path(args) -> str:
    """the PMC traffic table of this configuration (F = 8 frames per step): profiles/pmc_traffic.json
    for the default 1080p medium 8-bit step, profiles/pmc_traffic_<h>p_<preset>_<depth>bit.json else"""
    default = (args.width, args.height, args.depth, args.preset) == (1920, 1080, 8, "medium")
    name = "pmc_traffic.json" if default else f"pmc_traffic_{args.height}p_{args.preset}_{args.depth}bit.json"
    return os.path.join(ROOT, "profiles", name)


def pmc_traffic(launch_name: str, path: str):
    """per-launch HBM bytes of `launch_name` from a committed PMC summary
    (tools/pmc_workload.py + tools/pmc_parse.py, FETCH_SIZE and WRITE_SIZE in separate
    rocprofv3 passes, calibrated on known-byte kernels), if any"""
    if not os.path.exists(path):
        return None
    try:
        e = json.load(open(path)).get(launch_name)
        return int(e["hbm_bytes"]) if e else None
    except Exception:
        return None


def pick_census(args):
    """The reference encoder's per-frame call census for this resolution / preset / depth.

    Falls back to the 1080p medium census scaled by the pixel ratio when no census of the
    exact configuration has been recorded (oracle/run_census.py records them)."""
    from src.x265_amd.workload import load_census

    gold = os.path.join(ROOT, "tests", "golden")
    name = f"census_{args.height}p_{args.preset}{'_main10' if args.depth > 8 else ''}.json"
    for cand in (name, f"census_{args.height}p_{args.preset}.json"):
        if os.path.exists(os.path.join(gold, cand)):
            return load_census(os.path.join(gold, cand)), cand
    base = load_census()
    k = args.width * args.height / (1920 * 1080)
    return {key: v * k for key, v in base.items()}, f"census_1080p_medium.json x {k:.3f} (pixel ratio)"


def pipeline_rates(prims, args, census, local, skip=()):
    """Other forms of the frame-parallel step on this one GPU, beside `value` (N = 1): one open GOP of
    F = 32 pictures with whole-picture and 4-CTU-row bands, and 32 one-picture segments (32 I pictures:
    no references, one step) — the same pictures through the same graph machinery without any
    dependency."""
    import torch

    from src.x265_amd.frame_pipeline import GpuFramePipeline

    F = 32
    out = {"frames_per_step": F}
    for br, seg in ((0, 0), (4, 0), (0, 8), (0, 1)):
        if (br, seg) in skip:
            continue
        progress(f"pipeline form band_rows={br} segments={seg}")
        pipe = GpuFramePipeline(prims, args.width, args.height, args.depth, F, 1, 0, census=census,
                                band_rows=br or None, segment_frames=seg or None, streams=args.streams,
                                device=f"cuda:{local}")
        pipe.build(graphs=True)
        for _ in range(2):
            pipe.step()
        torch.cuda.synchronize()
        n = 10
        t0 = time.perf_counter()
        for _ in range(n):
            pipe.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        out[f"band_rows_{br or pipe.plan.band_rows}" + (f"_segments_of_{seg}" if seg else "")] = {
            "fps": round(F / dt, 1), "ms_per_step": round(dt * 1e3, 3), "bands_per_frame": pipe.plan.nbands,
            "schedule_steps": pipe.sched.nsteps, "launches_per_step": pipe.launches_per_step}
        pipe.close()
        del pipe
    return out


class ReplayStep:
    """The census of F frames of this rank as one set of independent grouped launches (one launch per
    kernel class), spread over S streams by measured launch time and captured in a hipGraph.  It gives
    the dominant launch of the workload (the roofline kernel: the committed PMC table was recorded on
    this step with F = 8) and the replay rate reported beside the pipeline `value`."""

    def __init__(self, prims, args, census, local, rank, F=8):
        import ctypes

        import torch

        from src.x265_amd import capture_graph
        from src.x265_amd.workload import FrameSet, WorkloadBuilder, census_batches, group_launches

        self.prims, self.F = prims, F
        fs = FrameSet(args.width, args.height, F, args.depth, device=f"cuda:{local}", first_frame=rank * F)
        self.batches, self.wb = census_batches(fs, frames=F, census=census, builder=WorkloadBuilder(fs, seed=11 + rank))
        self.launches = launches = list(self.batches) if args.no_group else group_launches(self.batches)
        self.bytes = sum(b.bytes for b in self.batches)
        self.calls = sum(b.n for b in self.batches)
        nstreams = max(1, args.streams)
        side = [torch.cuda.Stream() for _ in range(nstreams)] if nstreams > 1 else []
        solo, lanes, fork = [], [[] for _ in range(nstreams)], [False]

        def assign(first=None, weight=None):
            """lanes by longest-processing-time: launches in decreasing weight, each onto the least-loaded
            stream; the dominant launch runs alone first (not overlapped), so its in-step duration is
            its isolated duration and the rocprof summary of the same command agrees"""
            fork[0] = first is not None
            solo[:] = [first] if first is not None else []
            load = [0.0] * nstreams
            for lst in lanes:
                lst.clear()
            wt = weight or (lambda b: b.bytes)
            for b in sorted(launches, key=wt, reverse=True):
                if b is first:
                    continue
                i = min(range(nstreams), key=lambda k: load[k])
                lanes[i].append(b)
                load[i] += wt(b)

        def kernels():
            if not side or not fork[0]:
                for b in launches:
                    b.run(prims)
                return
            for b in solo:
                b.run(prims)
            cur = torch.cuda.current_stream()
            for s_, lst in zip(side, lanes):
                s_.wait_stream(cur)
                h = ctypes.c_void_p(s_.cuda_stream)
                for b in lst:
                    b.run(prims, h)
            for s_ in side:
                cur.wait_stream(s_)

        assign()
        for _ in range(max(1, args.warmup)):
            kernels()
        torch.cuda.synchronize()
        self.ktimes = kernel_times(launches, prims)
        self.dominant = max(launches, key=lambda b: self.ktimes[b.name])
        balance = os.environ.get("X265AMD_BENCH_BALANCE", "time")
        assign(self.dominant, (lambda b: self.ktimes[b.name]) if balance == "time" else None)
        self.kernels, self.graph = kernels, None
        if not args.no_graph:
            try:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    kernels()
                torch.cuda.current_stream().wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with capture_graph(g):
                    kernels()
                g.replay()
                torch.cuda.synchronize()
                self.graph = g
            except Exception as e:  # capture unsupported: measure eager launches instead
                print(f"[bench] hipGraph capture failed ({e}); eager launches", file=sys.stderr)

    def run(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self.kernels()

    def rate(self, seconds=1.0):
        """frames/s of this step alone (>= `seconds` of timed steps after a warm-up)"""
        import torch

        for _ in range(5):
            self.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.run()
        torch.cuda.synchronize()
        n = max(5, int(seconds / max(1e-5, time.perf_counter() - t0)))
        t0 = time.perf_counter()
        for _ in range(n):
            self.run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        return {"fps": round(self.F / dt, 1), "ms_per_step": round(dt * 1e3, 3), "frames_per_step": self.F,
                "steps": n, "launches_per_step": len(self.launches), "hipgraph": self.graph is not None}




def primitive_workload(width=1920, height=1080, depth=8, preset="medium", local=0, streams=8, seconds=1.0):
    """The census replay of 8 frames on this GPU (independent grouped launches in a hipGraph): its frame
    rate and the roofline of its dominant launch (calibrated PMC bytes / launch time, HIP events on the
    launch stream).  Informational beside the encoder headline."""
    import argparse

    import torch

    from src.x265_amd import Primitives

    args = argparse.Namespace(width=width, height=height, depth=depth, preset=preset, streams=streams, warmup=3,
                              no_group=False, no_graph=False)
    prims = Primitives(device=local)
    census, census_name = pick_census(args)
    rep = ReplayStep(prims, args, census, local, 0, F=8)
    rate = rep.rate(seconds)
    dominant = rep.dominant
    st = torch.cuda.current_stream()
    evs = []
    for _ in range(50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dominant.run(prims)
        e1.record(st)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    dom_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    ppath = pmc_traffic_path(args)
    traffic = pmc_traffic(dominant.name, ppath)
    achieved = traffic / (dom_ms * 1e-3) / 1e9 if traffic else None
    return {"workload": f"the x265-1.9 --preset {preset} per-frame primitive census ({height}p, "
                        f"tests/golden/{census_name}) of 8 frames replayed as independent batched gfx950 launches "
                        "(no encoder control flow: an upper bound on what the table's work costs on the GPU)",
            "fps": rate["fps"], "ms_per_step": rate["ms_per_step"], "launches_per_step": rate["launches_per_step"],
            "calls_per_step": rep.calls, "algorithmic_GB_per_step": round(rep.bytes / 1e9, 3),
            "roofline": {"bound": "hbm", "kernel": f"{dominant.kind}:{dominant.name}", "kernel_ms": round(dom_ms, 4),
                         "traffic": traffic, "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "achieved_algorithmic": round(dominant.bytes / (dom_ms * 1e-3) / 1e9, 1),
                         "basis": "calibrated PMC HBM bytes of the launch (" + os.path.relpath(ppath, ROOT) +
                                  ") / its mean time over 50 launches (HIP events on the launch stream)"}}
