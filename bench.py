#!/usr/bin/env python3
"""bench.py — x265 1.9 primitive hot path on MI355X, census-driven.

A *step* replays, for F synthetic frames resident in HBM (default 1080p), every
EncoderPrimitives call the reference encoder makes per frame at that
resolution and preset (exact per-entry census: tests/golden/census_<H>p_<preset>
[_main10].json, oracle/run_census.py; default 1080p medium), as one batched gfx950 launch per (table entry, block
shape) through the C ABI (include/x265_amd.h).  Entries that stay on the CPU
in this design (CABAC estimation, SAO, lowres init, ...) are excluded and
listed in the output.  `value` is frames per second of that primitive
workload over all ranks; Mpixel/s is reported beside it.

Modes (one process per GPU under torch.distributed.run; weak scaling, F pictures
per rank per step):
  pipeline (default, every N)  the frame-parallel shard of SURVEY §8(e): picture j
                    of a G*F-picture sequence on rank j mod G, closed --preset medium
                    GOPs of 8 pictures; every census job waits for the reference
                    bands it reads; finished reference bands (deblock, SAO, border
                    extension) go point to point over RCCL to every rank that reads
                    them (src/x265_amd/pipeline.py).  The same step form
                    at N = 1 and N > 1, so the driver's scaling ratio is like for like;
  replay            the census of this rank's F frames as one set of independent
                    grouped launches (no dependencies); at N = 1 its rate is
                    reported beside the pipeline line (`frame_parallel_pipeline.replay`).
Timing: W warmup steps, then K steps bracketed by barrier + device sync, max
over ranks.

Also reported (rank 0):
  roofline     — dominant kernel of the replay step (largest share): its calibrated
                 PMC HBM bytes per launch / its mean launch time, measured with HIP
                 events on the launch stream, against the 8 TB/s HBM peak.
  cpu_baseline — the path north_star names: the reference x265 1.9 CLI
                 (`x265 --preset medium`, C primitives; oracle/_ref/x265ref8,
                 compiled from the reference sources) encoding synthetic frames
                 of the same resolution on the box's host-core share and on one
                 core (N = 1 only); beside it the reference's C primitives
                 replaying the same census descriptors (`census_replay`).
  encoder_level — BASELINE's metric on the encoder itself: encoded fps of the
                 reference x265 encoder and of the same encoder with its lookahead
                 estimates and its large-PU motion searches on the MI355X
                 (integration/gpu_lookahead.cpp, integration/gpu_me.cpp), 64 synthetic
                 frames at 1080p and 2160p on the same host cores, 5 interleaved runs
                 per arm (min / median / max), bitstreams identical; plus the
                 per-call provider on a small clip.

`value` is frames/s of the PRIMITIVE WORKLOAD, not of an end-to-end encode: the
census's calls are batched per schedule step, while inside x265 they are serially
dependent (HEX rounds, sub-pel early exits, intra neighbours), so it bounds what the
table's work costs on the GPU; the encoder frame rate is `encoder_level`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def progress(msg: str) -> None:
    """a progress line on stderr (long phases — the encoder runs — must not look hung)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default K: >= 1 s of timed steps at the measured ~2.2 ms per 8-frame step
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per step per GPU (default: 32 in pipeline mode, 8 in replay mode)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--preset", default="medium", choices=("medium", "slow"),
                    help="selects the census of that x265 preset (tests/golden/census_<H>p_<preset>[_main10].json)")
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a hipGraph")
    ap.add_argument("--mode", default="", choices=("", "pipeline", "replay"),
                    help="pipeline (default, every N): frame-parallel GOP shard, pictures encoded band by band with "
                         "the reference-row dependencies and the RCCL reference exchange (src/x265_amd/pipeline.py), "
                         "closed GOP segments of 8; replay: the census of this rank's frames as one set of "
                         "independent grouped launches (reported beside the pipeline at N = 1)")
    ap.add_argument("--band-rows", type=int, default=0, help="CTU rows per pipeline band (default: whole pictures)")
    ap.add_argument("--segment-frames", type=int, default=0,
                    help="pictures per closed GOP segment in pipeline mode (default 8 with whole-picture bands)")
    ap.add_argument("--exchange", default="torch", choices=("torch", "rccl"),
                    help="pipeline reference exchange: torch.distributed P2P batches, or the native RCCL communicator "
                         "of the C ABI (x265amd_exchange, csrc/exchange.cpp)")
    ap.add_argument("--no-pipeline-check", action="store_true",
                    help="skip the N=1 measurement of the frame-parallel pipeline beside a replay run")
    ap.add_argument("--streams", type=int, default=8, help="HIP streams the step's independent launches spread over")
    ap.add_argument("--no-group", action="store_true", help="one launch per batch instead of grouped multi-shape launches")
    ap.add_argument("--census-cpu-seconds", type=float, default=5.0,
                    help="target duration of the census-replay CPU comparison")
    ap.add_argument("--no-encoder-level", action="store_true")
    ap.add_argument("--encoder-reps", type=int, default=5,
                    help="interleaved encoder runs per arm for encoder_level (SURVEY §8(d): median of >= 5)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--breakdown", type=str, default="", help="write per-batch timing JSON here")
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """--gpus N without a launcher: start N ranks with torch.distributed.run (a child process, before
    this process initialises the GPU) and return their exit status"""
    import socket
    import subprocess

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ))


def dist_setup(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        # the first collective of the group is one every rank joins (batch_isend_irecv, which only the
        # ranks with transfers in a step call, must not be the first NCCL call of the group)
        dist.barrier()
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(v: float, world: int) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


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


def host_cores() -> int:
    """Host CPUs this process may use, capped at the GPU box's per-GPU share (16):
    os.cpu_count() / nproc show the whole machine there."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _x265_run(exe, src, w, h, depth, frames, extra, env=None, one_core=False, timeout=300):
    """Run a reference x265 CLI build; returns (fps, bitstream md5, stderr)."""
    import hashlib
    import re
    import subprocess
    import tempfile

    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "o.hevc")
        cmd = [exe, "--input", src, "--input-res", f"{w}x{h}", "--input-depth", str(depth), "--fps", "30",
               "--frames", str(frames), "--no-info", "-o", out, *extra]
        if depth > 8:
            cmd += ["--output-depth", str(depth)]
        pre = None
        if one_core:
            cpu0 = min(os.sched_getaffinity(0))
            pre = lambda: os.sched_setaffinity(0, {cpu0})
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, preexec_fn=pre)
        if r.returncode != 0:
            raise RuntimeError(f"{os.path.basename(exe)} rc={r.returncode}: {r.stderr[-500:]}")
        m = re.search(r"encoded (\d+) frames in ([\d.]+)s \(([\d.]+) fps\)", r.stderr)
        md5 = hashlib.md5(open(out, "rb").read()).hexdigest()
        return float(m.group(3)), md5, r.stderr


def reference_encoder_baseline(args):
    """x265 1.9 --preset medium (C primitives) on synthetic frames of the bench resolution:
    the box's host-core share and one core."""
    import tempfile

    from src.x265_amd.synth import SyntheticSource

    exe = os.path.join(ROOT, "oracle", "_ref", "x265ref8")
    if args.depth != 8 or not os.path.exists(exe):
        return None
    cores = host_cores()
    n_all = 64 if args.width * args.height <= 1920 * 1080 else 16     # BASELINE config 0: 64 frames at 1080p
    n_one = 4 if args.width * args.height <= 1920 * 1080 else 2
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "src.yuv")
        SyntheticSource(args.width, args.height, n_all, 8).write_yuv(src)
        fps_all, _, _ = _x265_run(exe, src, args.width, args.height, 8, n_all,
                                  ["--preset", args.preset, "--pools", str(cores)])
        progress(f"cpu_baseline {cores} cores: {fps_all} fps")
        fps_one, _, _ = _x265_run(exe, src, args.width, args.height, 8, n_one,
                                  ["--preset", args.preset, "--pools", "1", "-F", "1"], one_core=True)
    return {"value": round(fps_all, 3), "unit": "fps", "cores": cores, "kind": "reference",
            "sample": f"x265 1.9 CLI --preset {args.preset} (C primitives, oracle/_ref/x265ref8 built from the "
                      f"reference sources; no asm) encoding {n_all} synthetic {args.width}x{args.height} frames with "
                      f"--pools {cores} (the box's per-GPU host-core share); one-core figure: {n_one} frames, "
                      f"--pools 1 -F 1 pinned to one CPU",
            "value_1core": round(fps_one, 3), "cpu_model": cpu_model(), "nproc_visible": os.cpu_count(),
            "mpix_per_s": round(fps_all * args.width * args.height / 1e6, 3)}


ENCODER_ARMS = (
    # (key, binary, extra environment, what runs on the MI355X)
    ("reference", "x265ref8", {}, "nothing: the unmodified reference encoder on the host cores"),
    ("mi355x_lookahead", "x265la8", {"X265AMD_ME": "cpu"},
     "LookaheadTLD::lowresIntraEstimate and every CostEstimateGroup estimate (P / B, lowres motion searches, "
     "batched per finishBatch)"),
    ("mi355x_lookahead_me", "x265la8", {"X265AMD_ME": "gpu"},
     "the lookahead estimates as above, plus the main encoder's motion searches of 64x64 PUs "
     "(Search::predInterSearch's per-reference motionEstimate calls of a CU in one device batch, "
     "integration/gpu_me.cpp)"),
)


def encoder_level(args, reps=5, width=None, height=None, frames=None, provider=True):
    """BASELINE's metric on the encoder itself: encoded fps of the reference x265 1.9 encoder
    (oracle/_ref/x265ref8, C primitives) and of the same encoder with parts of its work on the MI355X
    (oracle/_ref/x265la8: integration/gpu_lookahead.cpp and integration/gpu_me.cpp), on the same synthetic
    frames, the same host cores (--pools) and the default frame threads; `reps` runs per arm, interleaved
    arm by arm (median of >= 5, min / median / max reported); every bitstream must be
    identical.  A speed-up is stated as significant only when the arm's slowest run beats the reference's
    fastest.  Beside it, the per-call provider (every primitive one synchronous device round trip)."""
    import statistics
    import tempfile

    from src.x265_amd.synth import SyntheticSource

    arms = [(k, os.path.join(ROOT, "oracle", "_ref", b), env, what) for k, b, env, what in ENCODER_ARMS]
    if args.depth != 8 or not all(os.path.exists(exe) for _, exe, _, _ in arms):
        return None
    if os.environ.get("X265AMD_BENCH_ARMS"):
        keep = set(os.environ["X265AMD_BENCH_ARMS"].split(",")) | {"reference"}
        arms = [a for a in arms if a[0] in keep]
    cores = host_cores()
    W, H = width or args.width, height or args.height
    n = frames or (64 if W * H <= 1920 * 1080 else 16)
    extra = ["--preset", args.preset, "--pools", str(cores)]
    out = {"clip": f"{n} synthetic {W}x{H} 8-bit frames, --preset {args.preset}, --pools {cores}, "
                   f"default frame threads", "cores": cores, "cpu_model": cpu_model(), "runs_per_arm": reps}
    runs = {k: [] for k, _, _, _ in arms}
    md5 = {}
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "src.yuv")
        SyntheticSource(W, H, n, 8).write_yuv(src)
        for _ in range(reps):
            for k, exe, env, _ in arms:
                f, m, _ = _x265_run(exe, src, W, H, 8, n, extra, env=dict(os.environ, **env), timeout=600)
                progress(f"encoder_level {W}x{H} {k}: {f} fps")
                runs[k].append(f)
                md5.setdefault(k, set()).add(m)
    ref = runs["reference"]
    digests = set().union(*md5.values())
    for k, _, _, what in arms:
        r = runs[k]
        e = {"fps_min": min(r), "fps_median": statistics.median(r), "fps_max": max(r), "fps_runs": r,
             "mpix_per_s_median": round(statistics.median(r) * W * H / 1e6, 2), "on_the_gpu": what}
        if k != "reference":
            e["speedup_median"] = round(statistics.median(r) / statistics.median(ref), 3)
            e["speedup_significant"] = min(r) > max(ref)
        out[k] = e
    out["bitstreams_identical"] = len(digests) == 1
    # round-3 field names (reference / lookahead medians), kept for continuity
    out["reference_fps"] = statistics.median(ref)
    if "mi355x_lookahead" in runs:
        out["mi355x_lookahead_fps"] = statistics.median(runs["mi355x_lookahead"])
    out["host_side"] = "CU analysis, RDO, CABAC, loop filters and the remaining motion searches stay on the host cores"
    hip = os.path.join(ROOT, "oracle", "_ref", "x265hip8")
    if provider and os.path.exists(hip):
        w, h, n2 = 416, 240, 2
        small = ["--preset", "medium", "-F", "2", "--pools", "8"]
        with tempfile.TemporaryDirectory() as td:
            src = os.path.join(td, "src.yuv")
            SyntheticSource(w, h, n2, 8).write_yuv(src)
            c_fps, c_md5, _ = _x265_run(hip, src, w, h, 8, n2, small, env=dict(os.environ, X265AMD_PROVIDER="c"))
            g_fps, g_md5, _ = _x265_run(hip, src, w, h, 8, n2, small, env=dict(os.environ, X265AMD_PROVIDER="hip"),
                                        timeout=120)
        out["per_call_provider"] = {"clip": f"{w}x{h} 8-bit, {n2} frames, --preset medium -F 2", "c_table_fps": c_fps,
                                    "mi355x_per_call_provider_fps": g_fps, "bitstreams_identical": c_md5 == g_md5,
                                    "note": "every table call is one synchronous host->device->host round trip"}
    return out


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
        if dt >= args.census_cpu_seconds:
            break
    fps = frames * reps / dt
    return {"value": round(fps, 3), "unit": "fps", "cores": threads, "kind": kind,
            "sample": f"{reps} x the census workload of {frames} {args.width}x{args.height} frames ({sum(b.n for b in bs)} calls per "
                      f"pass, the same batch descriptors as the GPU path) in {dt:.1f}s on {threads} host threads "
                      f"({'x265 1.9 C primitives, oracle/_ref' if kind == 'reference' else 'oracle restatement'})",
            "mpix_per_s": round(fps * args.width * args.height / 1e6, 3)}


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
        del pipe
        torch.cuda.synchronize()
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


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args))
    if not args.mode:
        args.mode = "pipeline"
    if not args.frames:
        args.frames = 32 if args.mode == "pipeline" else 8
    if args.mode == "pipeline" and not args.segment_frames and not args.band_rows:
        # closed --preset medium GOP segments of 8 pictures: the same step form at every N
        args.segment_frames = 8
    import torch

    world, rank, local = dist_setup(args)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs the MI355X (no CPU fallback)")
    from src.x265_amd import Primitives

    prims = Primitives(device=local)
    census, census_name = pick_census(args)
    F = args.frames
    nstreams = max(1, args.streams)
    pipe = None
    if args.mode == "pipeline":
        # frame-parallel shard: picture j of a G*F-picture sequence on rank j mod G, band by band of CTU
        # rows, waiting on / publishing reconstructed reference bands (src/x265_amd/pipeline.py)
        from src.x265_amd.frame_pipeline import GpuFramePipeline

        pipe = GpuFramePipeline(prims, args.width, args.height, args.depth, F, world, rank, census=census,
                                band_rows=args.band_rows or None, segment_frames=args.segment_frames or None,
                                streams=nstreams, device=f"cuda:{local}", exchange=args.exchange)
        # slice (and reorder) the census batches per step and capture the step graphs FIRST
        pipe.build(graphs=not args.no_graph)
    # the replay step: the dominant launch for the roofline (and, in replay mode, the timed step)
    rep = ReplayStep(prims, args, census, local, rank, F=8 if pipe is not None else F)
    if pipe is not None:
        batches, wb, graph = pipe.batches, pipe.wb, bool(pipe.graphs) or None
        run = pipe.step
    else:
        batches, wb, graph = rep.batches, rep.wb, rep.graph
        run = rep.run
    step_bytes = sum(b.bytes for b in batches)
    calls = sum(b.n for b in batches)
    dominant, ktimes, launches = rep.dominant, rep.ktimes, rep.launches

    progress(f"timing {args.steps} steps ({args.mode})")
    for _ in range(args.warmup):
        run()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, world)

    # stability: after the K timed steps, three more windows of >= 1 s each (not part of `value`)
    per = max(1e-4, elapsed / args.steps)
    n_long = max(1, int(1.0 / per) + 1)
    windows = []
    for _ in range(3):
        barrier(world)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(n_long):
            run()
        torch.cuda.synchronize()
        barrier(world)
        windows.append(max_over_ranks(time.perf_counter() - t1, world))

    # dominant kernel, timed live on its launch stream (eager launches bracketed by HIP events)
    st = torch.cuda.current_stream()
    evs = []
    for _ in range(max(args.steps, 20)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dominant.run(prims)
        e1.record(st)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    dom_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)

    ms_per_step = elapsed * 1000.0 / args.steps
    fps = world * F * args.steps / elapsed
    if rank == 0:
        algo_gbps = dominant.bytes / (dom_ms * 1e-3) / 1e9
        kname = f"{dominant.kind}:{dominant.name}"
        # the committed PMC summaries were recorded on the replay step with 8 frames
        ppath = pmc_traffic_path(args) if rep.F == 8 else ""
        traffic = pmc_traffic(dominant.name, ppath) if ppath else None
        # A census launch re-reads blocks many times (x265 scores many candidates per fenc block), so its
        # algorithmic bytes exceed what reaches HBM and algorithmic/time can exceed the HBM
        # peak.  The HBM fraction is therefore taken from the calibrated PMC bytes of the same launch
        # (FETCH_SIZE / WRITE_SIZE passes); without a PMC record the algorithmic rate is reported beside a
        # null frac.
        achieved = traffic / (dom_ms * 1e-3) / 1e9 if traffic else None
        roofline = {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                    "traffic": traffic,
                    "basis": "PMC HBM bytes per launch / launch time" if traffic else
                             "no PMC record for this launch in " + (os.path.relpath(ppath, ROOT) if ppath else
                             "profiles/ (recorded with 8 frames per step)") + "; see achieved_algorithmic",
                    "achieved_algorithmic": round(algo_gbps, 1),
                    "kernel": kname, "kernel_ms": round(dom_ms, 4), "bytes_per_launch": int(dominant.bytes),
                    "launch_jobs": dominant.n,
                    "share_of_step": round(ktimes[dominant.name] / max(1e-9, sum(ktimes.values())), 3),
                    "workload": f"the census of {rep.F} frames as independent grouped launches (the replay step); "
                                "the same kernels make up the pipeline's per-step slices"}
        if traffic:
            roofline["traffic_over_algorithmic"] = round(traffic / dominant.bytes, 3)
        replay = None
        if world == 1:
            replay = rep.rate()
        step_traffic = [pmc_traffic(b.name, ppath) for b in launches] if ppath else []
        step_hbm = None
        rep_ms = replay["ms_per_step"] if replay else (ms_per_step if pipe is None else None)
        if rep_ms and step_traffic and all(t is not None for t in step_traffic):
            tb = sum(step_traffic)
            step_hbm = {"bytes_per_step": tb, "GBps": round(tb / (rep_ms * 1e-3) / 1e9, 1),
                        "frac": round(tb / (rep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "basis": f"sum of the replay step's launches' PMC HBM bytes ({rep.F} frames) / its "
                                 "ms_per_step"}
        caller = None
        if world == 1:
            try:
                from src.x265_amd.caller_bench import caller_rates
                caller = caller_rates(prims, args.width, args.height, args.depth, dev=f"cuda:{local}")
            except Exception as e:   # informational: never fails the bench line
                caller = {"error": str(e)}
        frame_parallel = None
        if world == 1 and not args.no_pipeline_check:
            try:
                skip = {(args.band_rows, args.segment_frames)} if pipe is not None else set()
                frame_parallel = pipeline_rates(prims, args, census, local, skip=skip)
            except Exception as e:   # informational
                frame_parallel = {"error": str(e)}
            if replay is not None:
                frame_parallel = dict(frame_parallel or {}, replay=replay)
        cpu, creplay, enc = None, None, None
        if world == 1 and not args.no_cpu:
            try:
                cpu = reference_encoder_baseline(args)
            except Exception as e:
                cpu = {"value": None, "error": str(e)}
            try:
                creplay = census_replay_cpu(args, census)
            except Exception as e:
                creplay = {"value": None, "error": str(e)}
            if cpu is None:
                cpu = creplay
            else:
                cpu["census_replay"] = creplay
        if world == 1 and not args.no_encoder_level:
            progress("encoder_level runs")
            try:
                enc = encoder_level(args, reps=args.encoder_reps)
                if (args.width, args.height) == (1920, 1080) and args.preset == "medium":
                    # BASELINE's 4K figure: 2160p medium, 64 frames (longer than the lookahead depth)
                    enc["2160p"] = encoder_level(args, reps=args.encoder_reps, width=3840, height=2160, frames=64,
                                                 provider=False)
            except Exception as e:
                enc = {"error": str(e)}
        if pipe is not None:
            workload = (f"primitive-workload fps of the frame-parallel step: the x265-1.9 --preset {args.preset} "
                        f"per-frame primitive census ({args.height}p, tests/golden/{census_name}) of {world * F} "
                        f"pictures as closed GOPs of {pipe.segment_frames} (I/P/B-ref/b, 3 refs, L1<=2), every job "
                        "waiting for the reference bands it reads (deblock/SAO/border final), batched gfx950 "
                        "kernels per schedule step; CPU-side entries (CABAC estimates, SAO RDO, lowres init) "
                        "excluded")
        else:
            workload = (f"primitive-workload fps: the x265-1.9 --preset {args.preset} per-frame primitive census "
                        f"({args.height}p, tests/golden/{census_name}) replayed as independent batched gfx950 "
                        "kernels; CPU-side entries (CABAC estimates, SAO RDO, lowres init) excluded")
        line = {
            "metric": f"primitive-workload fps (x265 1.9 --preset {args.preset} per-frame primitive census, "
                      f"{args.height}p {args.depth}-bit, frame-parallel GOP shard; not an end-to-end encode: "
                      f"see encoder_level) + Mpixels/s",
            "value": round(fps, 2),
            "unit": "fps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8" if args.depth == 8 else "u16",
            "data": "synthetic (src/x265_amd/synth.py), HBM-resident",
            "config": {
                "workload": workload,
                "resolution": f"{args.width}x{args.height}", "depth": args.depth, "frames_per_step_per_gpu": F,
                "calls_per_step_per_gpu": calls, "batches_per_step": len(batches),
                "launches_per_step": pipe.launches_per_step if pipe is not None else len(launches),
                "algorithmic_GB_per_step_per_gpu": round(step_bytes / 1e9, 3),
                "hipgraph": graph is not None, "streams": nstreams, "mode": args.mode,
                "parallelism": (f"frame-parallel GOP shard x{world}: {world * F // pipe.segment_frames} closed "
                                f"--preset medium GOPs of {pipe.segment_frames} pictures (I/P/B-ref/b, 3 refs, L1<=2), "
                                f"picture j on rank j mod {world}, bands of {pipe.plan.band_rows} CTU rows in "
                                f"{pipe.sched.nsteps} schedule steps, final reference bands (deblock/SAO/border) sent "
                                f"to every rank that reads them over "
                                f"{('RCCL P2P (' + args.exchange + ')') if world > 1 else 'in-place stores (one rank)'}"
                                if pipe is not None else
                                f"independent replay x{world}"),
                "frames_per_step_total": world * F,
            },
            "mpix_per_s": round(fps * args.width * args.height / 1e6, 1),
            "timed_region_s": round(elapsed, 4),
            "fps_1s_windows": [round(world * F * n_long / w, 1) for w in windows],
            "step_GBps_algorithmic": round(step_bytes * world / (elapsed / args.steps) / 1e9, 1),
            "step_hbm": step_hbm,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "encoder_level": enc,
            "frame_parallel_pipeline": frame_parallel,
            "caller_level_rates": caller,
            "cpu_excluded_calls_per_frame": round(sum(v for v in wb.skipped.values()) / F),
        }
        if pipe is not None and getattr(pipe, "comm", None) is not None:
            line["config"]["rccl_backend"] = getattr(pipe.comm, "backend", None)
        if args.breakdown:
            with open(args.breakdown, "w") as f:
                json.dump({b.name: {"ms": ktimes[b.name], "jobs": b.n, "bytes": b.bytes,
                                    "GBps": b.bytes / (ktimes[b.name] * 1e-3) / 1e9} for b in launches}, f, indent=1)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
