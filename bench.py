#!/usr/bin/env python3
"""bench.py — BASELINE's metric: encoded fps (+ Mpixel/s) of x265 1.9 --preset medium at 2160p 8-bit,
with the encoder's hot path on the MI355X.

A *step* is one encode of a 64-frame synthetic 3840x2160 8-bit clip (BASELINE config 0's clip length,
SURVEY §8(d) generator, src/x265_amd/synth.py) by the reference x265 1.9 encoder built from the
reference sources with the MI355X hooks (oracle/_ref/x265la8: integration/gpu_lookahead.cpp — every
lookahead cost estimate on the device — and integration/gpu_me.cpp — the motion searches of the 64x64
CUs posted to the device at CU start and batched over all worker threads by the launch service of
csrc/mesession.cpp), on the rank's share of the host cores (16 per GPU, `--pools 16`).  Every step's
bitstream must equal the plain reference encoder's on the same clip (checked on every rank).

`value` = frames encoded by all ranks / the slowest rank's wall time of the K timed steps, or null (and
exit status 1) when any warmup or timed encode's bitstream differs from the reference's.  At N > 1
each rank encodes its own closed 64-frame segment of the sequence (frames 64 r .. 64 r + 63) on its own
GPU and host-core slice: GOP-level frame parallelism with no data-path collective (independent closed
segments exchange nothing), weak scaling.  The frame-level shard inside one encoder (frame encoder i on
device session i mod G, X265AMD_GPUS) is exercised by the tests, not timed here.

Also reported (rank 0):
  roofline      — the dominant kernel of the encode, the batched motion search (k_motion_search): its
                  algorithmic bytes per launch (per full-pel evaluation 2 W H b, per sub-pel
                  evaluation ((W+7)(H+7) + W H) b, counted by the kernel) over its mean launch time (HIP
                  events around each launch on the service stream, inside the encoder process), against
                  the 8 TB/s HBM peak;
  cpu_baseline  — the plain reference encoder (oracle/_ref/x265ref8, C primitives) on the same clip and
                  the same cores (N = 1), and on one core (2 frames);
  resolutions   — BASELINE names 1080p and 2160p: the same measurement at 1920x1080 (64 frames, its own
                  reference encode and bitstream check) after the headline 2160p arm;
  encoder       — per-run fps (x265's own clock), the device-path worker time (forming / posting /
                  waiting), launch-service counters;
  primitive_workload — the round 1-4 census replay (src/x265_amd/replay_bench.py) at 1080p with its
                  PMC-calibrated roofline (N = 1; --no-replay skips it).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import re
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
CORES_PER_GPU = 16      # the GPU box's host-core share per GPU


def progress(msg: str) -> None:
    """a progress line on stderr (long phases — the encodes — must not look hung)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed encodes of the clip per rank")
    ap.add_argument("--warmup", type=int, default=1, help="untimed encodes before the timed ones")
    ap.add_argument("--frames", type=int, default=64, help="frames per encode (per rank)")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--preset", default="medium")
    ap.add_argument("--no-cpu", action="store_true", help="skip the reference encoder's one-core sample")
    ap.add_argument("--no-replay", action="store_true", help="skip the primitive-workload replay (N = 1)")
    ap.add_argument("--env", action="append", default=[], help="extra KEY=VALUE for the hooked encoder")
    ap.add_argument("--rdo", choices=["server", "off"], default="server",
                    help="inter residual coding of 64x64 CUs on the device through the resident server "
                         "(integration/gpu_rdo.cpp, X265AMD_RDO_SERVER; DESIGN §14), or on the host")
    ap.add_argument("--second-res", type=int, nargs=2, default=[1920, 1080], metavar=("W", "H"),
                    help="BASELINE's other resolution, timed after the headline one (reported under "
                         "`resolutions`; --second-res 0 0 skips it)")
    ap.add_argument("--host-rehearsal", action="store_true",
                    help="tests only: the hooks' host forms, no GPU (rank plumbing), value null")
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """--gpus N without a launcher: start N ranks with torch.distributed.run (a child process, before
    this process initialises the GPU) and return their exit status"""
    import socket

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ))


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # control only (start / stop barriers, max over ranks): the encodes exchange no data
        dist.init_process_group(backend="gloo")
        dist.barrier()
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

    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_true(v: bool, world: int) -> bool:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist

    t = torch.tensor([0 if v else 1], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item()) == 0


def core_slice(local: int, world: int):
    """this rank's host cores: a disjoint slice of CORES_PER_GPU of the process's affinity set when the
    node has that many for every rank (one GPU box shows the whole machine's CPUs); otherwise an equal
    disjoint share of the set per rank (at least one core), so ranks never contend for the same cores"""
    cpus = sorted(os.sched_getaffinity(0))
    world = max(1, world)
    per = CORES_PER_GPU if len(cpus) >= CORES_PER_GPU * world else max(1, len(cpus) // world)
    lo = (local * per) % max(1, len(cpus))
    return cpus[lo:lo + per] or cpus[:per]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def write_clip(path, w, h, depth, first, n):
    """frames first .. first + n - 1 of the synthetic sequence (a closed segment of rank r: first = n r)"""
    import numpy as np

    from src.x265_amd.synth import SyntheticSource

    src = SyntheticSource(w, h, first + n, depth)
    with open(path, "wb") as f:
        for i in range(first, first + n):
            for plane in src.frame(i):
                f.write(plane.astype("<u2" if depth > 8 else np.uint8).tobytes())


def x265_run(exe, src, w, h, depth, frames, extra, env=None, cpus=None, timeout=900):
    """One encode; returns (x265's fps, wall seconds, bitstream md5, stderr)."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "o.hevc")
        cmd = [exe, "--input", src, "--input-res", f"{w}x{h}", "--input-depth", str(depth), "--fps", "30",
               "--frames", str(frames), "--no-info", "-o", out, *extra]
        if depth > 8:
            cmd += ["--output-depth", str(depth)]
        pre = (lambda: os.sched_setaffinity(0, set(cpus))) if cpus else None
        t0 = time.perf_counter()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, preexec_fn=pre)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            raise RuntimeError(f"{os.path.basename(exe)} rc={r.returncode}: {r.stderr[-800:]}")
        m = re.search(r"encoded (\d+) frames in ([\d.]+)s \(([\d.]+) fps\)", r.stderr)
        md5 = hashlib.md5(open(out, "rb").read()).hexdigest()
        return float(m.group(3)), wall, md5, r.stderr


def parse_me_stats(err: str):
    """the hook's and the launch service's counters (integration/gpu_me.cpp print_stats)"""
    out = {}
    m = re.search(r"worker time on the device path: forming ([\d.]+) s, reference uploads ([\d.]+) s, posting "
                  r"([\d.]+) s, waiting for the device ([\d.]+) s \((\d+) waits\)", err)
    if m:
        out.update(form_s=float(m.group(1)), upload_s=float(m.group(2)), post_s=float(m.group(3)),
                   wait_s=float(m.group(4)), waits=int(m.group(5)))
    m = re.search(r"service: (\d+) launches, (\d+) requests \(([\d.]+) per launch, max (\d+)\), (\d+) searches, "
                  r"kernel ([\d.]+) ms per launch \(HIP events\), batch ([\d.]+) ms, queueing ([\d.]+) ms per request, "
                  r"(\d+) waits slept; (\d+) row uploads ([\d.]+) MB ([\d.]+) ms; sessions (\d+)(?:; evaluations (\d+) "
                  r"full-pel (\d+) sub-pel, ([\d.]+) GB algorithmic, longest launch ([\d.]+) ms)?", err)
    if m:
        g = m.groups()
        out.update(launches=int(g[0]), requests=int(g[1]), requests_per_launch=float(g[2]),
                   max_requests_per_launch=int(g[3]), searches=int(g[4]), kernel_ms_per_launch=float(g[5]),
                   batch_ms=float(g[6]), queue_ms_per_request=float(g[7]), waits_slept=int(g[8]),
                   row_uploads=int(g[9]), row_upload_MB=float(g[10]), sessions=int(g[12]))
        if g[13] is not None:
            out.update(evals_fpel=int(g[13]), evals_subpel=int(g[14]), algo_GB=float(g[15]),
                       longest_launch_ms=float(g[16]))
    m = re.search(r"stats prefetches (\d+) searches (\d+) memo hits (\d+) misses (\d+)", err)
    if m:
        out.update(prefetches=int(m.group(1)), memo_hits=int(m.group(3)), memo_misses=int(m.group(4)))
    # inter residual coding (integration/gpu_rdo.cpp print_stats)
    m = re.search(r"\[x265rdo\] stats CUs posted (\d+) coded on the host (\d+); transformNxN memo hits (\d+) misses (\d+);"
                  r".*?worker wait ([\d.]+) s", err)
    if m:
        rdo = dict(cus_on_device=int(m.group(1)), cus_on_host=int(m.group(2)), tq_memo_hits=int(m.group(3)),
                   tq_memo_misses=int(m.group(4)), worker_wait_s=float(m.group(5)))
        m = re.search(r"\[x265rdo\] early posts merge (\d+) inter (\d+) bidir (\d+); used (\d+), dropped (\d+)", err)
        if m:
            rdo.update(early_posts=int(m.group(1)) + int(m.group(2)) + int(m.group(3)), early_used=int(m.group(4)))
        m = re.search(r"\[x265rdo\] service: .*? batch ([\d.]+) ms, queueing ([\d.]+) ms per CU", err)
        if m:
            rdo.update(post_to_result_ms=float(m.group(1)), posting_ms_per_cu=float(m.group(2)))
        out["rdo"] = rdo
    return out


ME_TRAFFIC = os.path.join(ROOT, "profiles", "r05", "pmc_me_traffic.json")


def me_roofline(st, traffic_file=ME_TRAFFIC):
    """roofline of the batched motion-search launch from the encoder's own HIP-event timing; traffic = the
    launch's HBM bytes from the committed PMC passes (FETCH_SIZE x 2 per the gfx950 note + WRITE_SIZE, per
    dispatch) when that table exists"""
    if not st.get("launches") or "algo_GB" not in st:
        return None
    per_launch = st["algo_GB"] * 1e9 / st["launches"]
    ms = st["kernel_ms_per_launch"]
    achieved = per_launch / (ms * 1e-3) / 1e9
    traffic, tbasis = None, "no PMC table of this launch (profiles/r05/pmc_me_traffic.json)"
    if traffic_file and os.path.exists(traffic_file):
        with open(traffic_file) as f:
            t = json.load(f)
        traffic = int(t["traffic_bytes_per_launch"])
        tbasis = (f"traffic: HBM bytes per launch from {os.path.relpath(traffic_file, ROOT)} (rocprofv3 FETCH_SIZE x "
                  f"{t['fetch_correction']} + WRITE_SIZE per launch; {traffic / per_launch:.2f} of the algorithmic "
                  "bytes_per_launch: the algorithmic count charges every candidate evaluation its block and "
                  "reference window, and the overlapping windows of neighbouring candidates are served by L1 / L2, "
                  "so HBM sees each window about once)")
    # "bound" names the roof frac is measured against (the contract's hbm | mfma); what actually limits this
    # kernel is latency / occupancy ("limiter"): one workgroup per search, a few searches per launch
    return {"bound": "hbm", "limiter": "latency / occupancy (one workgroup of up to four waves per search, a few "
                                       "searches per launch on an otherwise idle GPU; not bandwidth)",
            "kernel": "k_motion_search (x265amd_motion_search, launch-service batches)",
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "bytes_per_launch": int(per_launch), "kernel_ms": ms, "launches": st["launches"],
            "searches_per_launch": round(st["searches"] / st["launches"], 2),
            "basis": "algorithmic bytes per launch (DESIGN.md §3c: 2WHb per full-pel evaluation, ((W+7)(H+7)+WH)b "
                     "per sub-pel evaluation, evaluations counted by the kernel) / mean launch time (HIP events "
                     "around each launch on the launch-service stream, in the encoder process; the kernel is "
                     "latency-bound: one workgroup of up to four waves per search, ~7 searches per launch); " + tbasis}


def run_arm(args, world, rank, la, ref, W, H, F, D, cpus, extra, env, ref_env, steps, warmup, tag):
    """one resolution: this rank's segment clip, the plain reference's bitstream (and fps) on it, `warmup`
    untimed and `steps` timed hooked encodes (bracketed by barriers; the elapsed time is the max over
    ranks), every bitstream compared with the reference's"""
    with tempfile.TemporaryDirectory(prefix=f"bench{rank}_{tag}_") as td:
        src = os.path.join(td, "clip.yuv")
        progress(f"rank {rank} [{tag}]: writing frames {F * rank}..{F * rank + F - 1} ({W}x{H} {D}-bit)")
        write_clip(src, W, H, D, F * rank, F)
        # the reference bitstream of this rank's segment (and, at N = 1, the cpu_baseline): the plain
        # reference encoder on the same clip and cores (Main10: the same binary with the hooks off)
        progress(f"rank {rank} [{tag}]: reference encode")
        if D == 8:
            ref_fps, ref_wall, ref_md5, _ = x265_run(ref, src, W, H, D, F, extra, env=ref_env, cpus=cpus)
        else:
            ref_fps, ref_wall, ref_md5, _ = x265_run(la, src, W, H, D, F, extra, env=ref_env, cpus=cpus)
        progress(f"rank {rank} [{tag}]: reference {ref_fps} fps")
        mismatches = 0
        for i in range(warmup):
            f, _, m, _ = x265_run(la, src, W, H, D, F, extra, env=env, cpus=cpus)
            mismatches += m != ref_md5
            progress(f"rank {rank} [{tag}]: warmup {i}: {f} fps")
        barrier(world)
        runs, walls, err = [], [], ""
        t0 = time.perf_counter()
        for i in range(steps):
            f, wall, m, err = x265_run(la, src, W, H, D, F, extra, env=env, cpus=cpus)
            mismatches += m != ref_md5
            runs.append(f)
            walls.append(wall)
            progress(f"rank {rank} [{tag}]: step {i}: {f} fps (wall {wall:.2f} s){'' if m == ref_md5 else ' BITSTREAM DIFFERS'}")
        elapsed = time.perf_counter() - t0
        barrier(world)
        elapsed = max_over_ranks(elapsed, world)
        identical = all_true(mismatches == 0, world)
        one_core = None
        if rank == 0 and world == 1 and not args.no_cpu and D == 8 and tag == "2160p" and not args.host_rehearsal:
            n1 = 2
            f1, _, _, _ = x265_run(ref, src, W, H, D, n1, ["--preset", args.preset, "--pools", "1", "-F", "1"],
                                   cpus=cpus[:1])
            one_core = {"fps": f1, "frames": n1}
    fps = world * F * steps / elapsed
    return {"fps": fps, "elapsed": elapsed, "identical": identical, "mismatching_encodes_this_rank": mismatches,
            "runs": runs, "walls": walls, "err": err, "ref_fps": ref_fps, "ref_wall": ref_wall, "one_core": one_core,
            "W": W, "H": H, "F": F, "steps": steps}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args))
    world, rank, local = dist_setup(args)
    W, H, F, D = args.width, args.height, args.frames, args.depth
    la = os.path.join(ROOT, "oracle", "_ref", "x265la8" if D == 8 else "x265la10")
    ref = os.path.join(ROOT, "oracle", "_ref", "x265ref8")
    if not os.path.exists(la):
        raise SystemExit(f"{la} missing (build with __graft_entry__.build())")
    if not args.host_rehearsal:
        import torch

        if not torch.cuda.is_available():
            raise SystemExit("bench.py needs the MI355X (no CPU fallback)")
    cpus = core_slice(local, world)
    pools = str(len(cpus))
    extra = ["--preset", args.preset, "--pools", pools]
    env = dict(os.environ, HIP_VISIBLE_DEVICES=str(local), X265AMD_ME_STATS="1")
    if args.rdo == "server":
        # each 64x64 inter CU's residual coding posted when its prediction is final and served by the resident
        # kernel (measured faster than the host and than per-CU launches)
        env.update(X265AMD_RDO="gpu", X265AMD_RDO_EARLY="1", X265AMD_RDO_LAUNCHERS="0", X265AMD_RDO_SERVER="1")
    if args.host_rehearsal:
        # the hooks' host forms (integration/: the same forming, posting and memo, the searches, estimates and
        # residual coding by the reference's own functions): the rank plumbing on a machine without the GPU,
        # NOT a measurement
        env.update(X265AMD_ME="host", X265AMD_LOOKAHEAD="host")
        env.update(X265AMD_RDO="host" if args.rdo == "server" else "cpu")
        for k in ("X265AMD_RDO_EARLY", "X265AMD_RDO_LAUNCHERS", "X265AMD_RDO_SERVER"):
            env.pop(k, None)
    env.update(kv.split("=", 1) for kv in args.env)
    ref_env = dict(os.environ, X265AMD_LOOKAHEAD="cpu", X265AMD_ME="cpu")

    head = run_arm(args, world, rank, la, ref, W, H, F, D, cpus, extra, env, ref_env, args.steps, args.warmup,
                   f"{H}p")
    second = None
    if args.second_res[0] > 0 and (args.second_res[0], args.second_res[1]) != (W, H):
        w2, h2 = args.second_res
        second = run_arm(args, world, rank, la, ref, w2, h2, F, D, cpus, extra, env, ref_env, args.steps, 1,
                         f"{h2}p")
    replay = None
    if rank == 0 and world == 1 and not args.no_replay and not args.host_rehearsal:
        progress("primitive-workload replay (1080p census)")
        try:
            from src.x265_amd.replay_bench import primitive_workload

            replay = primitive_workload(local=local)
        except Exception as e:   # informational: never fails the bench line
            replay = {"error": str(e)}

    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    identical = head["identical"] and (second is None or second["identical"])
    st = parse_me_stats(head["err"])
    ms_per_step = head["elapsed"] * 1000.0 / args.steps

    def arm_summary(a):
        sm = {"fps": round(a["fps"], 3), "mpix_per_s": round(a["fps"] * a["W"] * a["H"] / 1e6, 1),
              "resolution": f"{a['W']}x{a['H']}", "frames_per_step_per_gpu": a["F"], "steps": a["steps"],
              "timed_region_s": round(a["elapsed"], 3), "bitstreams_identical_to_reference": a["identical"],
              "fps_runs": a["runs"], "wall_s_runs": [round(w, 3) for w in a["walls"]],
              "speedup_vs_reference_same_cores": round(statistics.median(a["runs"]) / a["ref_fps"], 3),
              "device_path": parse_me_stats(a["err"])}
        if world == 1:
            sm["cpu_baseline"] = {"value": a["ref_fps"], "unit": "fps", "cores": len(cpus), "kind": "reference",
                                  "wall_s": round(a["ref_wall"], 3),
                                  "mpix_per_s": round(a["ref_fps"] * a["W"] * a["H"] / 1e6, 2)}
        if not a["identical"]:
            sm["fps"] = sm["mpix_per_s"] = None
        return sm

    res = {f"{head['H']}p": arm_summary(head)}
    if second is not None:
        res[f"{second['H']}p"] = arm_summary(second)
    what = (f"x265 1.9 --preset {args.preset}, {H}p {D}-bit, {F}-frame synthetic clip per GPU, reference encoder with "
            "its lookahead estimates, motion searches" + (" and inter residual coding" if args.rdo == "server" else "")
            + " on the MI355X")
    line = {
        # a bitstream that differs from the reference's on any rank voids the number: value null, exit 1
        "metric": f"encoded fps ({what}, " + ("bitstream identical to the reference" if identical else
                                             "BITSTREAM DIFFERS FROM THE REFERENCE: not a valid measurement")
                  + ") + Mpixels/s" + (" [HOST REHEARSAL: hooks in host mode, not a measurement]"
                                       if args.host_rehearsal else ""),
        "value": round(head["fps"], 3) if identical and not args.host_rehearsal else None,
        "unit": "fps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 1),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8" if D == 8 else "u16",
        "data": "synthetic (src/x265_amd/synth.py: SURVEY §8(d) generator), written per rank before timing",
        "config": {"workload": f"{F} frames {W}x{H} {D}-bit yuv420p per GPU, x265 --preset {args.preset} "
                               f"--pools {pools} (default frame threads), oracle/_ref/{os.path.basename(la)}",
                   "resolution": f"{W}x{H}", "depth": D, "frames_per_step_per_gpu": F, "preset": args.preset,
                   "parallelism": f"GOP shard x{world}: rank r encodes the closed segment of frames {F}r..{F}r+{F - 1} "
                                  "on its own GPU and host-core slice; no data-path collective (DESIGN.md §6)",
                   "host_cores_per_gpu": len(cpus), "cpu_model": cpu_model(),
                   "hooked_env": {k: v for k, v in env.items() if k.startswith("X265AMD")}},
        "mpix_per_s": round(head["fps"] * W * H / 1e6, 1) if identical else None,
        "timed_region_s": round(head["elapsed"], 3),
        "bitstreams_identical_to_reference": identical,
        "resolutions": res,
        "encoder": {"fps_runs": head["runs"], "fps_min": min(head["runs"]), "fps_median": statistics.median(head["runs"]),
                    "fps_max": max(head["runs"]), "wall_s_runs": [round(w, 3) for w in head["walls"]],
                    "device_path": st},
        "roofline": me_roofline(st),
        "cpu_baseline": {"value": head["ref_fps"], "unit": "fps", "cores": len(cpus), "kind": "reference",
                         "sample": f"x265 1.9 CLI --preset {args.preset} (C primitives, oracle/_ref/"
                                   f"{'x265ref8' if D == 8 else 'x265la10 with its hooks off'}, built from the reference "
                                   f"sources; no asm) encoding the same {F}-frame clip on the same {len(cpus)} cores "
                                   "(--pools), one run", "wall_s": round(head["ref_wall"], 3),
                         "mpix_per_s": round(head["ref_fps"] * W * H / 1e6, 2),
                         "one_core": head["one_core"]} if world == 1 else None,
        "speedup_vs_reference_same_cores": round(statistics.median(head["runs"]) / head["ref_fps"], 3),
        "primitive_workload": replay,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    if not identical:
        raise SystemExit("bench.py: a hooked encode's bitstream differs from the reference's")


if __name__ == "__main__":
    main()
