"""Encoded fps of the reference encoder (oracle/_ref/x265ref8) and the GPU-lookahead encoder
(oracle/_ref/x265la8) under a few x265 options / hook environments, to see where the host time
goes: each variant is run interleaved ref / la, `reps` times, median reported, with the bitstream
MD5 of both and the CPU seconds (user + sys of the child) per run.  The la runs set
X265AMD_LA_STATS=1 (per-kind call counts and wall time of the hook, stderr).

A variant is "x265 options|ENV=VALUE ENV=VALUE" (either part may be empty; "default" = none)."""
import argparse
import json
import os
import resource
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _cpu():
    r = resource.getrusage(resource.RUSAGE_CHILDREN)
    return r.ru_utime + r.ru_stime


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--variants", default="default;--no-cutree;--rc-lookahead 40;-F 8")
    ap.add_argument("--no-ref", action="store_true", help="only the la encoder")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    from bench import x265_run
    from src.x265_amd.replay_bench import host_cores

    def _x265_run(exe, src, w, h, depth, frames, extra, env=None):
        f, _, m, err = x265_run(exe, src, w, h, depth, frames, extra, env=env)
        return f, m, err
    from src.x265_amd.synth import SyntheticSource

    ref, la = (os.path.join(ROOT, "oracle", "_ref", b) for b in ("x265ref8", "x265la8"))
    cores = host_cores()
    w, h = a.width, a.height
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "src.yuv")
        SyntheticSource(w, h, a.frames, 8).write_yuv(src)
        for v in a.variants.split(";"):
            opts, _, envs = v.partition("|")
            extra = ["--preset", "medium", "--pools", str(cores)] + ([] if opts in ("default", "") else opts.split())
            env = dict(os.environ, X265AMD_LA_STATS="1")
            env.update(kv.split("=", 1) for kv in envs.split())
            fr, fl, cr, cl, md5, stats = [], [], [], [], set(), ""
            for _ in range(a.reps):
                if not a.no_ref:
                    c0 = _cpu()
                    f, m, _ = _x265_run(ref, src, w, h, 8, a.frames, extra)
                    cr.append(round(_cpu() - c0, 2))
                    fr.append(f)
                    md5.add(m)
                c0 = _cpu()
                f, m, err = _x265_run(la, src, w, h, 8, a.frames, extra, env=env)
                cl.append(round(_cpu() - c0, 2))
                fl.append(f)
                md5.add(m)
                stats = "\n".join(l for l in err.splitlines() if "x265la" in l)
            print(json.dumps({"variant": v, "reference_fps": statistics.median(fr) if fr else None,
                              "la_fps": statistics.median(fl), "runs_ref": fr, "runs_la": fl,
                              "cpu_s_ref": cr, "cpu_s_la": cl, "identical": len(md5) == 1}), flush=True)
            print(stats, flush=True)


if __name__ == "__main__":
    main()
