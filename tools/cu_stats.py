"""Where the hooked encoder's worker time goes: x265's own CU statistics (oracle/_ref/x265la8s, built with
DETAILED_CU_STATS) and, optionally, a gprof flat profile (oracle/_ref/x265la8p, every reference object built
with -pg), on the bench's budget (the GPU's 16 host cores, pinned) and the bench's hooks (bench.py's hooked
environment: device lookahead, motion searches and inter residual coding).

  python tools/cu_stats.py --out gpurun_out/cu --width 3840 --height 2160 --frames 64 [--gprof]

Writes <out>/cu_stats.txt (the "CU:" lines and the hook counter lines of one encode, plus the plain
reference's CU lines from oracle/_ref/x265ref8s) and, with --gprof, <out>/gprof_flat.txt."""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--gprof", action="store_true")
    a = ap.parse_args()
    import bench

    os.makedirs(a.out, exist_ok=True)
    cpus = bench.core_slice(0, 1)
    R = os.path.join(ROOT, "oracle", "_ref")
    # (bench.py's default hooked environment, --rdo server)
    env = dict(os.environ, X265AMD_ME_STATS="1", X265AMD_RDO="gpu", X265AMD_RDO_EARLY="1", X265AMD_RDO_LAUNCHERS="0",
               X265AMD_RDO_SERVER="1")
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "clip.yuv")
        bench.write_clip(src, a.width, a.height, 8, 0, a.frames)
        args = ["--input", src, "--input-res", f"{a.width}x{a.height}", "--fps", "30", "--frames", str(a.frames),
                "--preset", "medium", "--pools", str(len(cpus)), "-o", os.path.join(td, "o.hevc")]
        lines = []
        # (the bench's own binary first: its fps and hook counters beside the statistics build's)
        for name, exe, e in (("hooked, no statistics", "x265la8", env), ("hooked", "x265la8s", env),
                             ("reference", "x265ref8s", dict(os.environ))):
            r = subprocess.run(["taskset", "-c", ",".join(map(str, cpus)), os.path.join(R, exe), *args],
                               capture_output=True, text=True, env=e, timeout=900)
            if r.returncode:
                sys.stderr.write(r.stderr[-3000:])
                return r.returncode
            keep = [ln for ln in r.stderr.splitlines() if "CU:" in ln or ln.startswith(("[x265", "encoded"))]
            lines += [f"== {name} ({exe}, {a.width}x{a.height}, {a.frames} frames, --pools {len(cpus)}, pinned)"] + keep
            print(f"{name}: done", flush=True)
        with open(os.path.join(a.out, "cu_stats.txt"), "w") as f:
            f.write("\n".join(lines) + "\n")
        if a.gprof:
            r = subprocess.run(["taskset", "-c", ",".join(map(str, cpus)), os.path.join(R, "x265la8p"), *args],
                               capture_output=True, text=True, env=env, timeout=900, cwd=td)
            if r.returncode:
                sys.stderr.write(r.stderr[-3000:])
                return r.returncode
            g = subprocess.run(["gprof", "-b", "-p", os.path.join(R, "x265la8p"), os.path.join(td, "gmon.out")],
                               capture_output=True, text=True, timeout=300)
            with open(os.path.join(a.out, "gprof_flat.txt"), "w") as f:
                f.write("\n".join(g.stdout.splitlines()[:80]) + "\n")
            print("gprof: done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
