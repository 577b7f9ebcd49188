"""Where a bench step's wall time goes outside x265's own clock: the hooked encoder (oracle/_ref/x265la8) run as
bench.py runs it (pinned to the GPU's host cores, the bench's hooked environment) with X265AMD_PHASES=1, which
stamps main, encoder open, the first encode call, the close (sessions dropped, encoder closed) and exit; the
parent stamps the spawn and the reap.

  python tools/phases.py --width 3840 --height 2160 --frames 64 --reps 2"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import bench

    cpus = bench.core_slice(0, 1)
    env = dict(os.environ, X265AMD_ME_STATS="1", X265AMD_RDO="gpu", X265AMD_RDO_EARLY="1", X265AMD_RDO_LAUNCHERS="0",
               X265AMD_RDO_SERVER="1", X265AMD_PHASES="1")
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "clip.yuv")
        bench.write_clip(src, a.width, a.height, 8, 0, a.frames)
        cmd = ["taskset", "-c", ",".join(map(str, cpus)), os.path.join(ROOT, "oracle", "_ref", "x265la8"),
               "--input", src, "--input-res", f"{a.width}x{a.height}", "--fps", "30", "--frames", str(a.frames),
               "--preset", "medium", "--pools", str(len(cpus)), "-o", os.path.join(td, "o.hevc")]
        for rep in range(a.reps):
            t0 = time.time()
            r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=900)
            t1 = time.time()
            st = {}
            for m in re.finditer(r"\[phase\] (\w+) ([\d.]+)", r.stderr):
                st.setdefault(m.group(1), float(m.group(2)))      # (the first stamp of a name)
            enc = re.search(r"encoded \d+ frames in ([\d.]+)s", r.stderr)
            marks = ["spawn"] + [k for k in ("main", "open", "opened", "first_encode", "close", "me_dropped",
                                             "la_dropped", "sessions_dropped", "closed", "exit") if k in st] + ["reaped"]
            st["spawn"], st["reaped"] = t0, t1
            gaps = {f"{marks[i]}->{marks[i + 1]}": round(1e3 * (st[marks[i + 1]] - st[marks[i]]), 1)
                    for i in range(len(marks) - 1)}
            print(json.dumps({"rep": rep, "rc": r.returncode, "wall_ms": round(1e3 * (t1 - t0), 1),
                              "x265_ms": round(1e3 * float(enc.group(1)), 1) if enc else None, "gaps_ms": gaps}),
                  flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
