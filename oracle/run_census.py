"""Per-frame primitive call census of the reference encoder — MEASUREMENT INFRASTRUCTURE.

Builds nothing itself: run `make -C oracle census` first (reference CLI +
census_main.cpp, only where /root/reference exists).  Encodes the synthetic
source of src/x265_amd/synth.py with the reference x265 1.9
(`--preset medium --no-asm`) and counts every call of every EncoderPrimitives
slot exactly (census_main.cpp).  The per-frame averages are written to
tests/golden/census_<res>_<preset>.json and define the workload bench.py
replays on the GPU.

    python oracle/run_census.py --width 1920 --height 1080 --frames 16
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--preset", default="medium")
    ap.add_argument("--depth", type=int, default=8, choices=(8, 10))
    a = ap.parse_args()

    from src.x265_amd.synth import SyntheticSource

    exe = os.path.join(HERE, "_ref", "x265census" if a.depth == 8 else "x265census10")
    if not os.path.exists(exe):
        raise SystemExit(f"run `make -C oracle {'census' if a.depth == 8 else 'census10'}` first")
    with tempfile.TemporaryDirectory() as td:
        yuv = os.path.join(td, "in.yuv")
        SyntheticSource(a.width, a.height, a.frames, a.depth).write_yuv(yuv)
        out = os.path.join(td, "census.json")
        env = dict(os.environ, X265_CENSUS_OUT=out)
        cmd = [exe, "--input", yuv, "--input-res", f"{a.width}x{a.height}", "--fps", "30", "--preset", a.preset,
               *(["--input-depth", "10", "--output-depth", "10"] if a.depth == 10 else []),
               "--no-asm", "-o", os.path.join(td, "out.hevc")]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, check=True)
        counts = json.load(open(out))["counts"]
    per_frame = {k: v / a.frames for k, v in sorted(counts.items())}
    name = f"census_{a.height}p_{a.preset}{'' if a.depth == 8 else '_main10'}.json"
    doc = {
        "what": "calls per frame of every EncoderPrimitives slot, x265 1.9 C primitives (reference built by "
                "oracle/Makefile), exact counts via census_main.cpp",
        "command": " ".join(["x265"] + cmd[1:2] + ["<synthetic>"] + cmd[3:]),
        "source": f"src/x265_amd/synth.py {a.width}x{a.height} {a.frames} frames {a.depth}-bit 4:2:0",
        "encoder_summary": [l for l in r.stderr.splitlines() if "encoded" in l],
        "frames": a.frames,
        "per_frame": per_frame,
    }
    path = os.path.join(ROOT, "tests", "golden", name)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {path} ({len(per_frame)} slots, {sum(per_frame.values()):.0f} calls/frame)")


if __name__ == "__main__":
    main()
