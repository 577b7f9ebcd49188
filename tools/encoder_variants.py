"""Encoded fps of the reference encoder (oracle/_ref/x265ref8) and the GPU-lookahead encoder
(oracle/_ref/x265la8) under a few x265 options, to see where the host time goes: each variant is
run interleaved ref / la, `reps` times, median reported, with the bitstream MD5 of both.
The la runs set X265AMD_LA_STATS=1 (per-kind call counts and wall time of the hook, stderr)."""
import argparse
import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--variants", default="default;--no-cutree;--rc-lookahead 40;-F 8")
    a = ap.parse_args()
    from bench import _x265_run, host_cores
    from src.x265_amd.synth import SyntheticSource

    ref, la = (os.path.join(ROOT, "oracle", "_ref", b) for b in ("x265ref8", "x265la8"))
    cores = host_cores()
    w, h = 1920, 1080
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "src.yuv")
        SyntheticSource(w, h, a.frames, 8).write_yuv(src)
        for v in a.variants.split(";"):
            extra = ["--preset", "medium", "--pools", str(cores)] + ([] if v == "default" else v.split())
            fr, fl, md5, stats = [], [], set(), ""
            for _ in range(a.reps):
                f, m, _ = _x265_run(ref, src, w, h, 8, a.frames, extra)
                fr.append(f)
                md5.add(m)
                f, m, err = _x265_run(la, src, w, h, 8, a.frames, extra,
                                      env=dict(os.environ, X265AMD_LA_STATS="1"))
                fl.append(f)
                md5.add(m)
                stats = "\n".join(l for l in err.splitlines() if "x265la" in l)
            print(json.dumps({"variant": v, "reference_fps": statistics.median(fr), "la_fps": statistics.median(fl),
                              "runs_ref": fr, "runs_la": fl, "identical": len(md5) == 1}), flush=True)
            print(stats, flush=True)


if __name__ == "__main__":
    main()
