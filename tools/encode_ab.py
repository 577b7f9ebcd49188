"""Interleaved A/B of hooked-encoder variants on the bench's own budget (the GPU's 16 host cores, pinned, as
bench.py runs them): the plain reference once, then `reps` rounds of every variant in turn; per run x265's fps,
the wall time, whether the bitstream equals the reference's, and the hook counter lines.

  python tools/encode_ab.py --width 3840 --height 2160 --frames 64 --reps 3 \\
      --variant "base:" --variant "rdo6:X265AMD_RDO=gpu,X265AMD_RDO_MIN=6"

A variant is NAME:ENV=V,ENV=V[:x265 options].  One JSON line per run and a summary line per variant."""
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
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pools", type=int, default=0, help="x265 --pools (default: the core slice's size)")
    ap.add_argument("--variant", action="append", default=[])
    a = ap.parse_args()
    import bench

    cpus = bench.core_slice(0, 1)
    pools = a.pools or len(cpus)
    R = os.path.join(ROOT, "oracle", "_ref")
    out = {}
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "clip.yuv")
        bench.write_clip(src, a.width, a.height, 8, 0, a.frames)
        base = ["--preset", "medium", "--pools", str(len(cpus))]
        rf, rw, rmd5, _ = bench.x265_run(os.path.join(R, "x265ref8"), src, a.width, a.height, 8, a.frames, base,
                                         cpus=cpus)
        print(json.dumps({"variant": "reference", "fps": rf, "wall_s": round(rw, 3)}), flush=True)
        vs = []
        for v in a.variant:
            parts = v.split(":", 2)
            env = dict(kv.split("=", 1) for kv in parts[1].split(",") if kv) if len(parts) > 1 else {}
            extra = parts[2].split() if len(parts) > 2 else []
            vs.append((parts[0], env, extra))
        for rep in range(a.reps):
            for name, env, extra in vs:
                e = dict(os.environ, X265AMD_ME_STATS="1", **env)
                f, w, m, err = bench.x265_run(os.path.join(R, "x265la8"), src, a.width, a.height, 8, a.frames,
                                              ["--preset", "medium", "--pools", str(pools), *extra], env=e, cpus=cpus)
                lines = [ln for ln in err.splitlines() if ln.startswith(("[x265rdo]", "[x265la]", "[x265me] service", "[x265me] check"))
                         or "waiting for the device" in ln]
                print(json.dumps({"variant": name, "rep": rep, "fps": f, "wall_s": round(w, 3), "identical": m == rmd5,
                                  "hook": lines}), flush=True)
                out.setdefault(name, []).append((f, w, m == rmd5))
    for name, runs in out.items():
        fs = [r[0] for r in runs]
        print(json.dumps({"summary": name, "fps_median": statistics.median(fs), "fps_min": min(fs), "fps_max": max(fs),
                          "wall_median": statistics.median(r[1] for r in runs), "all_identical": all(r[2] for r in runs),
                          "reference_fps": rf, "cores": len(cpus), "pools": pools}), flush=True)


if __name__ == "__main__":
    main()
