"""bench.py's rank path without a GPU: `--gpus 2` with no launcher spawns two ranks with
torch.distributed.run (gloo), each encodes its own closed segment of the synthetic sequence with the hooked
reference encoder (oracle/_ref/x265la8) in the hooks' host form, checks its bitstream against the plain
reference's on the same segment, the elapsed time is the max over ranks, and rank 0 alone prints the line.
A bitstream that differs from the reference's voids the number (value null, exit status 1).

(Sizes: at 192x96 — two CTU rows — the plain reference encoder itself is not deterministic under load, 2 of 24
concurrent runs gave a second bitstream; 256x144 and 320x192 gave one in 24.)"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

LA = os.path.join(ROOT, "oracle", "_ref", "x265la8")
REF = os.path.join(ROOT, "oracle", "_ref", "x265ref8")


@pytest.mark.skipif(not (os.path.exists(LA) and os.path.exists(REF)), reason="reference encoders not built")
def test_bench_two_ranks_host_rehearsal():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--frames", "5", "--width", "256", "--height", "144", "--second-res", "320", "192", "--host-rehearsal",
           "--no-cpu", "--no-replay"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                      # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["warmup"] == 1
    assert line["bitstreams_identical_to_reference"] is True
    assert line["value"] is None and "HOST REHEARSAL" in line["metric"]
    assert line["config"]["parallelism"].startswith("GOP shard x2")
    assert set(line["resolutions"]) == {"144p", "192p"}
    for arm in line["resolutions"].values():
        assert arm["bitstreams_identical_to_reference"] is True and len(arm["fps_runs"]) == 2
        assert arm["fps"] > 0 and "cpu_baseline" not in arm          # cpu_baseline only at N = 1
    assert line["cpu_baseline"] is None
    # both ranks ran their own segment: the per-rank progress lines of ranks 0 and 1
    assert "rank 0 [144p]: writing frames 0..4" in r.stderr and "rank 1 [144p]: writing frames 5..9" in r.stderr


def test_mismatching_bitstream_voids_the_value(tmp_path, monkeypatch, capsys):
    ref_dir = tmp_path / "oracle" / "_ref"
    ref_dir.mkdir(parents=True)
    for exe in ("x265la8", "x265ref8"):
        (ref_dir / exe).write_text("")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    calls = []

    def fake_run(exe, src, w, h, depth, frames, extra, env=None, cpus=None, timeout=900):
        calls.append(os.path.basename(exe))
        hooked = os.path.basename(exe) == "x265la8"
        # the third hooked encode (a timed one) differs from the reference
        bad = hooked and calls.count("x265la8") == 3
        return 10.0, 1.0, "bad" if bad else "good", ""

    monkeypatch.setattr(bench, "x265_run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "2", "--warmup", "1", "--frames", "2", "--width", "64",
                                      "--height", "32", "--second-res", "0", "0", "--host-rehearsal", "--no-cpu",
                                      "--no-replay"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "differs" in str(e.value)
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["value"] is None and line["mpix_per_s"] is None
    assert line["bitstreams_identical_to_reference"] is False and "DIFFERS" in line["metric"]
    assert line["resolutions"]["32p"]["fps"] is None
