"""The drop-in proof: the reference's OWN harnesses run on the MI355X provider.

SURVEY.md §8(b)/(c): a replacement slots in where x265's assembly providers sit
(`x265_setup_primitives`, primitives.cpp:228-249).  Two reference programs are
compiled from /root/reference where they lie (oracle/Makefile `bridge`; the
binaries travel to the GPU box in oracle/_ref/, the sources do not):

* TestBench{8,10} — the reference TestBench (test/testbench.cpp:153-243, its four
  harnesses pixel / transforms / interp / intrapred) whose asm hook installs the
  provider (oracle/hip_bridge.cpp): every entry the provider implements is
  checked against the reference's C table `cprim` with the harness's own random
  / min / max inputs, iterations and whole-buffer compares;
* x265hip{8,10} — the reference CLI and encoder (x265_encoder_open /
  x265_encoder_encode, api.cpp:182) with the provider in the global table
  (oracle/hip_encoder_main.cpp).  The bitstream and the reconstructed frames must
  be identical to the same encoder on the C table: every primitive result the
  encoder consumes came from the GPU, and one differing bit anywhere would change
  a decision and the bitstream.
"""
import hashlib
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFBIN = os.path.join(ROOT, "oracle", "_ref")
sys.path.insert(0, ROOT)

W, H, FRAMES = 416, 240, 3
# -F 2: frame-parallel search-range clip (search.cpp:89-91) so the result does not
# depend on thread timing; --pools bounds the number of host threads (and so the
# provider's per-thread device contexts)
ENC_ARGS = ["--preset", "medium", "-F", "2", "--pools", "8", "--fps", "30", "--no-info"]


def _bin(name):
    p = os.path.join(REFBIN, name)
    if not os.path.exists(p):
        if os.path.isdir("/root/reference/x265_1.9/source"):
            from src.x265_amd import build as b

            b.build(verbose=False)
            subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "bridge"], check=True,
                           capture_output=True)
        else:
            pytest.skip(f"{name} not built (oracle/Makefile bridge needs /root/reference)")
    return p


def _source(tmp_path, depth):
    from src.x265_amd.synth import SyntheticSource

    path = tmp_path / f"src_{W}x{H}_{depth}.yuv"
    SyntheticSource(W, H, FRAMES, depth).write_yuv(str(path))
    return path


def _encode(exe, provider, src, depth, out_dir, timeout=600):
    env = dict(os.environ, X265AMD_PROVIDER=provider)
    bs, rec = out_dir / f"{provider}.hevc", out_dir / f"{provider}_recon.yuv"
    cmd = [exe, "--input", str(src), "--input-res", f"{W}x{H}", "--input-depth", str(depth), "--frames",
           str(FRAMES), *ENC_ARGS, "-o", str(bs), "--recon", str(rec)]
    if depth > 8:
        cmd += ["--output-depth", str(depth)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    m = re.search(r"encoded (\d+) frames in ([\d.]+)s \(([\d.]+) fps\)", r.stderr)
    assert m and int(m.group(1)) == FRAMES, r.stderr[-2000:]
    digest = lambda p: hashlib.md5(p.read_bytes()).hexdigest()
    return digest(bs), digest(rec), float(m.group(3)), r.stderr


def test_reference_cli_builds_agree_on_cpu(tmp_path):
    """(no GPU) the bridge binary on the C table encodes exactly like the plain reference CLI"""
    src = _source(tmp_path, 8)
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    a = _encode(_bin("x265ref8"), "c", src, 8, tmp_path / "a")
    b = _encode(_bin("x265hip8"), "c", src, 8, tmp_path / "b")
    assert a[:2] == b[:2]
    assert "provider=c" in b[3]


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
@pytest.mark.parametrize("harness", ["pixel", "transforms", "interp", "intrapred"])
def test_reference_testbench_on_hip_provider(depth, harness):
    exe = _bin(f"TestBench{depth}")
    env = dict(os.environ, X265AMD_TB_SPEED="0")
    r = subprocess.run([exe, "--cpuid", "SSE2", "--testbench", harness], capture_output=True, text=True, env=env,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    m = re.search(r"\[hip_bridge\] MI355X provider installed: (\d+) entries", out)
    assert m and int(m.group(1)) > 1000, out[-2000:]
    assert "Testing primitives: SSE2" in out
    assert "failed" not in out.lower(), out[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [8, 10])
def test_reference_encoder_on_hip_provider_is_bit_exact(tmp_path, depth):
    exe = _bin(f"x265hip{depth}")
    src = _source(tmp_path, depth)
    (tmp_path / "c").mkdir()
    (tmp_path / "h").mkdir()
    c_bs, c_rec, c_fps, _ = _encode(exe, "c", src, depth, tmp_path / "c")
    h_bs, h_rec, h_fps, log = _encode(exe, "hip", src, depth, tmp_path / "h", timeout=900)
    m = re.search(r"provider=hip entries=(\d+)", log)
    assert m and int(m.group(1)) > 1000, log[-2000:]
    print(f"\n[dropin] {W}x{H} {depth}-bit medium, {FRAMES} frames: C table {c_fps} fps, "
          f"MI355X per-call provider {h_fps} fps; bitstream md5 {h_bs}")
    assert h_bs == c_bs, "bitstream differs between the C table and the MI355X provider"
    assert h_rec == c_rec, "reconstructed frames differ"


def _run_enc(exe, src, depth, out_dir, env_extra, timeout=600):
    env = dict(os.environ, **env_extra)
    cmd = [exe, "--input", str(src), "--input-res", f"{W}x{H}", "--input-depth", str(depth), "--frames",
           str(FRAMES), *ENC_ARGS, "-o", str(out_dir / "o.hevc")]
    return subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)


def test_encoder_fails_loudly_without_device(tmp_path):
    """(no GPU) the provider cannot be installed: the encoder refuses to run (non-zero exit,
    the library's message) instead of silently encoding on the C table"""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is present")
    src = _source(tmp_path, 8)
    r = _run_enc(_bin("x265hip8"), src, 8, tmp_path, {"X265AMD_PROVIDER": "hip"})
    assert r.returncode != 0
    assert "x265amd_setup_primitives failed" in r.stderr, r.stderr[-2000:]
    assert not (tmp_path / "o.hevc").exists() or (tmp_path / "o.hevc").stat().st_size == 0


@pytest.mark.gpu
@pytest.mark.parametrize("fault", [{"X265AMD_FAULT": "alloc"}, {"X265AMD_FAULT_AFTER": "2000"}],
                         ids=["staging-alloc", "copy-after-2000-calls"])
def test_provider_failure_fails_the_encode(tmp_path, fault):
    """A failing staging allocation / device copy inside the per-call provider must surface as
    x265_encoder_encode() < 0 (x265.h:1351-1359), i.e. the CLI's exit code 4
    (x265.cpp:643-649), not as garbage primitive results in a 'successful' encode"""
    src = _source(tmp_path, 8)
    r = _run_enc(_bin("x265hip8"), src, 8, tmp_path, dict(fault, X265AMD_PROVIDER="hip"), timeout=900)
    assert r.returncode == 4, (r.returncode, r.stderr[-3000:])
    assert "MI355X provider failed" in r.stderr, r.stderr[-2000:]
    assert "x265_encoder_encode -> -1" in r.stderr
