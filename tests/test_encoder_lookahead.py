"""f1 in the RUNNING encoder: the reference x265 1.9 encoder with its lookahead cost estimates on
the MI355X (integration/gpu_lookahead.cpp over the x265amd_la_* session entries).

oracle/Makefile x265la links the reference CLI + encoder, compiled where its sources lie, with
LookaheadTLD::lowresIntraEstimate (slicetype.cpp:230-336) and
CostEstimateGroup::estimateFrameCost (slicetype.cpp:1977-2066) replaced by the hook.  Every
slice-type decision, cuTree propagation, rate-control and VBV figure of the encode is derived
from those estimates, so one differing cost anywhere changes the bitstream: the encode on the
device must be BIT-IDENTICAL to the plain reference encoder (oracle/_ref/x265ref8) on the same
input — at 1080p --preset medium (lookahead slices, b-adapt 2 batches, weightp, cuTree, AQ).

CPU tests pin the binding itself:
  * X265AMD_LOOKAHEAD=cpu  — the hooked binary calling the reference's original functions
    (objcopy aliases) equals the reference encoder;
  * X265AMD_LOOKAHEAD=host — the hook's restated control flow (cost cache, bDoSearch, weightp,
    coop-slice geometry, B bias, intra penalty) with the reference's per-CU loops equals the
    reference encoder, 416x240 (no lookahead slices) and 1080p (6 coop slices);
  * without a device the encode fails loudly (exit 4, x265_encoder_encode < 0).
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


def _bin(name):
    p = os.path.join(REFBIN, name)
    if not os.path.exists(p):
        if os.path.isdir("/root/reference/x265_1.9/source"):
            from src.x265_amd import build as b

            b.build(verbose=False)
            subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "ref", "bridge"], check=True,
                           capture_output=True)
        else:
            pytest.skip(f"{name} not built (oracle/Makefile bridge needs /root/reference)")
    return p


def _source(tmp_path, w, h, frames, depth=8, fade=0.0):
    from src.x265_amd.synth import SyntheticSource

    path = tmp_path / f"src_{w}x{h}_{frames}_{depth}_{fade}.yuv"
    if not path.exists():
        SyntheticSource(w, h, frames, depth, fade=fade).write_yuv(str(path))
    return path


def encode(exe, src, w, h, frames, out, env_extra=None, pools=8, depth=8, extra=(), timeout=900, preset="medium"):
    """run a reference-CLI build; returns (returncode, md5 of the bitstream or None, fps or None, stderr)"""
    env = dict(os.environ, **(env_extra or {}))
    cmd = [exe, "--input", str(src), "--input-res", f"{w}x{h}", "--input-depth", str(depth), "--fps", "30",
           "--frames", str(frames), "--preset", preset, "-F", "2", "--pools", str(pools), "--no-info", "-o",
           str(out), *extra]
    if depth > 8:
        cmd += ["--output-depth", str(depth)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
    # the device sessions must unregister the encoder's page-locked planes while they are still allocated
    # (oracle/hip_encoder_main.cpp closing(); src/x265_amd/csrc/hostreg.h): the binding reports any that
    # were already freed
    assert "page-locked host buffers were freed" not in r.stderr, r.stderr[-1500:]
    m = re.search(r"encoded (\d+) frames in ([\d.]+)s \(([\d.]+) fps\)", r.stderr)
    md5 = hashlib.md5(open(out, "rb").read()).hexdigest() if r.returncode == 0 and os.path.exists(out) else None
    return r.returncode, md5, (float(m.group(3)) if m else None), r.stderr


@pytest.mark.parametrize("size,frames", [((416, 240), 16), ((1920, 1080), 6)], ids=["240p", "1080p-coop-slices"])
@pytest.mark.parametrize("mode", ["cpu", "host"])
def test_hooked_encoder_equals_reference_on_cpu(tmp_path, size, frames, mode):
    w, h = size
    src = _source(tmp_path, w, h, frames)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, frames, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, frames, tmp_path / "la.hevc", {"X265AMD_LOOKAHEAD": mode})
    assert rc == 0, err[-2000:]
    assert f"[x265la] lookahead estimates on the CPU" in err
    assert got == ref, f"X265AMD_LOOKAHEAD={mode}: bitstream differs from the reference encoder"


def test_hooked_encoder_weighted_fade_equals_reference_on_cpu(tmp_path):
    """a luma fade: weightsAnalyse picks weights, so the hook's weighted paths run (the weighted P
    estimate on the thread's wbuffer, weighted B estimates on the host loop) — host control flow"""
    w, h, n = 640, 360, 24
    src = _source(tmp_path, w, h, n, fade=0.03)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    assert re.search(r"Weighted P-Frames: Y:[1-9]", err), "the fade clip must trigger weighted prediction"
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "la.hevc", {"X265AMD_LOOKAHEAD": "host"})
    assert rc == 0, err[-2000:]
    assert got == ref


def test_lookahead_encoder_fails_loudly_without_device(tmp_path):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is present")
    src = _source(tmp_path, 416, 240, 8)
    rc, _, _, err = encode(_bin("x265la8"), src, 416, 240, 8, tmp_path / "g.hevc")
    assert rc == 4, (rc, err[-2000:])
    assert "x265amd_la_create failed" in err


@pytest.mark.gpu
def test_gpu_lookahead_encode_1080p_medium_is_bit_exact(tmp_path):
    """BASELINE config 0's workload (64 synthetic 1080p frames, --preset medium, -F 2): the encode with
    the lookahead on the MI355X equals the reference encoder bit for bit"""
    w, h, n = 1920, 1080, 64
    src = _source(tmp_path, w, h, n)
    rc, ref, ref_fps, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc", pools=16)
    assert rc == 0, err[-2000:]
    rc, got, la_fps, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "la.hevc", pools=16)
    assert rc == 0, err[-3000:]
    assert "[x265la] lookahead estimates on the MI355X" in err
    print(f"\n[x265la] 1080p medium {n} frames, --pools 16: reference {ref_fps} fps, MI355X lookahead {la_fps} fps")
    assert got == ref, "bitstream with the MI355X lookahead differs from the reference encoder"


@pytest.mark.gpu
def test_gpu_lookahead_weighted_fade_is_bit_exact(tmp_path):
    """the weighted paths on the device — a luma fade makes weightsAnalyse choose weights, so
    P estimates run on the thread's weighted planes (x265amd_la_pcost with weighted_buffer) and weighted
    B estimates take the host loop; the encode equals the reference and the stats show both happened"""
    w, h, n = 640, 360, 24
    src = _source(tmp_path, w, h, n, fade=0.03)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "la.hevc", {"X265AMD_LA_STATS": "1"})
    assert rc == 0, err[-3000:]
    assert re.search(r"Weighted P-Frames: Y:[1-9]", err)
    m = re.search(r"stats P weighted\s+calls\s+(\d+)", err)
    assert m and int(m.group(1)) > 0, err[-3000:]
    assert got == ref, "weighted estimates on the device changed the bitstream"


@pytest.mark.gpu
def test_gpu_lookahead_encode_main10_is_bit_exact(tmp_path):
    """Main10 (HIGH_BIT_DEPTH build): the device lookahead equals the same binary's reference functions"""
    w, h, n = 1920, 1080, 12
    src = _source(tmp_path, w, h, n, depth=10)
    exe = _bin("x265la10")
    rc, ref, _, err = encode(exe, src, w, h, n, tmp_path / "ref.hevc", {"X265AMD_LOOKAHEAD": "cpu"}, depth=10)
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(exe, src, w, h, n, tmp_path / "la.hevc", depth=10)
    assert rc == 0, err[-3000:]
    assert got == ref
