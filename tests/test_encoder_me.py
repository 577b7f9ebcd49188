"""f2 in the RUNNING encoder: the reference x265 1.9 encoder with the motion searches of its large
PUs on the MI355X (integration/gpu_me.cpp over the x265amd_mes_* session entries).

oracle/Makefile links the reference CLI + encoder (x265la8 / x265la10) with
Search::predInterSearch (search.cpp:2050) and MotionEstimate::motionEstimate (motion.cpp:571)
hooked: the hook forms every search the reference loop is about to make for a 64x64 PU (X265AMD_ME_MIN),
runs them in one device launch, and hands each result to the reference's own predInterSearch
when it makes that exact call.  Every mode decision, RDO cost and bitstream bit downstream
depends on those searches, so the encode must be BIT-IDENTICAL to the plain reference encoder.

CPU tests pin the binding itself (X265AMD_ME=host: the hook's restated search setup with the
reference's motionEstimate, no device): equal bitstream, every prefetched call found in the memo.
GPU tests: 1080p and 2160p --preset medium, 64 frames, device lookahead + device searches, equal to
the reference encoder; X265AMD_ME=check compares every device search used with the host search.
"""
import os
import re

import pytest

from test_encoder_lookahead import _bin, _source, encode


def _stats(err):
    m = re.search(r"\[x265me\] stats prefetches (\d+) searches (\d+) memo hits (\d+) misses (\d+) host fallbacks (\d+) "
                  r"weighted-reference searches (\d+)", err)
    assert m, err[-3000:]
    return dict(zip(("prefetches", "searches", "hits", "misses", "fallbacks", "weighted"), map(int, m.groups())))


@pytest.mark.parametrize("size,frames,fade", [((640, 360), 16, 0.0), ((1920, 1080), 6, 0.0), ((640, 360), 24, 0.03)],
                         ids=["360p", "1080p", "360p-weighted-fade"])
def test_me_hook_host_prefetch_equals_reference_on_cpu(tmp_path, size, frames, fade):
    w, h = size
    src = _source(tmp_path, w, h, frames, fade=fade)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, frames, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, frames, tmp_path / "me.hevc",
                             {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "host", "X265AMD_ME_STATS": "1"})
    assert rc == 0, err[-2000:]
    assert "[x265me] motion searches of PUs >= 4096 pixels on the CPU (hook prefetch)" in err
    st = _stats(err)
    assert st["prefetches"] > 0 and st["hits"] > 0
    # every search the reference made after a prefetch was one of the prefetched ones, except those on
    # weighted references, which stay on the host
    assert st["misses"] == 0, st
    assert (st["weighted"] > 0) == (fade > 0), st
    assert got == ref, "X265AMD_ME=host: bitstream differs from the reference encoder"


def test_me_hook_cpu_mode_is_the_reference(tmp_path):
    w, h, n = 640, 360, 8
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "me.hevc", {"X265AMD_LOOKAHEAD": "cpu"})
    assert rc == 0, err[-2000:]
    assert "(reference functions)" in err and got == ref


def _gpu_encode_equals_reference(tmp_path, w, h, n, extra_env=None, depth=8):
    src = _source(tmp_path, w, h, n, depth=depth)
    if depth == 8:
        rc, ref, ref_fps, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc", pools=16)
        exe = _bin("x265la8")
    else:
        exe = _bin("x265la10")
        rc, ref, ref_fps, err = encode(exe, src, w, h, n, tmp_path / "ref.hevc",
                                       {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "cpu"}, pools=16, depth=10)
    assert rc == 0, err[-2000:]
    env = {"X265AMD_ME_STATS": "1", **(extra_env or {})}
    rc, got, fps, err = encode(exe, src, w, h, n, tmp_path / "me.hevc", env, pools=16, depth=depth)
    assert rc == 0, err[-3000:]
    assert "[x265me] motion searches of PUs >= 4096 pixels on the MI355X" in err
    st = _stats(err)
    print(f"\n[x265me] {w}x{h} {n} frames: reference {ref_fps} fps, MI355X lookahead + ME {fps} fps; {st}")
    assert st["prefetches"] > 0 and st["hits"] > 0 and st["misses"] == 0, st
    assert got == ref, "bitstream with the MI355X motion searches differs from the reference encoder"
    return err


@pytest.mark.gpu
def test_gpu_me_encode_1080p_medium_is_bit_exact(tmp_path):
    _gpu_encode_equals_reference(tmp_path, 1920, 1080, 64)


@pytest.mark.gpu
def test_gpu_me_encode_2160p_medium_is_bit_exact(tmp_path):
    """BASELINE's 4K configuration (3840x2160 8-bit --preset medium, 64 frames): device lookahead and
    device motion searches, bitstream identical to the reference encoder"""
    _gpu_encode_equals_reference(tmp_path, 3840, 2160, 64)


@pytest.mark.gpu
def test_gpu_me_check_mode_every_search_matches(tmp_path):
    """X265AMD_ME=check: every device search the encoder uses is recomputed on the host and compared"""
    err = _gpu_encode_equals_reference(tmp_path, 1280, 720, 12, {"X265AMD_ME": "check"})
    m = re.search(r"check: (\d+) mismatching searches", err)
    assert m and int(m.group(1)) == 0, err[-3000:]


@pytest.mark.gpu
def test_gpu_me_encode_main10_is_bit_exact(tmp_path):
    """Main10: the 16-bit search kernel behind the same hook, against the same binary's reference functions"""
    _gpu_encode_equals_reference(tmp_path, 1920, 1080, 12, depth=10)
