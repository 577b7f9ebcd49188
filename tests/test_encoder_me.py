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


@pytest.mark.parametrize("size,frames,fade,min_area", [((640, 360), 16, 0.0, 4096), ((1920, 1080), 6, 0.0, 4096),
                                                       ((640, 360), 24, 0.03, 4096), ((640, 360), 16, 0.0, 1024),
                                                       ((1280, 720), 8, 0.0, 1024)],
                         ids=["360p", "1080p", "360p-weighted-fade", "360p-32x32", "720p-32x32"])
def test_me_hook_host_prefetch_equals_reference_on_cpu(tmp_path, size, frames, fade, min_area):
    """X265AMD_ME=host: the hook's CU-start prefetch (64x64 at depth 0, and with X265AMD_ME_MIN=1024 the
    32x32 CUs at depth 1 through the checkMerge2Nx2N_rd0_4 hook) formed exactly as the reference loop makes
    its calls — every reference call after a prefetch is found in the memo, and the bitstream is the
    reference's"""
    w, h = size
    src = _source(tmp_path, w, h, frames, fade=fade)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, frames, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, frames, tmp_path / "me.hevc",
                             {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "host", "X265AMD_ME_STATS": "1",
                              "X265AMD_ME_MIN": str(min_area)})
    assert rc == 0, err[-2000:]
    assert f"[x265me] motion searches of PUs >= {min_area} pixels on the CPU (hook prefetch), prefetched at CU start" in err
    st = _stats(err)
    assert st["prefetches"] > 0 and st["hits"] > 0
    # every search the reference made after a prefetch was one of the prefetched ones, except those on
    # weighted references, which stay on the host
    assert st["misses"] == 0, st
    assert (st["weighted"] > 0) == (fade > 0), st
    assert got == ref, "X265AMD_ME=host: bitstream differs from the reference encoder"


def test_me_hook_two_device_sessions_on_cpu(tmp_path):
    """X265AMD_GPUS=2 (host mode): frame encoder i's searches go to device session i mod 2 — both sessions get
    searches (frames alternate between the encoder's frame threads, encoder.cpp:649-650) and the bitstream
    is the reference's"""
    w, h, n = 640, 360, 16
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "me.hevc",
                             {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "host", "X265AMD_ME_STATS": "1",
                              "X265AMD_GPUS": "2"})
    assert rc == 0, err[-2000:]
    m = re.search(r"searches per device session: (\d+) (\d+)", err)
    assert m and int(m.group(1)) > 0 and int(m.group(2)) > 0, err[-2000:]
    assert _stats(err)["misses"] == 0
    assert got == ref


def _twice(tmp_path, src, w, h, n, env, tag):
    import subprocess

    outs = [tmp_path / f"{tag}1.hevc", tmp_path / f"{tag}2.hevc"]
    r = subprocess.run([_bin("x265twice8"), str(src), str(w), str(h), str(n), str(outs[0]), str(outs[1])],
                       capture_output=True, text=True, timeout=600, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "page-locked host buffers were freed" not in r.stderr, r.stderr[-1500:]
    return [o.read_bytes() for o in outs], r.stderr


def test_two_encoders_in_one_process_on_cpu(tmp_path):
    """two encoders of one geometry opened one after the other in one process (oracle/twice_main.cpp, the
    x265 API): with the hooks' host forms, both bitstreams equal the hooks-off program's"""
    w, h, n = 640, 360, 12
    src = _source(tmp_path, w, h, n)
    ref, _ = _twice(tmp_path, src, w, h, n, {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "cpu"}, "ref")
    assert ref[0] == ref[1]
    got, _ = _twice(tmp_path, src, w, h, n, {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "host"}, "host")
    assert got[0] == ref[0] and got[1] == ref[0]


@pytest.mark.gpu
def test_gpu_two_encoders_in_one_process_are_bit_exact(tmp_path):
    """the second encoder reuses freed PicYuv / Lowres addresses with the same POCs; the
    binding's teardown after x265_encoder_close (x265amd_me_encoder_closed / x265amd_la_encoder_closed)
    drops the first encoder's device sessions, so the second encode's device searches and estimates see
    only its own pictures — both bitstreams equal the hooks-off program's"""
    w, h, n = 640, 360, 16
    src = _source(tmp_path, w, h, n)
    ref, _ = _twice(tmp_path, src, w, h, n, {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "cpu"}, "ref")
    got, err = _twice(tmp_path, src, w, h, n, {"X265AMD_ME_STATS": "1"}, "gpu")
    assert "lookahead estimates on the MI355X" in err and "on the MI355X" in err
    assert got[0] == ref[0], "first encoder differs"
    assert got[1] == ref[0], "second encoder in the same process differs (stale device pictures?)"


def test_me_hook_cpu_mode_is_the_reference(tmp_path):
    w, h, n = 640, 360, 8
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "me.hevc", {"X265AMD_LOOKAHEAD": "cpu"})
    assert rc == 0, err[-2000:]
    assert "(reference functions)" in err and got == ref


def _gpu_encode_equals_reference(tmp_path, w, h, n, extra_env=None, depth=8, min_area=4096, preset="medium",
                                 extra=()):
    src = _source(tmp_path, w, h, n, depth=depth)
    if depth == 8:
        rc, ref, ref_fps, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc", pools=16, preset=preset,
                                       extra=extra)
        exe = _bin("x265la8")
    else:
        exe = _bin("x265la10")
        rc, ref, ref_fps, err = encode(exe, src, w, h, n, tmp_path / "ref.hevc",
                                       {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "cpu"}, pools=16, depth=10,
                                       preset=preset, extra=extra)
    assert rc == 0, err[-2000:]
    env = {"X265AMD_ME_STATS": "1", **(extra_env or {})}
    rc, got, fps, err = encode(exe, src, w, h, n, tmp_path / "me.hevc", env, pools=16, depth=depth, preset=preset,
                               extra=extra)
    assert rc == 0, err[-3000:]
    assert f"[x265me] motion searches of PUs >= {min_area} pixels on the MI355X" in err
    st = _stats(err)
    print(f"\n[x265me] {w}x{h} {n} frames: reference {ref_fps} fps, MI355X lookahead + ME {fps} fps; {st}")
    assert st["prefetches"] > 0 and st["hits"] > 0 and st["misses"] == 0, st
    assert got == ref, "bitstream with the MI355X motion searches differs from the reference encoder"
    return err


@pytest.mark.gpu
def test_gpu_me_encode_1080p_medium_is_bit_exact(tmp_path):
    _gpu_encode_equals_reference(tmp_path, 1920, 1080, 64)


@pytest.mark.gpu
def test_gpu_sessions_unregister_planes_before_the_encoder_frees_them(tmp_path):
    """ADVICE r5 / the round-5 GPU-fault audit: the device sessions page-lock the encoder's PicYuv and Lowres
    planes; the binding must drop the sessions (uploads drained, planes unregistered) BEFORE
    x265_encoder_close frees them.  The library counts every unregister of a range that is no longer mapped
    (x265amd_host_unregister_stale, csrc/hostreg.h) and the binding prints it.  Default order: none (encode()
    asserts it).  The round-5 order (sessions dropped after the close, X265AMD_ROUND5_CLOSE_ORDER=1): the
    1080p planes are munmapped by then and the count is positive — the check catches the old code."""
    import subprocess

    w, h, n = 1920, 1080, 8
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "me.hevc", {"X265AMD_ME_STATS": "1"})
    assert rc == 0 and got == ref, err[-2000:]
    cmd = [_bin("x265la8"), "--input", str(src), "--input-res", f"{w}x{h}", "--input-depth", "8", "--fps", "30",
           "--frames", str(n), "--preset", "medium", "-F", "2", "--pools", "8", "--no-info", "-o",
           str(tmp_path / "old.hevc")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, X265AMD_ROUND5_CLOSE_ORDER="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    m = re.search(r"(\d+) page-locked host buffers were freed before their session unregistered them", r.stderr)
    assert m and int(m.group(1)) > 0, r.stderr[-2000:]


@pytest.mark.gpu
def test_gpu_me_encode_2160p_medium_is_bit_exact(tmp_path):
    """BASELINE's 4K configuration (3840x2160 8-bit --preset medium, 64 frames): device lookahead and
    device motion searches, bitstream identical to the reference encoder"""
    _gpu_encode_equals_reference(tmp_path, 3840, 2160, 64)


@pytest.mark.gpu
@pytest.mark.parametrize("transfer", ["3", "0", "1"])
def test_gpu_me_check_mode_every_search_matches(tmp_path, transfer):
    """X265AMD_ME=check: every device search the encoder uses is recomputed on the host and compared — for each
    form of the launch service's transfer (X265AMD_MES_ZEROCOPY): 3 the default, inputs written by the host into
    device memory through the BAR and outputs written by the kernel into host memory; 0 staged copies both
    ways; 1 the kernel reads and writes host memory"""
    err = _gpu_encode_equals_reference(tmp_path, 1280, 720, 12, {"X265AMD_ME": "check", "X265AMD_MES_ZEROCOPY": transfer})
    m = re.search(r"check: (\d+) mismatching searches", err)
    assert m and int(m.group(1)) == 0, err[-3000:]


@pytest.mark.gpu
def test_gpu_me_service_prefetch_32x32_check_mode(tmp_path):
    """the launch service with the CU-start prefetch at depth 0 and 1 (64x64 and 32x32 CUs), every used
    device search recomputed on the host: 0 mismatches, the prefetches were posted and collected (memo
    hits), and the bitstream is the reference's"""
    err = _gpu_encode_equals_reference(tmp_path, 1280, 720, 12, {"X265AMD_ME": "check", "X265AMD_ME_MIN": "1024"},
                                       min_area=1024)
    m = re.search(r"check: (\d+) mismatching searches", err)
    assert m and int(m.group(1)) == 0, err[-3000:]
    m = re.search(r"service: (\d+) launches, (\d+) requests", err)
    assert m and int(m.group(1)) > 0 and int(m.group(2)) >= int(m.group(1)), err[-3000:]
    assert re.search(r"posted [1-9]", err), err[-3000:]


@pytest.mark.gpu
def test_gpu_me_two_device_sessions_is_bit_exact(tmp_path):
    """X265AMD_GPUS=2 on the one-GPU box: two device sessions (frame encoder i on session i mod 2, each with
    its own reference-row copies) on device 0 — the frame-level shard of config 4 inside one encoder"""
    err = _gpu_encode_equals_reference(tmp_path, 1280, 720, 16, {"X265AMD_GPUS": "2", "X265AMD_GPU_LIST": "0,0"})
    m = re.search(r"searches per device session: (\d+) (\d+)", err)
    assert m and int(m.group(1)) > 0 and int(m.group(2)) > 0, err[-3000:]
    assert re.search(r"sessions 2", err), err[-3000:]


@pytest.mark.gpu
def test_gpu_me_round4_per_thread_form_is_bit_exact(tmp_path):
    """X265AMD_MES_LAUNCHERS=0: the round-4 form (each worker launching on its own stream, synchronous)"""
    _gpu_encode_equals_reference(tmp_path, 1280, 720, 8, {"X265AMD_MES_LAUNCHERS": "0"})


@pytest.mark.gpu
def test_gpu_me_encode_2160p_slow_is_bit_exact(tmp_path):
    """BASELINE config 3 (3840x2160 8-bit --preset slow, 64 frames): STAR searches with subme 3, whose sub-pel
    refine adds the 4:2:0 chroma SATD (motion.cpp:1204-1230) — the chroma session (reference chroma planes
    resident, the PU's chroma blocks posted with its searches); bitstream identical to the reference"""
    err = _gpu_encode_equals_reference(tmp_path, 3840, 2160, 64, preset="slow")
    m = re.search(r"evaluations (\d+) full-pel (\d+) sub-pel", err)
    assert m and int(m.group(2)) > 0, err[-3000:]


@pytest.mark.gpu
def test_gpu_me_slow_check_mode_chroma_satd(tmp_path):
    """--preset slow with the 32x32 CUs too, every used device search (chroma SATD included) recomputed on
    the host: 0 mismatches"""
    err = _gpu_encode_equals_reference(tmp_path, 1280, 720, 12, {"X265AMD_ME": "check", "X265AMD_ME_MIN": "1024"},
                                       min_area=1024, preset="slow")
    m = re.search(r"check: (\d+) mismatching searches", err)
    assert m and int(m.group(1)) == 0, err[-3000:]
    m = re.search(r"check: (\d+) search windows beyond", err)
    assert m and int(m.group(1)) == 0, err[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("preset,extra", [("medium", ("--me", "star")), ("medium", ("--me", "umh")),
                                          ("medium", ("--me", "dia")), ("veryslow", ())],
                         ids=["star", "umh", "dia", "veryslow"])
def test_gpu_me_check_mode_search_methods(tmp_path, preset, extra):
    """every search method of x265_param::searchMethod through the session (x265.h numbers UMH 2 and STAR 3,
    the kernel STAR 2 and UMH 3: the session maps them) and veryslow's subme 4 / merange, in check mode with
    the 32x32 CUs: 0 mismatches, 0 windows beyond the resident rows, the reference's bitstream"""
    err = _gpu_encode_equals_reference(tmp_path, 1280, 720, 8, {"X265AMD_ME": "check", "X265AMD_ME_MIN": "1024"},
                                       min_area=1024, preset=preset, extra=extra)
    m = re.search(r"check: (\d+) mismatching searches", err)
    assert m and int(m.group(1)) == 0, err[-3000:]
    m = re.search(r"check: (\d+) search windows beyond", err)
    assert m and int(m.group(1)) == 0, err[-3000:]


@pytest.mark.gpu
def test_gpu_me_encode_2160p_main10_is_bit_exact(tmp_path):
    """BASELINE config 5 (3840x2160 Main10 --preset medium, 64 frames): the 16-bit lookahead and search
    kernels behind the same hooks, against the same binary's reference functions"""
    _gpu_encode_equals_reference(tmp_path, 3840, 2160, 64, depth=10)


@pytest.mark.gpu
def test_gpu_me_encode_main10_is_bit_exact(tmp_path):
    """Main10: the 16-bit search kernel behind the same hook, against the same binary's reference functions"""
    _gpu_encode_equals_reference(tmp_path, 1920, 1080, 12, depth=10)
