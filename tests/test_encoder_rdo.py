"""Round 6: the inter residual coding of the running reference encoder on the device (integration/gpu_rdo.cpp over
the x265amd_rdo_* session, csrc/rdosession.cpp).

Search::encodeResAndCalcRdInterCU (search.cpp:2562) posts an eligible CU's source and prediction; the device runs
the fused TU chain of every TU (csrc/tu.hip) and the per-8x8 psy energies (csrc/pixel.hip); the reference's own
estimateResidualQT then runs with its Quant::transformNxN / invtransformNxN calls and the table's psy_cost_pp
answered from those results wherever the call's inputs are the device's.

CPU: X265AMD_RDO=host computes the same results with the reference's own functions and serves them through the
same memo — every call must hit and the bitstream must be the reference's (checks the binding's plumbing).
GPU: the bitstream equals the reference's, and in check mode every device answer equals the reference function's.
"""
import os
import re

import pytest

from test_encoder_lookahead import _bin, _source, encode


def _rdo_stats(err):
    m = re.search(r"\[x265rdo\] stats CUs posted (\d+) coded on the host (\d+); transformNxN memo hits (\d+) misses "
                  r"(\d+); invtransformNxN hits (\d+) misses (\d+); psy_cost_pp hits (\d+) misses (\d+)", err)
    assert m, err[-3000:]
    k = ("posts", "host", "tq_hit", "tq_miss", "itq_hit", "itq_miss", "psy_hit", "psy_miss")
    return dict(zip(k, map(int, m.groups())))


@pytest.mark.parametrize("min_log2", [6, 4])
def test_rdo_hook_host_memo_equals_reference_on_cpu(tmp_path, min_log2):
    w, h, n = 640, 360, 8
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "rdo.hevc",
                             {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "cpu", "X265AMD_RDO": "host",
                              "X265AMD_RDO_MIN": str(min_log2), "X265AMD_ME_STATS": "1"})
    assert rc == 0, err[-2000:]
    st = _rdo_stats(err)
    assert st["posts"] > 0 and st["tq_hit"] > 0 and st["itq_hit"] > 0 and st["psy_hit"] > 0, st
    assert st["tq_miss"] == st["itq_miss"] == st["psy_miss"] == 0, st
    assert got == ref, "X265AMD_RDO=host: bitstream differs from the reference encoder"


@pytest.mark.parametrize("size", [(640, 360), (456, 264)], ids=["360p", "456x264"])
def test_sao_hook_host_memo_equals_reference_on_cpu(tmp_path, size):
    """X265AMD_RDO_SAO=host: SAO::calcSaoStatsCu's hook computes each CTU's three planes at its first call (here by
    the reference's own function on zeroed statistics) and adds one plane's part per call, as the device path
    does — every CTU is served by the memo and the bitstream is the reference's; a picture whose size is no CTU
    multiple (456x264: partial right and bottom CTUs) included"""
    w, h = size
    n = 8
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc")
    assert rc == 0, err[-2000:]
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "sao.hevc",
                             {"X265AMD_LOOKAHEAD": "cpu", "X265AMD_ME": "cpu", "X265AMD_RDO_SAO": "host",
                              "X265AMD_ME_STATS": "1"})
    assert rc == 0, err[-2000:]
    m = re.search(r"\[x265rdo\] SAO statistics: (\d+) CTUs on the hook memo .*, (\d+) on the host", err)
    ctus = ((w + 63) // 64) * ((h + 63) // 64) * n
    assert m and int(m.group(1)) == ctus and int(m.group(2)) == 0, err[-2000:]
    assert got == ref, "X265AMD_RDO_SAO=host: bitstream differs from the reference encoder"


def _gpu(tmp_path, w, h, n, env, min_log2=6):
    src = _source(tmp_path, w, h, n)
    rc, ref, _, err = encode(_bin("x265ref8"), src, w, h, n, tmp_path / "ref.hevc", pools=16)
    assert rc == 0, err[-2000:]
    e = {"X265AMD_RDO_MIN": str(min_log2), "X265AMD_ME_STATS": "1"}
    e.update(env)
    rc, got, _, err = encode(_bin("x265la8"), src, w, h, n, tmp_path / "rdo.hevc", e, pools=16)
    assert rc == 0, err[-3000:]
    assert got == ref, "device residual coding: bitstream differs from the reference encoder\n" + err[-2000:]
    return err


@pytest.mark.gpu
@pytest.mark.parametrize("min_log2", [6, 4])
def test_gpu_rdo_encode_1080p_is_bit_exact(tmp_path, min_log2):
    """device lookahead, device motion searches and device inter residual coding together, 1080p medium"""
    err = _gpu(tmp_path, 1920, 1080, 16, {"X265AMD_RDO": "gpu"}, min_log2)
    st = _rdo_stats(err)
    assert st["posts"] > 0 and st["tq_hit"] > 0 and st["tq_miss"] == 0 and st["itq_miss"] == 0, st
    assert st["psy_miss"] == 0, st


@pytest.mark.gpu
def test_gpu_rdo_check_mode_every_answer_matches(tmp_path):
    """X265AMD_RDO=check: every coefficient block, numSig, inverse-transformed residual and psy energy the
    device supplied is recomputed by the reference's function when it is used: 0 mismatches"""
    err = _gpu(tmp_path, 1280, 720, 12, {"X265AMD_RDO": "check"}, 4)
    m = re.search(r"\[x265rdo\] check: (\d+) mismatches", err)
    assert m and int(m.group(1)) == 0, err[-3000:]
    assert _rdo_stats(err)["tq_hit"] > 0


def _early_stats(err):
    m = re.search(r"\[x265rdo\] early posts merge (\d+) inter (\d+) bidir (\d+); used (\d+), dropped (\d+)", err)
    assert m, err[-3000:]
    return dict(zip(("merge", "inter", "bidir", "used", "dropped"), map(int, m.groups())))


FORMS = {"service": {}, "direct": {"X265AMD_RDO_LAUNCHERS": "0"},
         "server": {"X265AMD_RDO_LAUNCHERS": "0", "X265AMD_RDO_SERVER": "1"}}


@pytest.mark.gpu
@pytest.mark.parametrize("form", list(FORMS))
@pytest.mark.parametrize("mode", ["gpu", "check"])
def test_gpu_rdo_early_posts_bit_exact(tmp_path, mode, form):
    """X265AMD_RDO_EARLY=1: each CU's request is posted when its prediction becomes final (2Nx2N search, bidir,
    best merge candidate) and taken by the encodeResAndCalcRdInterCU whose inputs it matches; the bitstream is the
    reference's, every kind of post is made and used, and in check mode every device answer matches.  Forms: the
    launch service, direct launches by the worker, and the resident server kernel (X265AMD_RDO_SERVER: no launch
    per CU; tu.hip k_rdo_server polls the slots)"""
    env = {"X265AMD_RDO": mode, "X265AMD_RDO_EARLY": "1", **FORMS[form]}
    err = _gpu(tmp_path, 1280, 720, 12, env, 5)
    st, es = _rdo_stats(err), _early_stats(err)
    assert es["merge"] > 0 and es["inter"] > 0 and es["bidir"] > 0 and es["used"] > 0, es
    assert st["posts"] == es["used"] and st["tq_hit"] > 0 and st["tq_miss"] == 0, (st, es)
    if mode == "check":
        m = re.search(r"\[x265rdo\] check: (\d+) mismatches", err)
        assert m and int(m.group(1)) == 0, err[-3000:]
    # the server form also computes every CTU's SAO statistics (SAO::calcSaoStatsCu; in check mode each plane's
    # statistics are recomputed by the reference and compared: the mismatch count above includes them)
    m = re.search(r"\[x265rdo\] SAO statistics: (\d+) CTUs on the device .*, (\d+) on the host", err)
    if form == "server":
        assert m and int(m.group(1)) > 0 and int(m.group(2)) == 0, err[-3000:]
    else:
        assert m is None, err[-3000:]
    # the server also returns every 8x8 block's sse_pp against the prediction and the reconstruction: the CU's
    # distortions (search.cpp:2591-2595, 2668-2679) are served from them (compared in check mode)
    m = re.search(r"\[x265rdo\] sse_pp memo hits (\d+) misses (\d+)", err)
    assert m, err[-3000:]
    if form == "server":
        assert int(m.group(1)) > 0 and int(m.group(2)) == 0, err[-3000:]
