"""bench.py's host-side helpers (no GPU): the parsing of the encoder hook's counters into the roofline of
the batched motion-search launch, the per-rank clip (a closed segment of the synthetic sequence) and the
per-rank host-core slices."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ERR = """[x265me] stats prefetches 123004 searches 496472 memo hits 489487 misses 0 host fallbacks 0 weighted-reference searches 0 posted 124740 dropped 1736
[x265me] worker time on the device path: forming 0.200 s, reference uploads 0.693 s, posting 0.308 s, waiting for the device 12.062 s (123004 waits)
[x265me] service: 55870 launches, 124740 requests (2.23 per launch, max 14), 502994 searches, kernel 0.093 ms per launch (HIP events), batch 0.131 ms, queueing 0.058 ms per request, 51098 waits slept; 653 row uploads 263.7 MB 115.3 ms; sessions 1; evaluations 7572921 full-pel 5042178 sub-pel, 108.108 GB algorithmic, longest launch 3.460 ms
"""


def test_parse_me_stats_and_roofline():
    st = bench.parse_me_stats(ERR)
    assert st["launches"] == 55870 and st["searches"] == 502994 and st["memo_misses"] == 0
    assert st["wait_s"] == 12.062 and st["evals_subpel"] == 5042178 and st["algo_GB"] == 108.108
    r = bench.me_roofline(st, traffic_file=None)
    per = 108.108e9 / 55870
    assert r["bytes_per_launch"] == int(per)
    assert abs(r["achieved"] - per / 0.093e-3 / 1e9) < 0.01
    assert abs(r["frac"] - r["achieved"] / bench.HBM_PEAK_GBS) < 1e-4
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"


def test_roofline_traffic_from_the_committed_pmc_table(tmp_path):
    import json

    t = tmp_path / "t.json"
    t.write_text(json.dumps({"traffic_bytes_per_launch": 600000, "fetch_correction": 2.0}))
    r = bench.me_roofline(bench.parse_me_stats(ERR), traffic_file=str(t))
    assert r["traffic"] == 600000 and "FETCH_SIZE" in r["basis"]


def test_roofline_absent_without_service_counters():
    assert bench.me_roofline(bench.parse_me_stats("encoded 64 frames")) is None


def test_rank_clip_is_a_segment_of_the_sequence(tmp_path):
    from src.x265_amd.synth import SyntheticSource

    w, h, n = 64, 32, 3
    p = tmp_path / "c.yuv"
    bench.write_clip(str(p), w, h, 8, n, n)          # rank 1's segment: frames 3..5
    data = np.fromfile(p, np.uint8)
    fs = w * h * 3 // 2
    src = SyntheticSource(w, h, 2 * n, 8)
    for i in range(n):
        y, u, v = src.frame(n + i)
        assert np.array_equal(data[i * fs:i * fs + w * h], y.reshape(-1))


def test_core_slices_are_disjoint_when_the_node_has_enough():
    cpus = sorted(os.sched_getaffinity(0))
    s0, s1 = bench.core_slice(0, 2), bench.core_slice(1, 2)
    if len(cpus) >= 2 * bench.CORES_PER_GPU:
        assert not set(s0) & set(s1) and len(s0) == bench.CORES_PER_GPU
    elif len(cpus) >= 2:
        # fewer cores than 16 per rank: an equal disjoint share each
        assert not set(s0) & set(s1) and len(s0) == len(s1) == len(cpus) // 2
    assert s0 and set(s0) <= set(cpus)


def test_core_slices_share_a_small_node_evenly(monkeypatch):
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda _: set(range(96)))
    slices = [bench.core_slice(r, 8) for r in range(8)]
    assert all(len(s) == 12 for s in slices)
    assert len(set().union(*map(set, slices))) == 96
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda _: set(range(256)))
    assert [len(bench.core_slice(r, 8)) for r in range(8)] == [16] * 8
