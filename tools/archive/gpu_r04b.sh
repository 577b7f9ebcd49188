# round 4, second box call: new GPU tests (session lifetime, native exchange, weighted lookahead,
# the encoder's motion searches on the device at 1080p / 2160p / Main10 / check mode), the 2160p
# DETAILED_CU_STATS breakdowns, and a bench line with all encoder arms
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_la_session.py tests/test_gpu_pipeline.py::test_gpu_native_exchange_loopback \
    tests/test_encoder_lookahead.py::test_gpu_lookahead_weighted_fade_is_bit_exact tests/test_encoder_me.py -m gpu -x -v -s \
    --timeout 300 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 || { tail -60 gpurun_out/r04b_tests.log; exit 1; }
grep -E "x265me\]|PASS|passed|failed" gpurun_out/r04b_tests.log | tail -20
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for run in "x265la8s X265AMD_ME=cpu" "x265la8s X265AMD_ME=gpu" "x265ref8s X265AMD_ME=cpu"; do
  set -- $run
  env $2 X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/$1 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
      --preset medium --pools 16 --no-info -o /tmp/o.hevc > gpurun_out/r04b_cu_stats_$1_$2.txt 2>&1 || { tail gpurun_out/r04b_cu_stats_$1_$2.txt; exit 1; }
  echo "== $run"; grep -E "encoded|CU:|x265me\] stats" gpurun_out/r04b_cu_stats_$1_$2.txt
done
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || { tail -30 gpurun_out/r04b_bench.err; exit 1; }
head -c 1500 gpurun_out/r04b_bench.json
