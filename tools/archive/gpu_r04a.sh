# round 4, first box call: the new GPU tests, the 2160p DETAILED_CU_STATS breakdown of the encoder
# with the device lookahead (and the reference beside it, same box), and a bench line in pipeline mode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_la_session.py tests/test_gpu_pipeline.py::test_gpu_native_exchange_loopback \
    tests/test_encoder_lookahead.py::test_gpu_lookahead_weighted_fade_is_bit_exact -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -40 gpurun_out/r04a_tests.log; exit 1; }
tail -5 gpurun_out/r04a_tests.log
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for exe in x265la8s x265ref8s; do
  timeout -k 10 200 oracle/_ref/$exe --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 --preset medium \
      --pools 16 --no-info -o /tmp/o.hevc > gpurun_out/r04a_cu_stats_$exe.txt 2>&1 || { tail gpurun_out/r04a_cu_stats_$exe.txt; exit 1; }
  grep -E "encoded|CU:" gpurun_out/r04a_cu_stats_$exe.txt
done
X265AMD_BENCH_ARMS=mi355x_lookahead timeout -k 10 500 python3 -u bench.py --encoder-reps 3 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -30 gpurun_out/r04a_bench.err; exit 1; }
cat gpurun_out/r04a_bench.json | head -c 3000
