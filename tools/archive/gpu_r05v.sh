# round 5: the landed interpolation rewrite (round 4's a052ed0 without its inline-asm dot starts) and the
# workers' stream-free uploads: interp parity + guarded outputs, the interpolation roofline, the encoder
# tests, and the pinned 2160p encode (3 runs)
set -o pipefail
mkdir -p gpurun_out/r05/v
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/v/parity.log 2>&1 || { grep -E "FAILED|mismatches|assert" gpurun_out/r05/v/parity.log | head; tail -20 gpurun_out/r05/v/parity.log; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/r05/v/parity.log)"
timeout -k 10 200 python3 -u tools/interp_diff.py > gpurun_out/r05/v/interp_diff.txt 2>&1 || { tail -20 gpurun_out/r05/v/interp_diff.txt; exit 1; }
grep -c " 0 differing" gpurun_out/r05/v/interp_diff.txt
timeout -k 10 300 python3 -u tools/kernel_roofline.py --only luma_hpp,luma_vpp,luma_hvpp 2>/dev/null | grep "{" | cut -c1-160 \
    | tee gpurun_out/r05/v/interp_roofline.txt || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_encoder_me.py tests/test_encoder_lookahead.py -m gpu -x -q --timeout 400 --timeout-method thread \
    > gpurun_out/r05/v/encoder_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/v/encoder_tests.log | head; tail -30 gpurun_out/r05/v/encoder_tests.log; exit 1; }
echo "encoder tests: $(tail -n 1 gpurun_out/r05/v/encoder_tests.log)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
for rep in 1 2 3; do
  X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
  echo "rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/v/encode_pinned.txt
  grep -E "worker time|waits by" /tmp/e.txt | tee -a gpurun_out/r05/v/encode_pinned.txt
done
