# round 5: motion searches of more than 64 4x4 units over 2 / 4 wavefronts of one workgroup
# (X265AMD_ME_GMAX=128 / 256): ME parity against the oracle at each setting, then the pinned 2160p medium
# encode 3 rounds interleaved (fps, kernel time per launch), then check mode at the faster setting
set -o pipefail
mkdir -p gpurun_out/r05/z
export TMPDIR=/tmp
for g in 256 128; do
  X265AMD_ME_GMAX=$g timeout -k 10 300 python3 -u -m pytest tests/test_me.py -m gpu -x -q --timeout 240 --timeout-method thread \
      > gpurun_out/r05/z/me_parity_g$g.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/r05/z/me_parity_g$g.log | head; tail -20 gpurun_out/r05/z/me_parity_g$g.log; exit 1; }
  echo "me parity gmax=$g: $(tail -n 1 gpurun_out/r05/z/me_parity_g$g.log)"
done
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
OUT=gpurun_out/r05/z/gmax_ab.txt
for rep in 1 2 3; do
  for g in 64 128 256; do
    X265AMD_ME_GMAX=$g X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "gmax=$g rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a $OUT
    grep -E "worker time|service:" /tmp/e.txt | tee -a $OUT | grep -o "kernel [0-9.]* ms per launch"
  done
done
X265AMD_ME_GMAX=256 timeout -k 10 600 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -q -k "check_mode" \
    --timeout 400 --timeout-method thread > gpurun_out/r05/z/encoder_check_g256.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/z/encoder_check_g256.log | head; tail -30 gpurun_out/r05/z/encoder_check_g256.log; exit 1; }
echo "check mode gmax=256: $(tail -n 1 gpurun_out/r05/z/encoder_check_g256.log)"
