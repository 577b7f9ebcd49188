# round 5: sub-pel refinement rounds costed four directions per call (8-bit, X265AMD_ME_SPB): ME parity, the
# encoder check modes, then the pinned 2160p medium encode 3 rounds interleaved against the one-per-call build
set -o pipefail
mkdir -p gpurun_out/r05/aa
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_me.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/r05/aa/me_parity.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/r05/aa/me_parity.log | head; tail -20 gpurun_out/r05/aa/me_parity.log; exit 1; }
echo "me parity: $(tail -n 1 gpurun_out/r05/aa/me_parity.log)"
timeout -k 10 600 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -q -k "check_mode or 2160p_medium" \
    --timeout 400 --timeout-method thread > gpurun_out/r05/aa/encoder_check.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/aa/encoder_check.log | head; tail -30 gpurun_out/r05/aa/encoder_check.log; exit 1; }
echo "encoder check: $(tail -n 1 gpurun_out/r05/aa/encoder_check.log)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
OUT=gpurun_out/r05/aa/spb_ab.txt
for rep in 1 2 3; do
  for v in tree spb0; do
    if [ $v = tree ]; then LP=""; else LP=$PWD/src/x265_amd/ab/spb0; fi
    LD_LIBRARY_PATH=$LP X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a $OUT
    grep -E "worker time|service:" /tmp/e.txt | tee -a $OUT | grep -o "kernel [0-9.]* ms per launch"
  done
done
