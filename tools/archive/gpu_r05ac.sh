# round 5: reference-row requests that need no upload answered without a HIP call (x265amd_mes_ref420 fast
# path) against the previous session, pinned 2160p medium 64-frame encode, 3 rounds interleaved; then the
# encoder's check-mode and 2160p bit-exact tests on the new session
set -o pipefail
mkdir -p gpurun_out/r05/ac
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
OUT=gpurun_out/r05/ac/ref420_fast_ab.txt
for rep in 1 2 3; do
  for v in tree r420old; do
    if [ $v = tree ]; then LP=""; else LP=$PWD/src/x265_amd/ab/r420old; fi
    LD_LIBRARY_PATH=$LP X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a $OUT
    grep -E "worker time|service:" /tmp/e.txt | tee -a $OUT | grep -o "reference uploads [0-9.]* s"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -q -k "check_mode or 2160p_medium" \
    --timeout 400 --timeout-method thread > gpurun_out/r05/ac/encoder_check.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/ac/encoder_check.log | head; tail -30 gpurun_out/r05/ac/encoder_check.log; exit 1; }
echo "encoder check: $(tail -n 1 gpurun_out/r05/ac/encoder_check.log)"
