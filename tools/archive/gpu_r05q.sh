# round 5: asynchronous reference-row uploads (ordered by per-picture events on the launch streams)
# against uploads waited for by the worker (X265AMD_MES_SYNC_UPLOAD=1), pinned to the bench's 16 cores,
# interleaved, 3 reps; process start-up cost (2-frame encodes, hooked vs reference); then the encoder
# check-mode / multi-session / two-encoder GPU tests
set -o pipefail
mkdir -p gpurun_out/r05/q
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --preset medium"
for rep in 1 2 3; do
  for v in "default" "X265AMD_MES_SYNC_UPLOAD=1"; do
    ENVV=""
    [ "$v" != default ] && ENVV="$v"
    env $ENVV X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K --frames 64 -o /tmp/o.hevc > /tmp/e.txt 2>&1 \
        || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/q/upload_pinned_ab.txt
    grep -E "worker time|service:|waits by|batches by" /tmp/e.txt | tee -a gpurun_out/r05/q/upload_pinned_ab.txt
  done
done
for exe in x265ref8 x265la8; do
  S=$(date +%s.%N)
  timeout -k 10 100 taskset -c $CORES oracle/_ref/$exe $E4K --frames 2 -o /tmp/t.hevc > /tmp/t.txt 2>&1 || { tail -5 /tmp/t.txt; exit 1; }
  E=$(date +%s.%N)
  echo "$exe 2 frames: wall $(python3 -c "print(round($E - $S, 3))") s; $(grep encoded /tmp/t.txt)" | tee -a gpurun_out/r05/q/startup.txt
done
timeout -k 10 900 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -v --timeout 400 --timeout-method thread \
    -k "search_methods or slow_check or check_mode_every or two_encoders or two_device or service_prefetch" > gpurun_out/r05/q/encoder_tests.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/q/encoder_tests.log | head; tail -30 gpurun_out/r05/q/encoder_tests.log; exit 1; }
echo "encoder tests: $(tail -n 1 gpurun_out/r05/q/encoder_tests.log)"
