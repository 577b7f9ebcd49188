# round 5: the launch service's waiting on the encoder's 16-core budget (pinned like bench.py): the new
# default (pause-spin, then a yield loop, sleep last; notifies only to sleepers) against the previous
# behaviour (X265AMD_MES_YIELD_US=0 X265AMD_MES_IDLE_US=0: sleep after the spin), interleaved, 3 reps;
# then the search-method check tests (the service changed)
set -o pipefail
mkdir -p gpurun_out/r05/p
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
for rep in 1 2 3; do
  for v in "default" "X265AMD_MES_YIELD_US=0 X265AMD_MES_IDLE_US=0"; do
    ENVV=""
    [ "$v" != default ] && ENVV="$v"
    env $ENVV X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 \
        || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/p/yield_pinned_ab.txt
    grep -E "worker time|service:|waits by|batches by" /tmp/e.txt | tee -a gpurun_out/r05/p/yield_pinned_ab.txt
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -v --timeout 400 --timeout-method thread \
    -k "search_methods or slow_check or check_mode_every or two_encoders or two_device" > gpurun_out/r05/p/methods.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/p/methods.log | head; tail -30 gpurun_out/r05/p/methods.log; exit 1; }
echo "encoder tests: $(tail -n 1 gpurun_out/r05/p/methods.log)"
