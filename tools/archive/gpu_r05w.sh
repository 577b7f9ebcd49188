# round 5: reference uploads done by a single launcher on its own stream (X265AMD_MES_LUPLOAD=1) against the
# workers' synchronous uploads with 2 and 1 launchers; the pinned 2160p medium 64-frame encode, 3 rounds
# interleaved, md5 of every stream, plus the check-mode encoder test in the new mode
set -o pipefail
mkdir -p gpurun_out/r05/w
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
OUT=gpurun_out/r05/w/lupload_ab.txt
for rep in 1 2 3; do
  for v in tree l1 l1up; do
    case $v in
      tree) ENV="";;
      l1) ENV="X265AMD_MES_LAUNCHERS=1";;
      l1up) ENV="X265AMD_MES_LAUNCHERS=1 X265AMD_MES_LUPLOAD=1";;
    esac
    env $ENV X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a $OUT
    grep -E "worker time|service:" /tmp/e.txt >> $OUT
  done
done
X265AMD_MES_LAUNCHERS=1 X265AMD_MES_LUPLOAD=1 timeout -k 10 600 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -q \
    --timeout 400 --timeout-method thread > gpurun_out/r05/w/encoder_me_lupload.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/w/encoder_me_lupload.log | head; tail -30 gpurun_out/r05/w/encoder_me_lupload.log; exit 1; }
echo "encoder_me (launcher uploads): $(tail -n 1 gpurun_out/r05/w/encoder_me_lupload.log)"
# sad_x4 lane-per-reference variants (X265AMD_SADX_LANES bits: 1 lane per reference, 2 8x8 units, 4 non-temporal)
for rep in 1 2; do
  for v in 0 1 3 5 7; do
    X265AMD_SADX_LANES=$v timeout -k 10 200 python3 -u tools/kernel_roofline.py --only sad_x4 2>/dev/null | grep "{" \
      | sed "s/^/lanes=$v rep=$rep /" | cut -c1-200 | tee -a gpurun_out/r05/w/sadx_lanes_ab.txt || exit 1
  done
done
