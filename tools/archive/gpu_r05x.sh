# round 5: reference-row uploads three ways on the pinned 2160p medium 64-frame encode, 3 rounds interleaved:
# the workers' synchronous copies (tree), the workers' own streams (X265AMD_MES_WSTREAM=1), and the two
# launchers copying the rows ahead of their batches (X265AMD_MES_LUPLOAD=1); then check mode in the last
set -o pipefail
mkdir -p gpurun_out/r05/x
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
OUT=gpurun_out/r05/x/upload_modes_ab.txt
for rep in 1 2 3; do
  for v in tree wstream lupload; do
    case $v in
      tree) ENV="X265AMD_MES_LUPLOAD=0";;
      wstream) ENV="X265AMD_MES_WSTREAM=1";;
      lupload) ENV="X265AMD_MES_LUPLOAD=1";;
    esac
    env $ENV X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a $OUT
    grep -E "worker time|service:|waits by" /tmp/e.txt >> $OUT
  done
done
X265AMD_MES_LUPLOAD=1 timeout -k 10 600 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -q \
    --timeout 400 --timeout-method thread > gpurun_out/r05/x/encoder_me_lupload.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/x/encoder_me_lupload.log | head; tail -30 gpurun_out/r05/x/encoder_me_lupload.log; exit 1; }
echo "encoder_me (launcher uploads): $(tail -n 1 gpurun_out/r05/x/encoder_me_lupload.log)"
