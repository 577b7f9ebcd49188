# round 5: the launch service with the kernel reading its descriptors and source blocks from the pinned staging
# and writing its results there (X265AMD_MES_ZEROCOPY=1: no upload / download copies per batch) against the
# default and the outputs-only form (=2), pinned 2160p medium encode, 3 rounds interleaved
set -o pipefail
mkdir -p gpurun_out/r05/ah
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
OUT=gpurun_out/r05/ah/zerocopy_ab.txt
for rep in 1 2 3; do
  for v in 0 1 2; do
    X265AMD_MES_ZEROCOPY=$v X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "zerocopy=$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a $OUT
    grep -E "worker time|service:" /tmp/e.txt | tee -a $OUT | grep -oE "waiting for the device [0-9.]* s|kernel [0-9.]* ms per launch"
  done
done
