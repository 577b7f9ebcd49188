# round 5: with the faster search kernel, does the 32x32 prefetch (X265AMD_ME_MIN=1024) pay now?
# 2160p medium 64 frames, interleaved, 3 reps
set -o pipefail
mkdir -p gpurun_out/r05/k
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
for rep in 1 2 3; do
  for m in 4096 1024; do
    X265AMD_ME_MIN=$m X265AMD_ME_STATS=1 timeout -k 10 150 oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 \
        || { tail -5 /tmp/e.txt; exit 1; }
    echo "min=$m rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/k/min_ab.txt
    grep -E "worker time|service" /tmp/e.txt | tee -a gpurun_out/r05/k/min_ab.txt
  done
done
