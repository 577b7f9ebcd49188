# round 5: cuTree's propagation on the device (X265AMD_LA_PROPAGATE=1) in the 2160p medium encode:
# bitstream identity and fps against the host propagation, interleaved, 3 reps
set -o pipefail
mkdir -p gpurun_out/r05/l
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
for rep in 1 2 3; do
  for pr in 0 1; do
    X265AMD_LA_PROPAGATE=$pr X265AMD_LA_STATS=1 timeout -k 10 150 oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 \
        || { tail -5 /tmp/e.txt; exit 1; }
    echo "propagate=$pr rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/l/propagate_ab.txt
    grep -E "^\[x265la\]" /tmp/e.txt | tail -4 | tee -a gpurun_out/r05/l/propagate_ab.txt
  done
done
