# round 4, not run (GPU access for this session ended before it): the whole GPU suite on the tree, then
# the two opt-in paths built this round — coalesced device motion searches (X265AMD_MES_COALESCE=1) and
# cuTree's propagation on the device (X265AMD_LA_PROPAGATE=1) — under their check modes and in an
# interleaved 2160p encoder A/B against the defaults
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04l_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04l_gpu_tests.log; exit 1; }
echo "gpu suite: $(tail -1 gpurun_out/r04l_gpu_tests.log)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(1280, 720, 24, 8).write_yuv('/tmp/s720.yuv')
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
X265AMD_MES_COALESCE=1 X265AMD_ME=check X265AMD_LA_PROPAGATE=1 X265AMD_LOOKAHEAD=check X265AMD_LA_STATS=1 timeout -k 10 300 \
    oracle/_ref/x265la8 --input /tmp/s720.yuv --input-res 1280x720 --fps 30 --frames 24 --preset medium --no-info -o /tmp/c.hevc \
    > gpurun_out/r04l_check.log 2>&1 || { tail -20 gpurun_out/r04l_check.log; exit 1; }
grep -E "check:|stats propagate" gpurun_out/r04l_check.log
for rep in 1 2 3; do
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    X265AMD_MES_COALESCE=$1 X265AMD_LA_PROPAGATE=$2 X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 --input /tmp/s2160.yuv \
        --input-res 3840x2160 --fps 30 --frames 64 --preset medium --pools 16 --no-info -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "rep=$rep coalesce=$1 propagate=$2: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8) $(grep -o '[0-9.]* ms/prefetch' /tmp/e.txt)" | tee -a gpurun_out/r04l_encoder_ab.txt
  done
  timeout -k 10 200 oracle/_ref/x265ref8 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
      --preset medium --pools 16 --no-info -o /tmp/r.hevc > /tmp/e.txt 2>&1 || exit 1
  echo "rep=$rep reference: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/r.hevc | cut -c1-8)" | tee -a gpurun_out/r04l_encoder_ab.txt
done
