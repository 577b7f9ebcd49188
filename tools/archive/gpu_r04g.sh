# round 4: interleaved 2160p encoder A/B of the device motion-search modes (CTU-start asynchronous
# submit vs synchronous per-CU batches, 64x64-only vs 32x32 + 64x64 PUs), and the intra 16 / 32
# lanes-per-job variants
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# hvpp: ring without the separate previous-row registers (all variants), rolling 4-ahead prefetch (PF=3),
# compiler held to four waves per SIMD (WPE=4); parity under each, then an interleaved A/B
for v in "1 4" "3 1" "3 4"; do
  set -- $v
  X265AMD_HVPP_PF=$1 X265AMD_HVPP_WPE=$2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -k "golden or interp_compact or oracle_random" > gpurun_out/r04g_parity_pf$1_wpe$2.log 2>&1 || { tail -30 gpurun_out/r04g_parity_pf$1_wpe$2.log; exit 1; }
  echo "parity pf=$1 wpe=$2: $(tail -1 gpurun_out/r04g_parity_pf$1_wpe$2.log)"
done
for rep in 1 2; do
  for v in "1 1" "1 4" "3 1" "3 4"; do
    set -- $v
    echo "== hvpp pf=$1 wpe=$2 rep=$rep"
    X265AMD_HVPP_PF=$1 X265AMD_HVPP_WPE=$2 timeout -k 10 200 python3 -u tools/kernel_roofline.py --only luma_hvpp 2>/dev/null | grep "{" | cut -c1-150 || exit 1
  done
done
for g in "4 4" "2 8" "4 8"; do
  set -- $g
  echo "== intra G16=$1 G32=$2"
  X265AMD_INTRA_G16=$1 X265AMD_INTRA_G32=$2 timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang_16x16,intra_ang_32x32 2>/dev/null | grep "{" | cut -c1-150 || exit 1
done
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
out=gpurun_out/r04g_me_ab.txt
: > $out
for rep in 1 2 3; do
  for cfg in "1 4096" "0 4096" "0 1024" "1 1024"; do
    set -- $cfg
    X265AMD_ME_ASYNC=$1 X265AMD_ME_MIN=$2 X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
        --preset medium --pools 16 --no-info -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "rep=$rep async=$1 min=$2: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8) $(grep -o 'prefetches [0-9]*' /tmp/e.txt) $(grep -o '[0-9.]* ms/prefetch' /tmp/e.txt)" | tee -a $out
  done
  timeout -k 10 200 oracle/_ref/x265ref8 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
      --preset medium --pools 16 --no-info -o /tmp/r.hevc > /tmp/e.txt 2>&1 || exit 1
  echo "rep=$rep reference: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/r.hevc | cut -c1-8)" | tee -a $out
done
