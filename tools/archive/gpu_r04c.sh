# round 4, third box call: interp row-prefetch variants (parity under each, then kernel roofline A/B),
# baseline SAD / sad_x4 rooflines, and encoder thread / PU-size variants of the device motion searches
set -o pipefail
mkdir -p gpurun_out
for pf in 1 2; do
  X265AMD_HVPP_PF=$pf timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -k "golden or interp_compact or oracle_random" > gpurun_out/r04c_parity_pf$pf.log 2>&1 || { tail -30 gpurun_out/r04c_parity_pf$pf.log; exit 1; }
  echo "parity pf=$pf: $(tail -1 gpurun_out/r04c_parity_pf$pf.log)"
done
for rep in 1 2; do
for pf in 0 1 2; do
  echo "== pf=$pf rep=$rep"
  X265AMD_HVPP_PF=$pf timeout -k 10 300 python3 -u tools/kernel_roofline.py --only luma_hvpp,luma_hpp,luma_vpp 2>/dev/null | grep "{" | cut -c1-160 || exit 1
done
done
echo "== compare kernels"
timeout -k 10 300 python3 -u tools/kernel_roofline.py --only sad_8x8,sad_64x64,sad_x4_8x8,satd_8x8 2>/dev/null | grep "{" | cut -c1-200 || exit 1
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for run in "ref 16 1024" "la 16 1024" "la 24 1024" "la 32 1024" "la 24 256" "la 16 4096"; do
  set -- $run
  exe=oracle/_ref/x265la8; [ $1 = ref ] && exe=oracle/_ref/x265ref8
  r=$(X265AMD_ME_MIN=$3 X265AMD_ME_STATS=1 timeout -k 10 200 $exe --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
      --preset medium --pools $2 --no-info -o /tmp/o.hevc 2>&1) || { echo "$r" | tail; exit 1; }
  echo "== $run: $(echo "$r" | grep -E 'encoded') $(md5sum /tmp/o.hevc | cut -c1-8) $(echo "$r" | grep -oE 'prefetches [0-9]+ searches [0-9]+|[0-9.]+ ms/prefetch')"
done
timeout -k 10 1000 python3 -u bench.py > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || { tail -30 gpurun_out/r04c_bench.err; exit 1; }
head -c 1500 gpurun_out/r04c_bench.json
