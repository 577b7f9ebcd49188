# round 4: SQ / HBM counters of hvpp / hpp / SAD / sad_x4 before and after the row prefetch and the
# 8x8 SAD units, hvpp strip-width A/B with the prefetch, and the 2160p
# DETAILED_CU_STATS breakdown with the CTU-start device searches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ONLY=luma_hvpp_16x16,luma_hvpp_64x64,luma_hpp_16x16,sad_8x8,sad_x4_8x8
for v in 0 1; do
  export X265AMD_HVPP_PF=$v X265AMD_SAD_UH8=$v
  d=gpurun_out/r04f_pmc_v$v
  rm -rf $d; mkdir -p $d
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY --output-format csv -d $d/k1 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k1.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/k2 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k2.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/k3 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k3.log 2>&1 &&
  python3 tools/pmc_kernels.py $d/k1 $d/k2 $d/k3 --out $d/pmc_kernels.json || exit 1
  echo "== pmc v=$v"; cat $d/pmc_kernels.json | head -c 2500
done
unset X265AMD_HVPP_PF X265AMD_SAD_UH8
for sw in 8 4; do
  echo "== hvpp sw=$sw (pf 1)"
  X265AMD_HVPP_SW=$sw timeout -k 10 300 python3 -u tools/kernel_roofline.py --only luma_hvpp 2>/dev/null | grep "{" | cut -c1-170 || exit 1
done
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8s --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
    --preset medium --pools 16 --no-info -o /tmp/o.hevc > gpurun_out/r04f_cu_stats_la8s_me_async.txt 2>&1 || exit 1
grep -E "encoded|CU:|x265me\] stats" gpurun_out/r04f_cu_stats_la8s_me_async.txt
timeout -k 10 1000 python3 -u bench.py > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -30 gpurun_out/r04f_bench.err; exit 1; }
head -c 600 gpurun_out/r04f_bench.json
