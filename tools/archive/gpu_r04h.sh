# round 4: fused TU variants — 8x8 / 16x16 grid-stride with the next TU's inputs prefetched
# (X265AMD_TU_PF=1), 32x32 int8 with the next TU prefetched (X265AMD_TU_I8=2): parity under each,
# then an interleaved roofline A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
X265AMD_TU_PF=1 X265AMD_TU_I8=2 timeout -k 10 300 python3 -u -m pytest tests/test_tu.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -k "gpu_matches_oracle or without_residual or golden or oracle_random" > gpurun_out/r04h_parity.log 2>&1 || { tail -30 gpurun_out/r04h_parity.log; exit 1; }
echo "parity tu pf: $(tail -1 gpurun_out/r04h_parity.log)"
for rep in 1 2; do
  for v in "0 1" "1 2"; do
    set -- $v
    echo "== tu pf=$1 i8=$2 rep=$rep"
    X265AMD_TU_PF=$1 X265AMD_TU_I8=$2 timeout -k 10 200 python3 -u tools/kernel_roofline.py --only tu_pipeline_8x8,tu_pipeline_16x16,tu_pipeline_32x32 2>/dev/null | grep "{" | cut -c1-150 || exit 1
  done
done
ONLY=tu_pipeline_8x8,tu_pipeline_32x32,intra_ang_32x32
d=gpurun_out/r04h_pmc
rm -rf $d; mkdir -p $d
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY --output-format csv -d $d/k1 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/k2 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/k3 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k3.log 2>&1 || exit 1
# instruction mix (its own pass; a counter this gfx950 build lacks only loses this pass)
k4=$d/k4
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $d/k4 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > $d/k4.log 2>&1 || { echo "instruction-mix pass failed: $(tail -3 $d/k4.log)"; k4=; }
python3 tools/pmc_kernels.py $d/k1 $d/k2 $d/k3 $k4 --out $d/pmc_kernels.json || exit 1
python3 -c "
import json; d=json.load(open('$d/pmc_kernels.json'))
for k,v in d.items():
    if 'x265amd' in k: print(k[:60], {a: round(b,3) for a,b in v.items() if 'frac' in a or a in ('waves_resident','fetch_bytes','write_bytes','SQ_INSTS_VALU','SQ_INSTS_LDS','SQ_INSTS_SALU','SQ_INSTS_VMEM_RD','SQ_INSTS_VMEM_WR','SQ_WAVES','SQ_LDS_BANK_CONFLICT','SQ_WAIT_INST_LDS')})"
# where a device motion search's wall time goes inside the encoder: kernel and copy durations
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 16, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
X265AMD_ME_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r04h_encprof -o enc -- \
    oracle/_ref/x265la8 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 16 --preset medium --pools 16 --no-info -o /tmp/o.hevc \
    > gpurun_out/r04h_encprof.log 2>&1 || { tail -20 gpurun_out/r04h_encprof.log; exit 1; }
grep -E "encoded|x265me\] stats" gpurun_out/r04h_encprof.log
find gpurun_out/r04h_encprof -name "*stats*.csv" | while read f; do echo "== $f"; head -12 "$f" | cut -c1-200; done
# copies on blit kernels in the compute queue (no SDMA engine hop) for the per-PU search round trips
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for rep in 1 2; do
  for sd in 1 0; do
    HSA_ENABLE_SDMA=$sd X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
        --preset medium --pools 16 --no-info -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "rep=$rep sdma=$sd: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8) $(grep -o '[0-9.]* ms/prefetch' /tmp/e.txt)" | tee -a gpurun_out/r04h_sdma_ab.txt
  done
done
