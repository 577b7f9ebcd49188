# round 4: int8 matrix-core transforms — the operand-map probe, parity of k_tr32_i8 (X265AMD_TR_I8=1)
# on the golden / random / fused cases, then the kernel roofline of dct / idct 32x32, f16 split vs int8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/probes/mfma_i8_probe | tee gpurun_out/r04d_probe.txt || exit 1
X265AMD_TR_I8=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -k "golden or oracle_random" > gpurun_out/r04d_parity_i8.log 2>&1 || { tail -30 gpurun_out/r04d_parity_i8.log; exit 1; }
echo "parity i8: $(tail -1 gpurun_out/r04d_parity_i8.log)"
for rep in 1 2; do
for v in 0 1; do
  echo "== i8=$v rep=$rep"
  X265AMD_TR_I8=$v timeout -k 10 300 python3 -u tools/kernel_roofline.py --only dct_32x32,idct_32x32 2>/dev/null | grep "{" | cut -c1-170 || exit 1
done
done
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for run in "la 16 1024 4 block" "la 16 4096 4 block" "la 16 4096 16 block" "la 24 4096 16 block" "la 16 4096 16 spin" "la 16 1024 16 block"; do
  set -- $run
  r=$(GPU_MAX_HW_QUEUES=$4 X265AMD_MES_SYNC=$5 X265AMD_ME_MIN=$3 X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 --input /tmp/s2160.yuv \
      --input-res 3840x2160 --fps 30 --frames 64 --preset medium --pools $2 --no-info -o /tmp/o.hevc 2>&1) || { echo "$r" | tail; exit 1; }
  echo "== $run: $(echo "$r" | grep -E 'encoded') $(md5sum /tmp/o.hevc | cut -c1-8) $(echo "$r" | grep -oE '[0-9.]+ ms/prefetch')"
done
