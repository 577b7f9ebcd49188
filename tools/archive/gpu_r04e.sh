# round 4: int8 matrix-core transforms with the transposed stage 2 (direct row stores) and the int8
# fused 32x32 TU — parity under X265AMD_TR_I8=1 X265AMD_TU_I8=1, then A/B on the kernel roofline;
# the frame pipeline with TU-coded reconstruction (test_gpu_pipeline)
set -o pipefail
mkdir -p gpurun_out
export X265AMD_TR_I8=1 X265AMD_TU_I8=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_tu.py -m gpu -x -q --timeout 250 --timeout-method thread \
    -k "golden or oracle_random or tu" > gpurun_out/r04e_parity_i8.log 2>&1 || { tail -30 gpurun_out/r04e_parity_i8.log; exit 1; }
echo "parity i8: $(tail -1 gpurun_out/r04e_parity_i8.log)"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04e_pipeline.log 2>&1 || { tail -40 gpurun_out/r04e_pipeline.log; exit 1; }
echo "pipeline: $(tail -1 gpurun_out/r04e_pipeline.log)"
for rep in 1 2; do
for v in 0 1; do
  echo "== i8=$v rep=$rep"
  X265AMD_TR_I8=$v X265AMD_TU_I8=$v timeout -k 10 300 python3 -u tools/kernel_roofline.py --only dct_32x32,idct_32x32,tu_pipeline_32x32 2>/dev/null | grep "{" | cut -c1-170 || exit 1
done
done
unset X265AMD_TR_I8 X265AMD_TU_I8
timeout -k 10 500 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/r04e_me_tests.log 2>&1 || { tail -40 gpurun_out/r04e_me_tests.log; exit 1; }
grep -E "x265me\] [0-9]|passed|failed" gpurun_out/r04e_me_tests.log
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for run in "1 4096" "0 4096" "1 1024" "1 4096"; do
  set -- $run
  r=$(X265AMD_ME_ASYNC=$1 X265AMD_ME_MIN=$2 X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 --input /tmp/s2160.yuv \
      --input-res 3840x2160 --fps 30 --frames 64 --preset medium --pools 16 --no-info -o /tmp/o.hevc 2>&1) || { echo "$r" | tail; exit 1; }
  echo "== async=$1 min=$2: $(echo "$r" | grep -E 'encoded') $(md5sum /tmp/o.hevc | cut -c1-8) $(echo "$r" | grep -oE 'misses [0-9]+|[0-9.]+ ms/prefetch' | tr '\n' ' ')"
done
for rep in 1 2; do
for v in 0 1; do
  echo "== sad_uh8=$v rep=$rep"
  X265AMD_SAD_UH8=$v timeout -k 10 300 python3 -u tools/kernel_roofline.py --only sad_8x8,sad_16x16,sad_64x64,sad_x4_8x8,sad_x4_16x16 2>/dev/null | grep "{" | cut -c1-200 || exit 1
done
done
