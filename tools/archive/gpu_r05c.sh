# round 5: (0) parity of the rewritten kernels (fused TU straight-line form, re-applied interpolation / intra
# rewrites, the search kernel's evaluation counts); (1) where the --preset slow check mismatches come from —
# STAR alone, subme 3 (chroma SATD) alone, slow with subme 2 — in check mode at 720p; (2) launch-service
# latency options at 2160p medium 64 frames: high-priority launch streams, zero-copy staging, polling
# launchers, interleaved; (3) kernel-roofline A/Bs: fused TU straight-line vs branchy, 16x16 DCT on the int8
# matrix cores vs the f16 split, intra against the round-4 kernels
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_tu.py tests/test_me.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "not fullsize" > gpurun_out/r05/c_parity.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/r05/c_parity.log | head; tail -20 gpurun_out/r05/c_parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/r05/c_parity.log)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(1280, 720, 16, 8).write_yuv('/tmp/s720.yuv')
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
echo "sources ready"
E720="--input /tmp/s720.yuv --input-res 1280x720 --fps 30 --frames 16 --no-info --pools 16"
for v in "--preset medium --me star" "--preset medium --subme 3" "--preset slow --subme 2" "--preset slow"; do
  X265AMD_ME=check X265AMD_ME_MIN=1024 timeout -k 10 120 oracle/_ref/x265la8 $E720 $v -o /tmp/c.hevc \
      > /tmp/c.log 2>&1 || { tail -20 /tmp/c.log; exit 1; }
  echo "== $v: $(grep -E 'mismatching searches|windows beyond' /tmp/c.log | tr '\n' ' ')" | tee -a gpurun_out/r05/c_slow_isolate.txt
  grep MISMATCH /tmp/c.log | head -4 | tee -a gpurun_out/r05/c_slow_isolate.txt
done
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 --preset medium --pools 16 --no-info"
for rep in 1 2; do
  for v in "0 0 0" "1 0 0" "0 1 0" "0 0 1" "1 1 1"; do
    set -- $v
    X265AMD_MES_PRIORITY=$1 X265AMD_MES_ZEROCOPY=$2 X265AMD_MES_LSPIN=$3 X265AMD_ME_STATS=1 timeout -k 10 150 \
        oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "rep=$rep prio=$1 zerocopy=$2 lspin=$3: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/c_service_ab.txt
    grep -E "worker time|service" /tmp/e.txt | tee -a gpurun_out/r05/c_service_ab.txt
  done
done
for rep in 1 2; do
  for bf in 0 1; do
    echo "== X265AMD_TU_BF=$bf rep=$rep" | tee -a gpurun_out/r05/c_tu_bf_ab.txt
    X265AMD_TU_BF=$bf timeout -k 10 200 python3 -u tools/kernel_roofline.py --only tu_pipeline 2>/dev/null | grep "{" | cut -c1-200 \
        | tee -a gpurun_out/r05/c_tu_bf_ab.txt || exit 1
  done
done
for rep in 1 2; do
  for i8 in 0 1; do
    echo "== X265AMD_TR_I8=$i8 rep=$rep" | tee -a gpurun_out/r05/c_tr16_i8_ab.txt
    X265AMD_TR_I8=$i8 timeout -k 10 200 python3 -u tools/kernel_roofline.py --only dct_16x16,idct_16x16,dct_32x32,idct_32x32 2>/dev/null \
        | grep "{" | cut -c1-200 | tee -a gpurun_out/r05/c_tr16_i8_ab.txt || exit 1
  done
done
ONLY=intra_ang_4,intra_ang_8,intra_ang_16,intra_ang_32
for rep in 1 2; do
  for v in r4 cur; do
    unset X265AMD_LIB
    [ $v = r4 ] && export X265AMD_LIB=$PWD/src/x265_amd/ab/libx265amd_r4.so
    echo "== $v rep=$rep" | tee -a gpurun_out/r05/c_intra_ab.txt
    timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-170 \
        | tee -a gpurun_out/r05/c_intra_ab.txt || exit 1
  done
done
unset X265AMD_LIB
