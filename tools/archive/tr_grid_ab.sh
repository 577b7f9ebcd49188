# MFMA transform grid cap sweep (X265AMD_TR_GRID; default 4096 workgroups) on the kernel-roofline shapes
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for g in 4096 1024 2048 8192 16384; do
  echo "== grid cap $g"
  X265AMD_TR_GRID=$g timeout -k 10 200 python3 -u tools/kernel_roofline.py --only dct_16,dct_32,idct_16,idct_32 2>/dev/null | grep "{" | grep -v mfma_TFLOPs | cut -c1-150 || exit 1
done
done
