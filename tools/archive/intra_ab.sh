# intra 16x16 / 32x32 kernel A/B: round-2 build vs current (block kernel / persistent wave kernel), twice each
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in r2 block wave8192; do
  unset X265AMD_INTRA_WAVE X265AMD_LIB
  case $v in r2) export X265AMD_LIB=$PWD/tools/bin/libx265amd_r2intra.so ;; wave8192) export X265AMD_INTRA_WAVE=8192 ;; esac
  echo "== $v"
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang_16,intra_ang_32 2>/dev/null | grep "{" | cut -c1-150 || exit 1
done
done
