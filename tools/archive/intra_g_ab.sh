# lanes per job of the 16x16 / 32x32 intra kernel (k_intra_quad): X265AMD_INTRA_G16 2 / 4 and
# X265AMD_INTRA_G32 4 / 8, twice each
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for g in "4 4" "2 8"; do
  set -- $g
  echo "== G16=$1 G32=$2"
  X265AMD_INTRA_G16=$1 X265AMD_INTRA_G32=$2 timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang_16,intra_ang_32 2>/dev/null | grep "{" | cut -c1-160 || exit 1
done
done
