# intra 8x8: the lane-per-job kernel (X265AMD_INTRA_G8=0) vs k_intra_quad with 2 lanes per job, twice each
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for g in 0 2; do
  echo "== G8=$g"
  X265AMD_INTRA_G8=$g timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang_8 2>/dev/null | grep "{" | cut -c1-160 || exit 1
done
done
