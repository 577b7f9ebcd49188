# round 5: unit-height sweep of the luma hpp / vpp kernels on the roofline shapes (X265AMD_UH_HPP / _VPP)
set -o pipefail
mkdir -p gpurun_out/r05/ai
export TMPDIR=/tmp
OUT=gpurun_out/r05/ai/interp_uh_sweep.txt
for rep in 1 2; do
  for uh in 0 1 2 8; do
    X265AMD_UH_HPP=$uh timeout -k 10 200 python3 -u tools/kernel_roofline.py --only luma_hpp 2>/dev/null | grep "{" | cut -c1-170 \
      | sed "s/^/hpp uh=$uh rep=$rep /" | tee -a $OUT || exit 1
  done
  for uh in 0 4 8; do
    X265AMD_UH_VPP=$uh timeout -k 10 200 python3 -u tools/kernel_roofline.py --only luma_vpp 2>/dev/null | grep "{" | cut -c1-170 \
      | sed "s/^/vpp uh=$uh rep=$rep /" | tee -a $OUT || exit 1
  done
done
