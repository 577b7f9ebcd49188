# k_hvpp_stream variants (interp.hip): row bands (X265AMD_HVPP_RB=4|8) and 4-wide staged strips
# (X265AMD_HVPP_SW=4) against the default: parity of every variant first (compact and random
# interp cases), then the hv_pp kernel-roofline shapes, twice each.
set -o pipefail
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"base rb4 rb8 sw4 sw4rb8"}
envof() { case $1 in base) echo "";; rb4) echo "X265AMD_HVPP_RB=4";; rb8) echo "X265AMD_HVPP_RB=8";;
  sw4) echo "X265AMD_HVPP_SW=4";; sw4rb8) echo "X265AMD_HVPP_SW=4 X265AMD_HVPP_RB=8";; esac; }
for v in $VARIANTS; do
  echo "== $v parity"
  env $(envof $v) timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread \
    -k "interp_compact or oracle_random" > gpurun_out/hvpp_$v.log 2>&1 || { tail -30 gpurun_out/hvpp_$v.log; exit 1; }
  tail -1 gpurun_out/hvpp_$v.log
done
for rep in 1 2; do
for v in $VARIANTS; do
  echo "== $v kernels"
  env $(envof $v) timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "${1:-luma_hvpp}" 2>/dev/null | grep "{" | cut -c1-150 || exit 1
done
done
