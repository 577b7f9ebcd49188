# unit-height sweep of the luma interpolation kernels (disjoint-operand roofline, tools/kernel_roofline.py)
set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python3 -u tools/kernel_roofline.py --gb 1.0 --reps 5 --only luma_hpp,luma_vpp,luma_hvpp 2>&1 | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['kernel'], d['ms'], d['frac_of_8TBps'])
"; }
run X265AMD_UH_HPP=0 &&
run X265AMD_UH_HPP=1 X265AMD_UH_VPP=1 X265AMD_UH_HVPP=1 &&
run X265AMD_UH_HPP=2 X265AMD_UH_VPP=2 X265AMD_UH_HVPP=2 &&
run X265AMD_UH_VPP=4 X265AMD_UH_HVPP=4
