# interp unit-height sweep including 8-row units (kernel_roofline shapes)
set -o pipefail
for cfg in "X265AMD_NONE=1" "X265AMD_UH_HPP=8" "X265AMD_UH_VPP=8" "X265AMD_UH_HPP=2"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python3 -u tools/kernel_roofline.py --reps 10 --only luma_hpp,luma_vpp > gpurun_out/uh.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/uh.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['kernel'], d['ms'], d['frac_of_8TBps'])
"
done
