# ME occupancy A/B: k_motion_search built with __launch_bounds__(256, W) for W = 2 / 3 / 4
# (alternate libraries under src/x265_amd/_ab, selected with X265AMD_LIB)
set -o pipefail
for lib in "" src/x265_amd/_ab/libx265amd_w2.so src/x265_amd/_ab/libx265amd_w3.so src/x265_amd/_ab/libx265amd_w4.so; do
  echo "== ${lib:-default}"
  X265AMD_LIB=$lib timeout -k 10 300 python3 -u tools/kernel_roofline.py --reps 5 --only me_hex,me_star,me_umh > gpurun_out/mw.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/mw.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['kernel'], d['ms'], d.get('pu_per_s'), d.get('gpu_matches_reference_on_sample'))
"
done
