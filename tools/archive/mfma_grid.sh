# MFMA transform grid-cap sweep (X265AMD_MFMA_GRID) on the kernel roofline shapes
set -o pipefail
for cap in 4096 1024 16384 65536 1000000; do
  echo "== cap $cap"
  X265AMD_MFMA_GRID=$cap timeout -k 10 200 python3 -u tools/kernel_roofline.py --reps 10 --only dct_16,dct_32 > gpurun_out/mg.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/mg.jsonl'):
    if l.startswith('{') and 'frac_of_8TBps' in l:
        d=json.loads(l); print(d['kernel'], d['ms'], d['frac_of_8TBps'])
"
done
