# quant / dequant jobs-per-lane-group sweep (X265AMD_COEF_JPG) on the kernel roofline shapes, plus parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_tu.py -m gpu > gpurun_out/coef_tests.log 2>&1; rc=$?; tail -2 gpurun_out/coef_tests.log; [ $rc -eq 0 ] || exit 1
for cw in 4 8; do for j in 1 2 4; do
  echo "== X265AMD_COEF_CW=$cw X265AMD_COEF_JPG=$j"
  X265AMD_COEF_CW=$cw X265AMD_COEF_JPG=$j timeout -k 10 200 python3 -u tools/kernel_roofline.py --reps 10 --only quant > gpurun_out/coef_${cw}_$j.jsonl 2>&1 || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/coef_${cw}_$j.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['kernel'], d['ms'], d['frac_of_8TBps'])
"
done; done
