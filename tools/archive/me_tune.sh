# ME kernel rates (tools/kernel_roofline.py, every 2Nx2N PU of a 1080p frame) and ME parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_me.py tests/test_golden_f1f4.py -m gpu > gpurun_out/me_tests.log 2>&1; rc=$?; tail -3 gpurun_out/me_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/kernel_roofline.py --reps 5 --only me_ 2>&1 | tee gpurun_out/me_roofline.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['kernel'], d['ms'], d.get('pu_per_s'), d.get('pixel_candidates_per_s'), d.get('cpu_reference_1core_pu_per_s'), d.get('gpu_matches_reference_on_sample'))
"
