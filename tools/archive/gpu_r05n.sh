# round 5: non-temporal loads in SAD / sad_x3 / sad_x4 (X265AMD_NT, default 1): parity, the kernel roofline
# of the SAD family with and without them, and the census replay (primitive workload: cache-resident
# re-reads) with and without them, interleaved, 2 reps
set -o pipefail
mkdir -p gpurun_out/r05/n
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/n/parity.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/n/parity.log | head; tail -20 gpurun_out/r05/n/parity.log; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/r05/n/parity.log)"
ONLY=sad_8x8,sad_16x16,sad_32x32,sad_64x64,sad_x4_8x8,sad_x4_16x16,sad_x4_64x64
for rep in 1 2; do
  for nt in 1 0; do
    echo "== X265AMD_NT=$nt rep=$rep" | tee -a gpurun_out/r05/n/sad_nt_ab.txt
    X265AMD_NT=$nt timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-190 \
        | tee -a gpurun_out/r05/n/sad_nt_ab.txt || exit 1
    X265AMD_NT=$nt timeout -k 10 300 python3 -u -c "
import json
from src.x265_amd.replay_bench import primitive_workload
r = primitive_workload()
print(json.dumps({'census_replay_fps': r.get('fps'), 'ms_per_step': r.get('ms_per_step')}))" 2>/dev/null | grep census | tee -a gpurun_out/r05/n/sad_nt_ab.txt || exit 1
  done
done
