# LDS-staged write-back (interp.hip / blockops.hip STG kernels): parity first, then an A/B of
# $STAGE_ENV=0 (direct stores; default X265AMD_INTERP_STAGE) against the default on the
# kernel-roofline shapes ($1) and the census bench step, twice each.
STAGE_ENV=${STAGE_ENV:-X265AMD_INTERP_STAGE}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "${TEST_K:-compact or oracle_random or fullsize_frame_batch and 1080p}" > gpurun_out/stage_tests.log 2>&1 || { tail -30 gpurun_out/stage_tests.log; exit 1; }
tail -2 gpurun_out/stage_tests.log
for rep in 1 2; do
for v in 0 1; do
  export $STAGE_ENV=$v
  echo "== stage=$v kernels"
  timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "${1:-luma_hpp,luma_vpp}" 2>/dev/null | grep "{" | cut -c1-150 || exit 1
  echo "== stage=$v bench"
  timeout -k 10 300 python3 bench.py --no-cpu --no-encoder-level --no-pipeline-check 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(json.dumps({'fps': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac']}))" || exit 1
done
done
