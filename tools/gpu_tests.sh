# the GPU test suite as the driver runs it (one process, per-test time limit), log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
exit $rc
