# round 5: the whole GPU suite on the round's tree (search kernel rewrites, launch-service waits, SAD
# non-temporal loads, cuTree propagation on by default), then smoke
set -o pipefail
mkdir -p gpurun_out/r05/r
export TMPDIR=/tmp
timeout -k 10 1050 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
    > gpurun_out/r05/r/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r05/r/gpu_tests.log | head -20; tail -30 gpurun_out/r05/r/gpu_tests.log; exit 1; }
echo "gpu suite: $(tail -n 1 gpurun_out/r05/r/gpu_tests.log)"
timeout -k 10 100 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/r/smoke.log 2>&1 || { tail -20 gpurun_out/r05/r/smoke.log; exit 1; }
tail -n 2 gpurun_out/r05/r/smoke.log
