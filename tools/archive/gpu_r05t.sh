# round 5: the whole GPU suite again (stop at the first failure so its traceback is kept), then smoke
set -o pipefail
mkdir -p gpurun_out/r05/t
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r05/t/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r05/t/gpu_tests.log | head -20; tail -60 gpurun_out/r05/t/gpu_tests.log; exit 1; }
echo "gpu suite: $(tail -n 1 gpurun_out/r05/t/gpu_tests.log)"
timeout -k 10 100 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/t/smoke.log 2>&1 || { tail -20 gpurun_out/r05/t/smoke.log; exit 1; }
tail -n 2 gpurun_out/r05/t/smoke.log
