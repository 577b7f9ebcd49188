# round 5: smoke() and the kernel parity files touched by the last changes (motion search, sad_x), on the final tree
set -o pipefail
mkdir -p gpurun_out/r05/af
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/af/smoke.log 2>&1 || { tail -20 gpurun_out/r05/af/smoke.log; exit 1; }
tail -n 1 gpurun_out/r05/af/smoke.log | cut -c1-200
timeout -k 10 500 python3 -u -m pytest tests/test_me.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/af/parity.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/af/parity.log | head; tail -30 gpurun_out/r05/af/parity.log; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/r05/af/parity.log)"
