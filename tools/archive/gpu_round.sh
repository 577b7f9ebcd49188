# full round check on the GPU box: GPU suite, smoke, default bench line (logs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 1500 gpurun_out/bench.json
