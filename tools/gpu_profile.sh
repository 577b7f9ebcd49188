# One GPU call: the default bench line, its rocprofv3 kernel-trace summary, and the
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) over the same launches (tools/pmc_workload.py).
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-encoder-level > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err &&
echo "kernel trace ok" &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json > gpurun_out/pmc_write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json > gpurun_out/pmc_sq.log 2>&1 &&
echo "pmc ok"
