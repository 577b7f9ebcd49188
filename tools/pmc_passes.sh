# The three PMC passes of tools/gpu_profile.sh alone (FETCH_SIZE, WRITE_SIZE, SQ) over tools/pmc_workload.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json > gpurun_out/pmc_write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/pmc_workload.py --order gpurun_out/pmc_order.json > gpurun_out/pmc_sq.log 2>&1 &&
echo "pmc ok"
