# SQ + HBM counters of the kernel-roofline shapes named by $1 (comma list for --only), one PMC pass each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ONLY=${1:-luma_,intra_ang}
rm -rf gpurun_out/pmc_k1 gpurun_out/pmc_k2 gpurun_out/pmc_k3
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_k1 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > gpurun_out/pmc_k1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_k2 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > gpurun_out/pmc_k2.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_k3 -o run -- python3 tools/kernel_roofline.py --only "$ONLY" --reps 2 > gpurun_out/pmc_k3.log 2>&1 &&
python3 tools/pmc_kernels.py gpurun_out/pmc_k1 gpurun_out/pmc_k2 gpurun_out/pmc_k3 --out gpurun_out/pmc_kernels.json
