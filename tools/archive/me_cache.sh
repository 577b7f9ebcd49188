# L1 (TCP) / L2 (TCC) hit counters of the motion-search launches of the kernel roofline's 64x64 block
# (HEX, STAR / subme 3, batched x8, UMH, FULL): do the lockstep searches' reference re-reads hit the caches?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_me1 gpurun_out/pmc_me2
timeout -s KILL 200 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_me1 -o run -- python3 tools/kernel_roofline.py --only me_hex_64 --reps 2 > gpurun_out/pmc_me1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_me2 -o run -- python3 tools/kernel_roofline.py --only me_hex_64 --reps 2 > gpurun_out/pmc_me2.log 2>&1 &&
echo "me pmc ok"
