# DCT / iDCT 16 / 32 A/B (previous kernels vs software-pipelined), then MFMA + SQ counters of the new ones
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_tu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tr_parity.log 2>&1 || { tail -20 gpurun_out/tr_parity.log; exit 1; }
tail -1 gpurun_out/tr_parity.log
for rep in 1 2; do
for v in old new; do
  unset X265AMD_LIB; test $v = old && export X265AMD_LIB=$PWD/tools/bin/libx265amd_oldtr.so
  echo "== $v"
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only dct_16,dct_32,idct_16,idct_32 2>/dev/null | grep "{" | cut -c1-170 || exit 1
done
done
unset X265AMD_LIB
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_tr -o run -- python3 tools/kernel_roofline.py --only dct_16,dct_32,idct_16,idct_32 --reps 2 > gpurun_out/pmc_tr.log 2>&1 && echo "pmc ok"
