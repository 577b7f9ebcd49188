set -o pipefail
mkdir -p gpurun_out
export X265AMD_TB_SPEED=0
for d in 8 10; do for h in pixel transforms interp intrapred; do
  s=$(date +%s.%N)
  timeout -k 10 400 oracle/_ref/TestBench$d --cpuid SSE2 --testbench $h > gpurun_out/tb${d}_$h.log 2>&1 || { echo "TB $d $h rc=$?"; exit 1; }
  echo "TB $d $h ok $(python3 -c "import time;print(round(time.time()-$s,1))")s"
done; done
timeout -k 10 900 python -u -m pytest tests/test_dropin.py -m gpu -x -v -s --timeout 900 --timeout-method thread -k encoder > gpurun_out/dropin_enc.log 2>&1
