# round 5: size-dependent unit heights for 8-bit luma hpp (64-wide: 1 row) and vpp (8x8: 8 rows): parity of
# every golden / random interp case, the oracle diff, the roofline shapes
set -o pipefail
mkdir -p gpurun_out/r05/aj
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/aj/parity.log 2>&1 || { grep -E "FAILED|mismatches|assert" gpurun_out/r05/aj/parity.log | head; tail -20 gpurun_out/r05/aj/parity.log; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/r05/aj/parity.log)"
timeout -k 10 200 python3 -u tools/interp_diff.py > gpurun_out/r05/aj/interp_diff.txt 2>&1 || { tail -20 gpurun_out/r05/aj/interp_diff.txt; exit 1; }
grep -c " 0 differing" gpurun_out/r05/aj/interp_diff.txt
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only luma_hpp,luma_vpp 2>/dev/null | grep "{" | cut -c1-170 \
    | sed "s/^/rep=$rep /" | tee -a gpurun_out/r05/aj/interp_roofline.txt || exit 1
done
