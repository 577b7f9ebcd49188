# round 5: sad_x3 / sad_x4 with one lane per (job, reference) for small blocks: parity (the golden and
# oracle cases of test_gpu_parity), then the kernel roofline of SAD / sad_x4 on the tree, with
# X265AMD_SADX_LANES=0 (lane per job), and the non-temporal-load build (SAD rows), 2 reps interleaved
set -o pipefail
mkdir -p gpurun_out/r05/j
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/j/parity.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/j/parity.log | head; tail -20 gpurun_out/r05/j/parity.log; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/r05/j/parity.log)"
ONLY=sad_8x8,sad_16x16,sad_64x64,sad_x4_8x8,sad_x4_16x16,sad_x4_64x64
for rep in 1 2; do
  for v in tree lanes0 nt; do
    unset X265AMD_LIB X265AMD_SADX_LANES
    [ $v = lanes0 ] && export X265AMD_SADX_LANES=0
    [ $v = nt ] && export X265AMD_LIB=$PWD/src/x265_amd/ab/libx265amd_nt.so
    echo "== $v rep=$rep" | tee -a gpurun_out/r05/j/sad_ab.txt
    timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-190 \
        | tee -a gpurun_out/r05/j/sad_ab.txt || exit 1
  done
done
unset X265AMD_LIB X265AMD_SADX_LANES
