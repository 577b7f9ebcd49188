# round 5: the round-4 interpolation rewrite without its inline-asm dot starts (a052b: the chain start
# passed to the builtin instead): differences against the oracle, golden parity with that library, and
# the interpolation kernel roofline against the tree's, interleaved, 2 reps
set -o pipefail
mkdir -p gpurun_out/r05/u
export TMPDIR=/tmp
LIB=$PWD/src/x265_amd/ab/libx265amd_a052b.so
X265AMD_LIB=$LIB timeout -k 10 200 python3 -u tools/interp_diff.py > gpurun_out/r05/u/interp_diff_a052b.txt 2>&1 || { tail -20 gpurun_out/r05/u/interp_diff_a052b.txt; exit 1; }
grep differing gpurun_out/r05/u/interp_diff_a052b.txt
X265AMD_LIB=$LIB timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/u/parity.log 2>&1 || { grep -E "FAILED|mismatches|assert" gpurun_out/r05/u/parity.log | head; tail -20 gpurun_out/r05/u/parity.log; exit 1; }
echo "parity (a052b): $(tail -n 1 gpurun_out/r05/u/parity.log)"
ONLY=luma_hpp,luma_vpp,luma_hvpp
for rep in 1 2; do
  for v in tree a052b; do
    unset X265AMD_LIB
    [ $v = a052b ] && export X265AMD_LIB=$LIB
    echo "== $v rep=$rep" | tee -a gpurun_out/r05/u/interp_ab.txt
    timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-160 \
        | tee -a gpurun_out/r05/u/interp_ab.txt || exit 1
  done
done
unset X265AMD_LIB
