# round 4: 8-bit intra angular with x8 weights (each pixel the high byte of its u16 / u32 sum: one
# v_perm per four pixels on the vertical path, VOP3P dots with the rounding as an SGPR operand on the
# transposed path): parity, then an interleaved roofline A/B against the previous intra kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB=$PWD/src/x265_amd/ab
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -k "golden or oracle_random" > gpurun_out/r04k_parity.log 2>&1 || { tail -30 gpurun_out/r04k_parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/r04k_parity.log)"
for rep in 1 2; do
  for lib in intraold default; do
    echo "== $lib rep=$rep"
    if [ $lib = default ]; then unset X265AMD_LIB; else export X265AMD_LIB=$AB/libx265amd_$lib.so; fi
    timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang 2>/dev/null | grep "{" | cut -c1-150 || exit 1
  done
done
unset X265AMD_LIB
