# round 5: the whole GPU suite on the tree (incl. the re-applied round-4 interpolation / intra rewrites, the
# launch-service / chroma-session encoder tests), smoke, then an interleaved kernel-roofline A/B of the
# interpolation and intra kernels against the round-4 kernels that ran on the box (src/x265_amd/ab/
# libx265amd_r4.so, tools/build_ab.py r4 fc10ce6 interp.hip intra.hip)
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r05/b_gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r05/b_gpu_tests.log | head -20; tail -30 gpurun_out/r05/b_gpu_tests.log; exit 1; }
echo "gpu suite: $(tail -1 gpurun_out/r05/b_gpu_tests.log)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/b_smoke.log 2>&1 || { tail -20 gpurun_out/r05/b_smoke.log; exit 1; }
tail -1 gpurun_out/r05/b_smoke.log
ONLY=${ONLY:-luma_hvpp_8x8,luma_hvpp_16x16,luma_hvpp_64x64,luma_hpp_8x8,luma_hpp_16x16,luma_hpp_64x64,luma_vpp_8x8,luma_vpp_16x16,luma_vpp_64x64,intra_ang_4,intra_ang_8,intra_ang_16,intra_ang_32}
for rep in 1 2; do
  for v in r4 cur; do
    unset X265AMD_LIB
    [ $v = r4 ] && export X265AMD_LIB=$PWD/src/x265_amd/ab/libx265amd_r4.so
    echo "== $v rep=$rep" | tee -a gpurun_out/r05/b_interp_intra_ab.txt
    timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-170 \
        | tee -a gpurun_out/r05/b_interp_intra_ab.txt || exit 1
  done
done
unset X265AMD_LIB
