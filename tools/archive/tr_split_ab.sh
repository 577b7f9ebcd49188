# DCT / iDCT 16 / 32 on MFMA: packed 10-bit operand split and MFMA results in VGPRs
# ($NEWLIB) against the in-tree library: parity of the new build on every transform test first,
# then the kernel-roofline transform shapes, twice each.
set -o pipefail
mkdir -p gpurun_out
NEWLIB=${NEWLIB:-$PWD/src/x265_amd/_ab_newtr.so}
X265AMD_LIB=$NEWLIB timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_tu.py tests/test_capi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tr_parity.log 2>&1 || { tail -20 gpurun_out/tr_parity.log; exit 1; }
tail -1 gpurun_out/tr_parity.log
X265AMD_LIB=$NEWLIB timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "transform or dct or tr_ or smoke" > gpurun_out/tr_parity2.log 2>&1 || { tail -20 gpurun_out/tr_parity2.log; exit 1; }
tail -1 gpurun_out/tr_parity2.log
for rep in 1 2; do
for v in old new; do
  unset X265AMD_LIB; test $v = new && export X265AMD_LIB=$NEWLIB
  echo "== $v"
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only ${ONLY:-dct_16,dct_32,idct_16,idct_32} 2>/dev/null | grep "{" | cut -c1-170 || exit 1
done
done
