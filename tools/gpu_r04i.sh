# round 4: dword-aligned filter-window loads (X265AMD_WIN_ALIGNED=1 build in src/x265_amd/ab/) for the
# 8-bit luma hpp / hvpp: parity, then an interleaved roofline A/B against the default library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AL=$PWD/src/x265_amd/ab/libx265amd_winal.so
X265AMD_LIB=$AL timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -k "golden or interp_compact or oracle_random" > gpurun_out/r04i_parity_winal.log 2>&1 || { tail -30 gpurun_out/r04i_parity_winal.log; exit 1; }
echo "parity winal: $(tail -1 gpurun_out/r04i_parity_winal.log)"
for rep in 1 2; do
  for lib in default winal; do
    echo "== $lib rep=$rep"
    if [ $lib = winal ]; then export X265AMD_LIB=$AL; else unset X265AMD_LIB; fi
    timeout -k 10 200 python3 -u tools/kernel_roofline.py --only luma_hpp,luma_hvpp 2>/dev/null | grep "{" | cut -c1-150 || exit 1
  done
done
