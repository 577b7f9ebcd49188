# round 4: interpolation instruction cuts — v_sat_pk_u8_i16 output packing, the sp rounding folded into
# the dot chains' starts, VOP3P dot forms with the start as an operand (default library) — against the
# library before them (src/x265_amd/ab/libx265amd_presat.so), and dword-aligned filter-window loads on
# top (X265AMD_WIN_ALIGNED=1 build, ab/libx265amd_winal.so): parity, then an interleaved roofline A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB=$PWD/src/x265_amd/ab
for lib in default winal; do
  if [ $lib = winal ]; then export X265AMD_LIB=$AB/libx265amd_winal.so; else unset X265AMD_LIB; fi
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
      -k "golden or interp_compact or oracle_random" > gpurun_out/r04i_parity_$lib.log 2>&1 || { tail -30 gpurun_out/r04i_parity_$lib.log; exit 1; }
  echo "parity $lib: $(tail -1 gpurun_out/r04i_parity_$lib.log)"
done
for rep in 1 2; do
  for lib in presat default winal; do
    echo "== $lib rep=$rep"
    if [ $lib = default ]; then unset X265AMD_LIB; else export X265AMD_LIB=$AB/libx265amd_$lib.so; fi
    timeout -k 10 200 python3 -u tools/kernel_roofline.py --only luma_hpp,luma_vpp,luma_hvpp 2>/dev/null | grep "{" | cut -c1-150 || exit 1
  done
done
unset X265AMD_LIB
