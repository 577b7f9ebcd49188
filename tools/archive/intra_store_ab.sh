# intra kernel A/B: a reference build ($1, default ablibs/libx265amd_ref.so) vs the current build, twice each
set -o pipefail
mkdir -p gpurun_out
REF=${1:-ablibs/libx265amd_ref.so}
for rep in 1 2; do
for v in ref cur; do
  unset X265AMD_LIB
  [ $v = ref ] && export X265AMD_LIB=$PWD/$REF
  echo "== $v"
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang_16,intra_ang_32,intra_ang_8 2>/dev/null | grep "{" | cut -c1-160 || exit 1
done
done
