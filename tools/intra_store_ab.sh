# intra kernel A/B: a reference build in ablibs/ (named by the case below) vs the current build, twice each
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in rows16 cur; do
  unset X265AMD_LIB
  case $v in rows16) export X265AMD_LIB=$PWD/ablibs/libx265amd_rows16.so ;; esac
  echo "== $v"
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only intra_ang_16,intra_ang_32,intra_ang_8 2>/dev/null | grep "{" | cut -c1-160 || exit 1
done
done
