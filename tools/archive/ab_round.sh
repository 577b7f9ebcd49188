# A/B of the current build against a reference build in ablibs/ ($1, e.g. ablibs/libx265amd_rows16.so):
# kernel-roofline shapes ($2, comma list for --only) and the default census bench step, both twice
set -o pipefail
mkdir -p gpurun_out
REF=$1
ONLY=${2:-intra_ang_16,intra_ang_32,satd_8x8,satd_64x64}
for rep in 1 2; do
for v in ref cur; do
  unset X265AMD_LIB
  [ $v = ref ] && export X265AMD_LIB=$PWD/$REF
  echo "== $v kernels"
  timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-170 || exit 1
  echo "== $v bench"
  timeout -k 10 300 python3 bench.py --no-cpu --no-encoder-level --no-pipeline-check 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(json.dumps({'fps': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac']}))" || exit 1
done
done
