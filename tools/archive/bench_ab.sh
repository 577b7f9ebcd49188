# census-step A/B of tuning knobs: one bench line per environment setting (same box, same process order)
set -o pipefail
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 400 --warmup 20 --no-cpu --no-encoder-level --no-pipeline-check > gpurun_out/ab.json 2>/dev/null || return 1
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'])
" "$@"
}
for cfg in "$@"; do run $cfg || exit 1; done
