# census replay step rate vs the number of lanes (bench.py --streams), time-balanced lanes, twice each
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for n in 4 6 8 10 12; do
  echo "== streams $n"
  timeout -k 10 300 python3 bench.py --streams $n --no-cpu --no-encoder-level --no-pipeline-check 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'fps': d['value'], 'ms_per_step': d['ms_per_step']}))" || exit 1
done
done
