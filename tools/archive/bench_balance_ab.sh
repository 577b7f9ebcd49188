# census replay lanes balanced by algorithmic bytes vs by measured launch time (bench.py
# X265AMD_BENCH_BALANCE), three runs each, interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in bytes time; do
  echo "== $v"
  X265AMD_BENCH_BALANCE=$v timeout -k 10 300 python3 bench.py --no-cpu --no-encoder-level --no-pipeline-check 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'fps': d['value'], 'ms_per_step': d['ms_per_step'], 'windows': d.get('fps_1s_windows')}))" || exit 1
done
done
