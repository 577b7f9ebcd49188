# N=1 throughput of the bench step modes (replay vs frame-parallel pipeline at several band sizes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in "--mode pipeline --band-rows 4 --streams 1" "--mode pipeline --band-rows 4 --streams 4" "--mode pipeline --band-rows 4 --one-graph" "--mode pipeline --band-rows 1 --one-graph" "--mode pipeline --band-rows 17 --one-graph"; do
  echo "== $m"
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu --no-encoder-level $m > gpurun_out/mode.json 2> gpurun_out/mode.err || { tail -20 gpurun_out/mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/mode.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['config']['launches_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_pipe -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-encoder-level --mode pipeline --band-rows 4 > gpurun_out/prof_pipe.json 2> gpurun_out/prof_pipe.err
