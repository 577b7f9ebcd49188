# bench lines of the BASELINE configs that fit one GPU: 1080p medium (config 2), 2160p slow (config 3),
# 2160p medium (the per-GPU work of config 4), 2160p Main10 medium (config 5)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_configs.jsonl
for cfg in "--height 1080 --width 1920 --preset medium --depth 8" \
           "--height 2160 --width 3840 --preset slow --depth 8" \
           "--height 2160 --width 3840 --preset medium --depth 8" \
           "--height 2160 --width 3840 --preset medium --depth 10"; do
  timeout -k 10 400 python3 -u bench.py $cfg --steps 200 --warmup 10 --no-cpu --no-encoder-level --no-pipeline-check > gpurun_out/bc.json 2>gpurun_out/bc.err || exit 1
  tail -1 gpurun_out/bc.json >> gpurun_out/bench_configs.jsonl
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/bc.json').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'], d['roofline']['frac'], d['config'].get('workload','')[:60])
" $cfg
done
