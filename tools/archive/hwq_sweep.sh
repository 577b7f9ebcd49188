set -o pipefail
for cfg in "4 8" "8 8" "16 16" "8 16" "4 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python3 -u bench.py --steps 400 --warmup 20 --streams $2 --no-cpu --no-encoder-level --no-pipeline-check > gpurun_out/hw.json 2>/dev/null || exit 1
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/hw.json').read().strip().splitlines()[-1]); print('hwq', sys.argv[1], 'streams', sys.argv[2], d['value'], d['ms_per_step'])
" $1 $2
done
