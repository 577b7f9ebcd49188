# round 5: launch-service options on the encoder's real budget — the 16 host cores bench.py pins the
# encode to (taskset, the same slice as core_slice) — 2160p medium 64 frames, interleaved, 3 reps:
# defaults (sleeping launchers, priority streams, 2 launchers), polling launchers, default-priority
# streams, one launcher, workers not spinning before they sleep; plus the reference on the same cores
set -o pipefail
mkdir -p gpurun_out/r05/m
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
CORES=$(python3 -c "import os; c = sorted(os.sched_getaffinity(0))[:16]; print(','.join(map(str, c)))")
echo "cores $CORES" | tee -a gpurun_out/r05/m/service_pinned_ab.txt
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
timeout -k 10 150 taskset -c $CORES oracle/_ref/x265ref8 $E4K -o /tmp/r.hevc > /tmp/r.txt 2>&1 || { tail -5 /tmp/r.txt; exit 1; }
echo "reference: $(grep encoded /tmp/r.txt) $(md5sum < /tmp/r.hevc | cut -c1-8)" | tee -a gpurun_out/r05/m/service_pinned_ab.txt
for rep in 1 2 3; do
  for v in "default" "X265AMD_MES_LSPIN=1" "X265AMD_MES_PRIORITY=0" "X265AMD_MES_LAUNCHERS=1" "X265AMD_MES_SPIN_US=0"; do
    ENVV=""
    [ "$v" != default ] && ENVV="$v"
    env $ENVV X265AMD_ME_STATS=1 timeout -k 10 150 taskset -c $CORES oracle/_ref/x265la8 $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 \
        || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/m/service_pinned_ab.txt
    grep -E "worker time|service:|waits by|batches by" /tmp/e.txt | tee -a gpurun_out/r05/m/service_pinned_ab.txt
  done
done
