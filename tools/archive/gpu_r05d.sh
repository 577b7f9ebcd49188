# round 5: the new bench.py (encoded fps of 2160p medium, 64 frames per step) end to end with a short
# step count, then rocprofv3 kernel-trace summary of the same bench command, then PMC passes (FETCH_SIZE,
# WRITE_SIZE, each its own run) on a 16-frame 2160p encode of the hooked encoder for the HBM traffic of the
# batched motion-search launch
set -o pipefail
mkdir -p gpurun_out/r05/d
export TMPDIR=/tmp
: 
: 
timeout -k 10 420 python3 -u bench.py --steps 2 --warmup 0 > gpurun_out/r05/d/bench_short.json 2> gpurun_out/r05/d/bench_short.err \
    || { tail -30 gpurun_out/r05/d/bench_short.err; exit 1; }
tail -c 2500 gpurun_out/r05/d/bench_short.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05/d/prof -o bench -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-replay --no-cpu \
    > $GRAFT_REPO_ROOT/gpurun_out/r05/d/bench_rocprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05/d/bench_rocprof.err \
    || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r05/d/bench_rocprof.err; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/r05/d/prof -name "*kernel_stats.csv" | head -5
find gpurun_out/r05/d/prof -type f ! -name "*_stats.csv" -delete
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 16, 8).write_yuv('/tmp/s16.yuv')" || exit 1
cd /tmp
for pmc in FETCH_SIZE WRITE_SIZE; do
  X265AMD_ME_STATS=1 timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_$pmc -o enc -- \
      $GRAFT_REPO_ROOT/oracle/_ref/x265la8 --input /tmp/s16.yuv --input-res 3840x2160 --fps 30 --frames 16 --preset medium \
      --pools 16 --no-info -o /tmp/p.hevc > $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_$pmc.log 2>&1 \
      || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_$pmc.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/tools/pmc_by_kernel.py $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_$pmc \
      > $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_${pmc}_by_kernel.json || exit 1
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_$pmc
  echo "pmc $pmc done"
  du -sh $GRAFT_REPO_ROOT/gpurun_out/r05/d
done
python3 $GRAFT_REPO_ROOT/tools/me_traffic.py $GRAFT_REPO_ROOT/gpurun_out/r05/d $GRAFT_REPO_ROOT/gpurun_out/r05/d/pmc_me_traffic.json || exit 1
X265AMD_ME_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05/d/hiptrace -o enc -- \
    $GRAFT_REPO_ROOT/oracle/_ref/x265la8 --input /tmp/s16.yuv --input-res 3840x2160 --fps 30 --frames 16 --preset medium \
    --pools 16 --no-info -o /tmp/p.hevc > $GRAFT_REPO_ROOT/gpurun_out/r05/d/hiptrace.log 2>&1 \
    || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r05/d/hiptrace.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r05/d/hiptrace -name "*_stats.csv" | head
find $GRAFT_REPO_ROOT/gpurun_out/r05/d/hiptrace -type f ! -name "*_stats.csv" -delete
cd $GRAFT_REPO_ROOT
