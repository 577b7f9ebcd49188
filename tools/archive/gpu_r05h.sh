# round 5: gprof flat profile of the hooked encoder (device lookahead + device motion searches) at 2160p
# medium, 32 frames: where the host worker time goes now
set -o pipefail
mkdir -p gpurun_out/r05/h
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 32, 8).write_yuv('/tmp/s32.yuv')" || exit 1
cd /tmp
X265AMD_ME_STATS=1 timeout -k 10 300 $GRAFT_REPO_ROOT/oracle/_ref/x265la8p --input /tmp/s32.yuv --input-res 3840x2160 --fps 30 \
    --frames 32 --preset medium --pools 16 --no-info -o /tmp/p.hevc > $GRAFT_REPO_ROOT/gpurun_out/r05/h/enc.log 2>&1 \
    || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r05/h/enc.log; exit 1; }
grep -E "encoded|worker time" $GRAFT_REPO_ROOT/gpurun_out/r05/h/enc.log
gprof -b -p $GRAFT_REPO_ROOT/oracle/_ref/x265la8p /tmp/gmon.out > $GRAFT_REPO_ROOT/gpurun_out/r05/h/flat.txt || exit 1
gprof -b -q $GRAFT_REPO_ROOT/oracle/_ref/x265la8p /tmp/gmon.out > /tmp/graph.txt || exit 1
head -c 3000000 /tmp/graph.txt > $GRAFT_REPO_ROOT/gpurun_out/r05/h/graph.txt
head -45 $GRAFT_REPO_ROOT/gpurun_out/r05/h/flat.txt
