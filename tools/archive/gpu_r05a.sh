# round 5, first box call (second try, every step under its own short limit): the launch-service motion
# searches (csrc/mesession.cpp, launchers) with the CU-start prefetch at depth 0 / 1
# (integration/gpu_me.cpp); the first 720p run traces the service's first posts / launches / waits
# (X265AMD_MES_TRACE); then check modes (ME, lookahead + the device cuTree propagation, --preset slow's
# chroma SATD), an interleaved 2160p medium 64-frame A/B against the round-4 form and the reference, and one
# DETAILED_CU_STATS run
set -o pipefail
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(1280, 720, 24, 8).write_yuv('/tmp/s720.yuv')" || exit 1
echo "720p source ready"
E720="--input /tmp/s720.yuv --input-res 1280x720 --fps 30 --frames 24 --no-info --pools 16"
timeout -k 10 100 oracle/_ref/x265ref8 $E720 --preset medium -o /tmp/r720.hevc > /dev/null 2>&1 || exit 1
echo "reference 720p $(md5sum < /tmp/r720.hevc | cut -c1-8)"
X265AMD_MES_TRACE=40 X265AMD_ME_STATS=1 timeout -k 10 100 oracle/_ref/x265la8 $E720 --preset medium -o /tmp/g.hevc \
    > gpurun_out/r05/a_trace.log 2>&1
rc=$?; echo "traced run rc=$rc $(md5sum < /tmp/g.hevc | cut -c1-8)"; grep -E "^\[mes\]|stats|service|worker" gpurun_out/r05/a_trace.log | head -60
[ $rc = 0 ] || exit 1
X265AMD_ME=check X265AMD_ME_MIN=1024 timeout -k 10 150 oracle/_ref/x265la8 $E720 --preset medium -o /tmp/c.hevc \
    > gpurun_out/r05/a_check.log 2>&1 || { tail -20 gpurun_out/r05/a_check.log; exit 1; }
grep -E "check|stats|service|worker time" gpurun_out/r05/a_check.log
echo "ME check bitstream: $(md5sum < /tmp/c.hevc | cut -c1-8)"
X265AMD_LA_PROPAGATE=1 X265AMD_LOOKAHEAD=check X265AMD_LA_STATS=1 timeout -k 10 150 oracle/_ref/x265la8 $E720 --preset medium \
    -o /tmp/p.hevc > gpurun_out/r05/a_check_propagate.log 2>&1 || { tail -20 gpurun_out/r05/a_check_propagate.log; exit 1; }
grep -E "check|stats propagate" gpurun_out/r05/a_check_propagate.log
echo "propagate check bitstream: $(md5sum < /tmp/p.hevc | cut -c1-8)"
# --preset slow: STAR, subme 3 (chroma SATD on the device through the chroma session)
timeout -k 10 150 oracle/_ref/x265ref8 $E720 --preset slow -o /tmp/r720s.hevc > /dev/null 2>&1 || exit 1
X265AMD_ME=check X265AMD_ME_MIN=1024 timeout -k 10 170 oracle/_ref/x265la8 $E720 --preset slow -o /tmp/cs.hevc \
    > gpurun_out/r05/a_check_slow.log 2>&1 || { tail -20 gpurun_out/r05/a_check_slow.log; exit 1; }
grep -E "check|stats|service|worker time" gpurun_out/r05/a_check_slow.log
echo "slow check bitstream: $(md5sum < /tmp/cs.hevc | cut -c1-8) reference $(md5sum < /tmp/r720s.hevc | cut -c1-8)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
echo "2160p source ready"
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 --preset medium --pools 16 --no-info"
for rep in 1 2; do
  for v in "0 0 4096" "2 1 4096" "2 1 1024"; do
    set -- $v
    X265AMD_MES_LAUNCHERS=$1 X265AMD_ME_ASYNC=$2 X265AMD_ME_MIN=$3 X265AMD_ME_STATS=1 timeout -k 10 150 oracle/_ref/x265la8 \
        $E4K -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "rep=$rep launchers=$1 async=$2 min=$3: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/a_encoder_ab.txt
    grep -E "worker time|service" /tmp/e.txt | tee -a gpurun_out/r05/a_encoder_ab.txt
  done
  timeout -k 10 150 oracle/_ref/x265ref8 $E4K -o /tmp/r.hevc > /tmp/e.txt 2>&1 || exit 1
  echo "rep=$rep reference: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/r.hevc | cut -c1-8)" | tee -a gpurun_out/r05/a_encoder_ab.txt
done
X265AMD_ME_STATS=1 timeout -k 10 150 oracle/_ref/x265la8s $E4K -o /tmp/s.hevc > gpurun_out/r05/a_cu_stats_la8s_default.txt 2>&1 || exit 1
grep -E "CU:|x265me" gpurun_out/r05/a_cu_stats_la8s_default.txt | head -30
