# round 5: (0) search-kernel parity after the STAR out-of-range-origin fix and the load-first sub-pel
# compare (tests/test_me.py incl. the far-MVP cases); (1) 720p check mode for STAR / slow / UMH / veryslow;
# (2) 2160p medium 64 frames, service counters (kernel ms per launch against 0.092 before), twice;
# (3) 2160p slow 16 frames hooked against the unhooked build, bitstream md5
set -o pipefail
mkdir -p gpurun_out/r05/e
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_me.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/e/parity.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/e/parity.log | head; tail -20 gpurun_out/r05/e/parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/r05/e/parity.log)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(1280, 720, 16, 8).write_yuv('/tmp/s720.yuv')
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
E720="--input /tmp/s720.yuv --input-res 1280x720 --fps 30 --frames 16 --no-info --pools 16"
for v in "--preset medium --me star" "--preset slow" "--preset medium --me umh" "--preset veryslow"; do
  X265AMD_ME=check X265AMD_ME_MIN=1024 timeout -k 10 200 oracle/_ref/x265la8 $E720 $v -o /tmp/c.hevc \
      > /tmp/c.log 2>&1 || { tail -20 /tmp/c.log; exit 1; }
  echo "== $v: $(grep -E 'mismatching searches|windows beyond' /tmp/c.log | tr '\n' ' ')" | tee -a gpurun_out/r05/e/check.txt
  grep MISMATCH /tmp/c.log | head -4 | tee -a gpurun_out/r05/e/check.txt
done
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info"
for rep in 1 2; do
  X265AMD_ME_STATS=1 timeout -k 10 150 oracle/_ref/x265la8 $E4K --frames 64 --preset medium -o /tmp/o.hevc > /tmp/e.txt 2>&1 \
      || { tail -5 /tmp/e.txt; exit 1; }
  echo "medium rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/e/medium.txt
  grep -E "worker time|service" /tmp/e.txt | tee -a gpurun_out/r05/e/medium.txt
done
X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 $E4K --frames 16 --preset slow -o /tmp/s1.hevc > /tmp/s1.txt 2>&1 \
    || { tail -5 /tmp/s1.txt; exit 1; }
X265AMD_ME=cpu X265AMD_LOOKAHEAD=cpu timeout -k 10 300 oracle/_ref/x265la8 $E4K --frames 16 --preset slow -o /tmp/s0.hevc > /tmp/s0.txt 2>&1 \
    || { tail -5 /tmp/s0.txt; exit 1; }
echo "slow 16f hooked: $(grep encoded /tmp/s1.txt) $(md5sum < /tmp/s1.hevc | cut -c1-8)" | tee -a gpurun_out/r05/e/slow.txt
echo "slow 16f host:   $(grep encoded /tmp/s0.txt) $(md5sum < /tmp/s0.hevc | cut -c1-8)" | tee -a gpurun_out/r05/e/slow.txt
grep -E "worker time|service|stats" /tmp/s1.txt | tee -a gpurun_out/r05/e/slow.txt
