# f1 in the running encoder on the GPU box: per-estimate check, stats, bit-exactness and timing
set -o pipefail
mkdir -p gpurun_out
python3 -c "
import sys; sys.path.insert(0,'.')
from src.x265_amd.synth import SyntheticSource
SyntheticSource(1920,1080,64,8).write_yuv('/tmp/s1080_64.yuv')
"
X=oracle/_ref
ENC="--input /tmp/s1080_64.yuv --input-res 1920x1080 --fps 30 --preset medium --pools 16 --no-info"
if [ "${CHECK:-1}" = 1 ]; then
  timeout -k 10 300 env X265AMD_LOOKAHEAD=check $X/x265la8 $ENC -F 2 --frames ${NCHK:-24} -o /tmp/chk.hevc > gpurun_out/la_check.log 2>&1
  rc=$?; echo "check rc=$rc mismatches=$(grep -c 'CHECK MISMATCH' gpurun_out/la_check.log)"; grep "MISMATCH\|fatal\|check:" gpurun_out/la_check.log | head -20
  test $rc = 0 || exit 1
fi
for F in ${FLIST:-2 0}; do
for b in x265ref8 x265la8; do
  FF=""; test $F = 0 || FF="-F $F"
  timeout -k 10 300 env X265AMD_LA_STATS=1 $X/$b $ENC $FF --frames 64 -o /tmp/$b.hevc > gpurun_out/la_${b}_F$F.log 2>&1 || exit 1
  echo "== $b -F $F"; grep "frame threads\|stats\|encoded" gpurun_out/la_${b}_F$F.log; md5sum /tmp/$b.hevc
done
done
