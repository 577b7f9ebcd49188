# round 4: coalesced device motion searches (one launch for the PUs of every waiting worker):
# the encoder ME tests (incl. check mode: every device search recomputed on the host), then an
# interleaved 2160p A/B against per-PU launches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_encoder_me.py tests/test_encoder_lookahead.py -x -q -m gpu --timeout 400 --timeout-method thread -s \
    > gpurun_out/r04j_me_tests.log 2>&1 || { tail -30 gpurun_out/r04j_me_tests.log; exit 1; }
grep -E "x265me\]|x265la\]|passed|failed" gpurun_out/r04j_me_tests.log | cut -c1-220
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
for rep in 1 2 3; do
  for co in 1 0; do
    X265AMD_MES_COALESCE=$co X265AMD_ME_STATS=1 timeout -k 10 200 oracle/_ref/x265la8 --input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --frames 64 \
        --preset medium --pools 16 --no-info -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "rep=$rep coalesce=$co: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8) $(grep -o 'prefetches [0-9]*' /tmp/e.txt) $(grep -o '[0-9.]* ms/prefetch' /tmp/e.txt)" | tee -a gpurun_out/r04j_coalesce_ab.txt
  done
done
