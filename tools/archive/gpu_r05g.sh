# round 5: (0) search-kernel parity of the tree's lib (sub-pel compare out of line with its state as values,
# DPP group reductions); (1) the method-mapping check tests; (2) search-kernel variants in the 2160p medium
# encode, interleaved, 2 reps: tree (by-value call, 4 units per round trip, DPP), nodpp (LDS shuffles), ku2
# (2 units per round trip for 64-lane groups), a657 (state by reference), ded9 (one unit per round trip)
set -o pipefail
mkdir -p gpurun_out/r05/g
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_me.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05/g/parity.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/g/parity.log | head; tail -20 gpurun_out/r05/g/parity.log; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/r05/g/parity.log)"
python3 -c "
from src.x265_amd.synth import SyntheticSource
SyntheticSource(3840, 2160, 64, 8).write_yuv('/tmp/s2160.yuv')" || exit 1
E4K="--input /tmp/s2160.yuv --input-res 3840x2160 --fps 30 --pools 16 --no-info --frames 64 --preset medium"
for rep in 1 2; do
  for v in tree nodpp ku2 a657 ded9; do
    LP=""
    [ $v != tree ] && LP=$PWD/src/x265_amd/ab/$v
    LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} X265AMD_ME_STATS=1 timeout -k 10 150 oracle/_ref/x265la8 $E4K \
        -o /tmp/o.hevc > /tmp/e.txt 2>&1 || { tail -5 /tmp/e.txt; exit 1; }
    echo "$v rep=$rep: $(grep encoded /tmp/e.txt) $(md5sum < /tmp/o.hevc | cut -c1-8)" | tee -a gpurun_out/r05/g/me_ab.txt
    grep -E "worker time|service" /tmp/e.txt | tee -a gpurun_out/r05/g/me_ab.txt
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -v --timeout 400 --timeout-method thread \
    -k "search_methods or slow_check" > gpurun_out/r05/g/methods.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/g/methods.log | head; tail -30 gpurun_out/r05/g/methods.log; exit 1; }
echo "methods: $(tail -n 1 gpurun_out/r05/g/methods.log)"
