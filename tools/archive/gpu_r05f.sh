# round 5: the search-method mapping (x265 UMH 2 / STAR 3 against the kernel's STAR 2 / UMH 3) in check mode
# for star / umh / dia / veryslow and --preset slow with chroma SATD, through the GPU tests
set -o pipefail
mkdir -p gpurun_out/r05/f
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_encoder_me.py -m gpu -x -v --timeout 400 --timeout-method thread \
    -k "search_methods or slow_check" > gpurun_out/r05/f/methods.log 2>&1 \
    || { grep -E "FAILED|Error|assert" gpurun_out/r05/f/methods.log | head; tail -30 gpurun_out/r05/f/methods.log; exit 1; }
echo "methods: $(tail -1 gpurun_out/r05/f/methods.log)"
