# round 5: the sad_x4 8x8 default (lane per reference, one 8x8 unit, non-temporal) on the roofline tool, then the
# whole GPU suite and smoke on the round's final tree
set -o pipefail
mkdir -p gpurun_out/r05/y
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/kernel_roofline.py --only sad_x4,sad_8x8 2>/dev/null | grep "{" | cut -c1-200 \
    | sed "s/^/rep=$rep /" | tee -a gpurun_out/r05/y/sadx_default.txt || exit 1
done
bash tools/gpu_r05t.sh || exit 1
mkdir -p gpurun_out/r05/y/t && cp gpurun_out/r05/t/* gpurun_out/r05/y/t/
