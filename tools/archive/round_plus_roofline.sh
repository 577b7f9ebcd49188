# GPU suite + smoke + default bench line (tools/gpu_round.sh), then the kernel-roofline rows of $1
set -o pipefail
bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "${1:-dct_16,dct_32,idct_16,idct_32,tu_pipeline}" > gpurun_out/roofline_sel.jsonl 2> gpurun_out/roofline_sel.err || { tail -20 gpurun_out/roofline_sel.err; exit 1; }
grep "{" gpurun_out/roofline_sel.jsonl | cut -c1-200
