# round 5: non-temporal loads of the 8-bit interpolation windows (the ntinterp A/B library, built with
# X265AMD_NT_INTERP=1): parity of the interp goldens with it, the kernel roofline of hpp / vpp / hvpp and
# the census replay with and without, interleaved, 2 reps
set -o pipefail
mkdir -p gpurun_out/r05/o
export TMPDIR=/tmp
NTL=$PWD/src/x265_amd/ab/libx265amd_ntinterp.so
X265AMD_LIB=$NTL timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not fullsize" > gpurun_out/r05/o/parity.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05/o/parity.log | head; tail -20 gpurun_out/r05/o/parity.log; exit 1; }
echo "parity (ntinterp lib): $(tail -n 1 gpurun_out/r05/o/parity.log)"
ONLY=luma_hpp,luma_vpp,luma_hvpp
for rep in 1 2; do
  for v in tree ntinterp; do
    unset X265AMD_LIB
    [ $v = ntinterp ] && export X265AMD_LIB=$NTL
    echo "== $v rep=$rep" | tee -a gpurun_out/r05/o/interp_nt_ab.txt
    timeout -k 10 300 python3 -u tools/kernel_roofline.py --only "$ONLY" 2>/dev/null | grep "{" | cut -c1-190 \
        | tee -a gpurun_out/r05/o/interp_nt_ab.txt || exit 1
    timeout -k 10 300 python3 -u -c "
import json
from src.x265_amd.replay_bench import primitive_workload
r = primitive_workload()
print(json.dumps({'census_replay_fps': r.get('fps'), 'ms_per_step': r.get('ms_per_step')}))" 2>/dev/null | grep census | tee -a gpurun_out/r05/o/interp_nt_ab.txt || exit 1
  done
done
unset X265AMD_LIB
