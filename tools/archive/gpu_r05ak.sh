# round 5: smoke() on the round's final tree
set -o pipefail
mkdir -p gpurun_out/r05/ak
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/ak/smoke.log 2>&1 || { tail -20 gpurun_out/r05/ak/smoke.log; exit 1; }
tail -n 1 gpurun_out/r05/ak/smoke.log | cut -c1-200
