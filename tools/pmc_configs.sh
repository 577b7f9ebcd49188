# FETCH_SIZE / WRITE_SIZE passes over the census steps of the other BASELINE configs (one pass each)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "3840 2160 8 slow" "3840 2160 8 medium" "3840 2160 10 medium"; do
  set -- $cfg
  tag="${2}p_${4}_${3}bit"
  args="--width $1 --height $2 --depth $3 --preset $4"
  rm -rf gpurun_out/pf_$tag gpurun_out/pw_$tag
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf_$tag -o run -- python3 tools/pmc_workload.py $args --order gpurun_out/po_$tag.json > gpurun_out/pf_$tag.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw_$tag -o run -- python3 tools/pmc_workload.py $args --order gpurun_out/po_$tag.json > gpurun_out/pw_$tag.log 2>&1 || exit 1
  echo "$tag ok"
done
