#!/bin/bash
# HBM traffic per kernel from PMC counters, one counter per pass (FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950: MI355X_MICROARCH.md §rocprofv3).
#   bash tools/pmc.sh <config> [stripes per GPU] [nkfs_tune k=v,... (tag suffix "t")]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
c=${1:-c2}
st=${2:-0}
tune=${3:-}
extra=""
[ "$st" != 0 ] && extra="--stripes $st --scaling weak"
[ -n "$tune" ] && extra="$extra --tune $tune"
tag=$c; [ "$st" != 0 ] && tag=${c}_$st
[ -n "$tune" ] && tag=${tag}_t
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${tag}_$ctr -o run -- \
    python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu $extra > gpurun_out/pmc_${tag}_$ctr.log 2>&1 \
    || { echo "pmc $ctr failed"; tail -20 gpurun_out/pmc_${tag}_$ctr.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE $( [ -z "$tune" ] && echo "--json gpurun_out/traffic.json" ) --config $c --stripes $st | tee gpurun_out/pmc_${tag}_summary.txt
