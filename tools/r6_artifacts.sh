#!/bin/bash
# Round-6 evidence on the current build: rocprofv3 kernel stats of the bench
# command and PMC HBM traffic of the configs whose kernels changed.
#   PMC_CONFIGS="w2 w3" bash tools/r6_artifacts.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6 -o run -- \
  python3 bench.py --no-cpu > gpurun_out/prof_r6.log 2>&1 || { tail -20 gpurun_out/prof_r6.log; exit 1; }
tail -1 gpurun_out/prof_r6.log | cut -c1-300
for c in ${PMC_CONFIGS:-w2 w3}; do bash tools/pmc.sh $c || exit 1; done
