#!/bin/bash
# Produce the round's committed evidence: default bench line (all configs,
# CPU baselines), rocprofv3 kernel stats of the same command, PMC traffic
# per config (one counter per pass).   bash tools/round_artifacts.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# progress marker for the box's hang detector (the bench prints one line at the end)
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- \
  python3 bench.py --no-cpu > gpurun_out/prof_default.log 2>&1 || { tail -20 gpurun_out/prof_default.log; exit 1; }
tail -1 gpurun_out/prof_default.log | cut -c1-300
for c in ${PMC_CONFIGS:-c3 c2 c4 c5 w1}; do bash tools/pmc.sh $c || exit 1; done
