#!/bin/bash
# Diagnostics pass: PMC traffic for the given configs and SQ counters for kbench shapes.
#   PMC="w1 w2" SQ="c2" bash tools/gpu_diag.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for c in $PMC; do bash tools/pmc.sh $c || exit 1; done
for c in $SQ; do bash tools/pmc_sq.sh $c || exit 1; done
