#!/bin/bash
# Round 4: GPU suite on the two-hash-wave default, then PMC traffic of the
# configs whose kernel changed (C3 and its strong shards, C4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
cp profiles/traffic.json gpurun_out/traffic.json
bash tools/pmc.sh c3 > /dev/null || exit 1
bash tools/pmc.sh c4 > /dev/null || exit 1
for s in 1024 2048 4096; do bash tools/pmc.sh c3 $s > /dev/null || exit 1; done
tail -n 3 gpurun_out/pmc_*_summary.txt
