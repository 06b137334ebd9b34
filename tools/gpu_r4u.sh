#!/bin/bash
# Round 4 final build: PMC traffic of the configs on the warp-specialised encoders.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cp profiles/traffic.json gpurun_out/traffic.json
bash tools/pmc.sh c3 > /dev/null || exit 1
bash tools/pmc.sh c4 > /dev/null || exit 1
for s in 1024 2048 4096; do bash tools/pmc.sh c3 $s > /dev/null || exit 1; done
head -n 1 gpurun_out/pmc_c3_summary.txt gpurun_out/pmc_c4_summary.txt gpurun_out/pmc_c3_1024_summary.txt gpurun_out/pmc_c3_2048_summary.txt gpurun_out/pmc_c3_4096_summary.txt | cut -c1-160
