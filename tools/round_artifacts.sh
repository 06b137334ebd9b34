#!/bin/bash
# Produce the round's committed evidence: default bench line (with CPU
# baseline and PCIe-inclusive rate), rocprofv3 kernel stats of the same
# command, PMC traffic per config.   bash tools/round_artifacts.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --pcie > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- \
  python3 bench.py --no-cpu > gpurun_out/prof_default.log 2>&1 || { tail -20 gpurun_out/prof_default.log; exit 1; }
tail -1 gpurun_out/prof_default.log
for c in ${PMC_CONFIGS:-c2 c3 c4}; do bash tools/pmc.sh $c || exit 1; done
