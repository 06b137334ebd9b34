#!/bin/bash
# C5 probe: GPU parity tests, ragged probe (uniform vs ragged, split on/off),
# C5 bench line.   bash tools/probe_c5.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/ragged_probe.py > gpurun_out/probe_split.txt 2>&1 || { cat gpurun_out/probe_split.txt; exit 1; }
cat gpurun_out/probe_split.txt
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log
