#!/bin/bash
# Round-3 evidence: GPU tests, default bench line (CPU baselines), rocprofv3
# kernel stats of the same command, PMC traffic (PMC_CONFIGS), dispatch-seam
# sweep under rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- \
  python3 bench.py --no-cpu > gpurun_out/prof_default.log 2>&1 || { tail -20 gpurun_out/prof_default.log; exit 1; }
for c in ${PMC_CONFIGS:-c5 c3}; do bash tools/pmc.sh $c || exit 1; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_seam -o run -- \
  python3 -u tools/seam_sweep.py > gpurun_out/seam_sweep.txt 2>&1 || { tail -20 gpurun_out/seam_sweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/seam_sweep.txt | tail -40
