#!/bin/bash
# Round 4 evidence after the GPU suite ran in the same call: smoke, default
# bench line, rocprofv3 kernel stats + per-(kernel, grid) summary of the same
# command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- \
  python3 bench.py --no-cpu > gpurun_out/prof_default.log 2>&1 || { tail -20 gpurun_out/prof_default.log; exit 1; }
python3 tools/grid_stats.py gpurun_out/prof_default/run_kernel_trace.csv > gpurun_out/bench_kernel_grid_stats.csv
head -12 gpurun_out/bench_kernel_grid_stats.csv | cut -c1-200
echo done
