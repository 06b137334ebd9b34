#!/bin/bash
# Round 4: decode plan over K lanes per stripe -- suite, plan kernel time, per-call cost.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_plan -o run -- python3 tools/kbench.py 1024:1048576:8:5 c3 > gpurun_out/prof_plan.log 2>&1 || { tail -20 gpurun_out/prof_plan.log; exit 1; }
python3 tools/grid_stats.py gpurun_out/prof_plan/run_kernel_trace.csv | grep -i "plan\|decode_slice" | cut -c1-200
grep -v amdgpu.ids gpurun_out/prof_plan.log | grep "decode"
timeout -k 10 120 tools/percall nkfs_amd/lib/libnkfs_crt.so lib 2>&1 | grep -v "^sink" | grep "split\|assemble"
