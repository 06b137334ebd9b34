#!/bin/bash
# Round 4: k_decode_prep (k > 8 plans) with first-offer selection and log-sum
# denominators -- parity, then its kernel time on W1/W2 decodes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_prep -o run -- python3 tools/kbench.py w2 w1 > gpurun_out/prof_prep.log 2>&1 || { tail -20 gpurun_out/prof_prep.log; exit 1; }
python3 tools/grid_stats.py gpurun_out/prof_prep/run_kernel_trace.csv | grep -i "prep\|decode_big\|decode_wide" | cut -c1-200
grep -v amdgpu.ids gpurun_out/prof_prep.log | grep "decode"
