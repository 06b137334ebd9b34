#!/bin/bash
# Round 4: wide_ws encoder with two chunks of loads in flight -- parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4m.log 2>&1 || { tail -30 gpurun_out/pytest_r4m.log; exit 1; }
tail -1 gpurun_out/pytest_r4m.log
AB_NODEC=1 AB_ROUNDS=5 timeout -k 10 400 python -u tools/ab_tune.py w1 256:1048576:20:16 4096:262144:12:8 c3 -- "enc_ws_prefetch=1" "enc_ws_prefetch=2" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_wide_pf.txt || { cat gpurun_out/ab_wide_pf.txt; exit 1; }
cat gpurun_out/ab_wide_pf.txt
