#!/bin/bash
# Round 4: nibble tables in the wide fused encoder / wide decoder -- parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4n.log 2>&1 || { tail -30 gpurun_out/pytest_r4n.log; exit 1; }
tail -1 gpurun_out/pytest_r4n.log
AB_NODEC= AB_ROUNDS=5 timeout -k 10 400 python -u tools/ab_tune.py w1 256:1048576:20:16 4096:262144:12:8 2048:1048576:16:10 -- "wide_nib=0" "wide_nib=0,enc_ws_prefetch=2" "wide_nib=1" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_wide_nib.txt || { cat gpurun_out/ab_wide_nib.txt; exit 1; }
cat gpurun_out/ab_wide_nib.txt
