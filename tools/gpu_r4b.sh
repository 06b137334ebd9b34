#!/bin/bash
# Round 4: the changed GPU tests, then the ws encoder's 2-deep load prefetch
# A/B on C3 / C4 shapes (same process, interleaved rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_csum.py tests/test_gpu_host.py "tests/test_gpu_parity.py::test_bench_kernels_against_oracle" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4b.log 2>&1 || { tail -30 gpurun_out/pytest_r4b.log; exit 1; }
tail -1 gpurun_out/pytest_r4b.log
AB_NODEC=1 AB_ROUNDS=5 timeout -k 10 400 python -u tools/ab_tune.py c3 c4 -- "enc_kernel=0" "enc_kernel=0,enc_ws_prefetch=2" "enc_kernel=3" "enc_kernel=3,enc_ws_prefetch=2" "enc_kernel=1" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_ws_pf.txt || { cat gpurun_out/ab_ws_pf.txt; exit 1; }
cat gpurun_out/ab_ws_pf.txt
