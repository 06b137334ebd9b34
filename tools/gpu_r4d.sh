#!/bin/bash
# Round 4: the fused k > 16 encoder with the XCD-local chain hand-off:
# correctness (test_gpu_big, pair tests), then the W2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py "tests/test_gpu_parity.py::test_pair_decode_matches" "tests/test_gpu_parity.py::test_pair_decode_ragged" "tests/test_gpu_parity.py::test_c5_bench_scale_default_dispatch" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4d.log 2>&1 || { tail -30 gpurun_out/pytest_r4d.log; exit 1; }
tail -1 gpurun_out/pytest_r4d.log
AB_NODEC=1 AB_ROUNDS=5 timeout -k 10 300 python -u tools/ab_tune.py w2 -- "enc_big_unfused=0" "enc_big_unfused=1" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_w2_fused.txt || { cat gpurun_out/ab_w2_fused.txt; exit 1; }
cat gpurun_out/ab_w2_fused.txt
