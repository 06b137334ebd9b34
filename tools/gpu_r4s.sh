#!/bin/bash
# Round 4: k > 16 encode with the XXH64 pass overlapped on a side stream -- parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4s.log 2>&1 || { tail -30 gpurun_out/pytest_r4s.log; exit 1; }
tail -1 gpurun_out/pytest_r4s.log
AB_NODEC=1 AB_ROUNDS=5 timeout -k 10 400 python -u tools/ab_tune.py w2 1024:1048576:48:32 64:4194304:40:33 -- "enc_big_overlap=0" "enc_big_overlap=2,enc_big_hash_form=1" "enc_big_overlap=4,enc_big_hash_form=1" "enc_big_overlap=8,enc_big_hash_form=1" "enc_big_overlap=4,enc_big_hash_form=2" "enc_big_overlap=8,enc_big_hash_form=2" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_big_overlap.txt || { cat gpurun_out/ab_big_overlap.txt; exit 1; }
cat gpurun_out/ab_big_overlap.txt
