#!/bin/bash
# Round 4: ws encoder variants next to this box's 5:8 stream (is there headroom
# above the two-hash-wave kernel on a box whose HBM is faster?); W2 parts hash pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_BOX=1 AB_NODEC=1 AB_ROUNDS=5 timeout -k 10 400 python -u tools/ab_tune.py c3 c4 -- "enc_kernel=3" "enc_kernel=3,enc_ws_prefetch=2" "enc_kernel=3,enc_ws_hash_waves=1" "enc_kernel=3,enc_ws_hash_waves=1,enc_ws_prefetch=2" "enc_kernel=1" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_ws_box.txt || { cat gpurun_out/ab_ws_box.txt; exit 1; }
cat gpurun_out/ab_ws_box.txt
timeout -k 10 120 python tools/kbench.py w2 2>&1 | grep -v amdgpu.ids
