#!/bin/bash
# Round 4: wide decoder with 12-byte LDS reads (k <= 12) vs 16-byte; C5 ragged
# encode with two hash waves on the ws share.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4j.log 2>&1 || { tail -30 gpurun_out/pytest_r4j.log; exit 1; }
tail -1 gpurun_out/pytest_r4j.log
AB_NODEC= AB_ROUNDS=5 bash tools/ab_two_libs.sh ab_libs/nob96/libnkfs_crt.so nkfs_amd/lib/libnkfs_crt.so w1 -- "dec_kernel=0" > gpurun_out/ab_w1_b96.txt 2>&1 || { cat gpurun_out/ab_w1_b96.txt; exit 1; }
cat gpurun_out/ab_w1_b96.txt
AB_NODEC=1 AB_ROUNDS=5 timeout -k 10 300 python -u tools/ab_tune.py c5 -- "enc_kernel=0" "enc_ragged_split=32768" "enc_ragged_split=8192" "enc_kernel=3" "enc_kernel=3,enc_ws_hash_waves=1" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_c5_ws2.txt || { cat gpurun_out/ab_c5_ws2.txt; exit 1; }
cat gpurun_out/ab_c5_ws2.txt
