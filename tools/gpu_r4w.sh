#!/bin/bash
# Round 4: tiny k >= 3 uniform decodes on the wave decoder -- suite, then the seam.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SWEEP_ENC=auto SWEEP_DEC=auto,slice,wave SWEEP_SHAPES=mid SWEEP_ROUNDS=3 timeout -k 10 600 python -u tools/seam_sweep.py 2>&1 | grep -v amdgpu.ids > gpurun_out/seam_dec_mid.txt || { tail -5 gpurun_out/seam_dec_mid.txt; exit 1; }
cat gpurun_out/seam_dec_mid.txt
