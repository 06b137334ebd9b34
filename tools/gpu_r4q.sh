#!/bin/bash
# Round 4: GPU suite on the quantization-aware ws rules, then the seams again.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SWEEP_ENC=auto,walk,ws SWEEP_DEC= SWEEP_SHAPES=mid SWEEP_ROUNDS=3 timeout -k 10 600 python -u tools/seam_sweep.py 2>&1 | grep -v amdgpu.ids > gpurun_out/seam_mid2.txt || { tail -5 gpurun_out/seam_mid2.txt; exit 1; }
SWEEP_ENC=auto,walk,ws SWEEP_DEC= SWEEP_SHAPES=n8 SWEEP_ROUNDS=3 timeout -k 10 600 python -u tools/seam_sweep.py 2>&1 | grep -v amdgpu.ids > gpurun_out/seam_n8_2.txt || { tail -5 gpurun_out/seam_n8_2.txt; exit 1; }
cat gpurun_out/seam_mid2.txt gpurun_out/seam_n8_2.txt
