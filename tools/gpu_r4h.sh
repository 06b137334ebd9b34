#!/bin/bash
# Round 4: seam sweep of the two-hash-wave ws encoder against the walk encoder (N8K5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SWEEP_ENC=auto,walk,ws,ws2 SWEEP_DEC= SWEEP_SHAPES=n8 SWEEP_ROUNDS=3 timeout -k 10 900 python -u tools/seam_sweep.py 2>&1 | grep -v amdgpu.ids > gpurun_out/seam_ws2.txt || { tail -5 gpurun_out/seam_ws2.txt; exit 1; }
cat gpurun_out/seam_ws2.txt
