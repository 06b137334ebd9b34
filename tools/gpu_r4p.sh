#!/bin/bash
# Round 4: ws / walk seam below 2,048 stripes (N8K5 20-256 KiB blocks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SWEEP_ENC=auto,walk,ws,ws2 SWEEP_DEC=auto,wave SWEEP_SHAPES=mid SWEEP_ROUNDS=3 timeout -k 10 600 python -u tools/seam_sweep.py > gpurun_out/seam_mid.txt 2>&1 || { tail -5 gpurun_out/seam_mid.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/seam_mid.txt
