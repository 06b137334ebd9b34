#!/bin/bash
# Round 4, first box: the GPU suite on the hardened build (private scratch
# pool, pipeline scratch, pin registry), then the C3 line with the guide's
# float4 anchor.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_anchor.sh
