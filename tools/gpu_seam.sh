#!/bin/bash
# GPU tests, then the dispatch-seam sweep (tools/seam_sweep.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python3 -u tools/seam_sweep.py > gpurun_out/seam_sweep.txt 2>&1 || { tail -20 gpurun_out/seam_sweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/seam_sweep.txt
if [ -d ab_libs ]; then
  timeout -k 10 300 python tools/ab_lib.py nkfs_amd/lib/libnkfs_crt.so ab_libs/*/libnkfs_crt.so ${AB_CONFIGS:-c2} 2>&1 | grep -v amdgpu.ids
fi
