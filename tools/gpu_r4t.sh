#!/bin/bash
# Round 4: 6-slot DMA ring for few-wave XXH64 passes -- parity, then A/B against the 4-slot build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_integrity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4t.log 2>&1 || { tail -30 gpurun_out/pytest_r4t.log; exit 1; }
tail -1 gpurun_out/pytest_r4t.log
for i in 1 2; do
  for lib in ab_libs/ring4/libnkfs_crt.so nkfs_amd/lib/libnkfs_crt.so; do
    echo "== $lib"
    NKFS_LIB=$lib timeout -k 10 200 python tools/kbench.py w2 256:1048576:20:17 clu 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
