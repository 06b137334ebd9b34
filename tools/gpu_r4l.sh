#!/bin/bash
# Round 4: batched XXH64 without per-round selects on whole chunks -- parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_integrity.py tests/test_gpu_big.py tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4l.log 2>&1 || { tail -30 gpurun_out/pytest_r4l.log; exit 1; }
tail -1 gpurun_out/pytest_r4l.log
for i in 1 2; do
  for lib in ab_libs/xsel/libnkfs_crt.so nkfs_amd/lib/libnkfs_crt.so; do
    echo "== $lib"
    NKFS_LIB=$lib timeout -k 10 200 python tools/kbench.py w2 clu 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
