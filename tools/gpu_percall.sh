#!/bin/bash
# GPU suite, then the per-call drop-in cost of each build (tools/percall.c) and the reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for lib in nkfs_amd/lib/libnkfs_crt.so ab_libs/*/libnkfs_crt.so oracle/_ref/libnkfs_ref.so; do
  [ -f "$lib" ] || continue
  timeout -k 10 120 tools/percall $lib $(basename $(dirname $lib)) 2>&1 | grep -v "^sink" || exit 1
done | tee gpurun_out/percall.txt
