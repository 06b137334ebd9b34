#!/bin/bash
# Round 4: copy/kernel timeline of the host PUT/GET pipeline (C3, 1 GiB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trace_put -o run -- \
  python3 tools/pcie_bench.py c3 > gpurun_out/trace_put.log 2>&1 || { tail -20 gpurun_out/trace_put.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_put.log | tail -2
ls gpurun_out/trace_put
