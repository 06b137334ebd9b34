#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_lib.py nkfs_amd/lib/libnkfs_crt.so ab_libs/*/libnkfs_crt.so 1024:1048576:8:5 2048:1048576:8:5 4096:524288:8:5 512:262144:8:5 2>&1 | grep -v amdgpu.ids || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python tools/pcie_bench.py c2 c3 c4 c5 pages lanes 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pcie.txt
