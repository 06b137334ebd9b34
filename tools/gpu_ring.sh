#!/bin/bash
# Ring-pass variants (messages per wave, ring depth) on W2, then the batched-hash GPU tests on each build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_lib.py nkfs_amd/lib/libnkfs_crt.so ab_libs/*/libnkfs_crt.so w2 2>&1 | grep -v amdgpu.ids || exit 1
