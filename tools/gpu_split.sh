#!/bin/bash
# A/B across builds: ragged encode split (C5, split* builds) and the batched
# XXH64 ring pass (W2, ring* builds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_lib.py nkfs_amd/lib/libnkfs_crt.so ab_libs/ring*/libnkfs_crt.so w2 2>&1 | grep -v amdgpu.ids || exit 1
for lib in nkfs_amd/lib/libnkfs_crt.so ab_libs/split*/libnkfs_crt.so; do
  echo "== $lib"
  AB_ROUNDS=5 timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
import nkfs_amd._lib as l; l.LIB_PATH = '$lib'
sys.argv = ['ab_tune', 'c5', '--', 'dec_kernel=0']
import ab_tune; ab_tune.main()" 2>&1 | grep -v amdgpu.ids || exit 1
done
