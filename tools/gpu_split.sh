#!/bin/bash
# Ragged encode split A/B (C5) across builds, ragged parity tests on each split build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in nkfs_amd/lib/libnkfs_crt.so ab_libs/*/libnkfs_crt.so; do
  echo "== $lib"
  NKFS_LIB="$lib" AB_ROUNDS=5 timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
import nkfs_amd._lib as l; l.LIB_PATH = '$lib'
sys.argv = ['ab_tune', 'c5', '--', 'dec_kernel=0']
import ab_tune; ab_tune.main()" 2>&1 | grep -v amdgpu.ids || exit 1
done
