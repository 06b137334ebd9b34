#!/bin/bash
# C5 ragged GET from host memory: run decoder (auto) vs the ragged slice grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for t in "dec_kernel=0" "dec_kernel=1" "dec_kernel=2" "dec_kernel=0" ; do
  echo "== $t"
  timeout -k 10 200 python -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
from nkfs_amd import _lib
k, v = '$t'.split('=')
_lib.lib(); _lib.check(_lib.lib().nkfs_gpu_init(0))
import pcie_bench
with _lib.tuned(**{k: int(v)}):
    sys.argv = ['pcie_bench', 'c5']
    pcie_bench.main()
" 2>&1 | grep -v amdgpu.ids || exit 1
done
