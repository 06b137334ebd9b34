#!/bin/bash
# Same tune variants through two builds of libnkfs_crt.so on one box:
#   bash tools/ab_two_libs.sh <libA.so> <libB.so> <configs...> -- <variants...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
a=$1; b=$2; shift 2
for lib in "$a" "$b"; do
  echo "== $lib"
  AB_NODEC=${AB_NODEC-1} AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
import nkfs_amd._lib as l; l.LIB_PATH = '$lib'
sys.argv = ['ab_tune'] + sys.argv[1:]
import ab_tune; ab_tune.main()" "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
