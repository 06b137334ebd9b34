#!/bin/bash
# bench.py --config <c> with two builds of the library on one box, interleaved:
#   bash tools/ab_bench_libs.sh <libA.so> <libB.so> <config> [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
a=$1; b=$2; c=$3; r=${4:-2}
for i in $(seq $r); do
  for lib in "$a" "$b"; do
    timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0, '.')
import nkfs_amd._lib as l; l.LIB_PATH = '$lib'
sys.argv = ['bench.py', '--config', '$c', '--no-cpu']
import io, contextlib
buf = io.StringIO()
with contextlib.redirect_stdout(buf):
    import bench; bench.main()
d = json.loads(buf.getvalue().strip().splitlines()[-1])
print('$lib'.split('/')[-2], '$c', d['value'], 'enc', d['roofline']['achieved'], 'dec', d['decode']['achieved_GBps'])
" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
