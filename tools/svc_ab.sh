#!/bin/bash
# A/B of the per-call digest path: the round-6 library before (ab_libs/svc_old) and after the service /
# chain changes, same box, interleaved.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/svc_ab.txt
: > $out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_csum.py > gpurun_out/svc_ab_pytest.log 2>&1
echo "csum tests ok" >> $out
for rep in 1 2; do
  for lib in ab_libs/svc_old/libnkfs_crt.so nkfs_amd/lib/libnkfs_crt.so; do
    for m in 0 2; do
      echo "== rep $rep lib $lib svc $m" >> $out
      PERCALL_SVC=$m timeout -k 10 120 ./tools/percall $lib "svc$m" 2>&1 > /tmp/pc.txt; grep -E "csum|4096 B" /tmp/pc.txt >> $out
    done
  done
done
NKFS_SVC_TRACE=1 PERCALL_SVC=2 timeout -k 10 120 ./tools/percall nkfs_amd/lib/libnkfs_crt.so trace2 >> $out 2>&1
echo done >> $out
