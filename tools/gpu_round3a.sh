#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/percall nkfs_amd/lib/libnkfs_crt.so mi355x > gpurun_out/percall.txt 2>&1 || exit 1
timeout -k 10 120 tools/percall oracle/_ref/libnkfs_ref.so reference >> gpurun_out/percall.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
