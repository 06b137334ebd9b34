#!/bin/bash
# wide kernels after a change: GPU suite, kbench of the wide shapes, W1 bench sub-config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wide_tests.txt 2>&1 || { tail -30 gpurun_out/wide_tests.txt; exit 1; }
tail -1 gpurun_out/wide_tests.txt
shapes="2048:1048576:16:12 4096:262144:12:8 8192:65536:10:8 1024:1048576:20:16 16384:65536:12:4 1:1048576:8:5 1:1048576:16:12"
timeout -k 10 300 python -u tools/kbench.py $shapes 2>&1 | grep -v amdgpu.ids > gpurun_out/wide_kbench2.txt || exit 1
cat gpurun_out/wide_kbench2.txt
timeout -k 10 300 python -u bench.py --config w1 --steps 10 --no-cpu > gpurun_out/bench_w1.log 2>&1 || { tail -5 gpurun_out/bench_w1.log; exit 1; }
tail -1 gpurun_out/bench_w1.log | cut -c1-900
