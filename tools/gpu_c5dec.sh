#!/bin/bash
# ragged slice decoder check: GPU suite, C5 decode slice vs wave A/B, C5 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c5dec_tests.txt 2>&1 || { tail -30 gpurun_out/c5dec_tests.txt; exit 1; }
tail -1 gpurun_out/c5dec_tests.txt
AB_NODEC=0 timeout -k 10 300 python -u tools/ab_tune.py c5 -- "dec_kernel=1" "dec_kernel=2" "dec_kernel=1,dec_units=4" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_c5dec.txt || { cat gpurun_out/ab_c5dec.txt; exit 1; }
cat gpurun_out/ab_c5dec.txt
timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-700
