#!/bin/bash
# Run decoder check: its parity tests, then decoder A/B (VARIANTS) on CONFIGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${TESTS:-run_decode or slice_decode or bench_kernels or ragged}" > gpurun_out/run_tests.txt 2>&1 || { tail -30 gpurun_out/run_tests.txt; exit 1; }
tail -2 gpurun_out/run_tests.txt
AB_ROUNDS=5 timeout -k 10 400 python -u tools/ab_tune.py ${CONFIGS:-c5} -- ${VARIANTS:-"dec_kernel=0" "dec_kernel=1"} 2>&1 \
  | grep -v amdgpu.ids > gpurun_out/ab_run.txt || { cat gpurun_out/ab_run.txt; exit 1; }
cat gpurun_out/ab_run.txt
