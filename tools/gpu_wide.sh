#!/bin/bash
# wide-encoder check on the GPU box: its parity tests, the rest of the GPU
# suite, then kernel timings of the wide shapes (default vs general kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wide_tests.txt 2>&1 || { tail -30 gpurun_out/wide_tests.txt; exit 1; }
tail -3 gpurun_out/wide_tests.txt
shapes="2048:1048576:16:12 4096:262144:12:8 8192:65536:10:8 1024:1048576:20:16 16384:65536:12:4 1:1048576:8:5 1:1048576:16:12"
timeout -k 10 300 python -u tools/kbench.py $shapes > gpurun_out/wide_kbench.txt 2>&1 || exit 1
KB_TUNE=enc_kernel=4,dec_kernel=3 timeout -k 10 300 python -u tools/kbench.py $shapes > gpurun_out/wide_kbench_generic.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/wide_kbench.txt gpurun_out/wide_kbench_generic.txt
