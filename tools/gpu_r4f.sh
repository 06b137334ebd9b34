#!/bin/bash
# Round 4: pair decoder with 4 waves per workgroup -- parity, then C2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_pair_decode_matches" "tests/test_gpu_parity.py::test_pair_decode_ragged" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4f.log 2>&1 || { tail -30 gpurun_out/pytest_r4f.log; exit 1; }
tail -1 gpurun_out/pytest_r4f.log
AB_NODEC= AB_ROUNDS=7 timeout -k 10 300 python -u tools/ab_tune.py c2 -- "dec_kernel=0" "dec_kernel=7,dec_pair_waves=4,dec_pair_stage=1" "dec_kernel=7,dec_pair_waves=4,dec_pair_stage=0" "dec_kernel=7,dec_pair_waves=1,dec_pair_stage=0" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_c2_pair4.txt || { cat gpurun_out/ab_c2_pair4.txt; exit 1; }
cat gpurun_out/ab_c2_pair4.txt
