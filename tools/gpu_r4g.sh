#!/bin/bash
# Round 4: two hash waves per warp-specialised workgroup -- parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_warp_specialised_encode_matches" "tests/test_gpu_parity.py::test_ragged_kernels_match" "tests/test_gpu_parity.py::test_bench_kernels_against_oracle" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4g.log 2>&1 || { tail -30 gpurun_out/pytest_r4g.log; exit 1; }
tail -1 gpurun_out/pytest_r4g.log
timeout -k 10 60 tools/xxh_rate > gpurun_out/xxh_rate.txt 2>&1 || exit 1
AB_NODEC=1 AB_ROUNDS=7 timeout -k 10 400 python -u tools/ab_tune.py c3 1024:1048576:8:5 c4 -- "enc_ws_hash_waves=1" "enc_ws_hash_waves=2" "enc_ws_hash_waves=2,enc_ws_prefetch=2" "enc_ws_hash_waves=1,enc_kernel=3" "enc_ws_hash_waves=2,enc_kernel=3" 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_ws_hash_waves.txt || { cat gpurun_out/ab_ws_hash_waves.txt; exit 1; }
cat gpurun_out/ab_ws_hash_waves.txt
timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --tune enc_ws_hash_waves=2 > gpurun_out/bench_c3_hw2.log 2>&1 || { tail -5 gpurun_out/bench_c3_hw2.log; exit 1; }
tail -1 gpurun_out/bench_c3_hw2.log | cut -c1-900
AB_NODEC= AB_ROUNDS=7 bash tools/ab_two_libs.sh nkfs_amd/lib/libnkfs_crt.so ab_libs/wpe8/libnkfs_crt.so c2 -- "dec_kernel=0" > gpurun_out/ab_c2_wpe8.txt 2>&1 || { cat gpurun_out/ab_c2_wpe8.txt; exit 1; }
cat gpurun_out/ab_c2_wpe8.txt
