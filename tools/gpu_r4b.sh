#!/bin/bash
# Round 4: the changed GPU tests, then A/B of the fused k > 16 encoder (W2),
# the k = 2 pair decoder (C2), the ragged size-class split (C5), the ws
# encoder's 2-deep load prefetch (C3 / C4), same process, interleaved
# rounds; then the PCIe link calibration and the host-pipeline depth sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_csum.py tests/test_gpu_host.py "tests/test_gpu_parity.py::test_bench_kernels_against_oracle" "tests/test_gpu_parity.py::test_pair_decode_matches" "tests/test_gpu_parity.py::test_pair_decode_ragged" "tests/test_gpu_parity.py::test_c5_bench_scale_default_dispatch" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4b.log 2>&1 || { tail -30 gpurun_out/pytest_r4b.log; exit 1; }
tail -1 gpurun_out/pytest_r4b.log
ab() {  # ab <out> <nodec> <configs...> -- <variants...>
  local out=$1 nodec=$2; shift 2
  AB_NODEC=$nodec AB_ROUNDS=5 timeout -k 10 300 python -u tools/ab_tune.py "$@" 2>&1 | grep -v amdgpu.ids > gpurun_out/$out || { cat gpurun_out/$out; return 1; }
  cat gpurun_out/$out
}
ab ab_w2_fused.txt 1 w2 -- "enc_big_unfused=0" "enc_big_unfused=1" || exit 1
ab ab_c2_pair.txt 0 c2 -- "dec_kernel=0" "dec_kernel=7,dec_pair_stage=1" "dec_kernel=7,dec_pair_stage=0" || exit 1
ab ab_c5_split.txt 0 c5 -- "enc_kernel=0" "enc_kernel=0,enc_ragged_split=32768" "enc_kernel=0,enc_ragged_split=8192" "enc_kernel=3" || exit 1
ab ab_ws_pf.txt 1 c3 c4 -- "enc_kernel=0" "enc_kernel=0,enc_ws_prefetch=2" "enc_kernel=0,enc_ws_waves=6" "enc_kernel=0,enc_ws_waves=6,enc_ws_prefetch=2" "enc_kernel=3,enc_ws_prefetch=2" "enc_kernel=1" || exit 1
timeout -k 10 400 python -u tools/pcie_bench.py link c3 depth c5 > gpurun_out/pcie_r4.txt 2>&1 || { tail -20 gpurun_out/pcie_r4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/pcie_r4.txt
