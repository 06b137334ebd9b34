#!/bin/bash
# Round 4: pair-decoder ragged diagnosis, then the A/Bs and the PCIe sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg_pair.py 2>&1 | grep -v amdgpu.ids > gpurun_out/dbg_pair.txt || { cat gpurun_out/dbg_pair.txt; exit 1; }
cat gpurun_out/dbg_pair.txt
ab() {  # ab <out> <nodec: 1 = encode only, "" = both> <configs...> -- <variants...>
  local out=$1 nodec=$2; shift 2
  AB_NODEC=$nodec AB_ROUNDS=5 timeout -k 10 300 python -u tools/ab_tune.py "$@" 2>&1 | grep -v amdgpu.ids > gpurun_out/$out || { cat gpurun_out/$out; return 1; }
  cat gpurun_out/$out
}
ab ab_w2_fused.txt 1 w2 -- "enc_big_unfused=0" "enc_big_unfused=1" || exit 1
ab ab_c2_pair.txt "" c2 -- "dec_kernel=0" "dec_kernel=7,dec_pair_stage=1" "dec_kernel=7,dec_pair_stage=0" || exit 1
timeout -k 10 400 python -u tools/pcie_bench.py link c2 c3 c4 c5 pages > gpurun_out/pcie_r4.txt 2>&1 || { tail -20 gpurun_out/pcie_r4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/pcie_r4.txt
