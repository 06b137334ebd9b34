#!/bin/bash
# Round 4: PCIe link calibration and the host-pipeline sweep (depth x lanes,
# sub-batch size, the few-big-stripes rule) on C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/pcie_bench.py link depth > gpurun_out/pcie_sweep.txt 2>&1 || { tail -20 gpurun_out/pcie_sweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/pcie_sweep.txt
