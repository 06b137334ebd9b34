#!/bin/bash
# SQ counter passes (<= 8 SQ counters per pass, one rocprofv3 run each) over
# any short command; summary via tools/pmc_ratios.py.
#   bash tools/pmc_sq_cmd.sh <tag> python3 tools/enc_probe.py c3 enc_kernel=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=$1; shift
passes=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
 "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SALU"
 "GRBM_GUI_ACTIVE GRBM_COUNT SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d gpurun_out/sq_${tag}_$i -o run -- "$@" \
    > gpurun_out/sq_${tag}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_${tag}_$i.log; exit 1; }
done
python3 tools/pmc_ratios.py gpurun_out/sq_${tag}_* | tee gpurun_out/sq_${tag}_summary.txt
