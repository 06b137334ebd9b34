#!/bin/bash
# SQ/GRBM counter passes (<= 8 SQ counters per pass) over tools/kbench.py.
#   bash tools/pmc_sq.sh c4                      (tools/kbench.py c4)
#   bash tools/pmc_sq.sh c5 python3 bench.py ...  (any program after the name)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
c=${1:-c4}
shift
cmd=("$@")
[ ${#cmd[@]} -eq 0 ] && cmd=(python3 tools/kbench.py "$c")
passes=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
 "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SALU"
 "GRBM_GUI_ACTIVE GRBM_COUNT SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d gpurun_out/sq_${c}_$i -o run -- \
    "${cmd[@]}" > gpurun_out/sq_${c}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_${c}_$i.log; exit 1; }
done
python3 tools/pmc_all.py gpurun_out/sq_${c}_? > gpurun_out/sq_${c}_raw.txt
python3 tools/pmc_ratios.py gpurun_out/sq_${c}_? | tee gpurun_out/sq_${c}_summary.txt
