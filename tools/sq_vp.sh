#!/bin/bash
# SQ / SQC counter passes over tools/kbench.py for one config with a tune
# override (the VALU encoder's A/B evidence).  bash tools/sq_vp.sh w2 "enc_bign=3" tag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
c=${1:-w2}
export KB_TUNE="${2:-enc_bign=3}"
tag=${3:-vp}
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INST_CYCLES_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d gpurun_out/sq_${tag}_$i -o run -- python3 tools/kbench.py $c > gpurun_out/sq_${tag}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_${tag}_$i.log; exit 1; }
done
python3 tools/pmc_all.py gpurun_out/sq_${tag}_? > gpurun_out/sq_${tag}_raw.txt 2>&1
python3 tools/pmc_ratios.py gpurun_out/sq_${tag}_? > gpurun_out/sq_${tag}_summary.txt 2>&1
