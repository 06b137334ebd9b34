#!/bin/bash
# Round 4: full seam sweep (encoder families incl. two hash waves, decoders) on this box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
SWEEP_ENC=auto,walk,fused,ws,ws2 SWEEP_ROUNDS=3 timeout -k 10 1000 python -u tools/seam_sweep.py > gpurun_out/seam_sweep_r04.txt 2>&1 || { tail -5 gpurun_out/seam_sweep_r04.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/seam_sweep_r04.txt
