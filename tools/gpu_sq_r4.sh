#!/bin/bash
# SQ counters (4 passes each) of the C3 encoder/decoder, the C2 decoder and
# the C5 ragged encoder/decoder, for profiles/r04.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_sq.sh c3 || exit 1
bash tools/pmc_sq.sh c2 || exit 1
bash tools/pmc_sq.sh c5 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu || exit 1
echo done
