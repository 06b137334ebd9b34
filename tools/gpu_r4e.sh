#!/bin/bash
# Round 4: big-encoder tests (fused on every shape), then PMC traffic of the
# strong-scaling C3 shards (per-GPU 1,024 / 2,048 / 4,096 stripes) and of W2
# with XXH64 fused.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4e.log 2>&1 || { tail -30 gpurun_out/pytest_r4e.log; exit 1; }
tail -1 gpurun_out/pytest_r4e.log
bash tools/pmc.sh w2 0 enc_big_fused=1 || exit 1
bash tools/pmc.sh c3 1024 || exit 1
bash tools/pmc.sh c3 2048 || exit 1
bash tools/pmc.sh c3 4096 || exit 1
cat gpurun_out/traffic.json
