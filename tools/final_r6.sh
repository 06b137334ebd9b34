#!/bin/bash
# Round-6 final evidence on the shipped build: GPU suite, smoke, bench line,
# SQ counters of the final W2 encoder/decoder.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final2.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_final2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final2.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final2.log 2>&1 || { tail -5 gpurun_out/smoke_final2.log; exit 1; }
tail -1 gpurun_out/smoke_final2.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final2.log 2>&1 || { tail -20 gpurun_out/bench_final2.log; exit 1; }
tail -1 gpurun_out/bench_final2.log | cut -c1-160
bash tools/sq_vp.sh w2 "enc_bign=-1" w2final || exit 1
grep -A4 "k_encode_bign\|k_decode_bign" gpurun_out/sq_w2final_summary.txt
