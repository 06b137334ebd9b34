#!/bin/bash
# GPU-box check: parity tests, bench per config, optional rocprofv3 kernel trace.
#   bash tools/gpu_check.sh [tests] [bench] [prof]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what="${*:-tests bench}"
if [[ " $what " == *" tests "* ]]; then
  timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { echo "PYTEST FAILED rc=$rc"; exit $rc; }
fi
if [[ " $what " == *" bench "* ]]; then
  for c in ${CONFIGS:-c2 c3 c4}; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$c.log 2>&1 \
      || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
    tail -1 gpurun_out/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:20], 'value', d['value'], 'enc GB/s', d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['us_per_launch'], 'dec', d['decode'], d['verified'])"
  done
fi
if [[ " $what " == *" prof "* ]]; then
  for c in ${PROF_CONFIGS:-c2}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o run -- \
      python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_$c.log 2>&1 \
      || { echo "prof $c failed"; tail -20 gpurun_out/prof_$c.log; exit 1; }
    find gpurun_out/prof_$c -name "*kernel_stats.csv" | head -1 | xargs -r head -8
  done
fi
