set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo PYTEST_RC=$? >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
for c in c2 c3 c4; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }; tail -1 gpurun_out/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:20], d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['us_per_launch'], d['decode'], d['verified'])"; done
