set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_CONFIGS="c2 c5" bash tools/round_artifacts.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_c5.log 2>&1 || { tail -20 gpurun_out/prof_c5.log; exit 1; }
tail -1 gpurun_out/prof_c5.log
timeout -k 10 400 python bench.py --config c5 --pcie > gpurun_out/bench_c5_full.log 2>&1 || { tail -20 gpurun_out/bench_c5_full.log; exit 1; }
tail -1 gpurun_out/bench_c5_full.log
