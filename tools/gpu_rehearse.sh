#!/bin/bash
# Round 4: the multi-rank bench path on real GPU kernels -- two ranks sharing
# the box's one GPU, control collectives over gloo (RCCL refuses two ranks
# on one GPU).  Validates rank ranges, per-rank spread, digest all-gather and
# cross-rank check, line composition; the timings are not a measurement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --cpu-seconds 1 \
  > gpurun_out/rehearse_w2.log 2>&1 || { tail -30 gpurun_out/rehearse_w2.log; exit 1; }
tail -1 gpurun_out/rehearse_w2.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('n_gpus', d['n_gpus'], 'value', d['value'], 'verified', d['verified'], 'ranks', d['verified_ranks'], d.get('backend'))
print('workload', d['config']['workload'])
print('per_rank', d['per_rank'])
print('cpu', d['cpu_baseline']['kind'], d['cpu_baseline']['cores'], 'traffic', d['roofline']['traffic'])
for k, v in d['configs'].items(): print(k, v['verified'], v['verified_ranks'], v['per_rank']['encode_us'])
"
