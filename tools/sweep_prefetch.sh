#!/bin/bash
# encode prefetch-depth sweep (NKFS_ENC_PREFETCH) per config
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for c in ${CONFIGS:-c2 c4}; do
  for p in ${PS:-1 2 3}; do
    NKFS_ENC_PREFETCH=$p timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/sw_${c}_$p.log 2>&1 || { echo fail $c $p; tail -5 gpurun_out/sw_${c}_$p.log; exit 1; }
    tail -1 gpurun_out/sw_${c}_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c P=$p value', d['value'], 'enc', d['roofline']['achieved'], d['roofline']['us_per_launch'], 'dec', d['decode']['achieved_GBps'], d['verified'])"
  done
done
