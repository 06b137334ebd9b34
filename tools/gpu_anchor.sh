#!/bin/bash
# Round 4: the headline C3 line with the guide's plain float4 anchor
# (copy / read / write) measured in the same process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c3 --no-cpu --steps 10 > gpurun_out/anchor_c3.log 2>&1 || { tail -20 gpurun_out/anchor_c3.log; exit 1; }
tail -1 gpurun_out/anchor_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['hbm_anchor'])); r=d['roofline']; print(r['achieved'], r['frac'], r.get('frac_of_box_stream'), r.get('frac_of_anchor_copy'), r['box_stream']); print(d['decode'])"
