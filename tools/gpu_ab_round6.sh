#!/bin/bash
# Round-6 A/B of k_encode_bign build knobs (hash waves, hash priority):
# tune variants through each ab_libs/<name> build, then the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
shapes=${SHAPES:-"w2 256:1048576:24:20 512:1048576:20:17"}
for l in ${LIBS:-hw4p3}; do echo "== $l"; AB_NODEC=1 AB_ROUNDS=5 NKFS_LIB=ab_libs/$l/libnkfs_crt.so timeout -k 10 300 python tools/ab_tune.py $shapes -- "enc_bign=-1" "enc_bign=3" 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "== in-tree"
AB_ROUNDS=5 AB_NODEC=1 timeout -k 10 300 python tools/ab_tune.py $shapes -- "enc_bign=-1" 2>&1 | grep -v amdgpu.ids
