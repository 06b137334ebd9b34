#!/bin/bash
# Per-call cost of two builds on one box, interleaved: percall_ab.sh libA libB [SVC mode]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2; do
  for l in "$1" "$2"; do
    PERCALL_SVC=${3:-2} timeout -k 10 120 tools/percall "$l" "$(basename $(dirname $l))" | grep csum || exit 1
  done
done
