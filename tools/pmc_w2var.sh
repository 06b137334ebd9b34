#!/bin/bash
# W2 encode HBM traffic per variant: FETCH_SIZE / WRITE_SIZE passes over tools/enc_probe.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  for ctr in FETCH_SIZE WRITE_SIZE; do
    NKFS_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/w2v_${tag}_$ctr -o run -- \
      python3 tools/enc_probe.py w2 "$@" reps=3 > gpurun_out/w2v_${tag}_$ctr.log 2>&1 || { echo "fail $tag $ctr"; tail -5 gpurun_out/w2v_${tag}_$ctr.log; exit 1; }
  done
  echo "== $tag"; python3 tools/pmc_summary.py gpurun_out/w2v_${tag}_FETCH_SIZE gpurun_out/w2v_${tag}_WRITE_SIZE --config w2 | grep -i "encode"
}
for v in ${W2VARIANTS:-hash}; do
  case $v in
    hash) run hash nkfs_amd/lib/libnkfs_crt.so enc_bign=1 || exit 1 ;;
    nohash) run nohash nkfs_amd/lib/libnkfs_crt.so enc_bign=1 nohash || exit 1 ;;
    unit) run unit nkfs_amd/lib/libnkfs_crt.so enc_bign=2 || exit 1 ;;
    old) run old nkfs_amd/lib/libnkfs_crt.so enc_bign=0 enc_big_fused=1 || exit 1 ;;
    *) run $v ab_libs/$v/libnkfs_crt.so enc_bign=1 || exit 1 ;;
  esac
done
