set -e
for cfg in "0 0" "4096 0" "768 0" "0 256" "0 1024" "4096 1024" "0 0"; do
  set -- $cfg
  echo "== BPAD=$1 PPAD=$2"
  AB_BPAD=$1 AB_PPAD=$2 timeout -k 10 200 python -u tools/ab_lib.py nkfs_amd/lib/libnkfs_crt.so c3 c4 2>&1 | grep -v amdgpu.ids
done
