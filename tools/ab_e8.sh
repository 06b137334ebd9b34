set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
AB_TUNE=enc_nib=0 timeout -k 10 200 python -u tools/ab_lib.py ab_libs/cur/libnkfs_crt.so ab_libs/e8/libnkfs_crt.so c2 2>&1 | grep -v amdgpu.ids
AB_TUNE=enc_nib=1 timeout -k 10 200 python -u tools/ab_lib.py ab_libs/cur/libnkfs_crt.so ab_libs/e8/libnkfs_crt.so c2 2>&1 | grep -v amdgpu.ids
