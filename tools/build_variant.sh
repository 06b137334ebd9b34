#!/bin/bash
# Build an experiment variant of libnkfs_crt.so into ab_libs/<name>/ (ships to the GPU box) that
# differs from the in-tree build only in the listed HIP sources, compiled
# with extra flags:  bash tools/build_variant.sh <name> "<flags>" nk8_ws.hip [...]
set -e
name=$1; flags=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
obj=/tmp/ab_obj_$name
rm -rf "$obj" && cp -a "$root/nkfs_amd/build" "$obj"
for f in "$@"; do rm -f "$obj/${f%.hip}.o"; done
make -s -C "$root/nkfs_amd/csrc" OUTDIR="$root/ab_libs/$name" OBJDIR="$obj" BASEOBJ="$obj" EXTRA_HIPFLAGS="$flags"
echo "built ab_libs/$name/libnkfs_crt.so"
