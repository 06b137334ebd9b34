#!/bin/bash
# Per-kernel VGPR / scratch / LDS of one built object (nkfs_amd/build/<file>.o):
#   bash tools/kres.sh nk8_walk [name-filter]
B=/opt/rocm/lib/llvm/bin
o=${1:-nk8_walk}; f=${2:-.}
d=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$d/fb "$(dirname "$0")/../nkfs_amd/build/$o.o"
$B/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$d/fb --output=$d/co
$B/llvm-readelf --notes $d/co > $d/notes
python3 - "$d/notes" "$f" <<'PY'
import re, subprocess, sys
t = open(sys.argv[1]).read()
for blk in t.split('- .agpr_count')[1:]:
    g = lambda k: re.search(r'\.' + k + r':\s+(\S+)', blk).group(1)
    dn = subprocess.run(['c++filt', g('name')], capture_output=True, text=True).stdout.strip()
    if re.search(sys.argv[2], dn):
        print(f"{g('vgpr_count'):>4} vgpr {g('sgpr_count'):>4} sgpr {g('private_segment_fixed_size'):>4} scratch "
              f"{g('group_segment_fixed_size'):>6} lds  {dn[:100]}")
PY
rm -rf $d
