"""Per-basic-block instruction histogram of one kernel in a hipcc -save-temps
.s file:  python tools/isa_blocks.py file.s kernel_substring [top_blocks]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
want = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 4
m = re.search(r"^([^\n:]*" + re.escape(want) + r"[^\n:]*):", s, re.M)
start = m.end()
end = s.index("s_endpgm", start)
body = s[start:end]
blocks = re.split(r"^(\.LBB[0-9_]+):", body, flags=re.M)
res = []
label = "entry"
for part in blocks:
    if part.startswith(".LBB"):
        label = part
        continue
    ops = collections.Counter(re.findall(r'^\s+([a-z_][a-z_0-9]*)', part, re.M))
    res.append((sum(ops.values()), label, ops))
for n, label, ops in sorted(res, key=lambda x: -x[0])[:top]:
    print(f"{label}: {n} instrs: " + ", ".join(f"{k} {v}" for k, v in ops.most_common(16)))
