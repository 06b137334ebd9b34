"""Mean of every PMC counter per kernel across rocprofv3 csv dirs."""
import csv
import glob
import os
import sys
from collections import defaultdict

vals = defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
per = defaultdict(dict)
for (k, c), v in vals.items():
    per[k][c] = sum(v) / len(v)
for k in sorted(per):
    if not any(s in k for s in ("k_encode", "k_decode", "k_hash", "k_xxh")):
        continue
    print(k[:90])
    for c in sorted(per[k]):
        print(f"   {c:32s} {per[k][c]:18.1f}")
