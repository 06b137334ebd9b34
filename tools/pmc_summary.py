"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel name.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md §HBM), so the summary also prints 2x FETCH_SIZE."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    return vals


out = {}
for d in sys.argv[1:]:
    for (k, c), v in load(d).items():
        out.setdefault(k, {})[c] = sum(v) / len(v)
for k, cs in sorted(out.items(), key=lambda kv: -sum(kv[1].values())):
    if not any(s in k for s in ("k_encode", "k_decode", "k_hash", "k_xxh", "k_synth")):
        continue
    f = cs.get("FETCH_SIZE", 0) * 1024
    w = cs.get("WRITE_SIZE", 0) * 1024
    print(f"{k[:70]:70s} FETCH {f/1e6:10.1f} MB (x2 {2*f/1e6:10.1f})  WRITE {w/1e6:10.1f} MB")
