"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel name.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR [--json out.json --config c2]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM),
so HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE; --json records that
for the encode and decode kernels under the config name (bench.py reads it
as roofline.traffic)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    return vals


ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--json")
ap.add_argument("--config")
ap.add_argument("--stripes", type=int, default=0, help="per-GPU stripes of the profiled run (bench --stripes)")
a = ap.parse_args()
out = {}
for d in a.dirs:
    for (k, c), v in load(d).items():
        out.setdefault(k, {})[c] = sum(v) / len(v)
rec = {}
for k, cs in sorted(out.items(), key=lambda kv: -sum(kv[1].values())):
    if not any(s in k for s in ("k_encode", "k_decode", "k_hash", "k_xxh", "k_synth")):
        continue
    f = cs.get("FETCH_SIZE", 0) * 1024
    w = cs.get("WRITE_SIZE", 0) * 1024
    print(f"{k[:70]:70s} FETCH {f/1e6:10.1f} MB (x2 {2*f/1e6:10.1f})  WRITE {w/1e6:10.1f} MB")
    # one encode (decode) call may be several kernels (a ragged batch split
    # by part size: k_encode_ws + k_encode_fast, each launched once per call),
    # so the per-call traffic is the sum of their per-dispatch means; the
    # batched XXH64 of the parts (k_xxh64_*) belongs to the encode call of the
    # general n, k path (nk8_wide.hip encodes, then hashes the parts)
    for kind in ("encode", "decode"):
        if f"k_{kind}" in k or (kind == "encode" and "k_xxh64" in k):
            rec[f"{kind}_kernel"] = (rec[f"{kind}_kernel"] + " + " + k) if f"{kind}_kernel" in rec else k
            for key, val in ((f"{kind}_bytes_per_launch", 2 * f + w), (f"{kind}_fetch_size_x2", 2 * f),
                             (f"{kind}_write_size", w)):
                rec[key] = rec.get(key, 0) + int(val)
if a.json and a.config:
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import CONFIGS
    # bench.py uses the figure only for this per-GPU batch size
    rec["stripes"] = a.stripes or CONFIGS[a.config][0]
    doc = {}
    if os.path.exists(a.json):
        doc = json.load(open(a.json))
    doc[f"{a.config}@{a.stripes}" if a.stripes else a.config] = rec
    json.dump(doc, open(a.json, "w"), indent=1, sort_keys=True)
