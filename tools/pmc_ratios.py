"""Derived ratios from tools/pmc_sq.sh output dirs (relative, for A/B)."""
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
    if not any(s in k for s in ("k_encode", "k_decode", "k_xxh")):
        continue
    p = per[k]
    wc = p.get("SQ_WAVE_CYCLES", 1)
    cyc = p.get("GRBM_GUI_ACTIVE", 1) / 8  # per XCD
    simd_cycles = cyc * 1024
    print(f"{k[:60]:60s} waves {p.get('SQ_WAVES',0):8.0f}  kernel {cyc/1e6:6.2f} Mcyc/XCD")
    print(f"   wave time: active {p.get('SQ_ACTIVE_INST_ANY',0)/wc:5.1%}  wait(waitcnt/barrier) {p.get('SQ_WAIT_ANY',0)/wc:5.1%}"
          f"  issue-stall {p.get('SQ_WAIT_INST_ANY',0)/wc:5.1%}")
    print(f"   VALU busy ~{2*p.get('SQ_INSTS_VALU',0)/simd_cycles:5.1%}  LDS active/CU ~{p.get('SQ_LDS_IDX_ACTIVE',0)/256/cyc:5.1%}"
          f"  LDS conflict share {p.get('SQ_LDS_BANK_CONFLICT',0)/max(1,p.get('SQ_LDS_IDX_ACTIVE',1)):5.1%}"
          f"  avg waves/CU {p.get('SQ_WAVE_CYCLES',0)*4/256/cyc:5.1f}")
    print(f"   insts per wave: VALU {p.get('SQ_INSTS_VALU',0)/p.get('SQ_WAVES',1):8.0f}  LDS {p.get('SQ_INSTS_LDS',0)/p.get('SQ_WAVES',1):7.0f}"
          f"  SALU {p.get('SQ_INSTS_SALU',0)/p.get('SQ_WAVES',1):7.0f}  VMEM rd {p.get('SQ_INSTS_VMEM_RD',0)/p.get('SQ_WAVES',1):6.0f} wr {p.get('SQ_INSTS_VMEM_WR',0)/p.get('SQ_WAVES',1):6.0f}"
          f"  vmem in flight/CU {p.get('SQ_INST_LEVEL_VMEM',0)/256/cyc:5.1f}")
