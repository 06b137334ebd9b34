"""A/B of plain vs non-temporal stores in one process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  python tools/ab_nt.py c2 c4"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from kbench import timeit  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402

L = _lib.lib()
_lib.check(L.nkfs_gpu_init(0))
for name in sys.argv[1:] or ["c2"]:
    S, B, n, k, _ = CONFIGS[name]
    ps = batch.part_size(B, k)
    blocks = batch.synth(S, B)
    ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
    avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
    parts = torch.empty((S * n, batch.part_pitch(B, k)), dtype=torch.uint8, device="cuda")
    dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
    out = torch.empty((S, B), dtype=torch.uint8, device="cuda")
    st = torch.empty(S, dtype=torch.int32, device="cuda")
    enc_b = S * (B + n * ps + 8 * n)
    dec_b = S * (k * ps + B + k)
    res = {}
    for rnd in range(4):
        for nt in ("0", "1"):
            os.environ["NKFS_STORE_NT"] = nt
            te = timeit(lambda: batch.encode(blocks, B, n, k, ids, parts, dig), 10)
            td = timeit(lambda: batch.decode(parts, n, ids, avail, k, B, out=out, status=st), 10)
            res.setdefault(nt, []).append((enc_b / te / 1e9, dec_b / td / 1e9))
    for nt, v in res.items():
        e = sorted(x[0] for x in v)
        d = sorted(x[1] for x in v)
        print(f"{name} NT={nt} encode GB/s median {e[len(e)//2]:.0f} (min {e[0]:.0f} max {e[-1]:.0f})  "
              f"decode median {d[len(d)//2]:.0f} (min {d[0]:.0f} max {d[-1]:.0f})")
    del blocks, parts, out
    torch.cuda.empty_cache()
