"""Debug: walk encoder vs fused encoder vs oracle on small shapes; prints
where parts / digests differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nkfs_amd import _lib, batch, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

L = _lib.lib()
_lib.check(L.nkfs_gpu_init(0))
for (S, B, n, k) in [(2500, 8192, 8, 5), (2500, 10240, 8, 5), (2500, 4096, 8, 5), (5000, 8192, 4, 2), (2100, 9999, 8, 5)]:
    blocks = batch.synth(S, B)
    ids_np = synth.batch_ids(S, n)
    print("ids", ids_np[-1].tolist())
    ids = torch.from_numpy(ids_np).cuda()
    ps = batch.part_size(B, k)
    res = {}
    for name, kern in (("fused", 2), ("walk", 1)):
        with _lib.tuned(enc_kernel=kern):
            parts, dig = batch.encode(blocks, B, n, k, ids)
            torch.cuda.synchronize()
            res[name] = (parts[:, :ps].cpu().numpy(), [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig.cpu().tolist()])
    bn = blocks[:, :B].cpu().numpy()
    for name in res:
        bad_p, bad_d = [], []
        for s in range(S):
            want = O.encode(bn[s], n, k, ids_np[s])
            for i in range(n):
                got = res[name][0][s * n + i]
                if not np.array_equal(got, want[i]):
                    diff = np.nonzero(got != want[i])[0]
                    bad_p.append((s, i, int(diff[0]), int(diff[-1]), len(diff)))
                if res[name][1][s * n + i] != O.xxh64(want[i]):
                    bad_d.append((s, i))
        print("   bad stripes", sorted(set(x[0] for x in bad_p))[:20], "bad dig stripes", sorted(set(x[0] for x in bad_d))[:20])
        for (s, i, *_r) in bad_p[:0]:
            got = res[name][0][s * n + i]
            for s2 in range(S):
                for variant in range(2):
                    idv = ids_np[s2].copy()
                    if variant:
                        idv = np.roll(ids_np[s2], 4)
                    w2 = O.encode(bn[s], n, k, idv)
                    for i2 in range(n):
                        if np.array_equal(got, w2[i2]):
                            print(f"   stripe {s} part {i} == oracle with ids of stripe {s2} roll {variant} part {i2}")
            zero = ids_np[s].copy(); zero[4:] = 0
            print("   ", got[:8].tolist(), O.encode(bn[s], n, k, ids_np[s])[i][:8].tolist(), bn[s][:10].tolist())
        print(f"S={S} B={B} n={n} k={k} ps={ps} {name}: bad parts {bad_p[:6]} ({len(bad_p)}) bad digests {bad_d[:6]} ({len(bad_d)})",
              flush=True)
