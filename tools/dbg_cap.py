import numpy as np, torch, sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from nkfs_amd import _lib, batch, synth
L = _lib.lib(); assert L.nk8_init() == 0
def dev(a): return torch.from_numpy(np.ascontiguousarray(a)).cuda()
n, k = 48, 32
for gap in (1, 0):
    sizes = synth.mixed_sizes(16)
    sizes[:5] = (4096, 65536, 1048576, 1, k + 1)
    boff = np.zeros(len(sizes), np.int64); poff = np.zeros(len(sizes), np.int64); pos = ppos = 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos; pos += int(B) + gap; ppos += n * batch.part_pitch(int(B), k)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(500 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=500)
    outs = {}
    for eb in (0, 1, 1, 1, 1, 1, 1, 1):
        parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
        dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
        with _lib.tuned(enc_bign=eb):
            batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts,
                                dev(poff), dig, int(sizes.max()))
        torch.cuda.synchronize()
        if eb == 0:
            ref = dig.cpu()
        else:
            bad = (dig.cpu() != ref).nonzero().flatten().tolist()
            print("gap", gap, "sizes", sizes.tolist(), flush=True) if eb == 1 and not outs else None
            outs[len(outs)] = bad
            print("bad", len(bad), sorted({b // n for b in bad}), bad[:12], flush=True)
