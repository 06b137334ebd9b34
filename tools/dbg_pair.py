"""Diagnose the k = 2 pair decoder on a ragged batch: which bytes differ from
the input, per stripe, for the staged and direct forms and the wave decoder."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nkfs_amd import _lib, batch, synth  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def main():
    L = _lib.lib()
    assert L.nk8_init() == 0
    n, k = 4, 2
    for gap in (0, 3):
        sizes = synth.mixed_sizes(40)
        sizes[:5] = (4096, 1, 3, 1048576, 70001)
        boff = np.zeros(len(sizes), np.int64)
        poff = np.zeros(len(sizes), np.int64)
        pos = ppos = 0
        for s, B in enumerate(sizes):
            boff[s], poff[s] = pos, ppos
            pos += int(B) + gap
            ppos += n * batch.part_pitch(int(B), k)
        host = np.zeros(pos + 16, np.uint8)
        for s, B in enumerate(sizes):
            host[boff[s]: boff[s] + B] = synth.stripe_bytes(700 + s, int(B))
        ids_np = synth.batch_ids(len(sizes), n, first=700)
        parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
        batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff),
                            None, int(sizes.max()))
        avail = synth.batch_survivors(len(sizes), n, 3, first=700)
        for kern, stage, order in (("wave", 1, 1), ("pair", 1, 1), ("pair", 0, 1), ("pair", 1, 0), ("pair", 0, 0)):
            out = torch.zeros(pos + 16, dtype=torch.uint8, device="cuda")
            with _lib.tuned(dec_kernel=_lib.DEC[kern], dec_pair_stage=stage, size_order=order):
                st = batch.decode_ragged(parts, dev(poff), n, dev(ids_np), dev(avail), k, out, dev(boff),
                                         dev(sizes.astype(np.int32)), int(sizes.max()))
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            bad = []
            for s, B in enumerate(sizes):
                d = np.nonzero(got[boff[s]: boff[s] + B] != host[boff[s]: boff[s] + B])[0]
                if len(d):
                    bad.append((s, int(B), len(d), d[:6].tolist(), d[-3:].tolist()))
            print(f"gap {gap} {kern} stage {stage} order {order}: status {int(st.abs().sum())} bad {bad}", flush=True)


if __name__ == "__main__":
    main()
