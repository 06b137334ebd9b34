"""Is the ragged path itself slower, or the size mix?  The same N8K5 1 MiB
stripes encoded (+XXH64) through the uniform and the ragged entry points,
then the C5 mix's 1 MiB stripes alone and together with its small ones.

    python tools/ragged_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402


def ragged(sizes, n, k, first=0):
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes.tolist()):
        boff[s], poff[s] = pos, ppos
        pos += (B + 255) // 256 * 256
        ppos += n * batch.part_pitch(B, k)
    blocks = torch.empty(pos, dtype=torch.uint8, device="cuda")
    blocks.random_(0, 256)
    ids = torch.from_numpy(synth.batch_ids(len(sizes), n, first=first)).cuda()
    parts = torch.empty(ppos, dtype=torch.uint8, device="cuda")
    dig = torch.empty(len(sizes) * n, dtype=torch.int64, device="cuda")
    bo, po = torch.from_numpy(boff).cuda(), torch.from_numpy(poff).cuda()
    sz = torch.from_numpy(sizes.astype(np.int32)).cuda()
    nbytes = int(sizes.sum()) + n * sum(batch.part_size(int(B), k) for B in sizes) + 8 * n * len(sizes)
    t = timeit(lambda: batch.encode_ragged(blocks, bo, sz, n, k, ids, parts, po, dig, int(sizes.max())), 5)
    return t, nbytes


def main():
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    n, k, B = 8, 5, 1048576
    for S in (2048, 3840):
        blocks = batch.synth(S, B)
        ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
        parts = torch.empty((S * n, batch.part_pitch(B, k)), dtype=torch.uint8, device="cuda")
        dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
        nb = S * (B + n * batch.part_size(B, k) + 8 * n)
        t = timeit(lambda: batch.encode(blocks, B, n, k, ids, parts, dig), 5)
        print(f"uniform {S} x 1 MiB        {t*1e6:9.1f} us {nb/t/1e9:7.1f} GB/s", flush=True)
        del blocks, parts
        torch.cuda.empty_cache()
        t, nb = ragged(np.full(S, B, np.uint32), n, k)
        print(f"ragged  {S} x 1 MiB        {t*1e6:9.1f} us {nb/t/1e9:7.1f} GB/s", flush=True)
        torch.cuda.empty_cache()
    sizes = synth.mixed_sizes(11520, (4096, 65536, 1048576))
    for split in ("0", "1", "2", "0", "1", "2"):
        os.environ["NKFS_ENC_SPLIT"] = split  # read per call by the dispatch
        t, nb = ragged(sizes, n, k)
        print(f"ragged  C5 mix ({len(sizes)}) split={split} {t*1e6:9.1f} us {nb/t/1e9:7.1f} GB/s", flush=True)
    os.environ.pop("NKFS_ENC_SPLIT")
    big = sizes[sizes == 1048576]
    t, nb = ragged(big, n, k)
    print(f"ragged  C5 big only ({len(big)}) {t*1e6:9.1f} us {nb/t/1e9:7.1f} GB/s", flush=True)
    small = sizes[sizes != 1048576]
    t, nb = ragged(small, n, k)
    print(f"ragged  C5 small only ({len(small)}) {t*1e6:9.1f} us {nb/t/1e9:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
