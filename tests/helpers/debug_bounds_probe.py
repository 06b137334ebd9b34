"""Run under the debug-bounds build (NKFS_LIB=nkfs_amd/lib/debug/
libnkfs_crt.so, `make DEBUG_BOUNDS=1`) by tests/test_gpu_debug_bounds.py,
in a process of its own (the library path is read at import).

The exact geometry of the round-3 GPU fault: N8K5 ragged
host PUT then GET of a 1 MiB + 1 B + 70,001 B + mixed batch (29 stripes),
block gap 24, part gap 48, one 32 MiB sub-batch; then the same stripes at
sub-batches of 1 MiB and 100,000 B.  The ragged walk encoder and the
ragged slice decoder of this build check every stripe's block and part
range against the caller's buffers (nkfs_geom.blocks_bytes / parts_bytes)
and print "nkfs bounds: ..." for a stripe that would leave them.  Outputs
are checked against the oracle (the test's checker, crt/nk8.c restated).
Prints "debug-bounds ok" at the end."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (binds the library to torch's HIP runtime)

from nkfs_amd import _lib, batch, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

SENT = 0xA5


def layout(sizes, n, k, block_gap, part_gap):
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos
        pos += int(B) + block_gap
        ppos += n * batch.part_pitch(int(B), k) + part_gap
    return boff, poff, pos, ppos


def main():
    assert os.path.realpath(_lib.LIB_PATH).endswith(os.path.join("lib", "debug", "libnkfs_crt.so")), _lib.LIB_PATH
    L = _lib.lib()
    assert L.nk8_init() == 0
    n, k = 8, 5
    sizes = synth.mixed_sizes(29)
    sizes[:3] = (1048576, 1, 70001)
    boff, poff, pos, ppos = layout(sizes, n, k, 24, 48)
    host = np.full(pos, SENT, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(900 + s, int(B))
    ids = synth.batch_ids(len(sizes), n, first=900)
    want = [[O.xxh64(p) for p in O.encode(host[boff[s]: boff[s] + B], n, k, ids[s])] for s, B in enumerate(sizes)]
    for chunk in (0, 1 << 20, 100000):
        parts = np.full(ppos, SENT, np.uint8)
        dig = np.zeros(len(sizes) * n, np.int64)
        batch.encode_ragged_host(host, boff, sizes.astype(np.int32), n, k, ids, parts, poff, dig, chunk_bytes=chunk)
        got = [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig]
        for s in range(len(sizes)):
            assert got[s * n:(s + 1) * n] == want[s], ("digests", chunk, s)
        rng = np.random.default_rng(chunk)
        avail = np.stack([rng.permutation(n) for _ in sizes]).astype(np.uint8)
        out = np.full(pos, SENT, np.uint8)
        status = np.full(len(sizes), 7, np.int32)
        assert batch.decode_ragged_host(parts, poff, n, ids, avail, n, k, out, boff, sizes.astype(np.int32),
                                        status=status, chunk_bytes=chunk) == 0
        assert (status == 0).all(), status
        assert np.array_equal(out, host), ("decode", chunk)
        print(f"chunk {chunk}: PUT + GET of {len(sizes)} stripes exact", flush=True)
    print("debug-bounds ok", flush=True)


if __name__ == "__main__":
    main()
