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

Round 6 adds the round-5 fault's geometry: N6K3 page-list
PUT/GET of 26 mixed stripes (1 MiB, 1 B, 512 B, 513 B, ...) in 512-byte
pages at 200,000-byte sub-batches; and a 4,096-stripe ragged N8K5 batch of
small blocks in one sub-batch, so the persistent warp-specialised encoder
(k_encode_wsp) and the run decoder (k_decode_run), both range-checked in
this build, run with the pipeline's buffer bounds.  Pageable buffers are
staged, pinned ones DMA'd directly: both kinds run.
Prints "debug-bounds ok" at the end."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (binds the library to torch's HIP runtime)

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

    # round 5's fault geometry: page lists, N6K3, 200,000-byte sub-batches
    n, k, page, chunk = 6, 3, 512, 200000
    rng = np.random.default_rng(page + n)
    sizes = synth.mixed_sizes(26)
    sizes[:4] = (1048576, 1, page, page + 1)
    blocks = [synth.stripe_bytes(2000 + s, int(B)) for s, B in enumerate(sizes)]
    npg = [max(1, -(-int(B) // page)) for B in sizes]
    arena = np.full(sum(npg) * page, SENT, np.uint8)
    slots = rng.permutation(sum(npg))
    pages = np.zeros(sum(npg), np.int64)
    first = np.zeros(len(sizes), np.int64)
    q = 0
    for s, b in enumerate(blocks):
        first[s] = q
        for i in range(npg[s]):
            pages[q] = arena.ctypes.data + int(slots[q]) * page
            c = b[i * page:(i + 1) * page]
            arena[int(slots[q]) * page: int(slots[q]) * page + len(c)] = c
            q += 1
    ids = synth.batch_ids(len(sizes), n, first=2000)
    _, poff, _, ppos = layout(sizes, n, k, 0, 16)
    sz32 = sizes.astype(np.int32)
    parts = np.full(ppos, SENT, np.uint8)
    dig = np.zeros(len(sizes) * n, np.int64)
    assert batch.encode_pages(pages, page, first, sz32, n, k, ids, parts, poff, dig, chunk_bytes=chunk) == 0
    for s in range(len(sizes)):
        want = [O.xxh64(p) for p in O.encode(blocks[s], n, k, ids[s])]
        assert [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig[s * n:(s + 1) * n]] == want, ("pages digests", s)
    avail = np.stack([rng.permutation(n)[:k] for _ in sizes]).astype(np.uint8)
    arena[:] = SENT
    status = np.full(len(sizes), 3, np.int32)
    assert batch.decode_pages(parts, poff, n, ids, avail, k, k, pages, page, first, sz32, status=status,
                              chunk_bytes=chunk) == 0
    assert (status == 0).all(), status
    for s, b in enumerate(blocks):
        got = np.concatenate([arena[int(pages[first[s] + i]) - arena.ctypes.data:][:page] for i in range(npg[s])])
        assert np.array_equal(got[:len(b)], b), ("pages decode", s)
    print("round-5 geometry (pages N6K3, 200,000-B sub-batches): PUT + GET exact", flush=True)

    # one 4,096-stripe ragged sub-batch: k_encode_wsp + k_decode_run under bounds
    n, k = 8, 5
    rng = np.random.default_rng(6)
    sizes = rng.integers(1, 12000, 4096).astype(np.int64)  # ~24 MB: one 32 MiB sub-batch
    boff, poff, pos, ppos = layout(sizes, n, k, 8, 16)
    for pinned in (False, True):
        if pinned:
            host = torch.empty(pos, dtype=torch.uint8, pin_memory=True).numpy()
            parts = torch.empty(ppos, dtype=torch.uint8, pin_memory=True).numpy()
            out = torch.empty(pos, dtype=torch.uint8, pin_memory=True).numpy()
        else:
            host, parts, out = (np.empty(pos, np.uint8), np.empty(ppos, np.uint8), np.empty(pos, np.uint8))
        host[:] = SENT
        for s, B in enumerate(sizes):
            host[boff[s]: boff[s] + B] = synth.stripe_bytes(7000 + s, int(B))
        ids = synth.batch_ids(len(sizes), n, first=7000)
        dig = np.zeros(len(sizes) * n, np.int64)
        batch.encode_ragged_host(host, boff, sizes.astype(np.int32), n, k, ids, parts, poff, dig, chunk_bytes=0)
        for s in range(0, len(sizes), 97):
            want = [O.xxh64(p) for p in O.encode(host[boff[s]: boff[s] + sizes[s]], n, k, ids[s])]
            assert [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig[s * n:(s + 1) * n]] == want, ("wsp digests", s)
        avail = np.stack([rng.permutation(n) for _ in sizes]).astype(np.uint8)
        out[:] = SENT
        status = np.full(len(sizes), 7, np.int32)
        assert batch.decode_ragged_host(parts, poff, n, ids, avail, n, k, out, boff, sizes.astype(np.int32),
                                        status=status, chunk_bytes=0) == 0
        assert (status == 0).all()
        assert np.array_equal(out, host), ("run decode", pinned)
        print(f"4,096-stripe ragged sub-batch ({'pinned' if pinned else 'pageable'}): PUT + GET exact", flush=True)
    print("debug-bounds ok", flush=True)


if __name__ == "__main__":
    main()
