"""GPU parity of the kernels for k > 16: the column-chunked ones
(nk8_big.hip, NKFS_ENC_BIG / NKFS_DEC_BIG) for any n <= 255 and
k <= 254 (crt/nk8.c:13-16; the reference's self test draws k up to 254,
crt/nk8.c:735-744).

Every case is checked bit-exact against the thread-per-row general kernels
(NKFS_ENC_GENERIC / NKFS_DEC_GENERIC) on all stripes and against the oracle
(oracle/nk8_port.c, pinned to the compiled reference) on sampled stripes:
one and several 16-column chunks, part groups of 16 (the last one partial),
k = n, k = 254 / n = 255, tails of every size, unaligned ragged offsets,
one-byte blocks, the small-k shapes pinned to the big kernels, the
first-k-distinct selection and the -EINVAL stripe.  The stage-free encoder
with a hash wave (nk8_bign.hip, k_encode_bign: the default for 16 < k <= 76
with digests, in units of 16 parts up to k = 32 and of 8 parts above; tune
enc_bign = 1 pins it for every k <= 76, with or without digests) is held to
the same cases.
"""
import numpy as np
import pytest

from nkfs_amd import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def L():
    from nkfs_amd import _lib
    lib = _lib.lib()
    assert lib.nk8_init() == 0, "nk8_init (GPU self test) failed"
    return lib


@pytest.fixture(scope="module")
def O():
    from oracle import oracle
    return oracle


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def u64(x):
    return int(x) & 0xFFFFFFFFFFFFFFFF


def _tuned(**kw):
    from nkfs_amd import _lib
    return _lib.tuned(**kw)


@pytest.mark.parametrize("n,k,B,S", [
    (48, 32, 1048576, 3),      # the bench's W2 shape: 2 chunks, 3 groups, slices
    (20, 17, 65536, 10),       # 2 chunks, the second one column wide
    (255, 254, 70001, 2),      # 16 chunks, 16 groups (the last 15 parts wide)
    (40, 33, 4099, 30),        # tail rows, k not a multiple of 4
    (18, 17, 1, 5),            # one-byte blocks
    (64, 50, 1000003, 2),      # B not a multiple of 4 / 16 / k
    (17, 17, 17 * 300 + 5, 7),  # k = n
    (16, 12, 65536, 10),       # k <= 16 pinned to the big kernel
    (8, 5, 4096, 50),          # n <= 8 pinned to the big kernel
    (24, 20, 65543, 5),        # k % 4 == 0: the stage-free encoder's contiguous row loads, tail row
    (30, 24, 24 * 4096, 4),
    (29, 28, 4099, 9),
    # 32 < k <= 76: the stage-free encoder in units of 8 parts (8-byte table entries)
    (64, 41, 1048576, 2),      # the bench's W3 shape
    (77, 76, 4099, 3),         # the largest k of that encoder, 10 part groups
    (100, 75, 65537, 2),       # 13 part groups, the last one 4 parts wide
    (34, 33, 1, 4),            # one-byte blocks
    (45, 36, 36 * 3840 * 2 + 7, 2),  # k % 4 == 0 above 32, slices + a tail row
])
def test_big_encode_matches(L, O, n, k, B, S):
    from nkfs_amd import _lib, batch
    blocks = batch.synth(S, B, first=300 + n)
    ids_np = synth.batch_ids(S, n, first=300 + n)
    ids = dev(ids_np)
    with _tuned(enc_kernel=_lib.ENC["generic"]):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_lib.ENC["big"], enc_big_fused=0):  # the XXH64 pass
        p1, d1 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_lib.ENC["big"], enc_big_fused=1):  # XXH64 fused, chained over the slices
        p3, d3 = batch.encode(blocks, B, n, k, ids)
    p2, d2 = batch.encode(blocks, B, n, k, ids)  # default dispatch
    with _tuned(enc_bign=1):  # the stage-free encoder, hash waves and no-digest forms
        p4, d4 = batch.encode(blocks, B, n, k, ids)
        p5, _ = batch.encode(blocks, B, n, k, ids, digests=False)
    with _tuned(enc_bign=3):  # diagonal (bank-conflict-free) tables at every 16 < k <= 32
        p6, d6 = batch.encode(blocks, B, n, k, ids)
        p7, _ = batch.encode(blocks, B, n, k, ids, digests=False)
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps]) and torch.equal(d0, d1)
    assert torch.equal(p0[:, :ps], p3[:, :ps]) and torch.equal(d0, d3)
    assert torch.equal(p0[:, :ps], p2[:, :ps]) and torch.equal(d0, d2)
    assert torch.equal(p0[:, :ps], p4[:, :ps]) and torch.equal(d0, d4)
    assert torch.equal(p0[:, :ps], p5[:, :ps])
    assert torch.equal(p0[:, :ps], p6[:, :ps]) and torch.equal(d0, d6)
    assert torch.equal(p0[:, :ps], p7[:, :ps])
    got = [u64(x) for x in d1.cpu().tolist()]
    for s in sorted({0, S - 1}):
        want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
        assert np.array_equal(p1[s * n:(s + 1) * n, :ps].cpu().numpy(), np.stack(want)), s
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s


@pytest.mark.parametrize("n,k,gap", [(24, 20, 0), (40, 33, 5), (19, 18, 3), (48, 32, 1), (64, 41, 3), (80, 70, 0)])
def test_big_encode_ragged(L, O, n, k, gap):
    """Ragged batches (mixed sizes, block offsets unaligned when gap != 0):
    the big kernel equals the general kernel, and the oracle per stripe."""
    from nkfs_amd import _lib, batch
    sizes = synth.mixed_sizes(16)
    sizes[:5] = (4096, 65536, 1048576, 1, k + 1)
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos, ppos = 0, 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos
        pos += int(B) + gap
        ppos += n * batch.part_pitch(int(B), k)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(500 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=500)
    outs = []
    for kern, fused, eb in (("generic", 0, 0), ("big", 0, 0), ("big", 1, 0), ("auto", 0, -1), ("auto", 0, 1),
                            ("auto", -1, -1), ("auto", 0, 3)):
        parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
        dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
        with _tuned(enc_kernel=_lib.ENC[kern], enc_big_fused=fused, enc_bign=eb):
            batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts,
                                dev(poff), dig, int(sizes.max()))
        torch.cuda.synchronize()
        outs.append((parts.cpu().numpy(), [u64(x) for x in dig.cpu().tolist()]))
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0]) and outs[0][1] == o[1]
    pn, got = outs[2]
    for s in (0, 2, 3, 4, len(sizes) - 1):
        B = int(sizes[s])
        want = O.encode(host[boff[s]: boff[s] + B], n, k, ids_np[s])
        pitch = batch.part_pitch(B, k)
        for i in range(n):
            off = int(poff[s]) + i * pitch
            assert np.array_equal(pn[off: off + len(want[i])], want[i]), (s, i)
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s


@pytest.mark.parametrize("n,k,B,S", [
    (48, 32, 1048576, 3),      # W2 shape
    (255, 254, 70001, 2),
    (40, 33, 4099, 30),        # rows of 33 bytes: byte-wise band stores
    (20, 17, 1000003, 3),
    (18, 18, 1, 5),            # one-byte blocks, k = n
    (36, 20, 17 * 1024, 9),
    (16, 12, 65536, 10),       # k <= 16 pinned to the big decoder
    (8, 5, 262144, 6),         # k <= 8 pinned to the big decoder
    (64, 41, 1048576, 3),      # W3 shape: 3 groups, rows of 41 bytes
    (12, 9, 65539, 6),         # one group, odd k, tail row
    (64, 64, 4099, 5),         # 4 groups, k = n = 64
    (70, 61, 70001, 4),        # 4 groups, the last 13 columns wide
    (40, 18, 1048576 + 7, 3),  # rows of 18 bytes (dword pairs straddle rows)
])
def test_big_decode_matches(L, O, n, k, B, S):
    """NKFS_DEC_BIG rebuilds every block like the general decoder from k
    seeded survivors offered in random order plus one extra slot; stripe 1
    offers a duplicate id (skipped, crt/nk8.c:512-537), stripe 2 one distinct
    id (status -EINVAL, block untouched)."""
    from nkfs_amd import _lib, batch
    blocks = batch.synth(S, B, first=60 + k)
    ids_np = synth.batch_ids(S, n, first=60 + k)
    parts, _ = batch.encode(blocks, B, n, k, dev(ids_np))
    keep = min(n, k + 1)
    av = synth.batch_survivors(S, n, keep, first=60 + k)
    ids2 = ids_np.copy()
    if S > 2 and keep > k:
        ids2[1, av[1, 1]] = ids2[1, av[1, 0]]
    if S > 2:
        ids2[2, :] = ids2[2, 0]
    outs = []
    # the column-chunked decoder, then the replicated-table decoder
    # (nk8_bign.hip) in its three table layouts
    for kern, mode in (("generic", -1), ("big", -1), ("auto", -1), ("big", 0), ("big", 1), ("big", 2), ("auto", 2),
                       ("auto", -2), ("big", 3), ("auto", 3), ("big", 4), ("auto", 4), ("auto", 5)):
        with _tuned(dec_kernel=_lib.DEC[kern], dec_bign=mode):
            out = torch.full((S, B), 0xEE, dtype=torch.uint8, device="cuda")
            _, st = batch.decode(parts, n, dev(ids2), dev(av), k, B, out=out)
            torch.cuda.synchronize()
            outs.append((out.cpu(), st.cpu().tolist()))
    for o, st in outs[1:]:
        assert st == outs[0][1]
        assert torch.equal(o, outs[0][0])
    o, st = outs[1]
    ref = blocks[:, :B].cpu()
    for s in range(S):
        if S > 2 and s == 2:
            assert st[s] == -22 and bool((o[s] == 0xEE).all())
        else:
            assert st[s] == 0 and torch.equal(o[s], ref[s]), s
    s = S - 1
    sel = [int(x) for x in av[s]]
    pn = parts[s * n:(s + 1) * n, :batch.part_size(B, k)].cpu().numpy()
    got = O.decode([pn[j] for j in sel], [int(ids_np[s, j]) for j in sel], k, B)
    assert np.array_equal(np.asarray(got), ref[s].numpy())


@pytest.mark.parametrize("n,k,gap", [(24, 17, 0), (40, 33, 5), (64, 41, 3), (48, 32, 1), (12, 11, 7)])
def test_bigr_decode_ragged(L, O, n, k, gap):
    """The all-groups stage-free decoder (dec_bign 3: every output column of
    a slice in one workgroup, rows through an LDS stage) on ragged batches
    with unaligned block offsets and stripes of 1, k + 1 and 1 MiB bytes:
    equal to the column-chunked decoder and the general one, blocks exact,
    bytes between blocks untouched."""
    from nkfs_amd import _lib, batch
    sizes = synth.mixed_sizes(14)
    sizes[:5] = (4096, 1048576, 1, k + 1, 3 * k + 2)
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos, ppos = 0, 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos
        pos += int(B) + gap
        ppos += n * batch.part_pitch(int(B), k)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(800 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=800)
    parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff), dig,
                        int(sizes.max()))
    av = synth.batch_survivors(len(sizes), n, k, first=800)
    outs = []
    for kern, mode in (("generic", -1), ("big", -1), ("big", 3), ("auto", 3), ("auto", 5)):
        out = torch.full((pos + 16,), 0xEE, dtype=torch.uint8, device="cuda")
        st = torch.full((len(sizes),), 5, dtype=torch.int32, device="cuda")
        with _tuned(dec_kernel=_lib.DEC[kern], dec_bign=mode):
            batch.decode_ragged(parts, dev(poff), n, dev(ids_np), dev(av), k, out, dev(boff),
                                dev(sizes.astype(np.int32)), int(sizes.max()), status=st)
        torch.cuda.synchronize()
        outs.append((out.cpu().numpy(), st.cpu().numpy()))
    blk = np.zeros(pos + 16, bool)
    for s, B in enumerate(sizes):
        blk[boff[s]: boff[s] + B] = True
    for o, st in outs:
        assert (st == 0).all()
        assert np.array_equal(o[blk], host[blk]) and (o[~blk] == 0xEE).all()


def test_big_round_trip_w2(L, O):
    """The bench's W2 batch (256 x 1 MiB, N48K32): the default encoder (the
    stage-free one with its hash wave), the column-chunked one with the
    separate hash pass and with XXH64 fused (each slice continuing its part
    group's chains from the previous slice's workgroup) give the same parts
    and digests, the oracle's digests on a sample; keep 32 seeded survivors
    -> default decode gives every block back."""
    from nkfs_amd import _lib, batch
    S, B, n, k = 256, 1048576, 48, 32
    blocks = batch.synth(S, B, first=11)
    ids_np = synth.batch_ids(S, n, first=11)
    ids = dev(ids_np)
    parts, dig = batch.encode(blocks, B, n, k, ids)
    for fused in (0, 1):
        with _tuned(enc_bign=0, enc_big_fused=fused):
            parts1, dig1 = batch.encode(blocks, B, n, k, ids)
        torch.cuda.synchronize()
        assert torch.equal(parts, parts1) and torch.equal(dig, dig1), fused
        del parts1
    got = [u64(x) for x in dig.cpu().tolist()]
    for s in (0, 137, S - 1):
        want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s
    avail = dev(synth.batch_survivors(S, n, k, first=11))
    out, status = batch.decode(parts, n, ids, avail, k, B)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert torch.equal(out, blocks[:, :B])
    for mode in (-1, 0, 1, 2, 3, 4, 5):  # the survivor-table decoder, the stage-free one's layouts
        with _tuned(dec_bign=mode):
            out2, status2 = batch.decode(parts, n, ids, avail, k, B)
        torch.cuda.synchronize()
        assert int(status2.abs().sum()) == 0 and torch.equal(out2, out), mode
        del out2
    assert torch.equal(out, blocks[:, :B])


@pytest.mark.parametrize("gap", [0, 1])
def test_bign_hash_handoff_repeated(L, gap):
    """The stage-free encoder's hash wave folds each slice from the L2 after
    every encoder wave published its progress count; a hand-off that let it
    read rows before they were visible gave one part group wrong digests in
    a few runs out of ten (round 5, an LDS capture variant, reverted).  Ten
    launches of a ragged N48K32 batch per block alignment: every digest
    equal to the column-chunked kernel's + hash pass."""
    from nkfs_amd import batch
    n, k = 48, 32
    sizes = synth.mixed_sizes(16)
    sizes[:5] = (4096, 65536, 1048576, 1, k + 1)
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos
        pos += int(B) + gap
        ppos += n * batch.part_pitch(int(B), k)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(900 + s, int(B))
    ids = dev(synth.batch_ids(len(sizes), n, first=900))
    args = (dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, ids)
    ref = None
    for run in range(11):
        parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
        dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
        with _tuned(enc_bign=0 if run == 0 else -1):
            batch.encode_ragged(*args, parts, dev(poff), dig, int(sizes.max()))
        torch.cuda.synchronize()
        if ref is None:
            ref = (parts.clone(), dig.clone())
        else:
            bad = (dig != ref[1]).nonzero().flatten().tolist()
            assert not bad and torch.equal(parts, ref[0]), (run, bad[:16])
