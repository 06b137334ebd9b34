"""GPU parity of the part-group encoders (nk8_wide.hip): NKFS_ENC_WIDE (row
slices + a second XXH64 pass; for a handful of big stripes) and
NKFS_ENC_WIDE_WS (XXH64 fused by a hash wave; the default for n > 8 or k > 8
with k <= 16 on batches that fill the chip).

Every case is checked bit-exact against the thread-per-row general kernel
(NKFS_ENC_GENERIC) on all stripes and against the oracle's parts and XXH64
(oracle/nk8_port.c, pinned to the compiled reference) on sampled stripes:
part groups (n = 9..255), k = 2..16, tails of every size (B not a multiple
of 16, k or 4; one-byte blocks), unaligned ragged block offsets, row slices
(few big stripes), and the encode -> erase -> decode round trip.
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


def _enc(name):
    from nkfs_amd import _lib
    return _lib.ENC[name]


@pytest.mark.parametrize("n,k,B,S", [
    (10, 8, 65536, 40),        # two groups, the second one 2 parts wide
    (16, 12, 1048576, 6),      # 1 MiB stripes, row slices
    (12, 5, 4099, 300),        # tail rows, many stripes
    (255, 16, 70001, 2),       # 32 groups, last group 7 parts
    (9, 2, 1, 5),              # one-byte blocks
    (20, 16, 1000003, 2),      # B not a multiple of 4 / 16 / k
    (16, 9, 17, 64),           # fewer rows than one lane's 16
    (8, 5, 262144, 20),        # n <= 8 pinned to the wide kernel
    (4, 2, 4096, 100),
    (11, 3, 4096 * 1024 + 3, 1),  # one big stripe: slices across the chip
])
def test_wide_encode_matches(L, O, n, k, B, S):
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=900 + n)
    ids_np = synth.batch_ids(S, n, first=900 + n)
    ids = dev(ids_np)
    with _tuned(enc_kernel=_enc("generic")):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("wide")):
        p1, d1 = batch.encode(blocks, B, n, k, ids)
        p2, _ = batch.encode(blocks, B, n, k, ids, digests=False)
    with _tuned(enc_kernel=_enc("wide_ws")):  # XXH64 fused (hash wave)
        p4, d4 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("wide_ws"), enc_ws_prefetch=2):  # two chunks of loads in flight
        p5, d5 = batch.encode(blocks, B, n, k, ids)
    p3, d3 = batch.encode(blocks, B, n, k, ids)  # default dispatch
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps]) and torch.equal(d0, d1)
    assert torch.equal(p0[:, :ps], p2[:, :ps])
    assert torch.equal(p0[:, :ps], p3[:, :ps]) and torch.equal(d0, d3)
    assert torch.equal(p0[:, :ps], p4[:, :ps]) and torch.equal(d0, d4)
    assert torch.equal(p0[:, :ps], p5[:, :ps]) and torch.equal(d0, d5)
    got = [u64(x) for x in d1.cpu().tolist()]
    for s in sorted({0, S // 2, S - 1}):
        want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
        assert np.array_equal(p1[s * n:(s + 1) * n, :ps].cpu().numpy(), np.stack(want)), s
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s


@pytest.mark.parametrize("n,k,gap", [(12, 6, 0), (17, 16, 5), (9, 4, 3)])
def test_wide_encode_ragged(L, O, n, k, gap):
    """Ragged batches (mixed sizes, block offsets unaligned when gap != 0):
    the wide kernel equals the general kernel, and the oracle per stripe."""
    from nkfs_amd import batch
    sizes = synth.mixed_sizes(20)
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
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(700 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=700)
    outs = []
    for kern, pf in (("generic", 1), ("wide", 1), ("wide_ws", 1), ("wide_ws", 2)):
        parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
        dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
        with _tuned(enc_kernel=_enc(kern), enc_ws_prefetch=pf):
            batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts,
                                dev(poff), dig, int(sizes.max()))
        torch.cuda.synchronize()
        outs.append((parts.cpu().numpy(), [u64(x) for x in dig.cpu().tolist()]))
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    assert np.array_equal(outs[0][0], outs[2][0]) and outs[0][1] == outs[2][1]
    assert np.array_equal(outs[0][0], outs[3][0]) and outs[0][1] == outs[3][1]
    pn, got = outs[1]
    for s in (0, 2, 3, 4, len(sizes) - 1):
        B = int(sizes[s])
        want = O.encode(host[boff[s]: boff[s] + B], n, k, ids_np[s])
        pitch = batch.part_pitch(B, k)
        for i in range(n):
            off = int(poff[s]) + i * pitch
            assert np.array_equal(pn[off: off + len(want[i])], want[i]), (s, i)
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s


@pytest.mark.parametrize("n,k,B,S", [(16, 12, 262144, 30), (10, 8, 65536, 200)])
def test_wide_round_trip(L, n, k, B, S):
    """Encode (default dispatch: wide) -> keep k seeded survivors -> decode
    gives the blocks back on every stripe."""
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=5)
    ids = dev(synth.batch_ids(S, n, first=5))
    parts, _ = batch.encode(blocks, B, n, k, ids)
    avail = dev(synth.batch_survivors(S, n, k, first=5))
    out, status = batch.decode(parts, n, ids, avail, k, B)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert torch.equal(out, blocks[:, :B])


@pytest.mark.parametrize("n,k,B,S", [
    (16, 12, 1048576, 6),      # row slices
    (20, 16, 1000003, 3),      # B not a multiple of 4 / 16 / k
    (12, 9, 4099, 200),
    (10, 10, 1, 5),            # one-byte blocks, k = n
    (16, 13, 17, 64),          # fewer rows than one lane's 16
    (8, 5, 262144, 20),        # k <= 8 pinned to the wide decoder
    (4, 2, 4096, 100),
])
def test_wide_decode_matches(L, O, n, k, B, S):
    """The survivor-table decoder (NKFS_DEC_WIDE: default for 8 < k <= 16)
    rebuilds every block like the thread-per-row general decoder, from k
    seeded survivors offered in random order plus one extra slot; stripe 1
    offers a duplicate id (skipped, crt/nk8.c:512-537) and stripe 2 only one
    distinct id (status -EINVAL, block left untouched)."""
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=40 + k)
    ids_np = synth.batch_ids(S, n, first=40 + k)
    parts, _ = batch.encode(blocks, B, n, k, dev(ids_np))
    keep = min(n, k + 1)
    av = synth.batch_survivors(S, n, keep, first=40 + k)
    ids2 = ids_np.copy()
    if S > 2 and keep > k:
        ids2[1, av[1, 1]] = ids2[1, av[1, 0]]
    if S > 2:
        ids2[2, :] = ids2[2, 0]
    outs = []
    for kern, mode in (("generic", -1), ("wide", -1), ("auto", -1), ("auto", 0), ("auto", 1), ("auto", 2),
                       ("auto", -2), ("auto", 4)):
        from nkfs_amd import _lib
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
        else:  # stripe 1: the extra offered slot stands in for the skipped duplicate
            assert st[s] == 0 and torch.equal(o[s], ref[s]), s
    # one stripe against the oracle's assemble (crt/nk8.c:446-599)
    s = S - 1
    sel = [int(x) for x in av[s]]
    pn = parts[s * n:(s + 1) * n, :batch.part_size(B, k)].cpu().numpy()
    got = O.decode([pn[j] for j in sel], [int(ids_np[s, j]) for j in sel], k, B)
    assert np.array_equal(np.asarray(got), ref[s].numpy())


@pytest.mark.parametrize("n,k,B,S", [(16, 12, 1048576, 600), (20, 16, 65536, 700), (12, 9, 4099, 2000)])
def test_wide_ws_default_dispatch_against_oracle(L, O, n, k, B, S):
    """Batches that fill the chip take the fused part-group encoder by
    default: parts and XXH64 against the oracle on a sample of stripes, and
    against the two-pass form on all of them."""
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=77 + k)
    ids_np = synth.batch_ids(S, n, first=77 + k)
    ids = dev(ids_np)
    p1, d1 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("wide")):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps]) and torch.equal(d0, d1)
    got = [u64(x) for x in d1.cpu().tolist()]
    for s in sorted({0, S // 3, S - 1}):
        want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
        assert np.array_equal(p1[s * n:(s + 1) * n, :ps].cpu().numpy(), np.stack(want)), s
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s
