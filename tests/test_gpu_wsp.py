"""The persistent warp-specialised encoder (nk8_wsp.hip, NKFS_ENC_WSP):
one resident workgroup per CU walking a stream of 4-stripe groups, a
scheduler wave publishing group descriptors ahead into LDS, uniform batches
walked statically and ragged batches taken in size order from a device-wide
counter.  Bit-exact against the fused kernel (another family) and the oracle
(crt/nk8.c:344-444, crt/xxhash.c:358-496), on shapes that give every
workgroup many groups (1-chunk groups, groups spanning chunk-count classes,
partial last groups, 1- and 2-byte stripes) and at both load depths."""
import numpy as np
import pytest

from nkfs_amd import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def L():
    from nkfs_amd import _lib
    lib = _lib.lib()
    assert lib.nk8_init() == 0
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


@pytest.mark.parametrize("S,B,n,k", [(2601, 1000, 8, 5), (1100, 262144, 8, 5), (4099, 20000, 6, 3),
                                     (3000, 4096, 8, 8), (2049, 8192, 4, 2), (1027, 70001, 3, 2), (5, 3, 8, 2),
                                     (1031, 2048, 7, 7)])
@pytest.mark.parametrize("pf", [1, 2])
def test_wsp_uniform_matches(L, O, S, B, n, k, pf):
    """Uniform batches (groups from the device-wide counter; static when
    every workgroup has one group: S = 5) against the fused kernel and the
    oracle."""
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=91)
    ids_np = synth.batch_ids(S, n, first=91)
    ids = dev(ids_np)
    with _tuned(enc_kernel=_enc("fused")):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("wsp"), enc_ws_prefetch=pf):
        p1, d1 = batch.encode(blocks, B, n, k, ids)
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps])
    assert torch.equal(d0, d1)
    got = [u64(x) for x in d1.cpu().tolist()]
    for s in (0, S // 2, S - 1):
        want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s
    del p0, p1, blocks
    torch.cuda.empty_cache()


def _ragged(sizes, n, k, gap, first):
    from nkfs_amd import batch
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes.tolist()):
        boff[s], poff[s] = pos, ppos
        pos += B + gap
        ppos += n * batch.part_pitch(B, k)
    hb = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes.tolist()):
        hb[boff[s]: boff[s] + B] = synth.stripe_bytes(first + s, B)
    return boff, poff, hb, ppos


@pytest.mark.parametrize("n,k,gap,mix", [(8, 5, 0, "c5"), (8, 5, 3, "wide"), (6, 3, 0, "tiny"), (5, 4, 16, "wide"),
                                         (4, 2, 0, "c5"), (8, 8, 0, "classes")])
@pytest.mark.parametrize("pf", [1, 2])
def test_wsp_ragged_matches(L, O, n, k, gap, mix, pf):
    """Ragged batches in size order from the group counter: the same parts
    and digests as the walk encoder (the ragged default) and the oracle on a
    sample of every size."""
    from nkfs_amd import batch
    rng = np.random.default_rng(len(mix) * 7 + n + pf)
    if mix == "c5":
        sizes = synth.mixed_sizes(3001, (4096, 65536, 1048576)).astype(np.int64)
    elif mix == "wide":
        sizes = rng.integers(1, 600000, 1500)
        sizes[::7] = 1
        sizes[3::11] = 2
    elif mix == "tiny":
        sizes = rng.integers(1, 5000, 4000)
    else:  # chunk-count classes that change inside groups: 1, 2, 3, ... chunks
        sizes = np.repeat(np.arange(1, 40) * 1024 * k - 7, 37)
        rng.shuffle(sizes)
    sizes = sizes.astype(np.uint32)
    boff, poff, hb, ppos = _ragged(sizes, n, k, gap, 500)
    rid = synth.batch_ids(len(sizes), n, first=500)
    outs = []
    for kern in ("walk", "wsp"):
        with _tuned(enc_kernel=_enc(kern), enc_ws_prefetch=pf):
            parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
            dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
            batch.encode_ragged(dev(hb), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(rid), parts, dev(poff),
                                dig, int(max(1, sizes.max())))
            torch.cuda.synchronize()
            outs.append((parts, dig))
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][0], outs[1][0])
    got = [u64(x) for x in outs[1][1].cpu().tolist()]
    order = np.argsort(sizes, kind="stable")
    for s in sorted({int(order[0]), int(order[len(order) // 2]), int(order[-1]), 0, len(sizes) - 1}):
        B = int(sizes[s])
        want = O.encode(hb[boff[s]: boff[s] + B], n, k, rid[s])
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], (s, B)


def test_wsp_default_dispatch_c5_scale(L, O):
    """enc_persist = 1 (default): the automatic choice takes the persistent
    encoder for C5 (ragged); at the bench's scale and layout (11,520 stripes,
    ~4 GiB) it gives the walk encoder's (enc_persist = 0) bytes."""
    from nkfs_amd import batch
    n, k = 8, 5
    sizes = synth.mixed_sizes(11520, (4096, 65536, 1048576))
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes.tolist()):
        boff[s], poff[s] = pos, ppos
        pos += (B + 255) // 256 * 256
        ppos += n * batch.part_pitch(B, k)
    S = len(sizes)
    blocks = torch.zeros(pos, dtype=torch.uint8, device="cuda")
    bo, po, sz = dev(boff), dev(poff), dev(sizes.astype(np.int32))
    batch.synth_ragged(blocks, bo, sz, first=0)
    ids_np = synth.batch_ids(S, n, first=0)
    ids = dev(ids_np)
    res = []
    for persist in (0, 1):
        with _tuned(enc_persist=persist):
            parts = torch.empty(ppos, dtype=torch.uint8, device="cuda")
            dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
            batch.encode_ragged(blocks, bo, sz, n, k, ids, parts, po, dig, int(sizes.max()))
            torch.cuda.synchronize()
            res.append((parts, dig))
    assert torch.equal(res[0][1], res[1][1])
    for s in np.nonzero(sizes == 1048576)[0][:8].tolist() + np.nonzero(sizes == 4096)[0][-8:].tolist():
        a, b_ = int(poff[s]), int(poff[s]) + n * batch.part_pitch(int(sizes[s]), k)
        assert torch.equal(res[0][0][a:b_], res[1][0][a:b_]), s
    got = [u64(x) for x in res[1][1].cpu().tolist()]
    for B in (4096, 65536, 1048576):
        for s in np.nonzero(sizes == B)[0][[0, -1]].tolist():
            want = O.encode(blocks[boff[s]: boff[s] + B].cpu().numpy(), n, k, ids_np[s])
            assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], (s, B)
    del res, blocks
    torch.cuda.empty_cache()
