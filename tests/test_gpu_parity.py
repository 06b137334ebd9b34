"""GPU parity: the HIP path through the C-ABI against the reference's golden
vectors and the pinned CPU oracle, bit-exact (integer/byte arithmetic).

Sizes: golden cases in full; BASELINE configs at full per-stripe size with
stripe counts the oracle checks in seconds; C2 (65,536 x 4 KiB) in full.
Full-size properties: encode -> erase -> decode round trips on the device.
"""
import ctypes as C
import hashlib

import numpy as np
import pytest

from nkfs_amd import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def L():
    from nkfs_amd import _lib
    lib = _lib.lib()
    assert lib.nk8_init() == 0, "nk8_init (GPU self test) failed"
    assert lib.nkfs_gpu_ready() == 1
    return lib


@pytest.fixture(scope="module")
def O():
    from oracle import oracle
    return oracle


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def u64(x):
    return int(x) & 0xFFFFFFFFFFFFFFFF


def encode_batch(blocks_np, n, k, ids_np, block_size):
    from nkfs_amd import batch
    blocks = dev(blocks_np)
    ids = dev(ids_np)
    parts, dig = batch.encode(blocks, block_size, n, k, ids)
    torch.cuda.synchronize()
    return blocks, parts, dig


# ------------------------------------------------------------------ golden

def test_encode_golden(L, golden):
    from nkfs_amd import batch
    for case in golden["encode"]:
        B, n, k = case["block_size"], case["n"], case["k"]
        blk = synth.stripe_bytes(case["stripe"], B)
        ids = np.frombuffer(bytes.fromhex(case["ids"]), dtype=np.uint8)[None, :]
        pitch = ((B + 15) // 16) * 16
        host = np.zeros((1, pitch), np.uint8)
        host[0, :B] = blk
        _, parts, dig = encode_batch(host, n, k, ids, B)
        ps = batch.part_size(B, k)
        got = parts[:, :ps].cpu().numpy()
        assert sha(got) == case["parts_sha256"], (B, n, k)
        assert [f"{u64(d):016x}" for d in dig.cpu().tolist()] == case["part_xxh64"], (B, n, k)


def test_decode_golden(L, golden, O):
    from nkfs_amd import batch
    enc = golden["encode"]
    for d in golden["decode"]:
        case = enc[d["case"]]
        B, n, k = case["block_size"], case["n"], case["k"]
        blk = synth.stripe_bytes(case["stripe"], B)
        ids = np.frombuffer(bytes.fromhex(case["ids"]), dtype=np.uint8)
        parts = O.encode(blk, n, k, ids)
        pitch = batch.part_pitch(B, k)
        slots = np.zeros((n, pitch), np.uint8)
        slots[:, : parts.shape[1]] = parts
        avail = np.array(d["order"], dtype=np.uint8)[None, :]
        navail = avail.shape[1]
        if navail < 2 or navail < k:
            # fewer offered parts than k: the API rejects like nk8_assemble_block
            assert d["err"] == -22
            continue
        out, status = batch.decode(dev(slots), n, dev(ids[None, :]), dev(avail), k, B)
        torch.cuda.synchronize()
        assert int(status[0]) == d["err"], (B, n, k, d["order"])
        if d["err"] == 0:
            assert sha(out[0].cpu().numpy()) == d["block_sha256"]


def test_xxh64_golden_batch_and_compat(L, golden):
    from nkfs_amd import batch, crt
    vecs = golden["xxh64"]
    datas = [synth.stripe_bytes(v["stripe"], v["len"]) if v["len"] else np.zeros(0, np.uint8) for v in vecs]
    # batch API, per seed
    for seed_hex in sorted({v["seed"] for v in vecs}):
        sel = [i for i, v in enumerate(vecs) if v["seed"] == seed_hex]
        offs, buf, pos = [], [], 0
        for i in sel:
            offs.append(pos)
            buf.append(datas[i])
            pad = (-len(datas[i])) % 8 + 8
            buf.append(np.zeros(pad, np.uint8))
            pos += len(datas[i]) + pad
        base = dev(np.concatenate(buf))
        off = dev(np.array(offs, np.uint64).view(np.int64))
        lens = dev(np.array([len(datas[i]) for i in sel], np.uint64).view(np.int64))
        got = batch.xxh64_batch(base, off, lens, seed=int(seed_hex, 16))
        want = [int(vecs[i]["digest"], 16) for i in sel]
        assert [u64(x) for x in got.cpu().tolist()] == want
    # drop-in one-shot XXH64 (seed 0 subset)
    for v, data in zip(vecs, datas):
        assert crt.xxh64(data, int(v["seed"], 16)) == int(v["digest"], 16)


def test_csum_streaming_matches_oracle(L, O):
    from nkfs_amd import crt
    rng = np.random.default_rng(3)
    for total in [0, 1, 31, 32, 33, 100, 4096, 65536 + 13]:
        data = rng.integers(0, 256, total, dtype=np.uint8)
        cs = crt.Csum()
        pos = 0
        while pos < total:
            step = int(rng.integers(1, 97))
            cs.update(data[pos: pos + step])
            pos += step
        assert cs.digest() == O.xxh64(data)


# -------------------------------------------------------------- drop-in API

def test_split_assemble_compat(L, O):
    from nkfs_amd import crt
    rng = np.random.default_rng(5)
    for B, n, k in [(4096, 4, 2), (1048576, 8, 5), (70000, 255, 254), (1, 2, 2), (13, 8, 5), (65537, 16, 9)]:
        blk = rng.integers(0, 256, B, dtype=np.uint8)
        parts, ids = crt.split_block(blk, n, k)
        assert len(set(ids.tolist())) == n and ids.min() >= 1
        want = O.encode(blk, n, k, ids)
        assert np.array_equal(np.stack(parts), want)
        sel = rng.permutation(n)[:k]
        out = crt.assemble_block([parts[i] for i in sel], ids[sel], k, k, B)
        assert np.array_equal(out, blk)
        # extra parts after the first k distinct are ignored, duplicates skipped
        order = [int(sel[0])] + [int(x) for x in rng.permutation(n)][: min(n, 254)]
        out2 = crt.assemble_block([parts[i] for i in order], ids[order], len(order), k, B)
        assert np.array_equal(out2, blk)


def test_compat_errors(L, golden):
    from nkfs_amd import crt
    for e in golden["split_errors"]:
        blk = np.zeros(max(e["block_size"], 1), np.uint8)[: e["block_size"]]
        with pytest.raises(OSError) as ei:
            crt.split_block(blk, e["n"], e["k"])
        assert -ei.value.errno == e["err"]
    parts, ids = crt.split_block(np.arange(100, dtype=np.uint8), 4, 3)
    with pytest.raises(OSError) as ei:  # two distinct ids offered, k = 3
        crt.assemble_block([parts[0], parts[0], parts[1], parts[1]], [ids[0], ids[0], ids[1], ids[1]], 4, 3, 100)
    assert ei.value.errno == 22


def test_synth_kernel_matches_numpy(L):
    from nkfs_amd import batch
    for B in (4096, 1000, 13):
        t = batch.synth(9, B, first=40)
        torch.cuda.synchronize()
        got = t[:, :B].cpu().numpy()
        assert np.array_equal(got, synth.batch_bytes(9, B, first=40))


# --------------------------------------------------------- BASELINE shapes

def _oracle_digests(O, blocks_np, ids_np, n, k, B):
    out = []
    for s in range(blocks_np.shape[0]):
        parts = O.encode(blocks_np[s, :B], n, k, ids_np[s])
        out.extend(O.xxh64(p) for p in parts)
    return out


def test_c2_full_batch_n4k2_4k(L, O):
    """configs[1]: N=4,K=2 encode of 64 Ki x 4 KiB stripes, every part's bytes
    checked through its XXH64 against the oracle, then erase 2 -> decode."""
    from nkfs_amd import batch
    S, B, n, k = 65536, 4096, 4, 2
    blocks = batch.synth(S, B)
    ids_np = synth.batch_ids(S, n)
    parts, dig = batch.encode(blocks, B, n, k, dev(ids_np))
    torch.cuda.synchronize()
    blocks_np = blocks.cpu().numpy()
    want = _oracle_digests(O, blocks_np, ids_np, n, k, B)
    got = [u64(x) for x in dig.cpu().tolist()]
    assert got == want
    # spot-check raw part bytes too
    for s in (0, 1, 12345, S - 1):
        assert np.array_equal(parts[s * n:(s + 1) * n, :2048].cpu().numpy(),
                              O.encode(blocks_np[s, :B], n, k, ids_np[s]))
    avail = dev(synth.batch_survivors(S, n, k))
    out, status = batch.decode(parts, n, dev(ids_np), avail, k, B)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert torch.equal(out, blocks[:, :B])


@pytest.mark.parametrize("S,B,n,k,keep", [
    (48, 1048576, 8, 5, 5),    # C3 shape: 1 MiB stripes, decode from 5 of 8
    (256, 262144, 8, 5, 5),    # C4: 256 KiB, 3 erased
    (512, 65536, 8, 5, 6),     # extra survivor offered
    (64, 70000, 255, 254, 254),
    (300, 777, 17, 16, 17),
    (1024, 20480, 8, 5, 6),    # small batches of 4 KiB parts (plan + slice grid)
    (300, 4096, 6, 3, 4),
    (1025, 20480, 8, 5, 5),
])
def test_uniform_shapes(L, O, S, B, n, k, keep):
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=7)
    ids_np = synth.batch_ids(S, n, first=7)
    parts, dig = batch.encode(blocks, B, n, k, dev(ids_np))
    torch.cuda.synchronize()
    blocks_np = blocks.cpu().numpy()
    check = list(range(0, S, max(1, S // 16)))
    for s in check:
        want = _oracle_digests(O, blocks_np[s:s + 1], ids_np[s:s + 1], n, k, B)
        got = [u64(x) for x in dig[s * n:(s + 1) * n].cpu().tolist()]
        assert got == want, s
    avail = dev(synth.batch_survivors(S, n, keep, first=7))
    out, status = batch.decode(parts, n, dev(ids_np), avail, k, B)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert torch.equal(out, blocks[:, :B])


def test_ragged_mixed_batch(L, O):
    """C5 shape: mixed 4 KiB / 64 KiB / 1 MiB stripes in one ragged batch,
    N=8,K=5 and the N=4,K=2 variant, digests against the oracle."""
    from nkfs_amd import batch
    for n, k in ((8, 5), (4, 2)):
        sizes = synth.mixed_sizes(40)
        sizes[:3] = (4096, 65536, 1048576)
        boff = np.zeros(len(sizes), np.int64)
        poff = np.zeros(len(sizes), np.int64)
        pos = ppos = 0
        for s, B in enumerate(sizes):
            boff[s] = pos
            poff[s] = ppos
            pos += ((int(B) + 15) // 16) * 16
            ppos += n * batch.part_pitch(int(B), k)
        host = np.zeros(pos, np.uint8)
        for s, B in enumerate(sizes):
            host[boff[s]: boff[s] + B] = synth.stripe_bytes(s, int(B))
        ids_np = synth.batch_ids(len(sizes), n)
        parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
        dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
        batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts,
                            dev(poff), dig, int(sizes.max()))
        torch.cuda.synchronize()
        got = [u64(x) for x in dig.cpu().tolist()]
        for s, B in enumerate(sizes):
            want = _oracle_digests(O, host[None, boff[s]: boff[s] + B], ids_np[s:s + 1], n, k, int(B))
            assert got[s * n:(s + 1) * n] == want, (s, B)


def _ragged_layout(sizes, n, k, block_gap=0, first_off=0):
    from nkfs_amd import batch
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos, ppos = first_off, 0
    for s, B in enumerate(sizes):
        boff[s] = pos
        poff[s] = ppos
        pos += int(B) + block_gap
        ppos += n * batch.part_pitch(int(B), k)
    return boff, poff, pos, ppos


@pytest.mark.parametrize("n,k,gap", [(8, 5, 0), (4, 2, 3), (6, 3, 16), (17, 16, 5)])
def test_ragged_decode_round_trip(L, O, n, k, gap):
    """nkfs_nk8_decode_ragged over the layout nkfs_nk8_encode_ragged writes:
    mixed 4 KiB / 64 KiB / 1 MiB stripes (C5) plus odd sizes, output blocks
    at unaligned offsets (gap), survivors in seeded random order with an
    extra slot offered; fast path (k <= 8) and general path (k = 16).  Each
    stripe must come back bit-exact; one stripe's parts are also checked
    against the oracle's assemble."""
    from nkfs_amd import batch
    sizes = synth.mixed_sizes(24)
    sizes[:6] = (4096, 65536, 1048576, 1, k + 1, 70001)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, gap)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(300 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=300)
    parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff),
                        None, int(sizes.max()))
    keep = min(n, k + 1)
    avail = synth.batch_survivors(len(sizes), n, keep, first=300)
    out = torch.zeros(pos + 16, dtype=torch.uint8, device="cuda")
    status = batch.decode_ragged(parts, dev(poff), n, dev(ids_np), dev(avail), k, out, dev(boff),
                                 dev(sizes.astype(np.int32)), int(sizes.max()))
    torch.cuda.synchronize()
    assert status.abs().sum().item() == 0
    got = out.cpu().numpy()
    for s, B in enumerate(sizes):
        assert np.array_equal(got[boff[s]: boff[s] + B], host[boff[s]: boff[s] + B]), (s, int(B))
    # gaps between blocks stay untouched (only B bytes per stripe are written)
    mask = np.ones(pos + 16, bool)
    for s, B in enumerate(sizes):
        mask[boff[s]: boff[s] + B] = False
    assert not got[mask].any()
    # the oracle rebuilds stripe 2 (1 MiB) from the same device parts
    s, B = 2, int(sizes[2])
    pitch = batch.part_pitch(B, k)
    pn = parts[poff[s]: poff[s] + n * pitch].cpu().numpy().reshape(n, pitch)[:, :batch.part_size(B, k)]
    sel = list(avail[s])
    assert np.array_equal(O.decode([pn[j] for j in sel], ids_np[s][sel], k, B), host[boff[s]: boff[s] + B])


def test_decode_status_too_few_distinct(L):
    from nkfs_amd import batch
    S, B, n, k = 4, 4096, 4, 2
    blocks = batch.synth(S, B)
    ids_np = synth.batch_ids(S, n)
    parts, _ = batch.encode(blocks, B, n, k, dev(ids_np), digests=False)
    ids_dup = ids_np.copy()
    ids_dup[1, 1] = ids_dup[1, 0]  # stripe 1: slots 0 and 1 share an id
    avail = np.tile(np.array([0, 1], np.uint8), (S, 1))
    out, status = batch.decode(parts, n, dev(ids_dup), dev(avail), k, B)
    torch.cuda.synchronize()
    st = status.cpu().tolist()
    assert st[1] == -22 and st[0] == st[2] == st[3] == 0
    assert torch.equal(out[0], blocks[0, :B]) and torch.equal(out[3], blocks[3, :B])


def test_xxh64_batch_blocks_and_ragged(L, O):
    """Batched XXH64 (csum seed 0) of 64 KiB blocks -- the core's per-block
    integrity sum (core/dio.c:26-37) -- plus ragged lengths and 8-byte (not
    16-byte) aligned offsets, against the oracle."""
    from nkfs_amd import batch
    rng = np.random.default_rng(9)
    nb = 512
    blocks = batch.synth(nb, 65536, first=99)
    off = torch.arange(nb, dtype=torch.int64, device="cuda") * blocks.stride(0)
    lens = torch.full((nb,), 65536, dtype=torch.int64, device="cuda")
    got = batch.xxh64_batch(blocks, off, lens)
    torch.cuda.synchronize()
    host = blocks.cpu().numpy()
    gl = [u64(x) for x in got.cpu().tolist()]
    for i in range(0, nb, 7):
        assert gl[i] == O.xxh64(host[i, :65536])
    # ragged: random lengths 0..5000 at 8-byte aligned (some 16-unaligned) offsets
    lens_np = rng.integers(0, 5000, 333)
    offs_np = np.zeros(333, np.int64)
    pos = 8
    for i, n_ in enumerate(lens_np):
        offs_np[i] = pos
        pos += int(n_) + 8 + (8 if i % 3 else 0)
        pos = (pos + 7) // 8 * 8
    buf = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    got = batch.xxh64_batch(dev(buf), dev(offs_np), dev(lens_np.astype(np.int64)), seed=12345)
    torch.cuda.synchronize()
    gl = [u64(x) for x in got.cpu().tolist()]
    for i in range(333):
        assert gl[i] == O.xxh64(buf[offs_np[i]: offs_np[i] + lens_np[i]], 12345), i


@pytest.mark.parametrize("n", range(2, 9))
def test_fast_path_every_shape(L, O, n):
    """Every (n <= 8, k <= n) the fused kernels are instantiated for, with
    block sizes that leave tails of every length and stripes spanning
    several chunks, encode + XXH64 + decode from a random survivor order."""
    from nkfs_amd import batch
    rng = np.random.default_rng(100 + n)
    for k in range(2, n + 1):
        for B in (1, k - 1 or 1, k + 1, 777, 4096 * k + 3, 300_001):
            S = 5
            blocks = batch.synth(S, B, first=1000 * n + k)
            ids_np = synth.batch_ids(S, n, first=1000 * n + k)
            parts, dig = batch.encode(blocks, B, n, k, dev(ids_np))
            torch.cuda.synchronize()
            host = blocks.cpu().numpy()
            ps = batch.part_size(B, k)
            got_parts = parts.cpu().numpy()
            got_dig = [u64(x) for x in dig.cpu().tolist()]
            for s in range(S):
                want = O.encode(host[s, :B], n, k, ids_np[s])
                assert np.array_equal(got_parts[s * n:(s + 1) * n, :ps], want), (n, k, B, s)
                assert got_dig[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], (n, k, B, s)
            avail = np.stack([rng.permutation(n)[:k] for _ in range(S)]).astype(np.uint8)
            out, status = batch.decode(parts, n, dev(ids_np), dev(avail), k, B)
            torch.cuda.synchronize()
            assert int(status.abs().sum()) == 0
            assert torch.equal(out, blocks[:, :B]), (n, k, B)


def test_ragged_small_n_and_unaligned(L, O):
    """Ragged batch for n <= 4 (4 stripes per wave) with block offsets that
    are not 16-byte aligned (the kernels' scalar load path)."""
    from nkfs_amd import batch
    n, k = 4, 3
    sizes = np.array([5, 4096, 70000, 13, 65536, 1, 9999, 300], np.uint32)
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = 3
    ppos = 0
    for s, B in enumerate(sizes):
        boff[s] = pos
        poff[s] = ppos
        pos += int(B) + 5
        ppos += n * batch.part_pitch(int(B), k)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(s, int(B))
    ids_np = synth.batch_ids(len(sizes), n)
    parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff), dig,
                        int(sizes.max()))
    torch.cuda.synchronize()
    got = [u64(x) for x in dig.cpu().tolist()]
    pn = parts.cpu().numpy()
    for s, B in enumerate(sizes):
        want = O.encode(host[boff[s]: boff[s] + B], n, k, ids_np[s])
        pitch = batch.part_pitch(int(B), k)
        for i in range(n):
            assert np.array_equal(pn[poff[s] + i * pitch: poff[s] + i * pitch + want.shape[1]], want[i]), (s, i)
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], s


def test_encode_host_pipeline(L, O):
    """nkfs_nk8_encode_host (host memory in/out, sub-batches overlapped on
    two streams) equals the device-resident encode, for pageable numpy
    input (registered for the call) and several sub-batch sizes."""
    from nkfs_amd import batch
    S, B, n, k = 3000, 4096, 4, 2
    blocks = batch.synth(S, B)
    ids_np = synth.batch_ids(S, n)
    parts_d, dig_d = batch.encode(blocks, B, n, k, dev(ids_np))
    torch.cuda.synchronize()
    host = np.ascontiguousarray(blocks.cpu().numpy())
    for chunk in (0, 1 << 20, 123457):
        parts_h, dig_h = batch.encode_host(host, B, n, k, ids_np, chunk_bytes=chunk)
        assert torch.equal(parts_h[:, :2048], parts_d[:, :2048].cpu())
        assert torch.equal(dig_h, dig_d.cpu())
    blk = host[17, :B]
    assert [O.xxh64(p) for p in O.encode(blk, n, k, ids_np[17])] == [u64(x) for x in dig_h[17 * n:18 * n].tolist()]


@pytest.mark.parametrize("S,B,n,k", [(64, 4096, 4, 2), (16, 262144, 8, 5), (40, 70001, 6, 3), (8, 30000, 16, 12),
                                     (33, 100, 8, 8)])
def test_decode_verify(L, S, B, n, k):
    """Integrity-checked decode: clean parts verify; a flipped byte in a
    part that is read fails its stripe with -EIO and flags exactly that slot;
    a flipped byte in a part that is not read changes nothing."""
    from nkfs_amd import batch
    rng = np.random.default_rng(S + B)
    blocks = batch.synth(S, B, first=5)
    ids_np = synth.batch_ids(S, n, first=5)
    ids = dev(ids_np)
    parts, dig = batch.encode(blocks, B, n, k, ids)
    avail_np = np.stack([rng.permutation(n)[:k] for _ in range(S)]).astype(np.uint8)
    avail = dev(avail_np)
    out, status, bad = batch.decode_verify(parts, n, ids, avail, k, B, dig)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 and int(bad.abs().sum()) == 0
    assert torch.equal(out, blocks[:, :B])
    ps = batch.part_size(B, k)
    s_used, s_unused = 1, 2
    used_slot = int(avail_np[s_used, 1])
    unused = [j for j in range(n) if j not in avail_np[s_unused]]
    parts[s_used * n + used_slot, ps - 1] ^= 0x5A
    if unused:
        parts[s_unused * n + unused[0], 0] ^= 0xA5
    out, status, bad = batch.decode_verify(parts, n, ids, avail, k, B, dig)
    torch.cuda.synchronize()
    st = status.cpu().tolist()
    bm = [u64(x) for x in bad.cpu().tolist()]
    assert st[s_used] == -5 and bm[s_used] == 1 << used_slot
    assert st[s_unused] == 0 and bm[s_unused] == 0
    assert all(v == 0 for i, v in enumerate(st) if i != s_used)
    assert torch.equal(out[s_unused], blocks[s_unused, :B])


ENC = None  # set lazily: nkfs_amd._lib.ENC / DEC kernel ids


def _tuned(**kw):
    from nkfs_amd import _lib
    return _lib.tuned(**kw)


def _enc(name):
    from nkfs_amd import _lib
    return _lib.ENC[name]


def _dec(name):
    from nkfs_amd import _lib
    return _lib.DEC[name]


@pytest.mark.parametrize("n,k,B,hw", [(4, 2, 4096, 1), (4, 3, 70001, 1), (8, 5, 262144, 1), (8, 6, 1000, 1),
                                      (8, 5, 262144, 2), (8, 6, 1000, 2), (5, 2, 70001, 2), (8, 8, 3, 2)])
def test_warp_specialised_encode_matches(L, n, k, B, hw):
    """The warp-specialised encoder (nk8_ws.hip: encoder waves + one or two
    hash waves per workgroup; chosen by the shape rules for grids of <= 2
    waves per SIMD of big stripes, forced here through struct nkfs_tune)
    writes the same parts and digests as the fused kernel, tails and partial
    workgroups (23 stripes: 5 workgroups of 4 + 3) included."""
    from nkfs_amd import batch
    for S in (23, 2, 1):
        blocks = batch.synth(S, B, first=77)
        ids = dev(synth.batch_ids(S, n, first=77))
        with _tuned(enc_kernel=_enc("fused")):
            p0, d0 = batch.encode(blocks, B, n, k, ids)
        with _tuned(enc_kernel=_enc("ws"), enc_ws_hash_waves=hw):
            p1, d1 = batch.encode(blocks, B, n, k, ids)
        torch.cuda.synchronize()
        ps = batch.part_size(B, k)
        assert torch.equal(p0[:, :ps], p1[:, :ps]), S
        assert torch.equal(d0, d1), S


@pytest.mark.parametrize("S,B", [(2200, 163840), (3500, 131072), (1700, 1048576), (768, 65536), (513, 20480),
                                 (300, 20480), (1536, 262144), (1025, 262144)])
def test_encode_dispatch_shapes_agree(L, O, S, B):
    """Grids the default dispatch sends to different kernels (N8K5: 1,100
    fused waves of 32 KiB parts -> warp-specialised; 1,750 waves of 26 KB
    parts -> nibble tables; 850 waves of 1 MiB stripes -> warp-specialised;
    round 4: 768 / 513 stripes -> two hash waves, 300 -> one, 1,536 x 256
    KiB -> walk, partial last workgroups), and the walk encoder, give the
    same parts and digests as the fused 256-entry-table kernel, and the
    oracle's on the first and last stripe."""
    from nkfs_amd import batch
    n, k = 8, 5
    blocks = batch.synth(S, B, first=5)
    ids_np = synth.batch_ids(S, n, first=5)
    ids = dev(ids_np)
    p1, d1 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("fused"), enc_nib=0):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("walk")):
        p2, d2 = batch.encode(blocks, B, n, k, ids)
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps]) and torch.equal(d0, d1)
    assert torch.equal(p0[:, :ps], p2[:, :ps]) and torch.equal(d0, d2)
    for s in (0, S - 1):
        want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
        assert [u64(x) for x in d1[s * n:(s + 1) * n].cpu().tolist()] == [O.xxh64(p) for p in want]


@pytest.mark.parametrize("n,k,B,S,waves", [(4, 2, 4096, 3000, 4), (8, 5, 8192, 2500, 4), (8, 5, 4096, 1500, 4),
                                           (8, 5, 9999, 1100, 4), (7, 3, 70001, 40, 8), (6, 4, 1000, 2100, 4),
                                           (8, 8, 777, 900, 4), (2, 2, 1, 5, 8), (8, 5, 13, 3, 8),
                                           (4, 2, 8192 + 4, 1500, 4), (5, 5, 1048576 + 3, 3, 8)])
def test_walk_encode_matches(L, O, n, k, B, S, waves):
    """The persistent walk encoder (nk8_walk.hip: one wave walks its stripes
    chunk by chunk, grid-stride, fused XXH64) equals the fused kernel and the
    oracle, parts and digests, with and without digests: several stripes per
    wave (waves per CU capped low so the grid is smaller than the batch),
    several chunks per stripe, tails of every size (B not a multiple of 4,
    16 or k), one-byte blocks."""
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=321)
    ids_np = synth.batch_ids(S, n, first=321)
    ids = dev(ids_np)
    with _tuned(enc_kernel=_enc("fused")):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("walk"), enc_waves_per_cu=waves):
        p1, d1 = batch.encode(blocks, B, n, k, ids)
        p2, _ = batch.encode(blocks, B, n, k, ids, digests=False)
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps]) and torch.equal(d0, d1)
    assert torch.equal(p0[:, :ps], p2[:, :ps])
    host = blocks.cpu().numpy()
    got = [u64(x) for x in d1.cpu().tolist()]
    for s in sorted({0, S // 2, S - 1}):
        want = O.encode(host[s, :B], n, k, ids_np[s])
        assert np.array_equal(p1[s * n:(s + 1) * n, :ps].cpu().numpy(), np.stack(want))
        assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want]


@pytest.mark.parametrize("n,k,B,S", [(4, 2, 4096, 300), (8, 5, 262144, 40), (8, 5, 1048576, 9), (6, 3, 70001, 33),
                                     (8, 8, 777, 100), (5, 4, 4099, 64), (3, 3, 1, 7), (8, 7, 65536 * 7 + 5, 5)])
def test_slice_decode_matches(L, O, n, k, B, S):
    """The one-shot slice decoder (nk8_walk.hip: k_decode_plan selects the
    first k distinct offered ids and inverts per stripe, k_decode_slice
    rebuilds 1,024-row units per wave through an LDS transpose) rebuilds the
    same blocks as the wave decoder, for 1, 2 and 4 units per wave, tails of
    every size, duplicate and too-few ids (status -EINVAL, block left
    untouched, crt/nk8.c:512-537)."""
    from nkfs_amd import batch
    blocks = batch.synth(S, B, first=11)
    ids_np = synth.batch_ids(S, n, first=11)
    ids = dev(ids_np)
    parts, _ = batch.encode(blocks, B, n, k, ids)
    av = synth.batch_survivors(S, n, k, first=11)
    # every slot offered: the survivors first, then the rest; stripe 1's
    # second offered slot repeats the first one's id (the selection skips it
    # and takes the next), stripe 2 offers a single distinct id (-EINVAL)
    av = np.stack([np.concatenate([r, [j for j in range(n) if j not in r]]) for r in av]).astype(np.uint8)
    ids_np2 = ids_np.copy()
    if S > 2:
        ids_np2[1, av[1, 1]] = ids_np2[1, av[1, 0]]
        ids_np2[2, :] = ids_np2[2, 0]
    outs = []
    for kern, units in (("wave", 2), ("slice", 1), ("slice", 2), ("slice", 4), ("run", 1), ("run", 2), ("run", 4),
                        ("run", 16)):
        with _tuned(dec_kernel=_dec(kern), dec_units=min(units, 4), dec_run_units=units):
            out = torch.full((S, B), 0xEE, dtype=torch.uint8, device="cuda")
            o, st = batch.decode(parts, n, dev(ids_np2), dev(np.ascontiguousarray(av)), k, B, out=out)
            torch.cuda.synchronize()
            outs.append((out.clone(), st.cpu().tolist()))
    for o, st in outs[1:]:
        assert st == outs[0][1]
        assert torch.equal(o, outs[0][0])
    st = outs[0][1]
    for s in range(S):
        if s == 2 or (s == 1 and n == k):
            continue  # stripe 1 with n == k has no spare slot to take instead
        assert st[s] == 0 and torch.equal(outs[0][0][s], blocks[s, :B]), s
    if S > 2:
        assert st[2] == -22 and bool((outs[0][0][2] == 0xEE).all())


@pytest.mark.parametrize("n,k,B", [(8, 5, 262144), (8, 8, 4096 * 8 + 5), (6, 3, 70001), (4, 2, 4096), (3, 3, 777),
                                   (7, 2, 1)])
def test_nibble_tables_match(L, O, n, k, B):
    """Encode with nibble product tables (struct nkfs_tune enc_nib = 1; on by
    rule for large n <= 8 grids of the fused kernel) equals the 256-entry-
    table kernel and the oracle, parts and digests, uniform and ragged
    (size-ordered) batches, fused and walk encoders."""
    from nkfs_amd import batch
    S = 20
    blocks = batch.synth(S, B, first=123)
    ids_np = synth.batch_ids(S, n, first=123)
    ids = dev(ids_np)
    with _tuned(enc_kernel=_enc("fused"), enc_nib=0):
        p0, d0 = batch.encode(blocks, B, n, k, ids)
    with _tuned(enc_kernel=_enc("fused"), enc_nib=1):
        p1, d1 = batch.encode(blocks, B, n, k, ids)
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    assert torch.equal(p0[:, :ps], p1[:, :ps]) and torch.equal(d0, d1)
    host = blocks.cpu().numpy()
    for s in (0, S - 1):
        want = O.encode(host[s, :B], n, k, ids_np[s])
        assert [u64(x) for x in d1[s * n:(s + 1) * n].cpu().tolist()] == [O.xxh64(p) for p in want]
    # ragged: mixed sizes through the same tables, both encoders
    sizes = np.array([B, 1, 4096, 65536, B // 3 + 1] * 3, np.uint32)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k)
    hb = np.zeros(pos + 16, np.uint8)
    for s_, Bs in enumerate(sizes):
        hb[boff[s_]: boff[s_] + Bs] = synth.stripe_bytes(900 + s_, int(Bs))
    rid = synth.batch_ids(len(sizes), n, first=900)
    outs = []
    for kern in ("fused", "walk"):
        for nib in (0, 1):
            with _tuned(enc_kernel=_enc(kern), enc_nib=nib):
                parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
                dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
                batch.encode_ragged(dev(hb), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(rid), parts, dev(poff),
                                    dig, int(sizes.max()))
                torch.cuda.synchronize()
                outs.append((parts, dig))
    for p_, d_ in outs[1:]:
        assert torch.equal(outs[0][0], p_) and torch.equal(outs[0][1], d_)


@pytest.mark.parametrize("n,k,chunk", [(8, 5, 0), (4, 2, 1 << 20), (6, 3, 100000)])
def test_ragged_host_pipeline(L, O, n, k, chunk):
    """nkfs_nk8_encode_ragged_host (host memory in/out, C5 mixed sizes,
    sub-batches of consecutive stripes overlapped on three streams) equals
    the device-resident ragged encode, parts and digests, for pageable
    numpy buffers and several sub-batch sizes (one stripe larger than a
    sub-batch included)."""
    from nkfs_amd import batch
    sizes = synth.mixed_sizes(37)
    sizes[:4] = (1048576, 1, 4096, 70001)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, block_gap=8)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(500 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=500)
    parts_d = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    dig_d = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts_d, dev(poff),
                        dig_d, int(sizes.max()))
    torch.cuda.synchronize()
    parts_h = np.zeros(ppos, np.uint8)
    dig_h = np.zeros(len(sizes) * n, np.int64)
    batch.encode_ragged_host(host, boff, sizes.astype(np.int32), n, k, ids_np, parts_h, poff, dig_h,
                             chunk_bytes=chunk)
    assert np.array_equal(dig_h, dig_d.cpu().numpy())
    pd = parts_d.cpu().numpy()
    for s, B in enumerate(sizes):
        pitch = batch.part_pitch(int(B), k)
        ps = batch.part_size(int(B), k)
        for i in range(n):
            a = poff[s] + i * pitch
            assert np.array_equal(parts_h[a: a + ps], pd[a: a + ps]), (s, i)
    want = [O.xxh64(p) for p in O.encode(host[boff[3]: boff[3] + 70001], n, k, ids_np[3])]
    assert [u64(x) for x in dig_h[3 * n: 4 * n].tolist()] == want


@pytest.mark.parametrize("n,k,gap,order", [(8, 5, 0, 1), (8, 5, 3, 1), (6, 3, 16, 0), (7, 2, 0, 0)])
def test_ragged_kernels_match(L, O, n, k, gap, order):
    """A ragged n <= 8 batch (sizes on either side of 64 KiB parts, 1 MiB,
    4 KiB, 1 byte, odd sizes) gives the same parts and digests from the walk
    encoder (the ragged default: one wave per stripe), the fused kernel, the
    warp-specialised kernel (one or two hash waves) and the ragged split
    across the two (part-size windows at 64 KiB, 13,108 B = C5's 64 KiB
    stripes, 1 B = every stripe on ws), launched largest-first or in batch order
    (struct nkfs_tune size_order), aligned or not; digests of a sample
    against the oracle (crt/nk8.c:344-444, crt/xxhash.c:358-496)."""
    from nkfs_amd import batch
    sizes = np.array([k * 65536, k * 65535, 1048576, 4096, 1, 65536, k * 65536 + 1, 300000, 777] * 2, np.uint32)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, block_gap=gap)
    hb = np.zeros(pos + 16, np.uint8)
    for s_, Bs in enumerate(sizes):
        hb[boff[s_]: boff[s_] + Bs] = synth.stripe_bytes(1300 + s_, int(Bs))
    rid = synth.batch_ids(len(sizes), n, first=1300)
    outs = []
    # ("walk", hw, split): the ragged split -- stripes whose parts reach
    # `split` bytes on the warp-specialised kernel, the rest on the walk
    # encoder, two launches over complementary part-size windows
    for kern, hw, split in (("walk", 1, 0), ("fused", 1, 0), ("ws", 1, 0), ("ws", 2, 0), ("walk", 1, 65536),
                            ("walk", 2, 65536), ("walk", 2, 13108), ("walk", 1, 1)):
        with _tuned(enc_kernel=_enc(kern), size_order=order, enc_ws_hash_waves=hw, enc_ragged_split=split):
            parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
            dig = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
            batch.encode_ragged(dev(hb), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(rid), parts, dev(poff),
                                dig, int(sizes.max()))
            torch.cuda.synchronize()
            outs.append((parts, dig))
    for p_, d_ in outs[1:]:
        assert torch.equal(outs[0][0], p_) and torch.equal(outs[0][1], d_)
    got = [u64(x) for x in outs[0][1].cpu().tolist()]
    for s in (0, 1, 6, 7, 8):
        B = int(sizes[s])
        want = _oracle_digests(O, hb[None, boff[s]: boff[s] + B], rid[s:s + 1], n, k, B)
        assert got[s * n:(s + 1) * n] == want, (s, B)


@pytest.mark.parametrize("n,k,units", [(8, 5, 2), (6, 3, 4), (8, 8, 1)])
def test_ragged_slice_decode_matches_wave(L, n, k, units):
    """Ragged batches on the slice decoder (persistent grid over the scanned
    (stripe, slice) map, size order) rebuild the same blocks and statuses as
    the wave decoder, with part regions at unaligned offsets (byte loads),
    output blocks at unaligned offsets, one-byte and k+1-byte stripes, and a
    stripe offering too few distinct ids (-EINVAL, block untouched)."""
    from nkfs_amd import batch
    sizes = synth.mixed_sizes(30)
    sizes[:5] = (1048576, 1, k + 1, 4096 + 3, 65536)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, 5)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(40 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=40)
    parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff),
                        None, int(sizes.max()))
    # the same parts at offsets shifted by 0..7 bytes per stripe
    shift = np.arange(len(sizes), dtype=np.int64) % 8
    poff2 = poff + np.cumsum(shift)
    parts2 = torch.zeros(ppos + int(shift.sum()) + 16, dtype=torch.uint8, device="cuda")
    for s, B in enumerate(sizes):
        ln = n * batch.part_pitch(int(B), k)
        parts2[poff2[s]: poff2[s] + ln] = parts[poff[s]: poff[s] + ln]
    avail = synth.batch_survivors(len(sizes), n, k, first=40)
    ids2 = ids_np.copy()
    ids2[3, :] = ids2[3, 0]  # stripe 3: one distinct id
    outs = []
    for kern, pp, po in (("wave", parts, poff), ("slice", parts, poff), ("slice", parts2, poff2), ("run", parts, poff),
                         ("run", parts2, poff2)):
        with _tuned(dec_kernel=_dec(kern), dec_units=units):
            out = torch.full((pos + 16,), 0xEE, dtype=torch.uint8, device="cuda")
            st = batch.decode_ragged(pp, dev(po), n, dev(ids2), dev(avail), k, out, dev(boff),
                                     dev(sizes.astype(np.int32)), int(sizes.max()))
            torch.cuda.synchronize()
            outs.append((out.cpu(), st.cpu().tolist()))
    for o, st in outs[1:]:
        assert st == outs[0][1]
        assert torch.equal(o, outs[0][0])
    o, st = outs[0]
    assert st[3] == -22 and bool((o[boff[3]: boff[3] + sizes[3]] == 0xEE).all())
    for s, B in enumerate(sizes):
        if s != 3:
            assert st[s] == 0 and np.array_equal(o[boff[s]: boff[s] + B].numpy(), host[boff[s]: boff[s] + B]), s


@pytest.mark.parametrize("n,k,units", [(8, 5, 2), (6, 4, 4)])
def test_ragged_slice_decode_past_2gib(L, n, k, units):
    """The ragged slice decoder's persistent grid over more slices than it has
    waves (every wave walks several slices, with the next slice's descriptor
    prefetched) and with block and part offsets past 2^31 (64-bit offsets
    carried through the prefetch): encode -> erase n-k -> decode round trip,
    bit-exact, and the same bytes as the wave decoder (crt/nk8.c:446-599)."""
    from nkfs_amd import batch
    base = (1 << 31) + 4096
    sizes = np.array([1048576] * 28 + [4096, 65536, 777, 1048575] * 3, np.uint32)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, 0, first_off=base)
    poff = poff + base
    host = np.zeros(pos - base, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s] - base: boff[s] - base + B] = synth.stripe_bytes(900 + s, int(B))
    blocks = torch.zeros(pos, dtype=torch.uint8, device="cuda")
    blocks[base:] = dev(host)
    ids_np = synth.batch_ids(len(sizes), n, first=900)
    parts = torch.zeros(base + ppos, dtype=torch.uint8, device="cuda")
    sz = dev(sizes.astype(np.int32))
    batch.encode_ragged(blocks, dev(boff), sz, n, k, dev(ids_np), parts, dev(poff), None, int(sizes.max()))
    avail = synth.batch_survivors(len(sizes), n, k, first=900)
    res = []
    for kern in ("slice", "wave", "run"):
        with _tuned(dec_kernel=_dec(kern), dec_units=units):
            out = torch.zeros(pos, dtype=torch.uint8, device="cuda")
            st = batch.decode_ragged(parts, dev(poff), n, dev(ids_np), dev(avail), k, out, dev(boff), sz,
                                     int(sizes.max()))
            torch.cuda.synchronize()
            assert int(st.abs().sum()) == 0
            res.append(out[base:].cpu())
            del out
    assert torch.equal(res[0], res[1]) and torch.equal(res[0], res[2])
    assert np.array_equal(res[0].numpy(), host)
    del parts, blocks
    torch.cuda.empty_cache()


@pytest.mark.parametrize("S,B", [(512, 1048576), (1024, 1048576), (512, 262144), (1024, 262144)])
def test_bench_kernels_against_oracle(L, O, S, B):
    """The kernels the bench times, pinned through struct nkfs_tune and
    compared with the oracle directly (not only with another kernel): the
    warp-specialised encoder (C3's default) and the walk encoder (C4's) on
    >= 512 stripes -- every part's bytes and XXH64 of a 16-stripe sample
    spread over the batch -- and the one-shot slice decoder rebuilding every
    block from the seeded 5-of-8 survivors (crt/nk8.c:344-444, 446-599)."""
    from nkfs_amd import batch
    n, k = 8, 5
    blocks = batch.synth(S, B, first=4242)
    ids_np = synth.batch_ids(S, n, first=4242)
    ids = dev(ids_np)
    ps = batch.part_size(B, k)
    sample = sorted({int(x) for x in np.linspace(0, S - 1, 16)})
    for kern, pf, ne, hw in (("ws", 1, 4, 1), ("ws", 2, 4, 1), ("ws", 1, 6, 1), ("ws", 2, 6, 1), ("ws", 1, 4, 2),
                             ("ws", 2, 4, 2), ("walk", 1, 4, 1), ("auto", 1, 4, 0)):
        with _tuned(enc_kernel=_enc(kern), enc_ws_prefetch=pf, enc_ws_waves=ne, enc_ws_hash_waves=hw):
            parts, dig = batch.encode(blocks, B, n, k, ids)
        torch.cuda.synchronize()
        got = [u64(x) for x in dig.cpu().tolist()]
        for s in sample:
            want = O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])
            assert np.array_equal(parts[s * n:(s + 1) * n, :ps].cpu().numpy(), np.stack(want)), (kern, pf, ne, s)
            assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], (kern, pf, ne, s)
    avail = dev(synth.batch_survivors(S, n, k, first=4242))
    for kern in ("slice", "run"):
        with _tuned(dec_kernel=_dec(kern)):
            out, status = batch.decode(parts, n, ids, avail, k, B)
        torch.cuda.synchronize()
        assert int(status.abs().sum()) == 0
        assert torch.equal(out, blocks[:, :B]), kern


@pytest.mark.parametrize("n,k,waves,units", [(8, 5, 12, 4), (4, 2, 12, 2), (6, 3, 1, 4), (8, 8, 32, 1),
                                             (5, 4, 2, 8), (3, 2, 32, 2), (8, 5, 8, 16)])
def test_run_decode_walks_across_stripes(L, O, n, k, waves, units):
    """The run decoder (nk8_walk.hip k_run_plan + k_decode_run): every
    resident wave walks one contiguous run of 1,024-row units across stripe
    boundaries, with the next stripe's descriptor loaded ahead.  Runs that
    start and end inside stripes, stripes with too few distinct ids
    (-EINVAL, skipped, block untouched) at run boundaries and in a row,
    one-byte / k+1-byte / unit-boundary sizes, more waves than units
    (waves = 32 on a small batch) and a few long runs (waves = 1): blocks
    equal to the oracle's input, statuses equal to the wave decoder's
    (crt/nk8.c:446-599)."""
    from nkfs_amd import batch
    sizes = synth.mixed_sizes(300, (4096, 65536, 1048576, 1, k + 1, 1024 * k, 1024 * k + 1, 3 * 1024 * k - 1))
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, 3)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(7000 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=7000)
    parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff),
                        None, int(sizes.max()))
    avail = synth.batch_survivors(len(sizes), n, k, first=7000)
    ids2 = ids_np.copy()
    bad = {0, 17, 18, 19, 150, len(sizes) - 1}
    for s in bad:
        ids2[s, :] = ids2[s, 0]
    outs = []
    for kern in ("wave", "run"):
        with _tuned(dec_kernel=_dec(kern), dec_run_units=units, dec_waves_per_cu=waves):
            out = torch.full((pos + 16,), 0xEE, dtype=torch.uint8, device="cuda")
            st = batch.decode_ragged(parts, dev(poff), n, dev(ids2), dev(avail), k, out, dev(boff),
                                     dev(sizes.astype(np.int32)), int(sizes.max()))
            torch.cuda.synchronize()
            outs.append((out.cpu(), st.cpu().tolist()))
    assert outs[1][1] == outs[0][1]
    assert torch.equal(outs[1][0], outs[0][0])
    o, st = outs[1]
    for s, B in enumerate(sizes):
        if s in bad:
            assert st[s] == -22 and bool((o[boff[s]: boff[s] + B] == 0xEE).all()), s
        else:
            assert st[s] == 0 and np.array_equal(o[boff[s]: boff[s] + B].numpy(), host[boff[s]: boff[s] + B]), s
    # uniform: C2's shape (two units per stripe) through the same walk
    S, B = 3000, 4096
    blocks = batch.synth(S, B, first=77)
    uid = synth.batch_ids(S, n, first=77)
    up, _ = batch.encode(blocks, B, n, k, dev(uid))
    uav = dev(synth.batch_survivors(S, n, k, first=77))
    with _tuned(dec_kernel=_dec("run"), dec_run_units=units, dec_waves_per_cu=waves):
        out, status = batch.decode(up, n, dev(uid), uav, k, B)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 and torch.equal(out, blocks[:, :B])


@pytest.mark.parametrize("n,B,S", [(4, 4096, 3000), (4, 1, 9), (3, 3, 40), (6, 4097, 77), (4, 65536 * 2 + 7, 9),
                                   (255, 2048 * 4 + 1, 5), (2, 1048576, 3)])
def test_pair_decode_matches(L, O, n, B, S):
    """The k = 2 decoder (nk8_pair.hip: d1 = (p_a ^ p_b) / (x_a ^ x_b),
    d0 = p_a ^ x_a d1 from one product-table lookup per row) rebuilds the
    same blocks as the wave decoder and the oracle, with and without its
    output stage: every slot offered (the survivors first), stripe 1's second
    offer repeating the first one's id (the selection takes the next distinct
    one, crt/nk8.c:512-537), stripe 2 offering a single distinct id (status
    -EINVAL, block untouched); odd block sizes and tails of every length, long
    stripes split into row slices; the persistent pipelined form
    (dec_pair_pipe) on the shapes it takes."""
    from nkfs_amd import batch
    k = 2
    blocks = batch.synth(S, B, first=21)
    ids_np = synth.batch_ids(S, n, first=21)
    parts, _ = batch.encode(blocks, B, n, k, dev(ids_np))
    av = synth.batch_survivors(S, n, k, first=21)
    av = np.stack([np.concatenate([r, [j for j in range(n) if j not in r]]) for r in av]).astype(np.uint8)
    ids2 = ids_np.copy()
    if S > 2:
        ids2[1, av[1, 1]] = ids2[1, av[1, 0]]
        ids2[2, :] = ids2[2, 0]
    outs = []
    # pipe > 0: the persistent pipelined form (uniform blocks <= 4 KiB; 2
    # waves per CU: 512 waves walking 5-6 stripes each on the 3,000-stripe case)
    for kern, stage, waves, pipe in (("wave", 1, 4, 0), ("pair", 1, 4, 0), ("pair", 0, 1, 0), ("pair", 1, 1, 0),
                                     ("pair", 0, 4, 0), ("pair", 1, 1, 2), ("pair", 0, 1, 2), ("auto", 1, 1, 16)):
        with _tuned(dec_kernel=_dec(kern), dec_pair_stage=stage, dec_pair_waves=waves, dec_pair_pipe=pipe):
            out = torch.full((S, B), 0xEE, dtype=torch.uint8, device="cuda")
            _, st = batch.decode(parts, n, dev(ids2), dev(av), k, B, out=out)
            torch.cuda.synchronize()
            outs.append((out.clone(), st.cpu().tolist()))
    for o, st in outs[1:]:
        assert st == outs[0][1]
        assert torch.equal(o, outs[0][0])
    o, st = outs[1]
    for s in range(S):
        if s == 2 or (s == 1 and n == k):
            continue
        assert st[s] == 0 and torch.equal(o[s], blocks[s, :B]), s
    if S > 2:
        assert st[2] == -22 and bool((o[2] == 0xEE).all())
    # the oracle's assemble of the last stripe from its first two offers
    s = S - 1
    sel = [int(x) for x in av[s][:2]]
    pn = parts[s * n:(s + 1) * n, :batch.part_size(B, k)].cpu().numpy()
    assert np.array_equal(np.asarray(O.decode([pn[j] for j in sel], ids_np[s][sel], k, B)), blocks[s, :B].cpu().numpy())


@pytest.mark.parametrize("gap,stage,waves", [(0, 1, 4), (3, 1, 1), (5, 0, 4), (0, 0, 1)])
def test_pair_decode_ragged(L, gap, stage, waves):
    """The k = 2 decoder on a ragged batch (size order applied, blocks at
    unaligned offsets): every stripe back bit-exact, gap bytes untouched."""
    from nkfs_amd import batch
    n, k = 4, 2
    sizes = synth.mixed_sizes(40)
    sizes[:5] = (4096, 1, 3, 1048576, 70001)
    boff, poff, pos, ppos = _ragged_layout(sizes, n, k, gap)
    host = np.zeros(pos + 16, np.uint8)
    for s, B in enumerate(sizes):
        host[boff[s]: boff[s] + B] = synth.stripe_bytes(700 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=700)
    parts = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    batch.encode_ragged(dev(host), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts, dev(poff),
                        None, int(sizes.max()))
    avail = synth.batch_survivors(len(sizes), n, 3, first=700)
    out = torch.zeros(pos + 16, dtype=torch.uint8, device="cuda")
    with _tuned(dec_kernel=_dec("pair"), dec_pair_stage=stage, dec_pair_waves=waves):
        status = batch.decode_ragged(parts, dev(poff), n, dev(ids_np), dev(avail), k, out, dev(boff),
                                     dev(sizes.astype(np.int32)), int(sizes.max()))
    torch.cuda.synchronize()
    assert status.abs().sum().item() == 0
    got = out.cpu().numpy()
    mask = np.ones(pos + 16, bool)
    for s, B in enumerate(sizes):
        assert np.array_equal(got[boff[s]: boff[s] + B], host[boff[s]: boff[s] + B]), (s, int(B))
        mask[boff[s]: boff[s] + B] = False
    assert not got[mask].any()


def test_c5_bench_scale_default_dispatch(L, O):
    """C5 at the bench's own scale and layout (11,520 ragged stripes, 4 KiB /
    64 KiB / 1 MiB, ~4 GiB, blocks 256-B aligned, parts at the library's
    pitch) through the DEFAULT dispatch -- the size-ordered walk encoder and
    the run decoder that only batches of >= 2,048 ragged stripes take
    (this path was checked only by the bench's own verify):
    every block back bit-exact after erasing n - k parts, every status 0,
    digests and parts of a sample of every size class against the oracle."""
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
    parts = torch.empty(ppos, dtype=torch.uint8, device="cuda")
    dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
    batch.encode_ragged(blocks, bo, sz, n, k, ids, parts, po, dig, int(sizes.max()))
    avail = dev(synth.batch_survivors(S, n, k, first=0))
    out = torch.zeros(pos, dtype=torch.uint8, device="cuda")
    status = batch.decode_ragged(parts, po, n, ids, avail, k, out, bo, sz, int(sizes.max()))
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert torch.equal(out, blocks)
    del out
    got = [u64(x) for x in dig.cpu().tolist()]
    for B in (4096, 65536, 1048576):
        for s in np.nonzero(sizes == B)[0][[0, -1]].tolist():
            blk = blocks[boff[s]: boff[s] + B].cpu().numpy()
            want = O.encode(blk, n, k, ids_np[s])
            assert got[s * n:(s + 1) * n] == [O.xxh64(p) for p in want], (s, B)
            pitch = batch.part_pitch(B, k)
            pn = parts[poff[s]: poff[s] + n * pitch].cpu().numpy().reshape(n, pitch)[:, :len(want[0])]
            assert np.array_equal(pn, np.stack(want)), (s, B)
