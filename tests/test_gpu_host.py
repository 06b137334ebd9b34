"""Host-memory entry points (include/nkfs_gpu.h, pipeline.c) through the
C-ABI: PUT/GET from contiguous host buffers and from page lists
(core/upages.c:91-148, core/net.c:145-265), several sub-batch sizes, device
lanes (nkfs_gpu_set_devices), and the write-back contract (bytes outside the
defined outputs keep the caller's contents).  Checked against the
device-resident entry points and the pinned oracle, bit-exact.
"""
import threading

import numpy as np
import pytest

from nkfs_amd import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SENT = 0xA5


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
    """numpy -> device through a pinned bounce (no DMA from pageable memory
    in the tests either: DESIGN.md §5.6)."""
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().cuda()


def host(t):
    """device tensor -> numpy through a pinned buffer."""
    out = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    out.copy_(t)
    return out.numpy()


def pinned_np(nbytes, fill=None):
    """a pinned (hipHostMalloc) uint8 numpy array: DMA'd directly by the
    host entry points, where pageable arrays are staged."""
    a = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()
    if fill is not None:
        a[:] = fill
    return a


@pytest.fixture(autouse=True)
def host_state_clean(L):
    """Every host call leaves nothing behind: no registry reference, lane or
    copy thread, and the same registrations and contexts as before
    (VERDICT r05 item 1)."""
    from nkfs_amd import batch
    before = batch.host_state()
    yield
    after = batch.host_state()
    assert after["call_refs"] == 0 and after["lanes"] == 0 and after["copy_threads"] == 0, after
    assert after["registered"] == before["registered"] and after["contexts"] == before["contexts"], (before, after)


def u64(x):
    return int(x) & 0xFFFFFFFFFFFFFFFF


def ragged_layout(sizes, n_slots, k, block_gap=0, part_gap=0):
    from nkfs_amd import batch
    boff = np.zeros(len(sizes), np.int64)
    poff = np.zeros(len(sizes), np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos
        pos += int(B) + block_gap
        ppos += n_slots * batch.part_pitch(int(B), k) + part_gap
    return boff, poff, pos, ppos


def scatter_pages(blocks, page_size, rng):
    """Put each block's bytes into its own 4 KiB pages, laid out in a
    shuffled arena (like core/upages.c's page arrays): returns the arena,
    the page address list and each stripe's first page index."""
    npg = [max(1, -(-len(b) // page_size)) for b in blocks]
    total = sum(npg)
    arena = np.full(total * page_size, SENT, np.uint8)
    slots = rng.permutation(total)
    base = arena.ctypes.data
    pages = np.zeros(total, np.int64)
    first = np.zeros(len(blocks), np.int64)
    p = 0
    for s, b in enumerate(blocks):
        first[s] = p
        for i in range(npg[s]):
            slot = int(slots[p])
            pages[p] = base + slot * page_size
            chunk = b[i * page_size:(i + 1) * page_size]
            arena[slot * page_size: slot * page_size + len(chunk)] = chunk
            p += 1
    return arena, pages, first


def gather_pages(arena, pages, first, sizes, page_size):
    base = arena.ctypes.data
    out = []
    for s, B in enumerate(sizes):
        b = np.empty(int(B), np.uint8)
        for i in range(-(-int(B) // page_size)):
            off = int(pages[first[s] + i]) - base
            n = min(page_size, int(B) - i * page_size)
            b[i * page_size: i * page_size + n] = arena[off: off + n]
        out.append(b)
    return out


# ---------------------------------------------------------------- GET, uniform

@pytest.mark.parametrize("S,B,n,k,chunk,pitch_pad", [(3000, 4096, 4, 2, 0, 0), (200, 262144, 8, 5, 1 << 20, 0),
                                                     (97, 70001, 6, 3, 300000, 13), (40, 30000, 16, 12, 0, 7)])
def test_decode_host_round_trip(L, O, S, B, n, k, chunk, pitch_pad):
    """nkfs_nk8_decode_host: the k survivors of every stripe (random subset,
    random order) shipped from host memory rebuild each block bit-exact;
    pitched output keeps the gap bytes; a stripe offered duplicate ids
    (fewer than k distinct) returns -EINVAL and keeps its block bytes."""
    from nkfs_amd import batch
    rng = np.random.default_rng(S + B)
    blocks = batch.synth(S, B, first=11)
    ids_np = synth.batch_ids(S, n, first=11)
    parts, _ = batch.encode(blocks, B, n, k, dev(ids_np))
    torch.cuda.synchronize()
    pitch = batch.part_pitch(B, k)
    pn = host(parts).reshape(S, n, pitch)
    # survivors: k random slots per stripe, packed as the caller holds them
    pick = np.stack([rng.permutation(n)[:k] for _ in range(S)])
    held = np.ascontiguousarray(pn[np.arange(S)[:, None], pick])          # [S, k, pitch]
    hid = np.ascontiguousarray(ids_np[np.arange(S)[:, None], pick])       # [S, k]
    avail = np.tile(np.arange(k, dtype=np.uint8), (S, 1))
    bad = 5 % S
    hid[bad, 1] = hid[bad, 0]  # duplicate id: fewer than k distinct
    bp = B + pitch_pad
    out = np.full(S * bp, SENT, np.uint8)
    status = np.full(S, 99, np.int32)
    rc = batch.decode_host(held.reshape(-1), pitch, k, hid.reshape(-1), avail.reshape(-1), k, k, B, out, bp,
                           status=status, chunk_bytes=chunk)
    assert rc == 0
    want = host(blocks)[:, :B]
    got = out.reshape(S, bp)
    ok = np.ones(S, bool)
    ok[bad] = False
    assert status[bad] == -22 and (status[ok] == 0).all()
    assert np.array_equal(got[ok, :B], want[ok])
    assert (got[bad] == SENT).all()
    if pitch_pad:
        assert (got[:, B:] == SENT).all()
    # one stripe through the oracle's assemble as well
    s = 1
    ob = O.decode([held[s, c, :batch.part_size(B, k)] for c in range(k)], hid[s], k, B)
    assert np.array_equal(ob, want[s])


def test_decode_host_verify(L):
    """GET with the part check fused in (h_expect): a flipped byte in a
    part that is used fails its stripe with -EIO and flags the slot."""
    from nkfs_amd import batch
    S, B, n, k = 300, 65536, 8, 5
    blocks = batch.synth(S, B, first=77)
    ids_np = synth.batch_ids(S, n, first=77)
    parts, dig = batch.encode(blocks, B, n, k, dev(ids_np))
    torch.cuda.synchronize()
    pitch = batch.part_pitch(B, k)
    pn = host(parts).copy().reshape(-1)
    dg = host(dig)
    pn[(9 * n + 2) * pitch + 100] ^= 1
    avail = np.tile(np.array([2, 0, 4, 6, 7, 1], np.uint8), (S, 1))
    out = np.zeros(S * B, np.uint8)
    status = np.zeros(S, np.int32)
    badmask = np.zeros(S, np.int64)
    assert batch.decode_host(pn, pitch, n, ids_np.reshape(-1), avail.reshape(-1), 6, k, B, out, B,
                             status=status, expect=dg, badmask=badmask, chunk_bytes=4 << 20) == 0
    assert status[9] == -5 and badmask[9] == 1 << 2
    others = np.arange(S) != 9
    assert (status[others] == 0).all() and (badmask[others] == 0).all()
    assert np.array_equal(out.reshape(S, B)[others], host(blocks)[others, :B])


# ---------------------------------------------------------------- ragged, gaps

@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("n,k,chunk", [(8, 5, 0), (4, 2, 1 << 20), (6, 3, 100000)])
def test_ragged_host_gaps_untouched(L, n, k, chunk, pinned):
    """PUT and GET of a ragged batch whose block and part ranges have gaps
    between stripes: parts/blocks equal the device-resident result and
    every gap byte keeps the caller's sentinel (pipeline.c);
    pageable buffers (staged) and pinned ones (direct DMA) alike."""
    from nkfs_amd import batch
    alloc = pinned_np if pinned else (lambda nb, fill: np.full(nb, fill, np.uint8))
    sizes = synth.mixed_sizes(29)
    sizes[:3] = (1048576, 1, 70001)
    boff, poff, pos, ppos = ragged_layout(sizes, n, k, block_gap=24, part_gap=48)
    hostb = alloc(pos, SENT)
    for s, B in enumerate(sizes):
        hostb[boff[s]: boff[s] + B] = synth.stripe_bytes(900 + s, int(B))
    host_ = hostb
    ids_np = synth.batch_ids(len(sizes), n, first=900)
    parts_h = alloc(ppos, SENT)
    dig_h = np.zeros(len(sizes) * n, np.int64)
    batch.encode_ragged_host(host_, boff, sizes.astype(np.int32), n, k, ids_np, parts_h, poff, dig_h,
                             chunk_bytes=chunk)
    parts_d = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    dig_d = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
    batch.encode_ragged(dev(host_), dev(boff), dev(sizes.astype(np.int32)), n, k, dev(ids_np), parts_d, dev(poff),
                        dig_d, int(sizes.max()))
    torch.cuda.synchronize()
    assert np.array_equal(dig_h, host(dig_d))
    pd = host(parts_d)
    inside = np.zeros(ppos, bool)
    for s, B in enumerate(sizes):
        pitch, ps = batch.part_pitch(int(B), k), batch.part_size(int(B), k)
        inside[poff[s]: poff[s] + n * pitch] = True
        for i in range(n):
            a = poff[s] + i * pitch
            assert np.array_equal(parts_h[a: a + ps], pd[a: a + ps]), (s, i)
    assert (parts_h[~inside] == SENT).all()
    # GET from every slot back into a sentinel-filled buffer with gaps
    rng = np.random.default_rng(n)
    avail = np.stack([rng.permutation(n) for _ in sizes]).astype(np.uint8)
    out = alloc(pos, SENT)
    status = np.full(len(sizes), 7, np.int32)
    assert batch.decode_ragged_host(parts_h, poff, n, ids_np, avail, n, k, out, boff, sizes.astype(np.int32),
                                    status=status, chunk_bytes=chunk) == 0
    assert (status == 0).all()
    blk = np.zeros(pos, bool)
    for s, B in enumerate(sizes):
        blk[boff[s]: boff[s] + B] = True
    assert np.array_equal(out[blk], host_[blk]) and (out[~blk] == SENT).all()


# ---------------------------------------------------------------- page lists

@pytest.mark.parametrize("n,k,chunk,page", [(8, 5, 0, 4096), (4, 2, 1 << 20, 4096), (6, 3, 200000, 512)])
def test_pages_put_get(L, O, n, k, chunk, page):
    """PUT from page lists (nkfs_nk8_encode_pages: each block spread over
    pages in a shuffled arena, as core/upages.c holds a payload) equals the
    device-resident ragged encode; GET back into fresh page lists
    (nkfs_nk8_decode_pages) rebuilds every block; digests of a sample
    against the oracle."""
    from nkfs_amd import batch
    rng = np.random.default_rng(page + n)
    sizes = synth.mixed_sizes(26)
    sizes[:4] = (1048576, 1, page, page + 1)
    blocks = [synth.stripe_bytes(2000 + s, int(B)) for s, B in enumerate(sizes)]
    arena, pages, first = scatter_pages(blocks, page, rng)
    ids_np = synth.batch_ids(len(sizes), n, first=2000)
    _, poff, _, ppos = ragged_layout(sizes, n, k, part_gap=16)
    parts_h = np.full(ppos, SENT, np.uint8)
    dig_h = np.zeros(len(sizes) * n, np.int64)
    sz32 = sizes.astype(np.int32)
    assert batch.encode_pages(pages, page, first, sz32, n, k, ids_np, parts_h, poff, dig_h, chunk_bytes=chunk) == 0
    # reference: the same bytes packed, device-resident ragged encode
    boff, _, pos, _ = ragged_layout(sizes, n, k)
    packed = np.concatenate(blocks)
    parts_d = torch.zeros(ppos, dtype=torch.uint8, device="cuda")
    dig_d = torch.zeros(len(sizes) * n, dtype=torch.int64, device="cuda")
    batch.encode_ragged(dev(packed), dev(boff), dev(sz32), n, k, dev(ids_np), parts_d, dev(poff), dig_d,
                        int(sizes.max()))
    torch.cuda.synchronize()
    assert np.array_equal(dig_h, host(dig_d))
    pd = host(parts_d)
    for s, B in enumerate(sizes):
        pitch, ps = batch.part_pitch(int(B), k), batch.part_size(int(B), k)
        for i in range(n):
            a = poff[s] + i * pitch
            assert np.array_equal(parts_h[a: a + ps], pd[a: a + ps]), (s, i)
    for s in (2, 3):
        want = [O.xxh64(p) for p in O.encode(blocks[s], n, k, ids_np[s])]
        assert [u64(x) for x in dig_h[s * n:(s + 1) * n]] == want
    # GET into fresh, differently shuffled pages (erase n-k slots per stripe)
    arena2, pages2, first2 = scatter_pages([np.zeros(int(B), np.uint8) for B in sizes], page, rng)
    arena2[:] = SENT
    avail = np.stack([rng.permutation(n)[:k] for _ in sizes]).astype(np.uint8)
    status = np.full(len(sizes), 3, np.int32)
    assert batch.decode_pages(parts_h, poff, n, ids_np, avail, k, k, pages2, page, first2, sz32, status=status,
                              chunk_bytes=chunk) == 0
    assert (status == 0).all()
    got = gather_pages(arena2, pages2, first2, sizes, page)
    for s in range(len(sizes)):
        assert np.array_equal(got[s], blocks[s]), s
    # page tails past each block keep the sentinel
    base = arena2.ctypes.data
    for s, B in enumerate(sizes):
        last = int(pages2[first2[s] + (int(B) - 1) // page]) - base
        used = int(B) - ((int(B) - 1) // page) * page
        assert (arena2[last + used: last + page] == SENT).all()


# ---------------------------------------------------------------- device lanes

def test_lanes_split_identical(L):
    """nkfs_gpu_set_devices with several lanes (the same device repeated on
    a one-GPU box, every visible device otherwise): the byte-balanced split
    gives the same parts, digests and rebuilt blocks as one lane."""
    from nkfs_amd import batch
    ndev = L.nkfs_gpu_count()
    lanes = [0, 0, 0] if ndev < 2 else list(range(min(ndev, 4)))
    S, B, n, k = 1000, 65536, 8, 5
    host_ = np.ascontiguousarray(host(batch.synth(S, B, first=3)))
    ids_np = synth.batch_ids(S, n, first=3)
    ref_parts, ref_dig = batch.encode_host(host_, B, n, k, ids_np, chunk_bytes=4 << 20)
    try:
        assert batch.set_devices(lanes) == 0
        assert batch.get_devices() == lanes
        parts, dig = batch.encode_host(host_, B, n, k, ids_np, chunk_bytes=4 << 20)
        assert torch.equal(parts[:, :batch.part_size(B, k)], ref_parts[:, :batch.part_size(B, k)])
        assert torch.equal(dig, ref_dig)
        out = np.zeros(S * B, np.uint8)
        status = np.zeros(S, np.int32)
        avail = np.tile(np.array([7, 6, 5, 4, 3], np.uint8), (S, 1))
        assert batch.decode_host(parts.numpy().reshape(-1), batch.part_pitch(B, k), n, ids_np.reshape(-1),
                                 avail.reshape(-1), k, k, B, out, B, status=status, chunk_bytes=4 << 20) == 0
        assert (status == 0).all() and np.array_equal(out.reshape(S, B), host_[:, :B])
        # ragged, byte-balanced over the lanes
        sizes = synth.mixed_sizes(300)
        boff, poff, pos, ppos = ragged_layout(sizes, n, k)
        hb = np.zeros(pos, np.uint8)
        for s, Bs in enumerate(sizes):
            hb[boff[s]: boff[s] + Bs] = synth.stripe_bytes(s, int(Bs))
        rid = synth.batch_ids(len(sizes), n)
        got = []
        for ln in (lanes, []):
            assert batch.set_devices(ln) == 0
            ph = np.zeros(ppos, np.uint8)
            dh = np.zeros(len(sizes) * n, np.int64)
            batch.encode_ragged_host(hb, boff, sizes.astype(np.int32), n, k, rid, ph, poff, dh, chunk_bytes=8 << 20)
            got.append((ph, dh))
        defined = np.zeros(ppos, bool)  # part bytes (the pitch padding is unspecified)
        for s, Bs in enumerate(sizes):
            pitch, ps = batch.part_pitch(int(Bs), k), batch.part_size(int(Bs), k)
            for i in range(n):
                defined[poff[s] + i * pitch: poff[s] + i * pitch + ps] = True
        assert np.array_equal(got[0][1], got[1][1])
        assert np.array_equal(got[0][0][defined], got[1][0][defined])
    finally:
        batch.set_devices([])
    assert batch.get_devices() == [L.nkfs_gpu_device()]


def test_set_devices_rejects_missing(L):
    from nkfs_amd import batch
    assert batch.set_devices([L.nkfs_gpu_count()]) == -19  # -ENODEV
    assert batch.get_devices() == [L.nkfs_gpu_device()]


# ---------------------------------------------------------------- pin registry

def test_concurrent_calls_share_pageable_buffer(L):
    """Several threads run the host pipeline on the same pageable buffers
    at once: the registration is reference counted, so no call unpins
    memory another call is still copying (pipeline.c pin())."""
    from nkfs_amd import batch
    S, B, n, k = 600, 65536, 8, 5
    host_ = np.ascontiguousarray(host(batch.synth(S, B, first=8)))
    ids_np = synth.batch_ids(S, n, first=8)
    ref, ref_dig = batch.encode_host(host_, B, n, k, ids_np)
    errs = []

    def work():
        try:
            for _ in range(3):
                p, d = batch.encode_host(host_, B, n, k, ids_np, chunk_bytes=2 << 20)
                assert torch.equal(d, ref_dig)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def test_host_register_api(L):
    buf = np.zeros(1 << 20, np.uint8)
    p = buf.ctypes.data
    assert L.nkfs_host_register(p, buf.nbytes) == 0
    assert L.nkfs_host_register(p, buf.nbytes) == 0   # second reference
    assert L.nkfs_host_unregister(p) == 0
    assert L.nkfs_host_unregister(p) == 0
    assert L.nkfs_host_unregister(p) == -2            # -ENOENT: released
    pinned = torch.empty(4096, dtype=torch.uint8, pin_memory=True)
    assert L.nkfs_host_register(pinned.data_ptr(), 4096) == -17  # -EEXIST: runtime-pinned


def test_partial_overlap_with_registration_is_staged(L):
    """A host call whose buffer starts inside a range registered through
    nkfs_host_register but runs past its end is staged through pinned
    scratch (no DMA touches it, so its owner may unregister at any time);
    the range inside the registration is DMA'd directly and holds a
    reference only while the call runs.  All three give the digests of an
    unrelated copy of the same bytes (round 6: nothing is registered for a
    call)."""
    from nkfs_amd import batch
    B, n, k = 65536, 8, 5
    buf = np.zeros(4 * B, np.uint8)
    buf[:] = np.frombuffer(np.random.default_rng(5).bytes(buf.nbytes), np.uint8)
    ids_np = synth.batch_ids(2, n, first=77)
    assert L.nkfs_host_register(buf.ctypes.data, 2 * B) == 0
    try:
        assert batch.host_state()["registered"] >= 1
        p_in, d_in = batch.encode_host(buf[: 2 * B].reshape(2, B), B, n, k, ids_np)
        p_st, d_st = batch.encode_host(buf[B: 3 * B].reshape(2, B), B, n, k, ids_np)
        assert batch.host_state()["call_refs"] == 0
    finally:
        assert L.nkfs_host_unregister(buf.ctypes.data) == 0
    p_ref, d_ref = batch.encode_host(np.ascontiguousarray(buf[B: 3 * B]).reshape(2, B), B, n, k, ids_np)
    p_r0, d_r0 = batch.encode_host(np.ascontiguousarray(buf[: 2 * B]).reshape(2, B), B, n, k, ids_np)
    assert torch.equal(d_st, d_ref) and torch.equal(d_in, d_r0)
    ps = batch.part_size(B, k)
    assert torch.equal(p_st[:, :ps], p_ref[:, :ps]) and torch.equal(p_in[:, :ps], p_r0[:, :ps])


def test_registration_overlap_refused(L):
    """nkfs_host_register of a range that partly overlaps a registered one
    is -EBUSY; the same range again is a second reference."""
    buf = np.zeros(1 << 18, np.uint8)
    p = buf.ctypes.data
    assert L.nkfs_host_register(p, 1 << 17) == 0
    try:
        assert L.nkfs_host_register(p + (1 << 16), 1 << 17) == -16
    finally:
        assert L.nkfs_host_unregister(p) == 0


@pytest.mark.parametrize("n,k,chunk", [(6, 3, 200000), (8, 5, 1 << 20)])
def test_staged_equals_direct(L, n, k, chunk):
    """The round-5 fault geometry (N6K3, 200,000-B sub-batches, mixed sizes
    with 1 MiB, 1 B and page-edge stripes) through every buffer kind: PUT and
    GET from pageable arrays (staged), pinned arrays (direct DMA) and a
    registered range give identical parts, digests and blocks."""
    from nkfs_amd import batch
    sizes = synth.mixed_sizes(26)
    sizes[:4] = (1048576, 1, 512, 513)
    boff, poff, pos, ppos = ragged_layout(sizes, n, k, block_gap=8, part_gap=16)
    src = np.full(pos, SENT, np.uint8)
    for s, B in enumerate(sizes):
        src[boff[s]: boff[s] + B] = synth.stripe_bytes(3000 + s, int(B))
    ids_np = synth.batch_ids(len(sizes), n, first=3000)
    sz32 = sizes.astype(np.int32)
    rng = np.random.default_rng(n)
    avail = np.stack([rng.permutation(n)[:k] for _ in sizes]).astype(np.uint8)
    results = []
    for kind in ("pageable", "pinned", "registered"):
        if kind == "pinned":
            bl, pa, out = pinned_np(pos, SENT), pinned_np(ppos, SENT), pinned_np(pos, SENT)
        else:
            bl, pa, out = np.full(pos, SENT, np.uint8), np.full(ppos, SENT, np.uint8), np.full(pos, SENT, np.uint8)
        bl[:] = src
        regs = []
        if kind == "registered":
            for a in (bl, pa, out):
                assert L.nkfs_host_register(a.ctypes.data, a.nbytes) == 0
                regs.append(a.ctypes.data)
        try:
            dg = np.zeros(len(sizes) * n, np.int64)
            batch.encode_ragged_host(bl, boff, sz32, n, k, ids_np, pa, poff, dg, chunk_bytes=chunk)
            st = np.full(len(sizes), 9, np.int32)
            assert batch.decode_ragged_host(pa, poff, n, ids_np, avail, k, k, out, boff, sz32, status=st,
                                            chunk_bytes=chunk) == 0
            assert (st == 0).all()
            assert batch.host_state()["call_refs"] == 0
        finally:
            for p in regs:
                assert L.nkfs_host_unregister(p) == 0
        assert np.array_equal(out, src), kind
        results.append((pa.copy(), dg.copy()))
    defined = np.zeros(ppos, bool)  # part bytes (the pitch padding is unspecified)
    for s, B in enumerate(sizes):
        pitch, ps = batch.part_pitch(int(B), k), batch.part_size(int(B), k)
        for i in range(n):
            defined[poff[s] + i * pitch: poff[s] + i * pitch + ps] = True
    for pa, dg in results[1:]:
        assert np.array_equal(dg, results[0][1])
        assert np.array_equal(pa[defined], results[0][0][defined])


# ---------------------------------------------------------------- general path, big parts

def test_generic_parts_beyond_grid_y(L, O):
    """n > 8 with parts past 16 MiB: the general kernels grid-stride over
    rows beyond 65,535 x 256.  Round trip, and part bytes at
    rows past that limit against the GF product table."""
    from nkfs_amd import batch
    n, k = 10, 9
    B = 9 * (17 << 20) + 5
    blocks = batch.synth(1, B, first=4)
    ids_np = np.array([[3, 9, 27, 81, 243, 1, 2, 4, 8, 16]], np.uint8)
    parts, dig = batch.encode(blocks, B, n, k, dev(ids_np))
    torch.cuda.synchronize()
    ps = batch.part_size(B, k)
    mul = O.gf_mul_table()
    blk = host(blocks[0, :B])
    pn = host(parts)
    for j in (0, 65535 * 256 + 3, ps - 1):
        row = np.zeros(k, np.uint8)
        seg = blk[j * k: j * k + k]
        row[:len(seg)] = seg
        for i in range(n):
            c, acc = 1, 0
            for m in range(k):
                acc ^= int(mul[c, row[m]])
                c = int(mul[c, ids_np[0, i]])
            assert pn[i, j] == acc, (i, j)
    avail = dev(np.array([[9, 7, 5, 3, 1, 0, 2, 4, 6]], np.uint8))
    out, st = batch.decode(parts, n, dev(ids_np), avail, k, B)
    torch.cuda.synchronize()
    assert int(st[0]) == 0 and torch.equal(out[0, :B], blocks[0, :B])


def test_synth_ragged_matches_uniform(L):
    """nkfs_synth_ragged (the bench's one-launch C5 input) gives every stripe
    the bytes of the synthetic stream (nkfs_amd/synth.py), gaps untouched."""
    from nkfs_amd import batch
    sizes = np.array([1, 7, 4096, 65536, 1048576, 300001, 8], np.uint32)
    boff, _, pos, _ = ragged_layout(sizes, 1, 1, block_gap=5)
    buf = torch.full((pos,), SENT, dtype=torch.uint8, device="cuda")
    batch.synth_ragged(buf, dev(boff), dev(sizes.astype(np.int32)), first=40)
    torch.cuda.synchronize()
    got = host(buf)
    inside = np.zeros(pos, bool)
    for s, B in enumerate(sizes):
        assert np.array_equal(got[boff[s]: boff[s] + B], synth.stripe_bytes(40 + s, int(B))), s
        inside[boff[s]: boff[s] + B] = True
    assert (got[~inside] == SENT).all()
