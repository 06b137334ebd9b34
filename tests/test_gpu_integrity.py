"""GPU parity for the core's integrity-path hash shapes (SURVEY.md §8(f)
rows 1-2): whole-cluster sums with the fused stored-sum compare
(nkfs_clu_sum_batch: core/dio.c:26-37, core/inode.c:561-575) and payload
dsums over scattered 4 KiB page lists (nkfs_pages_dsum_batch:
core/upages.c:124-148), against the reference's Config 1 fixture and the
pinned oracle, bit-exact.
"""
import numpy as np
import pytest

from nkfs_amd import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def B():
    from nkfs_amd import _lib, batch
    assert _lib.lib().nk8_init() == 0
    return batch


@pytest.fixture(scope="module")
def O():
    from oracle import oracle
    return oracle


def hexs(t):
    return [f"{v & 0xFFFFFFFFFFFFFFFF:016x}" for v in t.cpu().tolist()]


def c1_object(golden):
    c1 = golden["c1"]
    return c1, synth.stripe_bytes(c1["stripe"], c1["object_size"])


def test_c1_cluster_sums_and_check(B, golden):
    c1, obj = c1_object(golden)
    ch = c1["chunk"]
    nclu = (obj.size + ch - 1) // ch
    clus = np.zeros((nclu, ch), np.uint8)
    clus.reshape(-1)[:obj.size] = obj
    d = torch.from_numpy(clus).cuda()
    sums, st = B.clu_sum(d)
    assert st is None
    assert hexs(sums) == c1["cluster_sums"]
    # fused compare: one corrupted stored sum, one corrupted cluster
    expect = sums.clone()
    expect[3] ^= 1
    d[7, 65535] ^= 0x80
    sums2, st = B.clu_sum(d, expect=expect)
    st = st.cpu().tolist()
    bad = {i for i, v in enumerate(st) if v != 0}
    assert bad == {3, 7} and all(st[i] == -22 for i in bad)
    assert hexs(sums2)[:7] == c1["cluster_sums"][:7]


def test_c1_payload_dsums_over_scattered_pages(B, golden):
    c1, obj = c1_object(golden)
    ch, page = c1["chunk"], 4096
    npages = (obj.size + page - 1) // page
    rng = np.random.default_rng(11)
    slot = rng.permutation(npages + 37)[:npages]  # page p lives in pool slot slot[p]
    pool = np.zeros((npages + 37, page), np.uint8)
    padded = np.zeros(npages * page, np.uint8)
    padded[:obj.size] = obj
    pool[slot] = padded.reshape(npages, page)
    dpool = torch.from_numpy(pool).cuda()
    ptrs = torch.tensor([dpool.data_ptr() + int(s) * page for s in slot], dtype=torch.int64).cuda()
    offs = list(range(0, obj.size, ch))
    first = torch.tensor([o // page for o in offs], dtype=torch.int64).cuda()
    lens = torch.tensor([min(ch, obj.size - o) for o in offs], dtype=torch.int64).cuda()
    out = B.pages_dsum(ptrs, first, lens, page)
    assert hexs(out) == c1["chunk_dsums"]
    # the whole object as one page list (the server's dsum of a full PUT)
    whole = B.pages_dsum(ptrs, torch.zeros(1, dtype=torch.int64).cuda(),
                         torch.tensor([obj.size], dtype=torch.int64).cuda(), page)
    import xxhash
    assert hexs(whole) == [f"{xxhash.xxh64_intdigest(obj.tobytes()):016x}"]


@pytest.mark.parametrize("page", [512, 4096, 65536])
def test_pages_dsum_ragged_lengths(B, O, page):
    rng = np.random.default_rng(page)
    lens = [0, 1, 31, 32, 33, 511, 512, 513, page - 1, page, page + 1, 3 * page + 17, 100000]
    msgs = [synth.stripe_bytes(300 + i, L) if L else np.zeros(0, np.uint8) for i, L in enumerate(lens)]
    pages, first = [], []
    for m in msgs:
        first.append(len(pages))
        npg = max(1, (m.size + page - 1) // page)
        buf = np.zeros(npg * page, np.uint8)
        buf[:m.size] = m
        pages.extend(buf.reshape(npg, page))
    order = rng.permutation(len(pages))
    pool = np.stack([pages[i] for i in order])
    where = np.empty(len(pages), np.int64)
    where[order] = np.arange(len(pages))
    dpool = torch.from_numpy(pool).cuda()
    ptrs = torch.tensor([dpool.data_ptr() + int(w) * page for w in where], dtype=torch.int64).cuda()
    out = B.pages_dsum(ptrs, torch.tensor(first, dtype=torch.int64).cuda(),
                       torch.tensor(lens, dtype=torch.int64).cuda(), page)
    assert hexs(out) == [f"{O.xxh64(m):016x}" for m in msgs]


def test_cluster_batch_full_size_property(B, O):
    """8,192 x 64 KiB clusters (512 MiB): the strided batch equals the
    offset-list batch; a sample equals the oracle."""
    n, ch = 8192, 65536
    d = B.synth(n, ch)
    sums, _ = B.clu_sum(d)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * d.stride(0)
    lens = torch.full((n,), ch, dtype=torch.int64, device="cuda")
    ref = B.xxh64_batch(d, off, lens)
    assert torch.equal(sums, ref)
    for i in (0, 1, 4097, n - 1):
        assert hexs(sums[i:i + 1])[0] == f"{O.xxh64(synth.stripe_bytes(i, ch)):016x}"
    # a short logical size inside a wider pitch
    s2, _ = B.clu_sum(d, cluster_size=1000)
    for i in (0, 77):
        assert hexs(s2[i:i + 1])[0] == f"{O.xxh64(synth.stripe_bytes(i, ch)[:1000]):016x}"


def test_integrity_argument_errors(B):
    from nkfs_amd import _lib
    L = _lib.lib()
    d = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    out = torch.zeros(4, dtype=torch.int64, device="cuda")
    assert L.nkfs_pages_dsum_batch(d.data_ptr(), out.data_ptr(), out.data_ptr(), 1, 1000, out.data_ptr(),
                                   None) == -22
    assert L.nkfs_pages_dsum_batch(d.data_ptr(), out.data_ptr(), out.data_ptr(), 1, 256, out.data_ptr(),
                                   None) == -22
    assert L.nkfs_clu_sum_batch(d.data_ptr() + 4, 1024, 1024, 2, out.data_ptr(), None, None, None) == -22
    assert L.nkfs_clu_sum_batch(d.data_ptr(), 512, 1024, 2, out.data_ptr(), None, None, None) == -22
    assert L.nkfs_clu_sum_batch(d.data_ptr(), 1024, 1024, 2, out.data_ptr(), out.data_ptr(), None, None) == -22
    assert L.nkfs_clu_sum_batch(d.data_ptr(), 1024, 1024, 0, None, None, None, None) == 0
