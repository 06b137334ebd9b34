"""GPU parity of the per-call checksum ABI (crt/csum.c:3-27,
crt/xxhash.c:566-930; csum.c + xxh64_chain.hip): one GPU round trip per
message, messages pending on the GPU between XXH64_update and
XXH64_digest.

Checked against the oracle's XXH64 (oracle/nk8_port.c, pinned to the
compiled reference and the python xxhash package): long streams (20 MiB,
and 8 MiB + 17 bytes after a 5-byte partial update) across the
256 KiB fold chunks, random chunkings, more pending states than slots (the
synchronous fallback), digest-then-continue (the reference's digest leaves
the state usable), reset / free of a pending state, seeds, and threads.
"""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def _state(L, seed=0):
    st = L.XXH64_createState()
    assert st
    assert L.XXH64_reset(st, seed) == 0
    return st


def _upd(L, st, a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    assert L.XXH64_update(st, a.ctypes.data if a.size else None, a.size) == 0


def test_long_streams(L, O):
    from nkfs_amd import crt
    rng = np.random.default_rng(21)
    data = rng.integers(0, 256, (20 << 20) + 7, dtype=np.uint8)
    want = O.xxh64(data)
    assert crt.xxh64(data) == want                      # one-shot
    st = _state(L)
    _upd(L, st, data)                                    # one update
    assert L.XXH64_digest(st) == want
    L.XXH64_freeState(st)
    # 5-byte partial, then 8 MiB + 17 in one update, then the rest
    cs = crt.Csum()
    cs.update(data[:5])
    cs.update(data[5: 5 + (8 << 20) + 17])
    cs.update(data[5 + (8 << 20) + 17:])
    assert cs.digest() == want
    # random chunk sizes across the 256 KiB fold boundaries
    cs = crt.Csum()
    pos = 0
    while pos < data.size:
        step = int(rng.choice([1, 31, 33, 4096, 262143, 262144, 262177, 1 << 20]))
        cs.update(data[pos: pos + step])
        pos += step
    assert cs.digest() == want


@pytest.mark.parametrize("seed", [0, 1, 0x9E3779B185EBCA87, (1 << 64) - 1])
def test_seeds_and_lengths(L, O, seed):
    rng = np.random.default_rng(seed & 0xFFFF)
    for n in [0, 1, 31, 32, 33, 63, 64, 65, 262144 - 1, 262144, 262144 + 31, 262144 + 33, 3 * 262144 + 5]:
        data = rng.integers(0, 256, n, dtype=np.uint8)
        st = _state(L, seed)
        _upd(L, st, data)
        assert L.XXH64_digest(st) == O.xxh64(data, seed), n
        L.XXH64_freeState(st)


def test_digest_then_continue(L, O):
    """The reference's digest does not end the state (crt/xxhash.c:838-930):
    updates after a digest continue the same message."""
    rng = np.random.default_rng(4)
    a = rng.integers(0, 256, 100000, dtype=np.uint8)
    b = rng.integers(0, 256, 300001, dtype=np.uint8)
    st = _state(L)
    _upd(L, st, a)
    assert L.XXH64_digest(st) == O.xxh64(a)
    assert L.XXH64_digest(st) == O.xxh64(a)  # twice
    _upd(L, st, b)
    assert L.XXH64_digest(st) == O.xxh64(np.concatenate([a, b]))
    L.XXH64_freeState(st)


def test_reset_and_free_pending(L, O):
    rng = np.random.default_rng(6)
    a = rng.integers(0, 256, 70000, dtype=np.uint8)
    st = _state(L)
    _upd(L, st, a)                 # pending on the GPU
    assert L.XXH64_reset(st, 7) == 0  # abandons it
    _upd(L, st, a[:1000])
    assert L.XXH64_digest(st) == O.xxh64(a[:1000], 7)
    st2 = _state(L)
    _upd(L, st2, a)
    L.XXH64_freeState(st2)         # freed while pending: the slot is released


def test_more_pending_states_than_slots(L, O):
    """1,100 messages pending at once (64 slots, csum.c NSLOT): the rest
    fold synchronously; every digest, taken in reverse order, is exact."""
    from nkfs_amd import crt
    rng = np.random.default_rng(8)
    datas = [rng.integers(0, 256, int(rng.integers(32, 3000)), dtype=np.uint8) for _ in range(1100)]
    cs = []
    for d in datas:
        c = crt.Csum()
        c.update(d[:40])
        c.update(d[40:])
        cs.append(c)
    for c, d in reversed(list(zip(cs, datas))):
        assert c.digest() == O.xxh64(d)


def test_threads(L, O):
    """Eight host threads hash concurrently (ctypes drops the GIL): per-call
    contexts and slots are per message, the results exact."""
    from nkfs_amd import crt
    rng = np.random.default_rng(9)
    datas = [rng.integers(0, 256, int(rng.integers(1, 600000)), dtype=np.uint8) for _ in range(64)]
    want = [O.xxh64(d) for d in datas]
    got = [None] * len(datas)

    def work(t):
        for i in range(t, len(datas), 8):
            if i % 2:
                got[i] = crt.xxh64(datas[i])
            else:
                c = crt.Csum()
                for j in range(0, datas[i].size, 77777):
                    c.update(datas[i][j: j + 77777])
                got[i] = c.digest()

    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == want


def test_poisoned_state_fails_until_reset(L, O):
    """A failed update poisons the state (it would otherwise look
    valid and digest to a wrong sum): every later update returns XXH_ERROR
    until XXH64_reset, which clears it without touching any slot.  The poison
    word (PEND_MAGIC | 0xFFFF in the 88-byte state's padding, offset 84) is
    what csum.c writes on that path."""
    rng = np.random.default_rng(12)
    a = rng.integers(0, 256, 5000, dtype=np.uint8)
    st = _state(L)
    _upd(L, st, a[:10])  # buffered on the host: no slot held
    C.c_uint32.from_address(st + 84).value = 0xC5A1FFFF
    assert L.XXH64_update(st, a.ctypes.data, a.size) == 1  # XXH_ERROR
    assert L.XXH64_update(st, a.ctypes.data, a.size) == 1
    assert L.XXH64_reset(st, 0) == 0
    _upd(L, st, a)
    assert L.XXH64_digest(st) == O.xxh64(a)
    L.XXH64_freeState(st)


def test_concurrent_digests_of_one_state(L, O):
    """The reference's digest is read-only, so one state may be digested
    from several threads at once; a pending message is completed once, under
    its slot's lock, and every thread gets the same exact digest."""
    rng = np.random.default_rng(13)
    for trial in range(20):
        a = rng.integers(0, 256, int(rng.integers(64, 400000)), dtype=np.uint8)
        st = _state(L)
        _upd(L, st, a)  # pending on the GPU
        got = [None] * 4

        def dig(i):
            got[i] = L.XXH64_digest(st)

        th = [threading.Thread(target=dig, args=(i,)) for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert got == [O.xxh64(a)] * 4, trial
        L.XXH64_freeState(st)


def test_percall_service(L, O):
    """The opt-in resident service wave (nkfs_percall_service, k_xxh64_service):
    one-piece messages are posted to its host-memory mailbox instead of
    launched; longer ones (an earlier 256 KiB fold) keep the launch path.
    Digests match the oracle across lengths and seeds, from eight threads at
    once (requests serialised on the one mailbox), after the wave left on its
    20 ms idle timeout (the next request relaunches it), and after the
    service is switched off again."""
    import time
    from nkfs_amd import crt
    rng = np.random.default_rng(31)
    assert L.nkfs_percall_service(1) == 0
    try:
        for n in [0, 1, 31, 32, 64, 1000, 65536, 262144, 262144 + 33, 700001]:
            for seed in (0, 5):
                data = rng.integers(0, 256, n, dtype=np.uint8)
                assert crt.xxh64(data, seed) == O.xxh64(data, seed), (n, seed)
        time.sleep(0.1)  # past the idle timeout: the wave has left
        data = rng.integers(0, 256, 4096, dtype=np.uint8)
        assert crt.xxh64(data) == O.xxh64(data)
        cs = crt.Csum()
        cs.update(data[:10])
        cs.update(data[10:])
        assert cs.digest() == O.xxh64(data)
        datas = [rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8) for _ in range(256)]
        want = [O.xxh64(d) for d in datas]
        got = [None] * len(datas)

        def work(t):
            for i in range(t, len(datas), 8):
                got[i] = crt.xxh64(datas[i])

        th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert got == want
    finally:
        assert L.nkfs_percall_service(0) == 0
    data = rng.integers(0, 256, 777, dtype=np.uint8)
    assert crt.xxh64(data) == O.xxh64(data)


def test_percall_service_off_on(L, O):
    """switching the service off (a stop request uses a request
    number) and on again must not leave the next wave seeing a phantom
    request.  On, off, on -- each time with the wave just stopped -- then an
    inline message (<= 1 KiB) and one over 1 KiB against the oracle; and a
    request right after a stop that the old wave may still be leaving."""
    from nkfs_amd import crt
    rng = np.random.default_rng(32)
    for cycle in range(4):
        assert L.nkfs_percall_service(1) == 0
        try:
            for n in (33, 1000, 1024, 1025, 4096 + 7):
                data = rng.integers(0, 256, n, dtype=np.uint8)
                assert crt.xxh64(data, cycle) == O.xxh64(data, cycle), (cycle, n)
        finally:
            assert L.nkfs_percall_service(0) == 0
    assert L.nkfs_percall_service(1) == 0
    try:
        data = rng.integers(0, 256, 700, dtype=np.uint8)
        assert crt.xxh64(data) == O.xxh64(data)
    finally:
        assert L.nkfs_percall_service(0) == 0
    assert L.nkfs_percall_service(3) == -22


def test_percall_service_bar_mailbox(L, O):
    """Mode 2: the request half of the mailbox in
    uncached device memory written by the host through the BAR.  Back-to-back
    requests of different messages and lengths (a stale argument or inline
    byte would show as a wrong digest), a switch to mode 1 and back with the
    wave live, the idle relaunch, and eight threads at once."""
    import time
    from nkfs_amd import crt
    rng = np.random.default_rng(33)
    assert L.nkfs_percall_service(2) == 0
    try:
        for it in range(60):
            n = int(rng.integers(0, 3000))
            data = rng.integers(0, 256, n, dtype=np.uint8)
            assert crt.xxh64(data, it) == O.xxh64(data, it), (it, n)
        assert L.nkfs_percall_service(1) == 0  # switch with the wave live
        data = rng.integers(0, 256, 64, dtype=np.uint8)
        assert crt.xxh64(data) == O.xxh64(data)
        assert L.nkfs_percall_service(2) == 0
        assert crt.xxh64(data, 9) == O.xxh64(data, 9)
        time.sleep(0.1)  # past the idle timeout
        data = rng.integers(0, 256, 1025, dtype=np.uint8)
        assert crt.xxh64(data) == O.xxh64(data)
        datas = [rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8) for _ in range(128)]
        want = [O.xxh64(d) for d in datas]
        got = [None] * len(datas)

        def work(t):
            for i in range(t, len(datas), 8):
                got[i] = crt.xxh64(datas[i])

        th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert got == want
    finally:
        assert L.nkfs_percall_service(0) == 0
