"""Post-init thread safety (SURVEY.md §8(b) Threading; the reference's
tables are written once in nk8_init and never change, crt/nk8.c:3-5):
drop-in nk8_split_block / nk8_assemble_block from several threads while
another thread keeps rewriting struct nkfs_tune (nkfs_tune_set), so every
call's kernel choice changes under it.  Each launch takes one consistent
snapshot of the tune (runtime.c), every kernel family is bit-exact, so every
output must still equal the oracle's (crt/nk8.c:344-444, 446-599).
"""
import ctypes as C
import threading

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


def test_split_assemble_while_tune_changes(L, O):
    from nkfs_amd import _lib, crt
    shapes = [(8, 5, 5 * 4096), (8, 5, 5 * 65536 + 3), (4, 2, 4096), (12, 8, 100003), (20, 17, 40000)]
    blocks = [synth.stripe_bytes(500 + i, B) for i, (_, _, B) in enumerate(shapes)]
    saved = _lib.get_tune()
    stop = threading.Event()
    errs = []
    flips = [0]

    def toggler():
        t = _lib.get_tune()
        i = 0
        while not stop.is_set():
            # the default rules and the thread-per-row kernels: both run
            # every shape here (pinned families outside their tested shapes
            # are not this test's subject)
            t.enc_kernel = _lib.ENC["generic"] if i & 2 else _lib.ENC["auto"]
            t.dec_kernel = _lib.DEC["generic"] if i & 4 else _lib.DEC["auto"]
            t.size_order = i & 1
            if L.nkfs_tune_set(C.byref(t)) != 0:
                errs.append(("tune_set", i))
                return
            i += 1
            flips[0] = i

    def worker(w):
        try:
            for it in range(6):
                j = (w + it) % len(shapes)
                n, k, B = shapes[j]
                blk = blocks[j]
                parts, ids = crt.split_block(blk, n, k)
                want = O.encode(blk, n, k, ids)
                for i in range(n):
                    assert np.array_equal(parts[i], want[i]), (w, it, j, i)
                # the last k parts in reverse order: a different survivor set
                sel = list(range(n - 1, n - k - 1, -1))
                out = crt.assemble_block([parts[i] for i in sel], ids[sel], k, k, B)
                assert np.array_equal(out, blk), (w, it, j)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    tt = threading.Thread(target=toggler)
    tt.start()
    try:
        ws = [threading.Thread(target=worker, args=(w,)) for w in range(4)]
        for t in ws:
            t.start()
        for t in ws:
            t.join()
    finally:
        stop.set()
        tt.join()
        L.nkfs_tune_set(C.byref(saved))
    assert not errs, errs[:3]
    assert flips[0] > 10  # the tune really changed under the calls
