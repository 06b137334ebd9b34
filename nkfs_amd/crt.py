"""Python mirror of the reference's crt/ erasure + checksum interface.

Each function is a thin ctypes call into libnkfs_crt.so's drop-in symbols
(include/nkfs_crt.h), with the reference's names, argument meaning and error
behaviour: a negative errno from the C side raises OSError(errno).

    nk8_init()                                  crt/nk8.c:725-747
    split_block(block, n, k) -> (parts, ids)    crt/nk8.c:344-444
    assemble_block(parts, ids, n, k, size)      crt/nk8.c:446-599
    Csum / xxh64                                crt/csum.c:3-27, crt/xxhash.c
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib, u8p


def _as_u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return np.ascontiguousarray(data, dtype=np.uint8)


def nk8_init() -> int:
    return lib().nk8_init()


def nk8_release() -> None:
    lib().nk8_release()


def split_block(block, n: int, k: int):
    """Encode one block; returns (parts: list of n uint8 arrays, ids: uint8[n]).
    The C side allocates with crt_malloc; this wrapper copies and crt_frees,
    as a reference caller would (crt/nk8.c:706-717)."""
    L = lib()
    blk = _as_u8(block)
    pparts = C.POINTER(u8p)()
    pids = u8p()
    check(L.nk8_split_block(blk.ctypes.data_as(u8p), blk.size, n, k, C.byref(pparts), C.byref(pids)),
          "nk8_split_block")
    ps = blk.size // k + (1 if blk.size % k else 0)
    ids = np.ctypeslib.as_array(pids, shape=(n,)).copy()
    parts = []
    for i in range(n):
        parts.append(np.ctypeslib.as_array(pparts[i], shape=(ps,)).copy())
        L.crt_free(C.cast(pparts[i], C.c_void_p))
    L.crt_free(C.cast(pparts, C.c_void_p))
    L.crt_free(C.cast(pids, C.c_void_p))
    return parts, ids


def assemble_block(parts, ids, n: int, k: int, block_size: int) -> np.ndarray:
    L = lib()
    arrs = [_as_u8(p) for p in parts]
    ptrs = (u8p * max(len(arrs), 1))(*[a.ctypes.data_as(u8p) for a in arrs])
    idv = _as_u8(ids)
    out = np.zeros(block_size, dtype=np.uint8)
    check(L.nk8_assemble_block(ptrs, idv.ctypes.data_as(u8p), n, k, out.ctypes.data_as(u8p), block_size),
          "nk8_assemble_block")
    return out


class Csum:
    """struct csum_ctx + csum_reset/update/digest (crt/include/csum.h:10-17)."""

    def __init__(self):
        self._ctx = (C.c_longlong * 11)()  # XXH64_state_t, crt/include/xxhash.h:105
        self._keep = []
        lib().csum_reset(C.addressof(self._ctx))

    def reset(self) -> None:
        lib().csum_reset(C.addressof(self._ctx))

    def update(self, data) -> None:
        a = _as_u8(data)
        lib().csum_update(C.addressof(self._ctx), a.ctypes.data if a.size else None, a.size)

    def digest(self) -> int:
        out = C.c_uint64(0)
        lib().csum_digest(C.addressof(self._ctx), C.addressof(out))
        return int(out.value)


def xxh64(data, seed: int = 0) -> int:
    a = _as_u8(data)
    return int(lib().XXH64(a.ctypes.data if a.size else None, a.size, seed))
