"""oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end to the CPU restatement (oracle/nk8_port.c -> liboracle.so)
and, when built, to the reference's own compiled sources
(oracle/_ref/libnkfs_ref.so, see oracle/ref/Makefile).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / the timed CPU baseline -- never as the product.

Reference semantics restated (irqlevel/nkfs):
  encode  crt/nk8.c:344-444   (explicit ids instead of nk8_gen_part_ids)
  decode  crt/nk8.c:446-599
  XXH64   crt/xxhash.c:358-496 (one-shot), csum seed 0 crt/csum.c:3-21
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libnkfs_ref.so")

_u8p = C.POINTER(C.c_uint8)


def build(quiet: bool = True) -> None:
    out = subprocess.run(["make", "-C", HERE, "all", "ref"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_init.restype = C.c_int
        L.orc_encode.argtypes = [_u8p, C.c_uint32, C.c_int, C.c_int, _u8p, _u8p, C.c_uint64]
        L.orc_encode.restype = C.c_int
        L.orc_decode.argtypes = [C.POINTER(_u8p), _u8p, C.c_int, C.c_int, _u8p, C.c_uint32]
        L.orc_decode.restype = C.c_int
        L.orc_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_xxh64.restype = C.c_uint64
        L.orc_part_size.argtypes = [C.c_uint32, C.c_int]
        L.orc_part_size.restype = C.c_uint32
        L.orc_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.orc_gf_mul.restype = C.c_uint8
        L.orc_mul_table.restype = _u8p
        L.orc_bench_encode_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, _u8p, _u8p,
                                              C.c_uint32, C.c_int, C.c_int, C.c_uint64, C.c_int,
                                              C.POINTER(C.c_uint64)]
        L.orc_bench_encode_decode.restype = C.c_double
        assert L.orc_init() == 0
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def part_size(block_size: int, k: int) -> int:
    return block_size // k + (1 if block_size % k else 0)


def encode(block: np.ndarray, n: int, k: int, ids) -> np.ndarray:
    """[n, ps] uint8 parts of one block with explicit ids."""
    block = np.ascontiguousarray(block, dtype=np.uint8)
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    ps = part_size(len(block), k) if len(block) else 0
    parts = np.zeros((n, max(ps, 1)), dtype=np.uint8)
    err = lib().orc_encode(_ptr(block), len(block), n, k, _ptr(ids), _ptr(parts), parts.shape[1])
    if err:
        raise OSError(-err, os.strerror(-err))
    return parts[:, :ps]


def decode(parts, ids, k: int, block_size: int) -> np.ndarray:
    """Decode from parts (list of uint8 arrays) with matching ids, reference
    selection rule (first k distinct ids in order)."""
    arrs = [np.ascontiguousarray(p, dtype=np.uint8) for p in parts]
    ptrs = (_u8p * len(arrs))(*[_ptr(a) for a in arrs])
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    out = np.zeros(block_size, dtype=np.uint8)
    err = lib().orc_decode(ptrs, _ptr(ids), len(arrs), k, _ptr(out), block_size)
    if err:
        raise OSError(-err, os.strerror(-err))
    return out


def xxh64(data, seed: int = 0) -> int:
    a = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
    return int(lib().orc_xxh64(a.ctypes.data if a.size else None, a.size, seed))


def gf_mul_table() -> np.ndarray:
    return np.ctypeslib.as_array(lib().orc_mul_table(), shape=(256, 256)).copy()


# ---------------------------------------------------------------- reference

_ref = None


def ref_lib():
    """The reference's own crt/ sources compiled by oracle/ref/Makefile, or
    None when neither the reference tree nor a prebuilt copy is available."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PATH):
            try:
                build()
            except RuntimeError:
                return None
            if not os.path.exists(REF_PATH):
                return None
        R = C.CDLL(REF_PATH)
        R.crt_log_set_level.argtypes = [C.c_int]
        R.crt_log_set_level(10)  # CL_MAX (crt/include/clog.h:14): keep ds.log out of timings
        R.nk8_init.restype = C.c_int
        R.nk8_split_block.argtypes = [_u8p, C.c_uint32, C.c_int, C.c_int,
                                      C.POINTER(C.POINTER(_u8p)), C.POINTER(_u8p)]
        R.nk8_split_block.restype = C.c_int
        R.nk8_assemble_block.argtypes = [C.POINTER(_u8p), _u8p, C.c_int, C.c_int, _u8p, C.c_uint32]
        R.nk8_assemble_block.restype = C.c_int
        R.XXH64.argtypes = [C.c_void_p, C.c_size_t, C.c_ulonglong]
        R.XXH64.restype = C.c_ulonglong
        R.crt_free.argtypes = [C.c_void_p]
        err = R.nk8_init()
        if err:
            raise RuntimeError(f"reference nk8_init failed: {err}")
        _ref = R
    return _ref


def ref_split(block: np.ndarray, n: int, k: int):
    """Reference nk8_split_block: returns (ids[n], parts[n, ps])."""
    R = ref_lib()
    block = np.ascontiguousarray(block, dtype=np.uint8)
    pparts = C.POINTER(_u8p)()
    pids = _u8p()
    err = R.nk8_split_block(_ptr(block), len(block), n, k, C.byref(pparts), C.byref(pids))
    if err:
        raise OSError(-err, os.strerror(-err))
    ps = part_size(len(block), k)
    ids = np.array([pids[i] for i in range(n)], dtype=np.uint8)
    parts = np.zeros((n, ps), dtype=np.uint8)
    for i in range(n):
        C.memmove(parts[i].ctypes.data, pparts[i], ps)
        R.crt_free(pparts[i])
    R.crt_free(pparts)
    R.crt_free(pids)
    return ids, parts


def ref_assemble(parts, ids, k: int, block_size: int):
    R = ref_lib()
    arrs = [np.ascontiguousarray(p, dtype=np.uint8) for p in parts]
    ptrs = (_u8p * len(arrs))(*[_ptr(a) for a in arrs])
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    out = np.zeros(block_size, dtype=np.uint8)
    err = R.nk8_assemble_block(ptrs, _ptr(ids), len(arrs), k, _ptr(out), block_size)
    return err, out


def ref_xxh64(data: np.ndarray, seed: int = 0) -> int:
    a = np.ascontiguousarray(data, dtype=np.uint8)
    return int(ref_lib().XXH64(a.ctypes.data if a.size else None, a.size, seed))


# ------------------------------------------------------------- cpu baseline

def bench_encode_decode(blocks: np.ndarray, n: int, k: int, survivors=None, threads: int = 1,
                        kind: str = "reference"):
    """Time split + XXH64 of every part (+ assemble of every stripe from
    survivors[s] when given) over the rows of `blocks` ([count, B] uint8).
    kind "reference" times oracle/_ref (the reference's own code, its id
    draw from /dev/urandom and per-call mallocs included), "port" the
    restatement.  Returns (seconds, digest_xor)."""
    L = lib()
    if kind == "reference":
        R = ref_lib()
        if R is None:
            raise FileNotFoundError(REF_PATH)
        split = C.cast(R.nk8_split_block, C.c_void_p)
        hsh = C.cast(R.XXH64, C.c_void_p)
        rel = C.cast(R.crt_free, C.c_void_p)
        asm = C.cast(R.nk8_assemble_block, C.c_void_p)
    else:
        split = C.cast(L.orc_split_block, C.c_void_p)
        hsh = C.cast(L.orc_xxh64, C.c_void_p)
        rel = C.cast(L.orc_free, C.c_void_p)
        asm = C.cast(L.orc_assemble_block, C.c_void_p)
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    sv = None
    if survivors is not None:
        sv = np.ascontiguousarray(survivors, dtype=np.uint8)
        assert sv.shape == (blocks.shape[0], k)
    dx = C.c_uint64(0)
    secs = L.orc_bench_encode_decode(split, hsh, rel, asm if sv is not None else None,
                                     _ptr(sv) if sv is not None else None, _ptr(blocks), blocks.shape[1],
                                     n, k, blocks.shape[0], threads, C.byref(dx))
    if secs < 0:
        raise OSError(int(-secs), "cpu baseline failed")
    return secs, int(dx.value)
