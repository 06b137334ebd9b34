"""The drop-in boundary: libnkfs_crt.so loads, exports every function
include/*.h declares, validates arguments like the reference, and refuses to
compute without a GPU (no CPU fallback).  No compute calls happen here."""
import ctypes as C
import subprocess

import pytest

from conftest import has_gpu_device
from nkfs_amd import _lib

REFERENCE_SYMBOLS = [  # crt/include/nk8.h:4-11, csum.h:14-17, xxhash.h:86-132, crt.h:12-13
    "nk8_init", "nk8_release", "nk8_split_block", "nk8_assemble_block",
    "csum_reset", "csum_update", "csum_digest", "csum_u64",
    "XXH64", "XXH64_createState", "XXH64_freeState", "XXH64_reset", "XXH64_update", "XXH64_digest",
    "crt_malloc", "crt_free",
]


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    return {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}


def test_library_loads():
    assert _lib.lib() is not None


def test_every_header_function_is_exported():
    names = _lib.header_functions()
    assert len(names) >= 30
    syms = exported()
    missing = [n for n in names if n not in syms]
    assert not missing, missing
    # and nothing beyond the declared ABI leaks out
    assert syms <= set(names)


def test_reference_symbols_present():
    syms = exported()
    for s in REFERENCE_SYMBOLS:
        assert s in syms


def test_state_abi_size():
    # struct csum_ctx embeds XXH64_state_t by value: 11 long longs (xxhash.h:105)
    assert C.sizeof(C.c_longlong * 11) == 88


def test_argument_validation_matches_reference():
    L = _lib.lib()
    u8p = _lib.u8p
    buf = (C.c_uint8 * 16)()
    pp = C.POINTER(u8p)()
    pi = u8p()
    # crt/nk8.c:356-360 -- checked before the init check
    for B, n, k in [(0, 4, 2), (16, 4, 1), (16, 2, 3), (16, 256, 2), (16, 255, 255)]:
        assert L.nk8_split_block(buf, B, n, k, C.byref(pp), C.byref(pi)) == -22
    parts = (u8p * 4)()
    ids = (C.c_uint8 * 4)(1, 2, 3, 4)
    assert L.nk8_assemble_block(parts, ids, 1, 2, buf, 16) == -22


def test_host_decode_rejects_missing_slots():
    """The host-memory decode checks every offered slot exists before it
    touches the GPU (the kernels index the stripe's id row with it): an
    h_avail entry >= n_slots is -EINVAL, with or without a GPU."""
    L = _lib.lib()
    n, k, B, S = 4, 2, 4096, 3
    parts = (C.c_uint8 * (S * n * 2048))()
    blocks = (C.c_uint8 * (S * B))()
    ids = (C.c_uint8 * (S * n))(*([1, 2, 3, 4] * S))
    bad = (C.c_uint8 * (S * k))(0, 1, 2, 3, 1, 4)  # stripe 2 offers slot 4 of 4
    assert L.nkfs_nk8_decode_host(parts, 2048, n, ids, bad, k, k, B, blocks, B, S, None, None, None, 0) == -22
    ok = (C.c_uint8 * (S * k))(0, 1, 2, 3, 1, 3)
    rc = L.nkfs_nk8_decode_host(parts, 2048, n, ids, ok, k, k, B, blocks, B, S, None, None, None, 0)
    assert rc != -22


@pytest.mark.skipif(has_gpu_device(), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly():
    L = _lib.lib()
    assert L.nk8_init() == -19  # -ENODEV
    assert L.nkfs_gpu_ready() == 0
    u8p = _lib.u8p
    buf = (C.c_uint8 * 4096)()
    pp = C.POINTER(u8p)()
    pi = u8p()
    assert L.nk8_split_block(buf, 4096, 4, 2, C.byref(pp), C.byref(pi)) == -11  # -EAGAIN
    assert L.nkfs_nk8_encode(None, 4096, 4096, 1, 4, 2, None, None, 2048, None, None) == -11
    assert L.nkfs_clu_sum_batch(None, 65536, 65536, 1, None, None, None, None) == -11
    assert L.nkfs_pages_dsum_batch(None, None, None, 1, 4096, None, None) == -11
    assert L.nkfs_dev_alloc(16) is None


def test_part_geometry():
    L = _lib.lib()
    assert L.nkfs_part_size(1048576, 5) == 209716
    assert L.nkfs_part_pitch(1048576, 5) == 209920
    assert L.nkfs_part_size(4096, 2) == 2048
    assert L.nkfs_part_pitch(1, 2) == 256


def test_walk_offset_bound():
    """The walk encoder drops a store by setting bit 31 of its buffer offset,
    so every offset it forms must stay below 2^31 (the digest
    array's bound was 2^32).  Host-side check, no GPU needed."""
    import ctypes as C
    from nkfs_amd import _lib
    f = _lib.lib().nkfs_walk_offsets_fit
    f.restype = C.c_int
    f.argtypes = [C.c_uint64] * 4
    assert f(1 << 20, 8 * 209920, 8192, 8) == 1
    # digests: nstripes * n * 8 bytes
    assert f(4096, 4 * 2048, (1 << 31) // 64 - 1, 8) == 1
    assert f(4096, 4 * 2048, (1 << 31) // 64, 8) == 0
    assert f(4096, 4 * 2048, (1 << 28) + 1, 1) == 0
    # a stripe's part span and the block reach
    assert f(4096, (1 << 31), 1, 8) == 0
    assert f((1 << 31) - 2048 * 8, 16, 1, 2) == 0


def test_decode_workspace_covers_every_plan_layout():
    """nkfs_decode_workspace(nstripes, k) holds the k + k*k plan bytes per
    stripe of the slice / general decoders and the run decoder's layout
    (plans at a dword stride, then a u32 chunk prefix per stripe and a u32
    total per 256-stripe group, each region 16-byte aligned)."""
    L = _lib.lib()
    for S in (1, 7, 255, 256, 257, 11520, 65536):
        for k in (2, 3, 5, 8, 12, 32, 254):
            w = L.nkfs_decode_workspace(S, k)
            assert w >= S * (k + k * k)
            stride = (k + k * k + 3) & ~3
            loc = (S * stride + 15) & ~15
            gsum = (loc + 4 * S + 15) & ~15
            assert w >= gsum + 4 * ((S + 255) // 256), (S, k)


def _ragged(sizes, n_slots, k, block_gap, part_gap):
    import numpy as np
    L = _lib.lib()
    boff = np.zeros(len(sizes), np.uint64)
    poff = np.zeros(len(sizes), np.uint64)
    pos = ppos = 0
    for s, B in enumerate(sizes):
        boff[s], poff[s] = pos, ppos
        pos += int(B) + block_gap
        ppos += n_slots * L.nkfs_part_pitch(int(B), k) + part_gap
    return boff, poff


def _plan(decode, boff, sizes, n, k, navail, poff, page, chunk):
    import numpy as np
    L = _lib.lib()
    sz = np.ascontiguousarray(sizes, np.uint32)
    msg = C.create_string_buffer(256)
    rc = L.nkfs_pipeline_check(decode, None if boff is None else boff.ctypes.data, sz.ctypes.data, int(sz.max()),
                               len(sz), n, k, navail, poff.ctypes.data, page, chunk, msg, 256)
    return rc, msg.value.decode()


def test_pipeline_plan_round3_fault_geometry():
    """CPU replay of the host pipeline's plan (sub-batch cuts, device layout,
    shifted ragged offsets: pipeline.c issue()) for the geometry of the
    round-3 fault (test_ragged_host_gaps_untouched[8-5-0]: N8K5, 1 MiB + 1 B
    + 70,001 B + mixed sizes, block gap 24, part gap 48): every kernel access
    and copy of every sub-batch stays inside its region, for PUT and GET and
    the three sub-batch sizes the GPU test uses."""
    from nkfs_amd import synth
    for n, k in ((8, 5), (4, 2), (6, 3)):
        sizes = synth.mixed_sizes(29)
        sizes[:3] = (1048576, 1, 70001)
        boff, poff = _ragged(sizes, n, k, 24, 48)
        for chunk in (0, 1 << 20, 100000, 1):
            for dec in (0, 1):
                rc, msg = _plan(dec, boff, sizes, n, k, n, poff, 0, chunk)
                assert rc == 0, (n, k, chunk, dec, msg)
                assert msg.startswith("ok")


def test_pipeline_plan_random_geometries():
    """The same replay over random ragged batches: sizes 1 B .. 2 MiB,
    unaligned block gaps, 16-byte part gaps, page-list staging, sub-batch
    sizes from one stripe to all of them."""
    import numpy as np
    rng = np.random.default_rng(4)
    for trial in range(60):
        n = int(rng.integers(2, 17))
        k = int(rng.integers(2, n + 1))
        S = int(rng.integers(1, 120))
        sizes = np.where(rng.random(S) < 0.2, rng.integers(1, 64, S), rng.integers(1, 2 << 20, S)).astype(np.uint32)
        boff, poff = _ragged(sizes, n, k, int(rng.integers(0, 97)), 16 * int(rng.integers(0, 9)))
        chunk = int(rng.choice([0, 1, 4096, 1 << 20, 7 << 20]))
        page = int(rng.choice([0, 0, 4096, 512]))
        rc, msg = _plan(int(trial & 1), None if page else boff, sizes, n, k, n, poff, page, chunk)
        assert rc == 0, (trial, msg)


def test_pipeline_plan_rejects_bad_geometry():
    import numpy as np
    sizes = np.array([4096, 4096], np.uint32)
    boff, poff = _ragged(sizes, 4, 2, 0, 0)
    poff[1] += 8  # part bases must be 16-byte aligned
    assert _plan(0, boff, sizes, 4, 2, 4, poff, 0, 0)[0] == -22
    boff, poff = _ragged(sizes, 4, 2, 0, 0)
    boff[1] -= 1  # blocks overlap
    assert _plan(0, boff, sizes, 4, 2, 4, poff, 0, 0)[0] == -22


@pytest.mark.timeout(900)
def test_debug_bounds_build_compiles():
    """the debug-bounds build (make DEBUG_BOUNDS=1: the
    ragged walk encoder's and slice decoder's range reports)
    compiles from the current sources and exports the product's ABI, so
    tests/test_gpu_debug_bounds.py can load it on the GPU box.  Incremental:
    build() normally made it already."""
    import os
    csrc = os.path.join(os.path.dirname(_lib.LIB_PATH), "..", "csrc")
    r = subprocess.run(["make", "-C", csrc, "DEBUG_BOUNDS=1", "-j", str(min(8, os.cpu_count() or 2))],
                       capture_output=True, text=True, timeout=880)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    dbg = os.path.join(os.path.dirname(_lib.LIB_PATH), "debug", "libnkfs_crt.so")
    out = subprocess.run(["nm", "-D", "--defined-only", dbg], capture_output=True, text=True, check=True)
    syms = {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}
    assert syms == exported()
    # the range checks are really compiled in: their report format is in the device code
    for o in ("nk8_walk_k5.o", "nk8_wsp.o", "nk8_run.o"):  # round 6: wsp + run decoder checked too
        strings = subprocess.run(["strings", os.path.join(csrc, "..", "build", "debug", o)],
                                 capture_output=True, text=True, check=True).stdout
        obj = subprocess.run(["grep", "-c", "nkfs bounds"], input=strings, capture_output=True, text=True)
        assert int(obj.stdout.strip() or 0) >= 1, o
    # and none in the product's objects (no shared objects)
    for o in ("nk8_wsp.o", "nk8_run.o"):
        strings = subprocess.run(["strings", os.path.join(csrc, "..", "build", o)],
                                 capture_output=True, text=True, check=True).stdout
        assert "nkfs bounds" not in strings, o


def test_host_lane_plan_interleaves_devices():
    """the host lanes of a host-memory call go round-robin over
    the devices, so the lane cap (16) drops whole rounds, never a device:
    8 devices x 3 lanes -> every device gets 2 lanes; 9+ devices at 2 lanes
    each keep every device."""
    L = _lib.lib()

    def plan(devs, per, cap=16):
        d = (C.c_int * len(devs))(*devs)
        out = (C.c_int * cap)()
        n = L.nkfs_host_lane_plan(d, len(devs), per, out, cap)
        return list(out[:n])

    assert plan([0], 2) == [0, 0]
    assert plan([0, 1], 1) == [0, 1]
    p = plan(list(range(8)), 3)
    assert len(p) == 16 and all(p.count(d) == 2 for d in range(8))
    p = plan(list(range(10)), 2)
    assert len(p) == 16 and set(p) == set(range(10))
    assert plan(list(range(4)), 4) == [0, 1, 2, 3] * 4
    assert plan([], 2) == [] and plan([3], 0) == [3]


def test_tune_struct_and_ranges():
    """struct nkfs_tune (include/nkfs_gpu.h) and its ctypes mirror have the
    same int fields in the same order, the round-5 defaults are the measured
    ones, and nkfs_tune_set rejects out-of-range values (-EINVAL, the state
    unchanged).  CPU only: the tune state needs no device."""
    import os
    import re
    from conftest import ROOT
    hdr = open(os.path.join(ROOT, "include", "nkfs_gpu.h")).read()
    body = hdr[hdr.index("struct nkfs_tune {"): hdr.index("};", hdr.index("struct nkfs_tune {"))]
    names = re.findall(r"^\s*int\s+(\w+);", body, re.M)
    assert names == [f for f, _ in _lib.Tune._fields_]
    t0 = _lib.get_tune()
    assert (t0.enc_persist, t0.dec_bign, t0.enc_bign, t0.dec_pair_pipe) == (1, -2, -1, 0)
    L = _lib.lib()
    for field, bad, good in (("enc_bign", 4, 3), ("enc_bign", -2, 0), ("dec_pair_pipe", 33, 8),
                             ("dec_pair_pipe", -1, 0), ("dec_bign", 6, 5), ("enc_persist", 3, 2)):
        t = _lib.get_tune()
        setattr(t, field, bad)
        assert L.nkfs_tune_set(C.byref(t)) == -22, field
        assert getattr(_lib.get_tune(), field) == getattr(t0, field)
        setattr(t, field, good)
        assert L.nkfs_tune_set(C.byref(t)) == 0, field
        assert L.nkfs_tune_set(C.byref(t0)) == 0
