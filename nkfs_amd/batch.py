"""Device-resident batch API over torch tensors (include/nkfs_gpu.h).

torch is only the allocator and stream provider here: every computation is
a HIP kernel inside libnkfs_crt.so, launched on torch's current stream.

Layout of a uniform batch (see include/nkfs_gpu.h):
    blocks  uint8 [nstripes, block_pitch]     interleaved user data
    ids     uint8 [nstripes, n]               part evaluation points
    parts   uint8 [nstripes * n, part_pitch]  planar parts
    digests int64 [nstripes * n]              XXH64(part) (seed 0)
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import check, lib

U8 = torch.uint8


def gpu_init(device: int = -1) -> None:
    check(lib().nkfs_gpu_init(device), "nkfs_gpu_init")


def part_size(block_size: int, k: int) -> int:
    return int(lib().nkfs_part_size(block_size, k))


def part_pitch(block_size: int, k: int) -> int:
    return int(lib().nkfs_part_pitch(block_size, k))


def _stream(stream) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _need(t, dtype, name):
    if not (t.is_cuda and t.dtype == dtype and t.is_contiguous()):
        raise ValueError(f"{name}: expected a contiguous {dtype} CUDA tensor")


def encode(blocks: torch.Tensor, block_size: int, n: int, k: int, ids: torch.Tensor,
           parts: torch.Tensor | None = None, digests: bool | torch.Tensor = True, stream=None):
    """Encode (+ XXH64 of every part).  Returns (parts, digests|None)."""
    _need(blocks, U8, "blocks")
    _need(ids, U8, "ids")
    nstripes = blocks.shape[0]
    pitch = part_pitch(block_size, k)
    if parts is None:
        parts = torch.empty((nstripes * n, pitch), dtype=U8, device=blocks.device)
    _need(parts, U8, "parts")
    if digests is True:
        digests = torch.empty(nstripes * n, dtype=torch.int64, device=blocks.device)
    elif digests is False:
        digests = None
    check(lib().nkfs_nk8_encode(blocks.data_ptr(), blocks.stride(0) if blocks.dim() > 1 else block_size,
                                block_size, nstripes, n, k, ids.data_ptr(), parts.data_ptr(),
                                parts.stride(0), _ptr(digests), _stream(stream)), "nkfs_nk8_encode")
    return parts, digests


def encode_ragged(blocks: torch.Tensor, block_off: torch.Tensor, block_sizes: torch.Tensor, n: int, k: int,
                  ids: torch.Tensor, parts: torch.Tensor, part_off: torch.Tensor,
                  digests: torch.Tensor | None, max_block_size: int, stream=None):
    for t, dt, nm in ((blocks, U8, "blocks"), (block_off, torch.int64, "block_off"),
                      (block_sizes, torch.int32, "block_sizes"), (ids, U8, "ids"), (parts, U8, "parts"),
                      (part_off, torch.int64, "part_off")):
        _need(t, dt, nm)
    check(lib().nkfs_nk8_encode_ragged(blocks.data_ptr(), block_off.data_ptr(), block_sizes.data_ptr(),
                                       max_block_size, block_sizes.numel(), n, k, ids.data_ptr(),
                                       parts.data_ptr(), part_off.data_ptr(), _ptr(digests), _stream(stream)),
          "nkfs_nk8_encode_ragged")


def decode_workspace(nstripes: int, k: int, device) -> torch.Tensor:
    return torch.empty(max(int(lib().nkfs_decode_workspace(nstripes, k)), 1), dtype=U8, device=device)


def decode(parts: torch.Tensor, n_slots: int, ids: torch.Tensor, avail: torch.Tensor, k: int, block_size: int,
           out: torch.Tensor | None = None, work: torch.Tensor | None = None,
           status: torch.Tensor | None = None, stream=None):
    """Decode every stripe from the slots listed in avail[s] (first k with
    distinct ids).  Returns (blocks [nstripes, block_size], status int32)."""
    _need(parts, U8, "parts")
    _need(ids, U8, "ids")
    _need(avail, U8, "avail")
    nstripes = avail.shape[0]
    navail = avail.shape[1]
    dev = parts.device
    if out is None:
        out = torch.empty((nstripes, block_size), dtype=U8, device=dev)
    if work is None:
        work = decode_workspace(nstripes, k, dev)
    if status is None:
        status = torch.empty(nstripes, dtype=torch.int32, device=dev)
    check(lib().nkfs_nk8_decode(parts.data_ptr(), parts.stride(0), n_slots, ids.data_ptr(), avail.data_ptr(),
                                navail, k, block_size, out.data_ptr(), out.stride(0) if out.dim() > 1 else block_size,
                                nstripes, work.data_ptr(), status.data_ptr(), _stream(stream)), "nkfs_nk8_decode")
    return out, status


def decode_ragged(parts: torch.Tensor, part_off: torch.Tensor, n_slots: int, ids: torch.Tensor, avail: torch.Tensor,
                  k: int, out: torch.Tensor, block_off: torch.Tensor, block_sizes: torch.Tensor,
                  max_block_size: int, work: torch.Tensor | None = None, status: torch.Tensor | None = None,
                  stream=None):
    """Decode a ragged batch laid out as encode_ragged writes it into out
    (uint8, stripe s at block_off[s], block_sizes[s] bytes).  Returns status."""
    for t, dt, nm in ((parts, U8, "parts"), (part_off, torch.int64, "part_off"), (ids, U8, "ids"),
                      (avail, U8, "avail"), (out, U8, "out"), (block_off, torch.int64, "block_off"),
                      (block_sizes, torch.int32, "block_sizes")):
        _need(t, dt, nm)
    nstripes, navail = avail.shape[0], avail.shape[1]
    if work is None:
        work = decode_workspace(nstripes, k, parts.device)
    if status is None:
        status = torch.empty(nstripes, dtype=torch.int32, device=parts.device)
    check(lib().nkfs_nk8_decode_ragged(parts.data_ptr(), part_off.data_ptr(), n_slots, ids.data_ptr(),
                                       avail.data_ptr(), navail, k, out.data_ptr(), block_off.data_ptr(),
                                       block_sizes.data_ptr(), max_block_size, nstripes, work.data_ptr(),
                                       status.data_ptr(), _stream(stream)), "nkfs_nk8_decode_ragged")
    return status


def decode_verify(parts: torch.Tensor, n_slots: int, ids: torch.Tensor, avail: torch.Tensor, k: int,
                  block_size: int, expect: torch.Tensor, out: torch.Tensor | None = None,
                  work: torch.Tensor | None = None, status: torch.Tensor | None = None, stream=None):
    """decode() that also checks each part it reads against expect
    [nstripes * n_slots] (int64 XXH64 digests).  Returns (blocks, status,
    badmask): status -EIO and badmask bit j for a mismatching slot j."""
    _need(parts, U8, "parts")
    _need(ids, U8, "ids")
    _need(avail, U8, "avail")
    _need(expect, torch.int64, "expect")
    nstripes, navail = avail.shape[0], avail.shape[1]
    dev = parts.device
    if out is None:
        out = torch.empty((nstripes, block_size), dtype=U8, device=dev)
    if work is None:
        work = decode_workspace(nstripes, k, dev)
    if status is None:
        status = torch.empty(nstripes, dtype=torch.int32, device=dev)
    bad = torch.empty(nstripes, dtype=torch.int64, device=dev)
    check(lib().nkfs_nk8_decode_verify(parts.data_ptr(), parts.stride(0), n_slots, ids.data_ptr(),
                                       avail.data_ptr(), navail, k, block_size, out.data_ptr(),
                                       out.stride(0) if out.dim() > 1 else block_size, nstripes, work.data_ptr(),
                                       status.data_ptr(), expect.data_ptr(), bad.data_ptr(), _stream(stream)),
          "nkfs_nk8_decode_verify")
    return out, status, bad


def encode_host(blocks, block_size: int, n: int, k: int, ids, chunk_bytes: int = 0, digests: bool = True,
                out=None):
    """Host-memory encode (+XXH64): blocks uint8 [nstripes, pitch] and ids
    uint8 [nstripes, n] as numpy arrays or CPU tensors (pinned is fastest);
    streams through the GPU in sub-batches (nkfs_nk8_encode_host).  out =
    (parts, digests|None) reuses caller buffers (pinned: no per-call pin).
    Returns (parts [nstripes*n, part_pitch] CPU tensor, digests or None)."""
    bt = torch.as_tensor(blocks)
    it = torch.as_tensor(ids)
    if bt.dtype != U8 or it.dtype != U8 or bt.is_cuda or it.is_cuda or not bt.is_contiguous():
        raise ValueError("blocks/ids: contiguous uint8 host arrays")
    nstripes = bt.shape[0]
    pitch = part_pitch(block_size, k)
    if out is not None:
        parts, dig = out
        if parts.shape != (nstripes * n, pitch) or parts.dtype != U8 or parts.is_cuda or not parts.is_contiguous():
            raise ValueError("out parts: contiguous uint8 host tensor [nstripes*n, part_pitch]")
        if dig is not None and (dig.numel() != nstripes * n or dig.dtype != torch.int64 or dig.is_cuda):
            raise ValueError("out digests: int64 host tensor [nstripes*n]")
    else:
        parts = torch.empty((nstripes * n, pitch), dtype=U8, pin_memory=torch.cuda.is_available())
        dig = torch.empty(nstripes * n, dtype=torch.int64, pin_memory=torch.cuda.is_available()) if digests else None
    check(lib().nkfs_nk8_encode_host(bt.data_ptr(), bt.stride(0) if bt.dim() > 1 else block_size, block_size,
                                     nstripes, n, k, it.contiguous().data_ptr(), parts.data_ptr(), pitch,
                                     _ptr(dig), chunk_bytes), "nkfs_nk8_encode_host")
    return parts, dig


def encode_ragged_host(blocks, block_off, block_sizes, n: int, k: int, ids, parts, part_off, digests=None,
                       max_block_size: int | None = None, chunk_bytes: int = 0):
    """Host-memory ragged encode (+XXH64): every argument a contiguous host
    numpy array or CPU tensor (uint8 blocks/ids/parts, int64 offsets, int32
    sizes, int64 digests or None); offsets non-decreasing in stripe order.
    Writes parts/digests in place (nkfs_nk8_encode_ragged_host)."""
    t = [torch.as_tensor(x) for x in (blocks, block_off, block_sizes, ids, parts, part_off)]
    for x, dt, nm in zip(t, (U8, torch.int64, torch.int32, U8, U8, torch.int64),
                         ("blocks", "block_off", "block_sizes", "ids", "parts", "part_off")):
        if x.is_cuda or x.dtype != dt or not x.is_contiguous():
            raise ValueError(f"{nm}: contiguous {dt} host array")
    dg = None if digests is None else torch.as_tensor(digests)
    if dg is not None and (dg.is_cuda or dg.dtype != torch.int64 or not dg.is_contiguous()):
        raise ValueError("digests: contiguous int64 host array")
    nstripes = t[2].numel()
    mb = int(t[2].max()) if max_block_size is None and nstripes else (max_block_size or 1)
    check(lib().nkfs_nk8_encode_ragged_host(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), mb, nstripes, n, k,
                                            t[3].data_ptr(), t[4].data_ptr(), t[5].data_ptr(), _ptr(dg),
                                            chunk_bytes), "nkfs_nk8_encode_ragged_host")


def _host(x, dt, nm):
    t = torch.as_tensor(x)
    if t.is_cuda or t.dtype != dt or not t.is_contiguous():
        raise ValueError(f"{nm}: contiguous {dt} host array")
    return t


def encode_pages(pages, page_size: int, first_page, block_sizes, n: int, k: int, ids, parts, part_off,
                 digests=None, max_block_size: int | None = None, chunk_bytes: int = 0):
    """PUT from page lists (nkfs_nk8_encode_pages): pages int64 [npages]
    host page addresses, block s = first block_sizes[s] bytes of pages
    first_page[s], first_page[s]+1, ...; parts/digests written in place."""
    pg, fp, sz = _host(pages, torch.int64, "pages"), _host(first_page, torch.int64, "first_page"), \
        _host(block_sizes, torch.int32, "block_sizes")
    it, pt, po = _host(ids, U8, "ids"), _host(parts, U8, "parts"), _host(part_off, torch.int64, "part_off")
    dg = None if digests is None else _host(digests, torch.int64, "digests")
    mb = int(sz.max()) if max_block_size is None and sz.numel() else (max_block_size or 1)
    return lib().nkfs_nk8_encode_pages(pg.data_ptr(), page_size, fp.data_ptr(), sz.data_ptr(), mb, sz.numel(), n, k,
                                       it.data_ptr(), pt.data_ptr(), po.data_ptr(), _ptr(dg), chunk_bytes)


def decode_host(parts, part_pitch: int, n_slots: int, ids, avail, navail: int, k: int, block_size: int, blocks,
                block_pitch: int | None = None, status=None, expect=None, badmask=None, chunk_bytes: int = 0):
    """GET from host memory (nkfs_nk8_decode_host); blocks written in place.
    Returns the library's return code."""
    pt, it, av, bt = _host(parts, U8, "parts"), _host(ids, U8, "ids"), _host(avail, U8, "avail"), \
        _host(blocks, U8, "blocks")
    st = None if status is None else _host(status, torch.int32, "status")
    ex = None if expect is None else _host(expect, torch.int64, "expect")
    bm = None if badmask is None else _host(badmask, torch.int64, "badmask")
    nstripes = it.numel() // n_slots
    return lib().nkfs_nk8_decode_host(pt.data_ptr(), part_pitch, n_slots, it.data_ptr(), av.data_ptr(), navail, k,
                                      block_size, bt.data_ptr(), block_pitch or block_size, nstripes, _ptr(st),
                                      _ptr(ex), _ptr(bm), chunk_bytes)


def decode_ragged_host(parts, part_off, n_slots: int, ids, avail, navail: int, k: int, blocks, block_off,
                       block_sizes, status=None, expect=None, badmask=None, max_block_size: int | None = None,
                       chunk_bytes: int = 0):
    """GET of a ragged batch from host memory (nkfs_nk8_decode_ragged_host)."""
    pt, po, it, av = _host(parts, U8, "parts"), _host(part_off, torch.int64, "part_off"), _host(ids, U8, "ids"), \
        _host(avail, U8, "avail")
    bt, bo, sz = _host(blocks, U8, "blocks"), _host(block_off, torch.int64, "block_off"), \
        _host(block_sizes, torch.int32, "block_sizes")
    st = None if status is None else _host(status, torch.int32, "status")
    ex = None if expect is None else _host(expect, torch.int64, "expect")
    bm = None if badmask is None else _host(badmask, torch.int64, "badmask")
    mb = int(sz.max()) if max_block_size is None and sz.numel() else (max_block_size or 1)
    return lib().nkfs_nk8_decode_ragged_host(pt.data_ptr(), po.data_ptr(), n_slots, it.data_ptr(), av.data_ptr(),
                                             navail, k, bt.data_ptr(), bo.data_ptr(), sz.data_ptr(), mb, sz.numel(),
                                             _ptr(st), _ptr(ex), _ptr(bm), chunk_bytes)


def decode_pages(parts, part_off, n_slots: int, ids, avail, navail: int, k: int, pages, page_size: int, first_page,
                 block_sizes, status=None, expect=None, badmask=None, max_block_size: int | None = None,
                 chunk_bytes: int = 0):
    """GET into page lists (nkfs_nk8_decode_pages)."""
    pt, po, it, av = _host(parts, U8, "parts"), _host(part_off, torch.int64, "part_off"), _host(ids, U8, "ids"), \
        _host(avail, U8, "avail")
    pg, fp, sz = _host(pages, torch.int64, "pages"), _host(first_page, torch.int64, "first_page"), \
        _host(block_sizes, torch.int32, "block_sizes")
    st = None if status is None else _host(status, torch.int32, "status")
    ex = None if expect is None else _host(expect, torch.int64, "expect")
    bm = None if badmask is None else _host(badmask, torch.int64, "badmask")
    mb = int(sz.max()) if max_block_size is None and sz.numel() else (max_block_size or 1)
    return lib().nkfs_nk8_decode_pages(pt.data_ptr(), po.data_ptr(), n_slots, it.data_ptr(), av.data_ptr(), navail,
                                       k, pg.data_ptr(), page_size, fp.data_ptr(), sz.data_ptr(), mb, sz.numel(),
                                       _ptr(st), _ptr(ex), _ptr(bm), chunk_bytes)


def host_state() -> dict:
    """nkfs_host_state: registered ranges, registry references held by calls
    in flight, host lane threads and copy threads running, contexts handed
    out (a host call that returned leaves the middle three at zero)."""
    arr = (C.c_uint64 * 5)()
    lib().nkfs_host_state(arr, 5)
    return dict(zip(("registered", "call_refs", "lanes", "copy_threads", "contexts"), (int(v) for v in arr)))


def set_devices(devices) -> int:
    """nkfs_gpu_set_devices: device lanes of the host-memory entry points."""
    arr = (C.c_int * max(1, len(devices)))(*devices)
    return lib().nkfs_gpu_set_devices(arr, len(devices))


def get_devices() -> list[int]:
    arr = (C.c_int * 16)()
    n = lib().nkfs_gpu_get_devices(arr, 16)
    return list(arr[:n])


def xxh64_batch(base: torch.Tensor, off: torch.Tensor, lens: torch.Tensor, seed: int = 0, stream=None):
    _need(base, U8, "base")
    out = torch.empty(off.numel(), dtype=torch.int64, device=base.device)
    check(lib().nkfs_xxh64_batch(base.data_ptr(), off.data_ptr(), lens.data_ptr(), off.numel(), seed,
                                 out.data_ptr(), _stream(stream)), "nkfs_xxh64_batch")
    return out


def clu_sum(clusters: torch.Tensor, cluster_size: int | None = None, expect: torch.Tensor | None = None,
            stream=None):
    """dio_clu_sum over every row of clusters (uint8 [count, pitch]): XXH64 of
    the first cluster_size bytes (default: the whole row).  With expect
    (int64 [count]) also returns the per-cluster status (0 / -EINVAL) of
    nkfs_inode_block_check_sum.  Returns (sums, status|None)."""
    _need(clusters, U8, "clusters")
    count = clusters.shape[0]
    size = clusters.shape[1] if cluster_size is None else cluster_size
    sums = torch.empty(count, dtype=torch.int64, device=clusters.device)
    status = None
    if expect is not None:
        _need(expect, torch.int64, "expect")
        status = torch.empty(count, dtype=torch.int32, device=clusters.device)
    check(lib().nkfs_clu_sum_batch(clusters.data_ptr(), clusters.stride(0), size, count, sums.data_ptr(),
                                   _ptr(expect), _ptr(status), _stream(stream)), "nkfs_clu_sum_batch")
    return sums, status


def pages_dsum(pages: torch.Tensor, first_page: torch.Tensor, lens: torch.Tensor, page_size: int = 4096,
               stream=None):
    """nkfs_pages_dsum over page lists: pages int64 [npages] device pointers,
    payload i = first lens[i] bytes of pages[first_page[i]:]."""
    for t, nm in ((pages, "pages"), (first_page, "first_page"), (lens, "lens")):
        _need(t, torch.int64, nm)
    out = torch.empty(lens.numel(), dtype=torch.int64, device=lens.device)
    check(lib().nkfs_pages_dsum_batch(pages.data_ptr(), first_page.data_ptr(), lens.data_ptr(), lens.numel(),
                                      page_size, out.data_ptr(), _stream(stream)), "nkfs_pages_dsum_batch")
    return out


def synth(nstripes: int, block_size: int, pitch: int | None = None, seed: int | None = None, first: int = 0,
          device="cuda", stream=None) -> torch.Tensor:
    from .synth import SEED
    pitch = pitch or ((block_size + 15) // 16) * 16
    t = torch.empty((nstripes, pitch), dtype=U8, device=device)
    check(lib().nkfs_synth_blocks(t.data_ptr(), pitch, block_size, nstripes, SEED if seed is None else seed,
                                  first, _stream(stream)), "nkfs_synth_blocks")
    return t


def synth_ragged(blocks: torch.Tensor, block_off: torch.Tensor, block_sizes: torch.Tensor, seed: int | None = None,
                 first: int = 0, stream=None) -> torch.Tensor:
    """Fill a packed ragged batch in place (one launch): stripe s = the
    synthetic stripe first + s, block_sizes[s] bytes at block_off[s]."""
    from .synth import SEED
    _need(blocks, U8, "blocks")
    _need(block_off, torch.int64, "block_off")
    _need(block_sizes, torch.int32, "block_sizes")
    check(lib().nkfs_synth_ragged(blocks.data_ptr(), block_off.data_ptr(), block_sizes.data_ptr(), block_sizes.numel(),
                                  SEED if seed is None else seed, first, _stream(stream)), "nkfs_synth_ragged")
    return blocks


def digests_u64(d: torch.Tensor):
    """int64 digest tensor -> list of Python unsigned ints."""
    return [v & 0xFFFFFFFFFFFFFFFF for v in d.cpu().tolist()]
