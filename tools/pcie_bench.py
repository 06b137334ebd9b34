"""PCIe-inclusive rates of the host-memory entry points (include/nkfs_gpu.h):
the path's real ends, SURVEY.md §8(f) row 2.  User bytes (block bytes) per
second, host buffers pinned once (a server's page pool), outputs verified
against the inputs after timing.

    python tools/pcie_bench.py [link c2 c3 c4 c5 pages lanes depth c2pg c3pg c4pg]

link  = the raw pinned link on this box: hipMemcpyAsync H2D alone, D2H alone,
        and both at once on two streams (1 GiB each way); every PUT / GET line
        then carries the bound the link puts on it (user GiB/s such that the
        H2D bytes, the D2H bytes and their sum each fit the measured rates)
        and the fraction of it reached.
depth = C3 PUT / GET at host_depth 3 / 6 x host_lanes 1 / 2 (struct nkfs_tune)
c3pg  = C3 from pageable caller buffers (staged through pinned scratch, round 6)

PUT  = nkfs_nk8_encode_host: blocks H2D -> encode + XXH64 -> parts + digests D2H
GET  = nkfs_nk8_decode_host: k survivor parts per stripe H2D -> decode -> blocks D2H
       (+ verify: the part digests checked inside the rebuild)
pages = the same through 4 KiB page lists (nkfs_nk8_encode_pages /
       nkfs_nk8_decode_pages: gathered into / scattered from pinned staging)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import C5_SIZES, CONFIGS  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402

GIB = 2**30
LINK = {}


def link(parts=4):
    """Raw pinned PCIe rates (GiB/s): H2D, D2H, and both directions at once,
    each direction as `parts` streams x (1 GiB / parts) copies (one stream
    serialises behind one DMA queue; the pipeline keeps several in flight
    too).  The best of the stream counts tried is kept for the bounds."""
    nbytes = 1 << 30
    q = nbytes // parts
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    up = [torch.cuda.Stream() for _ in range(parts)]
    down = [torch.cuda.Stream() for _ in range(parts)]

    def run(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]

    def h2d():
        for i, st in enumerate(up):
            with torch.cuda.stream(st):
                d[i * q:(i + 1) * q].copy_(h[i * q:(i + 1) * q], non_blocking=True)

    def d2h():
        for i, st in enumerate(down):
            with torch.cuda.stream(st):
                h2[i * q:(i + 1) * q].copy_(d2[i * q:(i + 1) * q], non_blocking=True)

    def both():
        h2d()
        d2h()

    r = {"h2d": nbytes / run(h2d) / GIB, "d2h": nbytes / run(d2h) / GIB, "bidir_total": 2 * nbytes / run(both) / GIB}
    for key, v in r.items():
        LINK[key] = max(LINK.get(key, 0.0), v)
    print(f"link (pinned, 1 GiB each way, {parts} streams per direction)  H2D {r['h2d']:6.2f} GiB/s   "
          f"D2H {r['d2h']:6.2f} GiB/s   both at once {r['bidir_total']:6.2f} GiB/s in all", flush=True)
    del h, h2, d, d2


def bound(h2d_per_user, d2h_per_user):
    """User GiB/s the measured link allows when every user byte moves
    h2d_per_user bytes host->device and d2h_per_user bytes device->host."""
    if not LINK:
        return None
    return min(LINK["h2d"] / h2d_per_user, LINK["d2h"] / d2h_per_user,
               LINK["bidir_total"] / (h2d_per_user + d2h_per_user))


def frac(rate, b):
    return f"{rate / b:5.3f}" if b else "  n/a"


def timed(fn, reps=3):
    fn()  # warm-up: pooled contexts and scratch
    t0 = time.perf_counter()
    for _ in range(reps):
        rc = fn()
        assert rc in (None, 0) or isinstance(rc, tuple), rc
    return (time.perf_counter() - t0) / reps


def uniform(name, user_bytes=1 << 30, lanes=None, tune=None, pinned=True):
    """pinned=False: pageable caller buffers, which the library stages
    through its pinned scratch by host copies (round 6)."""
    S0, B, n, k, _ = CONFIGS[name]
    S = min(S0, user_bytes // B)
    pitch = batch.part_pitch(B, k)
    pin = (lambda t: t.pin_memory()) if pinned else (lambda t: t.clone())
    blocks = pin(batch.synth(S, B).cpu()[:, :B].contiguous())
    ids = pin(torch.from_numpy(synth.batch_ids(S, n)))
    parts = pin(torch.empty((S * n, pitch), dtype=torch.uint8))
    dig = pin(torch.empty(S * n, dtype=torch.int64))
    if lanes is not None:
        _lib.check(batch.set_devices(lanes))
    tune = dict(tune or {})
    chunk = tune.pop("chunk", 0)  # sub-batch bytes (0: the library's default)
    tuned = _lib.tuned(**tune)
    tuned.__enter__()
    t_put = timed(lambda: batch.encode_host(blocks, B, n, k, ids, out=(parts, dig), chunk_bytes=chunk))
    # GET: the k survivors each stripe holds, packed (n_slots = k)
    surv = synth.batch_survivors(S, n, k).astype(np.int64)
    pv = parts.view(S, n, pitch)
    idx = torch.from_numpy(surv)
    held = pin(torch.gather(pv, 1, idx[:, :, None].expand(S, k, pitch)).contiguous())
    hid = pin(torch.gather(ids.view(S, n).long(), 1, idx).to(torch.uint8).contiguous())
    hexp = pin(torch.gather(dig.view(S, n), 1, idx).contiguous())
    avail = pin(torch.arange(k, dtype=torch.uint8).repeat(S, 1).contiguous())
    out = pin(torch.empty((S, B), dtype=torch.uint8))
    st = pin(torch.empty(S, dtype=torch.int32))
    bad = pin(torch.empty(S, dtype=torch.int64))
    t_get = timed(lambda: batch.decode_host(held, pitch, k, hid, avail, k, k, B, out, B, status=st, chunk_bytes=chunk))
    ok = bool(torch.equal(out, blocks)) and int(st.abs().sum()) == 0
    t_getv = timed(lambda: batch.decode_host(held, pitch, k, hid, avail, k, k, B, out, B, status=st, expect=hexp,
                                             badmask=bad, chunk_bytes=chunk))
    ok = ok and bool(torch.equal(out, blocks)) and int(st.abs().sum()) == 0
    tuned.__exit__(None, None, None)
    if lanes is not None:
        batch.set_devices([])
    ub = S * B
    tag = f"{name} lanes={lanes}" if lanes is not None else name
    if not pinned:
        tag += " pageable"
    if tune or chunk:
        tag += " " + ",".join(f"{a}={b}" for a, b in tune.items()) + (f",chunk={chunk >> 20}M" if chunk else "")
    put, get, getv = ub / t_put / GIB, ub / t_get / GIB, ub / t_getv / GIB
    bp, bg = bound(1.0, n * pitch / B), bound(k * pitch / B, 1.0)
    print(f"{tag:18s} {S:6d} x {B:8d}  PUT {put:6.2f} GiB/s   GET {get:6.2f} GiB/s   "
          f"GET+verify {getv:6.2f} GiB/s   in/out per GiB user: PUT {1 + n * pitch / B:.2f} GiB, "
          f"GET {1 + k * pitch / B:.2f} GiB   link bound PUT {bp or 0:6.2f} ({frac(put, bp)}) "
          f"GET {bg or 0:6.2f} ({frac(get, bg)})   verified={ok}", flush=True)


def ragged(user_bytes=1 << 30, pages=False, page=4096):
    n, k = 8, 5
    sizes = synth.mixed_sizes(CONFIGS["c5"][0], C5_SIZES)
    keep = int(np.searchsorted(np.cumsum(sizes.astype(np.int64)), user_bytes)) + 1
    sizes = sizes[:keep]
    S = len(sizes)
    boff = np.zeros(S, np.int64)
    poff = np.zeros(S, np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes.tolist()):
        boff[s], poff[s] = pos, ppos
        pos += (B + 255) // 256 * 256
        ppos += n * batch.part_pitch(B, k)
    host = torch.zeros(pos, dtype=torch.uint8).pin_memory()
    for s, B in enumerate(sizes.tolist()):
        host[boff[s]: boff[s] + B] = torch.from_numpy(synth.stripe_bytes(s, B))
    ids = torch.from_numpy(synth.batch_ids(S, n)).pin_memory()
    parts = torch.empty(ppos, dtype=torch.uint8).pin_memory()
    dig = torch.empty(S * n, dtype=torch.int64).pin_memory()
    sz = torch.from_numpy(sizes.astype(np.int32))
    bo, po = torch.from_numpy(boff), torch.from_numpy(poff)
    avail = torch.from_numpy(synth.batch_survivors(S, n, k))
    st = torch.empty(S, dtype=torch.int32)
    ub = int(sizes.sum())
    if not pages:
        t_put = timed(lambda: batch.encode_ragged_host(host, bo, sz, n, k, ids, parts, po, dig))
        out = torch.zeros(pos, dtype=torch.uint8).pin_memory()
        t_get = timed(lambda: batch.decode_ragged_host(parts, po, n, ids, avail, k, k, out, bo, sz, status=st))
        ok = bool(torch.equal(out, host)) and int(st.abs().sum()) == 0
        ps_all = float(n * sum(batch.part_pitch(B, k) for B in sizes.tolist())) / ub
        bp, bg = bound(1.0, ps_all), bound(ps_all, 1.0)
        put, get = ub / t_put / GIB, ub / t_get / GIB
        print(f"c5 ragged          {S:6d} stripes  PUT {put:6.2f} GiB/s   GET {get:6.2f} GiB/s"
              f"   (GET ships all {n} slots)   link bound PUT {bp or 0:6.2f} ({frac(put, bp)}) "
              f"GET {bg or 0:6.2f} ({frac(get, bg)})   verified={ok}", flush=True)
        return
    # page lists: every block in its own 4 KiB pages of a pinned pool
    npg = [(B + page - 1) // page for B in sizes.tolist()]
    first = np.concatenate([[0], np.cumsum(npg)[:-1]]).astype(np.int64)
    pool = torch.zeros(int(sum(npg)) * page, dtype=torch.uint8).pin_memory()
    rng = np.random.default_rng(7)
    slot = rng.permutation(int(sum(npg)))
    pg = torch.from_numpy(pool.data_ptr() + slot.astype(np.int64) * page)
    pn = pool.numpy()
    for s, B in enumerate(sizes.tolist()):
        src = host[boff[s]: boff[s] + B].numpy()
        for i in range(npg[s]):
            o = int(slot[first[s] + i]) * page
            c = src[i * page:(i + 1) * page]
            pn[o: o + len(c)] = c
    fp = torch.from_numpy(first)
    t_put = timed(lambda: batch.encode_pages(pg, page, fp, sz, n, k, ids, parts, po, dig))
    pool2 = torch.zeros_like(pool).pin_memory()
    pg2 = torch.from_numpy(pool2.data_ptr() + slot.astype(np.int64) * page)
    t_get = timed(lambda: batch.decode_pages(parts, po, n, ids, avail, k, k, pg2, page, fp, sz, status=st))
    ok = bool(torch.equal(pool2, pool)) or all(
        np.array_equal(pool2.numpy()[int(slot[first[s]]) * page: int(slot[first[s]]) * page + min(B, page)],
                       host[boff[s]: boff[s] + min(B, page)].numpy()) for s, B in enumerate(sizes.tolist()))
    print(f"c5 pages ({page} B)  {S:6d} stripes  PUT {ub / t_put / GIB:6.2f} GiB/s   GET {ub / t_get / GIB:6.2f} GiB/s"
          f"   verified={ok}", flush=True)


def main():
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    what = sys.argv[1:] or ["link", "c2", "c3", "c4", "c5", "pages", "lanes", "depth"]
    for w in what:
        if w == "link":
            for parts in (2, 4, 8):
                link(parts)
        elif w == "depth":
            for tune in ({"host_depth": 3, "host_lanes": 1}, {"host_depth": 6, "host_lanes": 2},
                         {"host_depth": 6, "host_lanes": 2, "enc_few_max": 8},
                         {"host_depth": 6, "host_lanes": 2, "chunk": 64 << 20},
                         {"host_depth": 4, "host_lanes": 2, "chunk": 64 << 20, "enc_few_max": 8}):
                uniform("c3", tune=tune)
        elif w in ("c2", "c3", "c4"):
            uniform(w)
        elif w in ("c2pg", "c3pg", "c4pg"):  # pageable caller buffers (staged)
            uniform(w[:2], pinned=False)
        elif w == "c5":
            ragged()
        elif w == "pages":
            ragged(pages=True)
        elif w == "lanes":
            uniform("c3", lanes=[0, 0])
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
