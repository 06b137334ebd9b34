"""bench.py -- device-resident N-K encode(+XXH64 of every part)+decode
throughput on MI355X, one process per GPU, stripes partitioned over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config all|c2|c3|c4|c5|w1|w2|w3]
                    [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Headline (BASELINE.json metric, configs[2] = SURVEY.md §8(d) C3): N=8, K=5,
1 MiB stripes, 8,192 stripes (8 GiB) in all, split evenly over the GPUs
(strong scaling, as SURVEY.md §8(d) defines C3; --scaling weak keeps 8,192
per GPU).  Step = one pass of the hot path over the batch resident in HBM:
  nkfs_nk8_encode  (fused encode + XXH64 of every part), then
  nkfs_nk8_decode  (per-stripe K x K inverse + apply) from the seeded
                   survivors (n-k parts erased per stripe).
value = user bytes of the whole job x K steps / max-over-ranks wall time.

The same line carries the other configs as sub-objects under "configs"
(c3s8: the 1,024-stripe per-GPU shard of the strong N=8 run, timed on one
GPU; C2: 65,536 x 4 KiB N4K2; C4: 16,384 x 256 KiB N8K5; C5: the ragged
4 KiB / 64 KiB / 1 MiB mix, byte-balanced over the ranks; W1/W2/W3: the general
n, k paths, W3 with k = 41 > 32), each timed over at least 200 ms with its own roofline.

The dominant kernel's roofline is measured live with HIP events on the
stream the library launches on (torch's current stream); algorithmic bytes
per stripe are SURVEY.md §8(d)'s: encode+hash B + n*ps + 8n.  Next to the
8 TB/s spec every roofline carries `box_stream`: the rate this box sustains,
in the same process, for the kernel's read:write mix with the arithmetic
stripped (nkfs_amd/csrc/boxprobe.hip), and the kernel's fraction of it.  The
CPU baseline (rank 0, N=1) times the reference's own code (oracle/_ref) on a
bounded sample of the same workload on this box's host cores: one thread
and the box's CPU share.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident N-K encode+decode, 4KiB–1MiB stripes, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MIN_TIMED_S = 0.25     # sub-configs: at least this much timed work each (>= 200 ms measured)

CONFIGS = {
    # name: (stripes per GPU, block size, n, k, description)
    "c2": (65536, 4096, 4, 2, "C2: N=4,K=2 encode(+XXH64/part)+decode(2 erased), 65536 x 4 KiB stripes per GPU"),
    "c3": (8192, 1048576, 8, 5, "C3: N=8,K=5 encode(+XXH64/part)+decode(3 erased), 8192 x 1 MiB stripes (8 GiB) "
                                "per GPU"),
    "c4": (16384, 262144, 8, 5, "C4: N=8,K=5 encode(+XXH64/part)+decode(3 erased), 16384 x 256 KiB stripes per GPU"),
    # beyond the BASELINE configs: n > 8, k > 8 (SURVEY.md §8 a5/a8 for general n, k) on the
    # part-group encoder with XXH64 fused (k_encode_wide_ws) and the survivor-table decoder (nk8_wide.hip)
    "w1": (2048, 1048576, 16, 12, "W1: N=16,K=12 encode(+XXH64/part)+decode(4 erased), 2048 x 1 MiB stripes per "
                                  "GPU (general n,k path; not a BASELINE config)"),
    # k > 16 (the reference allows k <= 254, crt/nk8.c:13-16; its self test draws k uniform in [2, 254],
    # crt/nk8.c:735-744): the column-chunked kernels (nk8_big.hip), XXH64 a second pass over the parts
    "w2": (256, 1048576, 48, 32, "W2: N=48,K=32 encode(+XXH64/part)+decode(16 erased), 256 x 1 MiB stripes per "
                                 "GPU (k > 16 path; not a BASELINE config)"),
    # k > 32 with rows of an odd byte count (most of the reference's k domain, its self
    # test's k uniform in [2, 254], lies above 32)
    "w3": (256, 1048576, 64, 41, "W3: N=64,K=41 encode(+XXH64/part)+decode(23 erased), 256 x 1 MiB stripes per "
                                 "GPU (k > 32, odd k path; not a BASELINE config)"),
    # ragged: block size of every stripe drawn from C5_SIZES (synth.mixed_sizes)
    "c5": (11520, None, 8, 5, "C5: N=8,K=5 encode(+XXH64/part)+decode(3 erased) of a ragged batch, stripe sizes "
                              "uniform over {4 KiB, 64 KiB, 1 MiB}, ~4 GiB per GPU, byte-balanced over the GPUs"),
}
C5_SIZES = (4096, 65536, 1048576)
HEADLINE = "c3"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30, help="timed steps of the headline config")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="all", choices=["all"] + sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=4.0, help="target duration of each CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pcie", action="store_true", help="also time the host-memory (PCIe-inclusive) path")
    ap.add_argument("--stripes", type=int, default=0, help="override the stripes per GPU of a single --config")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="control collectives: nccl (RCCL over xGMI, the real run) or gloo (CPU; rehearses the "
                         "multi-rank path with ranks sharing GPUs, e.g. 2 ranks on a 1-GPU box -- not a measurement)")
    ap.add_argument("--tune", default="", help="experiments only: struct nkfs_tune fields to set, k=v,k=v "
                    "(recorded in the line; the default line uses the library's defaults)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="headline C3: strong = 8,192 stripes in all split over the GPUs (SURVEY.md §8(d)); "
                         "weak = 8,192 per GPU")
    return ap.parse_args()


# ------------------------------------------------------------ distributed

def dist_setup(backend: str):
    """(rank, world, local_rank); initialises torch.distributed when the
    launcher set WORLD_SIZE > 1."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local


def stripe_range(rank: int, per_rank: int):
    """Rank r owns stripes [r*per_rank, (r+1)*per_rank) (weak scaling)."""
    return rank * per_rank, per_rank


def strong_range(rank: int, world: int, total: int):
    """Strong scaling (8,192 stripes total split evenly
    across the G GPUs): rank r owns the contiguous range [lo, hi) of the
    global batch, sizes differing by at most one stripe."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi - lo


def byte_balanced_ranges(sizes, world: int):
    """Contiguous stripe ranges [lo, hi) per rank with (nearly) equal user
    bytes (ranges byte-balanced for mixed batches)."""
    import numpy as np
    csum = np.concatenate([[0], np.cumsum(np.asarray(sizes, dtype=np.int64))])
    total = int(csum[-1])
    cuts = [0] + [int(np.searchsorted(csum, total * r / world, side="left")) for r in range(1, world)] + [len(sizes)]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


_CDEV = None  # collectives' device when it differs from the data's (--backend gloo: the CPU)


def cdev(device):
    """Device the control collectives run on: the rank's GPU under RCCL
    (backend nccl), the CPU under gloo (a rehearsal of the multi-rank path)."""
    return _CDEV if _CDEV is not None else device


def rank_spread(enc_s: float, dec_s: float, device) -> dict:
    """Every rank's mean encode / decode launch time (µs), all-gathered, so
    that a line at N > 1 shows the imbalance between ranks (max and min next
    to the per-rank list; the headline's roofline is rank 0's launches)."""
    import torch
    import torch.distributed as dist
    v = torch.tensor([enc_s * 1e6, dec_s * 1e6], dtype=torch.float64, device=cdev(device))
    if dist.is_available() and dist.is_initialized():
        out = [torch.zeros_like(v) for _ in range(dist.get_world_size())]
        dist.all_gather(out, v)
    else:
        out = [v]
    enc = [round(float(t[0]), 2) for t in out]
    dec = [round(float(t[1]), 2) for t in out]
    return {"encode_us": enc, "decode_us": dec, "encode_us_max": max(enc), "encode_us_min": min(enc),
            "decode_us_max": max(dec), "decode_us_min": min(dec)}


def reduce_max(value: float, device) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=cdev(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_digest_xor(local_xor: int, device) -> list[int]:
    """All-gather each rank's 64-bit xor-of-part-digests (the control
    collective: 8 bytes per rank)."""
    import torch
    import torch.distributed as dist
    v = torch.tensor([local_xor - (1 << 64) if local_xor >= (1 << 63) else local_xor], dtype=torch.int64,
                     device=cdev(device))
    if not (dist.is_available() and dist.is_initialized()):
        return [local_xor]
    out = [torch.zeros_like(v) for _ in range(dist.get_world_size())]
    dist.all_gather(out, v)
    return [int(x.item()) & 0xFFFFFFFFFFFFFFFF for x in out]


def gather_digests(local, device):
    """All-gather every rank's per-part digests (int64, 8n bytes per stripe:
    SURVEY.md §8(e) collective (2)) -> list of CPU tensors, one per rank.
    Ranks may hold different stripe counts (C5): padded to the largest."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [local.cpu()]
    world = dist.get_world_size()
    device = cdev(device)
    cnt = torch.tensor([local.numel()], dtype=torch.int64, device=device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    m = max(int(c.item()) for c in cnts)
    pad = torch.zeros(m, dtype=torch.int64, device=device)
    pad[:local.numel()] = local.to(device)
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad)
    return [t[:int(c.item())].cpu() for t, c in zip(out, cnts)]


def check_rank_digests(gathered, n, expect_fn, samples=8):
    """Rank 0's cross-rank check: for a sample of every rank's stripes the
    oracle's XXH64 of the regenerated parts (synth is a pure function of the
    global stripe index) equals that rank's digests.  expect_fn(rank, s) ->
    the expected n digests of that rank's local stripe s.  Returns the number
    of ranks verified, or -1 on a mismatch."""
    for r, dig in enumerate(gathered):
        d = [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig.tolist()]
        count = len(d) // n
        for s in range(0, count, max(1, count // samples)):
            if d[s * n:(s + 1) * n] != expect_fn(r, s):
                return -1
    return len(gathered)


_BARRIER_GPU = None  # the rank's GPU for RCCL barriers (set in main; None under gloo)


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        if _BARRIER_GPU is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[_BARRIER_GPU])  # the communicator's own GPU, no guess by rank
        else:
            dist.barrier()


# ----------------------------------------------------------------- timing

def phase(name, fn, check, device):
    """Run one library call of a step.  With `check` (the first warmup step)
    the device is synchronised after it, so an asynchronous fault is reported
    against the call that caused it instead of the next call that happens to
    read the runtime's sticky error."""
    import torch
    try:
        fn()
        if check:
            torch.cuda.synchronize(device)
    except (OSError, RuntimeError) as ex:
        raise RuntimeError(f"{name}: {ex}") from ex


def timed_steps(step, steps, warmup, device, stream, nev=2):
    """W untimed steps, then exactly `steps` timed steps bracketed by a
    barrier + synchronize on both sides (max over ranks).  Returns
    (elapsed_s, [per-launch seconds for each of the nev events gaps])."""
    import torch
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(nev + 1)] for _ in range(steps)]
    for _ in range(warmup):
        step(None)
    torch.cuda.synchronize(device)
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(steps):
        step(ev[i])
    torch.cuda.synchronize(device)
    barrier()
    t1 = time.perf_counter()
    elapsed = reduce_max(t1 - t0, device)
    per = [sum(e[j].elapsed_time(e[j + 1]) for e in ev) / 1e3 / steps for j in range(nev)]
    return elapsed, per


def auto_steps(step, device, min_steps):
    """Steps so that the timed region lasts >= MIN_TIMED_S (one probe step
    after the warmup sets the estimate)."""
    import torch
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    step(None)
    torch.cuda.synchronize(device)
    est = max(time.perf_counter() - t0, 1e-6)
    # every rank must time the same number of steps
    est = reduce_max(est, device)
    return max(min_steps, int(math.ceil(MIN_TIMED_S / est)))


_PROBE = None


def probe_lib():
    """nkfs_amd/lib/libnkfs_boxprobe.so (nkfs_amd/csrc/boxprobe.hip): the
    arithmetic-free stream bench.py calibrates each box with; None if absent."""
    global _PROBE
    if _PROBE is None:
        import ctypes as C
        path = os.path.join(ROOT, "nkfs_amd", "lib", "libnkfs_boxprobe.so")
        if not os.path.exists(path):
            return None
        P = C.CDLL(path)
        P.nkfs_probe_stream.restype = C.c_int
        P.nkfs_probe_stream.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_double)]
        _PROBE = P
    return _PROBE


MIXES = ((4, 8), (5, 8), (6, 8), (8, 8), (8, 4))


def box_stream(src, dst, read_bytes, write_bytes, stream):
    """HBM rate (GB/s) this box sustains, in this process, for the kernel's
    read:write mix with the arithmetic stripped: contiguous 1 KiB runs, a
    compact chip-wide front, 8 and 16 resident waves per CU (the better one
    is kept).  `src` / `dst` are the kernel's own input / output tensors
    (their contents are overwritten: call after verification).  The spec
    peak is 8 TB/s; this is the ceiling the box really offers the mix."""
    import ctypes as C
    P = probe_lib()
    if P is None:
        return None
    ratio = read_bytes / max(1, write_bytes)
    L, S = min(MIXES, key=lambda c: abs(c[0] / c[1] - ratio))
    best = 0.0
    for wpc in (8, 16):
        ms, nb = C.c_float(0), C.c_double(0)
        rc = P.nkfs_probe_stream(src.data_ptr(), src.numel() * src.element_size(), dst.data_ptr(),
                                 dst.numel() * dst.element_size(), L, S, wpc, 9, stream.cuda_stream, C.byref(ms),
                                 C.byref(nb))
        if rc == 0 and ms.value > 0:
            best = max(best, nb.value / (ms.value * 1e-3) / 1e9)
    if best <= 0:
        return None
    return {"GBps": round(best, 1), "read_write_kib": [L, S], "frac_of_peak": round(best / HBM_PEAK_GBS, 4)}


_ANCHOR = {}
_BOX = {}


def hbm_anchor(src, dst, stream):
    """The microarch guide's own anchor (MI355X_MICROARCH.md: 6.29 TB/s
    measured for a float4 copy), measured once per process on this box:
    plain grid-stride float4 copy, pure read and pure write kernels
    (boxprobe.hip nkfs_probe_plain), best of three grid sizes, over up to 4
    GiB of the headline's own buffers (past the 256 MB Infinity Cache).  It
    anchors `box_stream` independently of the product's access shape."""
    import ctypes as C
    if _ANCHOR:
        return _ANCHOR
    P = probe_lib()
    if P is None or not hasattr(P, "nkfs_probe_plain"):
        return None
    P.nkfs_probe_plain.restype = C.c_int
    P.nkfs_probe_plain.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                   C.POINTER(C.c_float), C.POINTER(C.c_double)]
    nbytes = min(src.numel() * src.element_size(), dst.numel() * dst.element_size(), 4 << 30) // 4096 * 4096
    cus = 256
    try:
        import torch
        cus = torch.cuda.get_device_properties(src.device).multi_processor_count
    except Exception:  # noqa: BLE001 -- property lookup only
        pass
    out = {"bytes_per_buffer": nbytes}
    for kind, name in ((0, "copy"), (1, "read"), (2, "write")):
        best, best_grid = 0.0, 0
        for per_cu in (4, 8, 32):
            ms, moved = C.c_float(0), C.c_double(0)
            rc = P.nkfs_probe_plain(src.data_ptr(), dst.data_ptr(), nbytes, kind, per_cu * cus, 7,
                                    stream.cuda_stream, C.byref(ms), C.byref(moved))
            if rc == 0 and ms.value > 0 and moved.value / (ms.value * 1e-3) / 1e9 > best:
                best, best_grid = moved.value / (ms.value * 1e-3) / 1e9, per_cu
        out[f"{name}_GBps"] = round(best, 1)
        out[f"{name}_wg_per_cu"] = best_grid
    out["kernel"] = "boxprobe.hip k_copy4/k_read4/k_write4: grid-stride float4, 256 threads/WG"
    _ANCHOR.update(out)
    return _ANCHOR


def box_clock(stream):
    """CU count, the runtime's peak shader clock and the clock a busy grid
    runs at on this box (boxprobe.hip k_clock: s_memtime cycles against the
    100 MHz s_memrealtime) -- VERDICT r05 item 4: box-to-box swings of the
    same kernels are attributed with it."""
    import ctypes as C
    P = probe_lib()
    if P is None or not hasattr(P, "nkfs_probe_clock"):
        return None
    P.nkfs_probe_clock.restype = C.c_int
    P.nkfs_probe_clock.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    mhz, cus, peak = C.c_double(0), C.c_int(0), C.c_int(0)
    if P.nkfs_probe_clock(stream.cuda_stream, C.byref(mhz), C.byref(cus), C.byref(peak)) != 0:
        return None
    return {"cus": cus.value, "sclk_peak_mhz": peak.value, "sclk_loaded_mhz": round(mhz.value, 1),
            "probe": "boxprobe.hip k_clock: 4 waves per CU, dependent integer chain, s_memtime vs s_memrealtime"}


def anchor_mix(read_bytes, write_bytes):
    """The HBM bound this box's anchor gives a kernel's read:write mix,
    independent of the product's access shape: (r + w) / (r / read_GBps +
    w / write_GBps) from the plain float4 read and write kernels
    (hbm_anchor).  None before the anchor ran or for an empty mix."""
    rd, wr = _ANCHOR.get("read_GBps"), _ANCHOR.get("write_GBps")
    if not rd or not wr or read_bytes + write_bytes <= 0:
        return None
    return (read_bytes + write_bytes) / (read_bytes / rd + write_bytes / wr)


def with_box(roof, box, rw=None):
    """Attach the box's own ceilings to a roofline dict: `box_stream` (the
    kernel's read:write mix through k_mix, the product's access shape; its
    spread between buffers of one process is a few %), the
    fraction of the guide's plain float4 copy, and -- rw = (read bytes,
    write bytes) of one launch -- `frac_of_anchor_mix`, the fraction of the
    bound the anchor's read and write rates give that mix (anchor_mix)."""
    if box:
        roof["box_stream"] = box
        roof["frac_of_box_stream"] = round(roof["achieved"] / box["GBps"], 4)
    if _ANCHOR.get("copy_GBps"):
        roof["frac_of_anchor_copy"] = round(roof["achieved"] / _ANCHOR["copy_GBps"], 4)
    if rw is not None:
        bound = anchor_mix(*rw)
        if bound:
            roof["anchor_mix_GBps"] = round(bound, 1)
            roof["frac_of_anchor_mix"] = round(roof["achieved"] / bound, 4)
    return roof


def roofline(kernel, nbytes, secs, traffic):
    return {"bound": "hbm", "kernel": kernel, "achieved": round(nbytes / secs / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(nbytes / secs / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": nbytes, "us_per_launch": round(secs * 1e6, 2)}


# --------------------------------------------------------------- workload

def workload(name, rank, world, stripes=0, strong_total=0):
    """(first global stripe, stripes on this rank, workload label) of a
    uniform config: strong scaling splits strong_total stripes over the
    ranks, weak scaling gives every rank `stripes` (default the config's)."""
    S, B, n, k, desc = CONFIGS[name]
    head = desc.split(", ")[0]  # "C3: N=8,K=5 encode(+XXH64/part)+decode(3 erased)"
    if strong_total:
        first, S = strong_range(rank, world, strong_total)
        return first, S, (f"{head}, {strong_total} x {B // 1024} KiB stripes in all, split evenly over {world} "
                          f"GPU(s) (strong scaling; {S} on this GPU)")
    if stripes:
        S = stripes
        desc = f"{head}, {S} x {B // 1024} KiB stripes per GPU"
    elif world > 1:
        desc = f"{desc} (weak scaling: {S * world} in all over {world} GPUs)"
    first, _ = stripe_range(rank, S)
    return first, S, desc


def uniform_result(name, args, rank, world, device, S, B, n, k, desc, strong_total, steps, elapsed, enc_s, dec_s,
                   box_enc, box_dec, ok, ranks_ok, gathered):
    """The result dict of one uniform config from what run_uniform measured
    (elapsed = max-over-ranks wall time of `steps` steps; enc_s / dec_s =
    this rank's mean encode / decode launch): value, roofline (this rank's
    launches, algorithmic bytes per SURVEY.md §8(d)), per-rank launch times
    (a collective: every rank calls this), and on rank 0 the CPU baseline at
    every world size.  Pure bookkeeping: tests/test_dist.py runs it at world
    2 over gloo."""
    ps = B // k + (1 if B % k else 0)
    enc_bytes = S * (B + n * ps + 8 * n)
    dec_bytes = S * (k * ps + B + k)
    # user bytes of the whole job: weak = every rank's S; strong = the total
    total_stripes = strong_total if strong_total else S * world
    user_bytes = total_stripes * B * steps
    dec = with_box({"achieved": round(dec_bytes / dec_s / 1e9, 1), "achieved_GBps": round(dec_bytes / dec_s / 1e9, 1),
                    "frac": round(dec_bytes / dec_s / 1e9 / HBM_PEAK_GBS, 4), "us_per_launch": round(dec_s * 1e6, 2),
                    "bytes_per_launch": dec_bytes}, box_dec, (S * k * ps, S * B))
    res = {
        "value": round(user_bytes / elapsed / 2**30, 3), "unit": "GiB/s", "steps": steps,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "timed_ms": round(elapsed * 1e3, 1),
        "scaling": "strong" if strong_total else "weak",
        "config": {"workload": desc, "n": n, "k": k, "block_size": B, "stripes_per_gpu": S, "part_size": ps,
                   "erased_per_stripe": n - k, "parallelism": f"stripe-partition x{world}",
                   "stripes_all_gpus": total_stripes},
        "roofline": with_box(roofline("nkfs_nk8_encode (encode + XXH64 per part)", enc_bytes, enc_s,
                                      pmc_traffic(name, S, world)), box_enc, (S * B, S * n * ps + 8 * S * n)),
        "decode": dec,
        "verified": ok, "verified_ranks": ranks_ok, "digest_xor_per_rank": [f"{x:016x}" for x in gathered],
        "per_rank": rank_spread(enc_s, dec_s, device),
    }
    if rank == 0 and not args.no_cpu:  # at every world size (rank 0's host cores)
        res["cpu_baseline"] = cpu_baseline(S, B, n, k, args.cpu_seconds)
    return res


def run_uniform(name, args, rank, world, device, steps, stripes=0, strong_total=0):
    """One uniform config: returns the result dict (value, roofline, ...).
    Weak scaling: `stripes` (default the config's) per GPU.  Strong scaling
    (strong_total > 0): that many stripes in all, split over the ranks."""
    import torch
    from nkfs_amd import batch, synth
    _, B, n, k, _ = CONFIGS[name]
    first, S, desc = workload(name, rank, world, stripes, strong_total)
    ps = batch.part_size(B, k)
    stream = torch.cuda.current_stream(device)

    blocks = batch.synth(S, B, first=first, device=device)
    ids_np = synth.batch_ids(S, n, first=first)
    ids = torch.from_numpy(ids_np).to(device)
    avail = torch.from_numpy(synth.batch_survivors(S, n, k, first=first)).to(device)
    parts = torch.empty((S * n, batch.part_pitch(B, k)), dtype=torch.uint8, device=device)
    digests = torch.empty(S * n, dtype=torch.int64, device=device)
    out = torch.empty((S, B), dtype=torch.uint8, device=device)
    work = batch.decode_workspace(S, k, device)
    status = torch.empty(S, dtype=torch.int32, device=device)

    def step(e, check=False):
        if e:
            e[0].record(stream)
        phase(f"{name} encode", lambda: batch.encode(blocks, B, n, k, ids, parts, digests, stream=stream), check,
              device)
        if e:
            e[1].record(stream)
        phase(f"{name} decode", lambda: batch.decode(parts, n, ids, avail, k, B, out=out, work=work, status=status,
                                                     stream=stream), check, device)
        if e:
            e[2].record(stream)

    for w in range(args.warmup):
        step(None, check=w == 0)
    if steps is None:
        steps = auto_steps(step, device, args.steps)
    elapsed, (enc_s, dec_s) = timed_steps(step, steps, 0, device, stream)

    # correctness of what was timed: decode == input, digests vs oracle on a sample
    ok = bool(torch.equal(out, blocks[:, :B])) and int(status.abs().sum()) == 0
    from oracle import oracle as O
    dig = digests.cpu()
    dx = 0
    for d in dig.tolist():
        dx ^= d & 0xFFFFFFFFFFFFFFFF
    for s in range(0, S, max(1, S // 16)):
        want = [O.xxh64(p) for p in O.encode(blocks[s, :B].cpu().numpy(), n, k, ids_np[s])]
        ok &= [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig[s * n:(s + 1) * n].tolist()] == want
    gathered = gather_digest_xor(dx, device)
    all_dig = gather_digests(digests, device)
    ranks_ok = None
    if rank == 0:
        def expect(r, s):
            g = (strong_range(r, world, strong_total)[0] if strong_total else r * S) + s
            return [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, B), n, k, synth.stripe_ids(g, n))]
        ranks_ok = check_rank_digests(all_dig, n, expect)
    ok &= ranks_ok != -1
    # the box's own ceiling for each kernel's read:write mix, on the
    # kernel's own buffers (after verification: the probe overwrites them)
    hbm_anchor(blocks, parts, stream)
    if not _BOX:
        _BOX.update(box_clock(stream) or {})
    box_enc = box_stream(blocks, parts, S * B, S * n * ps, stream)
    box_dec = box_stream(parts, out, S * k * ps, S * B, stream)
    res = uniform_result(name, args, rank, world, device, S, B, n, k, desc, strong_total, steps, elapsed, enc_s,
                         dec_s, box_enc, box_dec, ok, ranks_ok, gathered)
    if rank == 0 and args.pcie:
        res["pcie_inclusive_GiBps"] = pcie_rate(batch, blocks, S, B, n, k, ids)
    del blocks, parts, out, digests
    torch.cuda.empty_cache()
    return res


def c5_layout(world, per_rank):
    """Global C5 batch of world*per_rank stripes (sizes from the size
    stream), cut into byte-balanced contiguous ranges, one per rank."""
    from nkfs_amd import synth
    sizes = synth.mixed_sizes(world * per_rank, C5_SIZES)
    return sizes, byte_balanced_ranges(sizes, world)


def run_ragged(args, rank, world, device, steps):
    """C5: one ragged batch of mixed 4 KiB / 64 KiB / 1 MiB stripes, packed
    back to back in HBM (block s at block_off[s], parts at part_off[s] with
    the 256-B part pitch), encoded (+XXH64 of every part) with
    nkfs_nk8_encode_ragged and decoded from n-k erased with
    nkfs_nk8_decode_ragged each step.  The global batch is byte-balanced
    over the ranks; stripe g of the global batch is synth stripe g."""
    import numpy as np
    import torch
    from nkfs_amd import batch, synth

    S0, _, n, k, desc = CONFIGS["c5"]
    gsizes, ranges = c5_layout(world, S0)
    lo, hi = ranges[rank]
    sizes = gsizes[lo:hi]
    S = hi - lo
    boff = np.zeros(S, np.int64)
    poff = np.zeros(S, np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes.tolist()):
        boff[s], poff[s] = pos, ppos
        pos += (B + 255) // 256 * 256
        ppos += n * batch.part_pitch(B, k)
    stream = torch.cuda.current_stream(device)
    # every stripe generated on the device in one launch (synth stripe =
    # global stripe index)
    blocks = torch.zeros(pos, dtype=torch.uint8, device=device)
    batch.synth_ragged(blocks, torch.from_numpy(boff).to(device), torch.from_numpy(sizes.astype(np.int32)).to(device),
                       first=lo, stream=stream)
    ids_np = synth.batch_ids(S, n, first=lo)
    ids = torch.from_numpy(ids_np).to(device)
    avail = torch.from_numpy(synth.batch_survivors(S, n, k, first=lo)).to(device)
    sz = torch.from_numpy(sizes.astype(np.int32)).to(device)
    bo = torch.from_numpy(boff).to(device)
    po = torch.from_numpy(poff).to(device)
    parts = torch.empty(ppos, dtype=torch.uint8, device=device)
    digests = torch.empty(S * n, dtype=torch.int64, device=device)
    out = torch.zeros(pos, dtype=torch.uint8, device=device)
    work = batch.decode_workspace(S, k, device)
    status = torch.empty(S, dtype=torch.int32, device=device)
    maxB = int(gsizes.max())

    def step(e, check=False):
        if e:
            e[0].record(stream)
        phase("c5 encode_ragged", lambda: batch.encode_ragged(blocks, bo, sz, n, k, ids, parts, po, digests, maxB,
                                                              stream=stream), check, device)
        if e:
            e[1].record(stream)
        phase("c5 decode_ragged", lambda: batch.decode_ragged(parts, po, n, ids, avail, k, out, bo, sz, maxB,
                                                              work=work, status=status, stream=stream), check, device)
        if e:
            e[2].record(stream)

    for w in range(args.warmup):
        step(None, check=w == 0)
    if steps is None:
        steps = auto_steps(step, device, args.steps)
    elapsed, (enc_s, dec_s) = timed_steps(step, steps, 0, device, stream)

    ok = bool(torch.equal(out, blocks)) and int(status.abs().sum()) == 0
    dig = digests.cpu()
    from oracle import oracle as O
    for B in C5_SIZES:  # oracle digests on a sample of every size class
        for s in np.nonzero(sizes == B)[0][:4].tolist():
            blk = blocks[boff[s]: boff[s] + B].cpu().numpy()
            ok &= [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig[s * n:(s + 1) * n].tolist()] == \
                [O.xxh64(p) for p in O.encode(blk, n, k, ids_np[s])]
    dx = 0
    for d in dig.tolist():
        dx ^= d & 0xFFFFFFFFFFFFFFFF
    gathered = gather_digest_xor(dx, device)
    all_dig = gather_digests(digests, device)
    ranks_ok = None
    if rank == 0:
        def expect(r, s):
            g = ranges[r][0] + s
            B = int(gsizes[g])
            return [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, B), n, k, synth.stripe_ids(g, n))]
        ranks_ok = check_rank_digests(all_dig, n, expect)
    ok &= ranks_ok != -1
    ps = [batch.part_size(B, k) for B in sizes.tolist()]
    user = int(sizes.sum())
    enc_bytes = user + n * sum(ps) + 8 * n * S
    dec_bytes = k * sum(ps) + user + k * S
    total_user = reduce_sum(user, device)
    hbm_anchor(blocks, parts, stream)
    box_enc = box_stream(blocks, parts, user, n * sum(ps), stream)
    box_dec = box_stream(parts, out, k * sum(ps), user, stream)
    res = {
        "value": round(total_user * steps / elapsed / 2**30, 3), "unit": "GiB/s", "steps": steps,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "timed_ms": round(elapsed * 1e3, 1),
        "config": {"workload": desc, "n": n, "k": k, "block_sizes": list(C5_SIZES), "stripes_this_gpu": S,
                   "user_bytes_this_gpu": user, "user_bytes_all_gpus": total_user, "erased_per_stripe": n - k,
                   "parallelism": f"stripe-partition x{world} (byte-balanced ranges)"},
        "scaling": "weak",
        "roofline": with_box(roofline("nkfs_nk8_encode_ragged (encode + XXH64 per part)", enc_bytes, enc_s,
                                      pmc_traffic("c5", S, world)), box_enc, (user, n * sum(ps) + 8 * n * S)),
        "decode": with_box({"achieved": round(dec_bytes / dec_s / 1e9, 1), "achieved_GBps": round(dec_bytes / dec_s / 1e9, 1),
                            "frac": round(dec_bytes / dec_s / 1e9 / HBM_PEAK_GBS, 4),
                            "us_per_launch": round(dec_s * 1e6, 2), "bytes_per_launch": dec_bytes}, box_dec,
                           (k * sum(ps), user)),
        "verified": ok, "verified_ranks": ranks_ok, "digest_xor_per_rank": [f"{x:016x}" for x in gathered],
        "per_rank": rank_spread(enc_s, dec_s, device),
    }
    if rank == 0 and not args.no_cpu:  # at every world size (rank 0's host cores)
        res["cpu_baseline"] = cpu_baseline_mixed(sizes, n, k, args.cpu_seconds)
    if rank == 0 and args.pcie:
        res["pcie_inclusive_GiBps"] = pcie_rate_ragged(batch, blocks, boff, poff, sizes, ids_np, n, k, ppos)
    del blocks, parts, out, digests
    torch.cuda.empty_cache()
    return res


def reduce_sum(value: int, device) -> int:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.int64, device=cdev(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def compose_line(args, rank, world, top, subs):
    """The one JSON line (driver contract) from the headline result and the
    sub-configs: metric, value, timing, the headline's roofline and CPU
    baseline, the box's HBM anchor, the CPU model on rank 0."""
    top = dict(top)
    result = {
        "metric": METRIC, "value": top.pop("value"), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": top.pop("ms_per_step"), "higher_is_better": True,
        "scaling": top.pop("scaling"), "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 stripes generated on device, seed 0x6E6B3846)",
    }
    top.pop("steps")
    top.pop("unit")
    result.update(top)
    if subs:
        result["configs"] = subs
        result["verified"] = bool(result["verified"]) and all(v["verified"] for v in subs.values())
    if _ANCHOR:
        result["hbm_anchor"] = dict(_ANCHOR)
    if _BOX:
        result["box"] = dict(_BOX)
    if rank == 0 and not args.no_cpu:
        result["cpu_model"] = cpu_model()
    if getattr(args, "tune", ""):
        result["tune"] = args.tune
    if getattr(args, "backend", "nccl") != "nccl":
        result["backend"] = f"{args.backend} (rehearsal: ranks may share a GPU; not a measurement)"
    return result


def main():
    args = parse()
    import torch

    # the rank's GPU is selected before the process group exists, so RCCL's
    # communicator binds to it (one process per GPU)
    global _CDEV, _BARRIER_GPU
    ngpu = max(1, torch.cuda.device_count())
    gpu = int(os.environ.get("LOCAL_RANK", "0")) % ngpu  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(gpu)
    rank, world, local = dist_setup(args.backend)
    if args.backend == "gloo":
        _CDEV = torch.device("cpu")
    else:
        _BARRIER_GPU = gpu
    device = torch.device("cuda", gpu)
    os.environ["NKFS_DEVICE"] = str(gpu)
    local = gpu

    from nkfs_amd import _lib
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(local), "nkfs_gpu_init")
    if args.tune:
        t = _lib.get_tune()
        for kv in args.tune.split(","):
            key, val = kv.split("=")
            setattr(t, key, int(val))
        _lib.check(L.nkfs_tune_set(t), "nkfs_tune_set")

    head = HEADLINE if args.config == "all" else args.config
    strong = CONFIGS[HEADLINE][0] if (args.scaling == "strong" and head == HEADLINE and not args.stripes) else 0

    def run(name, steps, stripes=0, strong_total=0):
        if name == "c5":
            return run_ragged(args, rank, world, device, steps)
        return run_uniform(name, args, rank, world, device, steps, stripes, strong_total)

    top = run(head, args.steps, args.stripes if args.config != "all" else 0, strong)
    subs = {}
    if args.config == "all":
        if world == 1:
            # the per-GPU shard of the headline's strong N=8 run, timed on one
            # GPU now (kernel choice and per-GPU efficiency at 1,024 stripes)
            subs["c3s8"] = run("c3", None, CONFIGS["c3"][0] // 8)
        for name in ("c2", "c4", "c5", "w1", "w2", "w3"):
            subs[name] = run(name, None)
    result = compose_line(args, rank, world, top, subs)
    if rank == 0:
        print(json.dumps(result), flush=True)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


# -------------------------------------------------------------- baselines

def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> tuple[int, int]:
    """(threads used, CPUs visible).  The GPU box gives a job its CPU share
    through OMP_NUM_THREADS (16 per GPU) while nproc shows the whole
    machine; the baseline uses the share (never more than the affinity)."""
    visible = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or visible
    return max(1, min(share, visible)), os.cpu_count() or visible


def _time_cpu(blocks, sv, n, k, threads, kind, target_s):
    """Passes over `blocks` until ~target_s; returns (GiB/s, secs, passes)."""
    from oracle import oracle as O
    t, _ = O.bench_encode_decode(blocks, n, k, sv, threads, kind)
    passes = max(1, int(round(target_s / max(t, 1e-9))))
    total = t
    for _ in range(passes - 1):
        t2, _ = O.bench_encode_decode(blocks, n, k, sv, threads, kind)
        total += t2
    return blocks.shape[0] * blocks.shape[1] * passes / total / 2**30, total, passes


def cpu_baseline(S, B, n, k, target_s):
    """The reference's own split + XXH64 + assemble (oracle/_ref), on a
    bounded sample of this workload, on this box's host cores: one thread and
    the box's CPU share."""
    from nkfs_amd import synth
    from oracle import oracle as O
    kind = "reference" if O.ref_lib() is not None else "port"
    threads, visible = cpu_threads()
    count = int(max(threads, min(S, (128 << 20) // B)))
    blocks = synth.batch_bytes(count, B)
    sv = synth.batch_survivors(count, n, k)
    one, t1, p1 = _time_cpu(blocks[: max(1, count // threads)], sv[: max(1, count // threads)], n, k, 1, kind,
                            target_s)
    many, tm, pm = _time_cpu(blocks, sv, n, k, threads, kind, target_s)
    return {"value": round(many, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1_thread": round(one, 4), "cpus_visible": visible,
            "sample": f"{count} stripes x {B} B (N={n},K={k}), nk8_split_block + XXH64 of every part + "
                      f"nk8_assemble_block from {k} survivors: {pm} pass(es) on {threads} pthreads ({tm:.1f} s), "
                      f"{p1} pass(es) over {max(1, count // threads)} stripes on 1 thread ({t1:.1f} s)"}


def cpu_baseline_mixed(sizes, n, k, target_s):
    """The reference's split + XXH64 + assemble on a bounded sample of the
    C5 mix: per size class, stripes timed for the class's share (by bytes in
    the batch) of ~target_s; GiB/s over the mix, 1 thread and the share."""
    from nkfs_amd import synth
    from oracle import oracle as O
    kind = "reference" if O.ref_lib() is not None else "port"
    threads, visible = cpu_threads()
    rates = {}
    for th in (1, threads):
        total_t = total_b = 0.0
        for B in C5_SIZES:
            share = float((sizes == B).sum() * B) / float(sizes.sum())
            count = max(th, min(int((sizes == B).sum()), (32 << 20) // B))
            blocks = synth.batch_bytes(count, B)
            sv = synth.batch_survivors(count, n, k)
            rate, _, _ = _time_cpu(blocks, sv, n, k, th, kind, target_s * share)
            total_t += share / rate
            total_b += share
        rates[th] = total_b / total_t
    return {"value": round(rates[threads], 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1_thread": round(rates[1], 4), "cpus_visible": visible,
            "sample": f"C5 mix (N={n},K={k}): per size class {list(C5_SIZES)}, nk8_split_block + XXH64 of every "
                      f"part + nk8_assemble_block from {k} survivors, weighted by the batch's bytes per class, "
                      f"~{target_s:.0f} s per thread count"}


def pmc_traffic(config, stripes=None, world=1):
    """Per-launch HBM bytes of the encode kernel from the committed rocprofv3
    PMC summary (tools/pmc.sh: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    FETCH_SIZE halving corrected per MI355X_MICROARCH.md §HBM), or None.
    A launch's traffic depends only on the batch one GPU holds, so an entry
    is attached to any line -- at any world size -- whose per-GPU stripe
    count is the profiled run's: "c3@1024" is the c3 kernel on 1,024
    stripes (the N = 8 strong shard), "c3" the full 8,192."""
    del world  # per-GPU traffic: the PMC pass of the same per-GPU batch on one GPU
    path = os.path.join(ROOT, "profiles", "traffic.json")
    want = CONFIGS[config][0] if stripes is None else stripes
    try:
        with open(path) as f:
            doc = json.load(f)
        for key in (f"{config}@{want}", config):
            entry = doc.get(key)
            if entry is not None and entry.get("stripes") == want:
                return entry["encode_bytes_per_launch"]
        return None
    except (OSError, ValueError, KeyError):
        return None


def pcie_rate(batch, blocks, S, B, n, k, ids):
    """Host-memory path (nkfs_nk8_encode_host): pinned host blocks -> H2D ->
    fused encode+XXH64 -> D2H of parts and digests, sub-batches pipelined on
    three streams.  User GiB/s; DESIGN.md records it (never the headline)."""
    import torch
    cnt = min(S, (1 << 30) // B)  # 1 GiB of user data from host memory
    host_in = blocks[:cnt, :B].cpu().pin_memory()
    ids_h = ids[:cnt].cpu().pin_memory()
    out = batch.encode_host(host_in, B, n, k, ids_h)  # warm-up: pinned outputs, pooled streams/scratch
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        batch.encode_host(host_in, B, n, k, ids_h, out=out)
    t1 = time.perf_counter()
    del out
    torch.cuda.empty_cache()
    return round(cnt * B * reps / (t1 - t0) / 2**30, 3)


def pcie_rate_ragged(batch, blocks, boff, poff, sizes, ids_np, n, k, ppos):
    """C5 from host memory (nkfs_nk8_encode_ragged_host): pinned packed
    blocks -> H2D -> ragged encode+XXH64 -> D2H of parts and digests, in
    sub-batches of consecutive stripes on three streams.  User GiB/s."""
    import torch
    host = blocks.cpu().pin_memory()
    bo = torch.from_numpy(boff).pin_memory()
    po = torch.from_numpy(poff).pin_memory()
    sz = torch.from_numpy(sizes.astype("int32")).pin_memory()
    ids = torch.from_numpy(ids_np).pin_memory()
    parts = torch.empty(ppos, dtype=torch.uint8).pin_memory()
    dig = torch.empty(len(sizes) * n, dtype=torch.int64).pin_memory()
    batch.encode_ragged_host(host, bo, sz, n, k, ids, parts, po, dig)  # warm-up
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        batch.encode_ragged_host(host, bo, sz, n, k, ids, parts, po, dig)
    t1 = time.perf_counter()
    return round(int(sizes.sum()) * reps / (t1 - t0) / 2**30, 3)


if __name__ == "__main__":
    main()
