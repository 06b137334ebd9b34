"""bench.py -- device-resident N-K encode(+XXH64 of every part)+decode
throughput on MI355X, one process per GPU, weak scaling over stripes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Step = one pass of the hot path over one batch resident in HBM:
  nkfs_nk8_encode  (fused encode + XXH64 of every part), then
  nkfs_nk8_decode  (per-stripe K x K inverse + apply) from the seeded
                   survivors (n-k parts erased per stripe).
value = user bytes of all ranks x steps / max-over-ranks wall time (GiB/s).

The dominant kernel's roofline is measured live with HIP events on the
stream the library launches on (torch's current stream); algorithmic bytes
per stripe are SURVEY.md §8(d)'s: encode+hash B + n*ps + 8n.  The CPU
baseline (rank 0, N=1) times the reference's own code (oracle/_ref) on a
bounded sample of the same workload on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident N-K encode+decode, 4KiB–1MiB stripes, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (stripes per GPU, block size, n, k, description)
    "c2": (65536, 4096, 4, 2, "C2: N=4,K=2 encode(+XXH64/part)+decode(2 erased), 65536 x 4 KiB stripes per GPU"),
    "c3": (2048, 1048576, 8, 5, "C3: N=8,K=5 encode(+XXH64/part)+decode(3 erased), 2048 x 1 MiB stripes per GPU"),
    "c4": (16384, 262144, 8, 5, "C4: N=8,K=5 encode(+XXH64/part)+decode(3 erased), 16384 x 256 KiB stripes per GPU"),
    # ragged: block size of every stripe drawn from C5_SIZES (synth.mixed_sizes)
    "c5": (11520, None, 8, 5, "C5: N=8,K=5 encode(+XXH64/part)+decode(3 erased) of a ragged batch, stripe sizes "
                              "uniform over {4 KiB, 64 KiB, 1 MiB}, 11520 stripes (~4 GiB) per GPU"),
}
C5_SIZES = (4096, 65536, 1048576)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pcie", action="store_true", help="also time the host-memory (PCIe-inclusive) path")
    ap.add_argument("--strong-total", type=int, default=0,
                    help="strong scaling: this many stripes in total, split evenly over the ranks "
                         "(SURVEY.md 8(d) C3: 8192 x 1 MiB); default = the config's stripes per GPU (weak)")
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
    """Rank r owns stripes [r*per_rank, (r+1)*per_rank) (weak scaling: a
    fixed per_rank; strong: per_rank = total / world)."""
    return rank * per_rank, per_rank


def per_rank_stripes(config_stripes: int, strong_total: int, world: int) -> int:
    """Stripes per rank: the config's per-GPU count (weak scaling) or an even
    share of a fixed total (strong scaling)."""
    if not strong_total:
        return config_stripes
    if strong_total % world:
        raise SystemExit(f"--strong-total {strong_total} does not split evenly over {world} ranks")
    return strong_total // world


def reduce_max(value: float, device) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_digest_xor(local_xor: int, device) -> list[int]:
    """All-gather each rank's 64-bit xor-of-part-digests (the control
    collective: 8 bytes per rank)."""
    import torch
    import torch.distributed as dist
    v = torch.tensor([local_xor - (1 << 64) if local_xor >= (1 << 63) else local_xor], dtype=torch.int64,
                     device=device)
    if not (dist.is_available() and dist.is_initialized()):
        return [local_xor]
    out = [torch.zeros_like(v) for _ in range(dist.get_world_size())]
    dist.all_gather(out, v)
    return [int(x.item()) & 0xFFFFFFFFFFFFFFFF for x in out]


def gather_digests(local, device):
    """All-gather every rank's per-part digests (int64 [stripes*n], 8n bytes
    per stripe: SURVEY.md §8(e) collective (2)) -> list of CPU tensors, one
    per rank."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [local.cpu()]
    out = [torch.empty_like(local) for _ in range(dist.get_world_size())]
    dist.all_gather(out, local.to(device))
    return [t.cpu() for t in out]


def check_rank_digests(gathered, per_rank, B, n, k, samples=8):
    """Rank 0's cross-rank check: for a sample of every rank's stripes, the
    oracle's parts and XXH64 of the regenerated input (synth is a pure
    function of the global stripe index) equal the digests that rank
    produced.  Returns the number of ranks verified, or -1 on a mismatch."""
    from nkfs_amd import synth
    from oracle import oracle as O
    for r, dig in enumerate(gathered):
        d = [int(x) & 0xFFFFFFFFFFFFFFFF for x in dig.tolist()]
        for s in range(0, per_rank, max(1, per_rank // samples)):
            g = r * per_rank + s
            want = [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, B), n, k, synth.stripe_ids(g, n))]
            if d[s * n:(s + 1) * n] != want:
                return -1
    return len(gathered)


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


# --------------------------------------------------------------- workload

def main():
    args = parse()
    import torch

    # the rank's GPU is selected before the process group exists, so RCCL's
    # communicator binds to it (one process per GPU)
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    rank, world, local = dist_setup("nccl")
    device = torch.device("cuda", local)
    os.environ["NKFS_DEVICE"] = str(local)

    from nkfs_amd import _lib, batch, synth
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(local), "nkfs_gpu_init")

    if args.config == "c5":
        if args.strong_total:
            raise SystemExit("--strong-total applies to the uniform configs (c2-c4)")
        return run_ragged(args, rank, world, device)
    S, B, n, k, desc = CONFIGS[args.config]
    S = per_rank_stripes(S, args.strong_total, world)
    if args.strong_total:
        desc = (f"{desc.rsplit(', ', 1)[0]}, {args.strong_total} x {B // 1024} KiB stripes in total "
                f"split over {world} GPU(s) (strong scaling)")
    first, _ = stripe_range(rank, S)
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

    # HIP events around every launch of the timed region, on the stream the
    # library launches on (torch's current stream): per-kernel live timing
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(e=None):
        if e:
            e[0].record(stream)
        batch.encode(blocks, B, n, k, ids, parts, digests, stream=stream)
        if e:
            e[1].record(stream)
        batch.decode(parts, n, ids, avail, k, B, out=out, work=work, status=status, stream=stream)
        if e:
            e[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(ev[i])
    torch.cuda.synchronize(device)
    barrier()
    t1 = time.perf_counter()
    elapsed = reduce_max(t1 - t0, device)
    enc_s = sum(e[0].elapsed_time(e[1]) for e in ev) / 1e3 / args.steps
    dec_s = sum(e[1].elapsed_time(e[2]) for e in ev) / 1e3 / args.steps

    # correctness of what was timed: decode == input, digests vs oracle sample
    ok = bool(torch.equal(out, blocks[:, :B])) and int(status.abs().sum()) == 0
    dig = [int(x) & 0xFFFFFFFFFFFFFFFF for x in digests.cpu().tolist()]
    from oracle import oracle as O
    blocks_np = blocks[:, :B].cpu().numpy()
    for s in range(0, S, max(1, S // 64)):
        want = [O.xxh64(p) for p in O.encode(blocks_np[s], n, k, ids_np[s])]
        ok &= dig[s * n:(s + 1) * n] == want
    dx = 0
    for d in dig:
        dx ^= d
    gathered = gather_digest_xor(dx, device)
    all_dig = gather_digests(digests, device)
    ranks_ok = check_rank_digests(all_dig, S, B, n, k) if rank == 0 else None
    ok &= ranks_ok != -1
    enc_bytes = S * (B + n * ps + 8 * n)
    dec_bytes = S * (k * ps + B + k)

    user_bytes = S * B * world * args.steps
    value = user_bytes / elapsed / 2**30
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.strong_total else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded splitmix64 stripes generated on device, seed 0x6E6B3846)",
        "config": {"workload": desc, "n": n, "k": k, "block_size": B, "stripes_per_gpu": S,
                   "part_size": ps, "erased_per_stripe": n - k, "parallelism": f"stripe-partition x{world}"},
        "roofline": {
            "bound": "hbm",
            "kernel": "nkfs_nk8_encode (encode + XXH64 per part)",
            "achieved": round(enc_bytes / enc_s / 1e9, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(enc_bytes / enc_s / 1e9 / HBM_PEAK_GBS, 4),
            # PMC traffic is measured on the config's own batch; another
            # batch size (--strong-total) has none of its own
            "traffic": pmc_traffic(args.config) if S == CONFIGS[args.config][0] else None,
            "bytes_per_launch": enc_bytes,
            "us_per_launch": round(enc_s * 1e6, 2),
        },
        "decode": {"achieved_GBps": round(dec_bytes / dec_s / 1e9, 1), "us_per_launch": round(dec_s * 1e6, 2),
                   "bytes_per_launch": dec_bytes},
        "verified": ok,
        "verified_ranks": ranks_ok,
        "digest_xor_per_rank": [f"{x:016x}" for x in gathered],
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(S, B, n, k, args.cpu_seconds)
    if rank == 0 and args.pcie:
        result["pcie_inclusive_GiBps"] = pcie_rate(batch, blocks_np, S, B, n, k, ids, avail, device, stream)
    if rank == 0:
        print(json.dumps(result), flush=True)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def run_ragged(args, rank, world, device):
    """C5: one ragged batch of mixed 4 KiB / 64 KiB / 1 MiB stripes, packed
    back to back in HBM (block s at block_off[s], parts at part_off[s] with
    the 256-B part pitch), encoded (+XXH64 of every part) with
    nkfs_nk8_encode_ragged and decoded from n-k erased with
    nkfs_nk8_decode_ragged each step."""
    import numpy as np
    import torch
    from nkfs_amd import batch, synth

    S, _, n, k, desc = CONFIGS["c5"]
    first, _ = stripe_range(rank, S)
    sizes = synth.mixed_sizes(first + S, C5_SIZES)[first:]
    boff = np.zeros(S, np.int64)
    poff = np.zeros(S, np.int64)
    pos = ppos = 0
    for s, B in enumerate(sizes.tolist()):
        boff[s], poff[s] = pos, ppos
        pos += (B + 255) // 256 * 256
        ppos += n * batch.part_pitch(B, k)
    stream = torch.cuda.current_stream(device)
    # stripes generated on the device, one uniform batch per size class
    # (stripe ids first + class offset + i), scattered into the packed
    # buffer in 256-byte rows: a few launches, not one per stripe
    blocks = torch.zeros(pos, dtype=torch.uint8, device=device)
    rows = blocks.view(-1, 256)
    for ci, B in enumerate(C5_SIZES):
        idx = np.nonzero(sizes == B)[0]
        if not len(idx):
            continue
        data = batch.synth(len(idx), B, first=first + ci * S, device=device)
        r = (torch.from_numpy(boff[idx] // 256).to(device)[:, None] +
             torch.arange(B // 256, device=device)[None, :]).reshape(-1)
        rows[r] = data[:, :B].reshape(-1, 256)
        del data, r
    ids_np = synth.batch_ids(S, n, first=first)
    ids = torch.from_numpy(ids_np).to(device)
    avail = torch.from_numpy(synth.batch_survivors(S, n, k, first=first)).to(device)
    sz = torch.from_numpy(sizes.astype(np.int32)).to(device)
    bo = torch.from_numpy(boff).to(device)
    po = torch.from_numpy(poff).to(device)
    parts = torch.empty(ppos, dtype=torch.uint8, device=device)
    digests = torch.empty(S * n, dtype=torch.int64, device=device)
    out = torch.zeros(pos, dtype=torch.uint8, device=device)
    work = batch.decode_workspace(S, k, device)
    status = torch.empty(S, dtype=torch.int32, device=device)
    maxB = int(sizes.max())
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(e=None):
        if e:
            e[0].record(stream)
        batch.encode_ragged(blocks, bo, sz, n, k, ids, parts, po, digests, maxB, stream=stream)
        if e:
            e[1].record(stream)
        batch.decode_ragged(parts, po, n, ids, avail, k, out, bo, sz, maxB, work=work, status=status, stream=stream)
        if e:
            e[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(ev[i])
    torch.cuda.synchronize(device)
    barrier()
    t1 = time.perf_counter()
    elapsed = reduce_max(t1 - t0, device)
    enc_s = sum(e[0].elapsed_time(e[1]) for e in ev) / 1e3 / args.steps
    dec_s = sum(e[1].elapsed_time(e[2]) for e in ev) / 1e3 / args.steps

    ok = bool(torch.equal(out, blocks)) and int(status.abs().sum()) == 0
    dig = [int(x) & 0xFFFFFFFFFFFFFFFF for x in digests.cpu().tolist()]
    from oracle import oracle as O
    for B in C5_SIZES:  # oracle digests on a sample of every size class
        for s in np.nonzero(sizes == B)[0][:4].tolist():
            blk = blocks[boff[s]: boff[s] + B].cpu().numpy()
            ok &= dig[s * n:(s + 1) * n] == [O.xxh64(p) for p in O.encode(blk, n, k, ids_np[s])]
    dx = 0
    for d in dig:
        dx ^= d
    gathered = gather_digest_xor(dx, device)
    ps = [batch.part_size(B, k) for B in sizes.tolist()]
    user = int(sizes.sum())
    enc_bytes = user + n * sum(ps) + 8 * n * S
    dec_bytes = k * sum(ps) + user + k * S
    value = user * world * args.steps / elapsed / 2**30
    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 stripes generated on device, seed 0x6E6B3846; sizes from the "
                "separate size stream)",
        "config": {"workload": desc, "n": n, "k": k, "block_sizes": list(C5_SIZES), "stripes_per_gpu": S,
                   "user_bytes_per_gpu": user, "erased_per_stripe": n - k,
                   "parallelism": f"stripe-partition x{world}"},
        "roofline": {"bound": "hbm", "kernel": "nkfs_nk8_encode_ragged (encode + XXH64 per part)",
                     "achieved": round(enc_bytes / enc_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(enc_bytes / enc_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("c5"),
                     "bytes_per_launch": enc_bytes, "us_per_launch": round(enc_s * 1e6, 2)},
        "decode": {"achieved_GBps": round(dec_bytes / dec_s / 1e9, 1), "us_per_launch": round(dec_s * 1e6, 2),
                   "bytes_per_launch": dec_bytes},
        "verified": ok,
        "digest_xor_per_rank": [f"{x:016x}" for x in gathered],
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline_mixed(sizes, n, k, args.cpu_seconds)
    if rank == 0 and args.pcie:
        result["pcie_inclusive_GiBps"] = pcie_rate_ragged(batch, blocks, boff, poff, sizes, ids_np, n, k, pos, ppos)
    if rank == 0:
        print(json.dumps(result), flush=True)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def cpu_baseline_mixed(sizes, n, k, target_s):
    """The reference's split + XXH64 + assemble on a bounded sample of the
    C5 mix: per size class, a few stripes timed until the class's share
    (by bytes in the batch) of ~target_s is spent; GiB/s over the mix."""
    from nkfs_amd import synth
    from oracle import oracle as O
    kind = "reference" if O.ref_lib() is not None else "port"
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    total_t = 0.0
    total_b = 0
    for B in C5_SIZES:
        share = float((sizes == B).sum() * B) / float(sizes.sum())
        count = max(threads, min(int((sizes == B).sum()), (64 << 20) // B))
        blocks = synth.batch_bytes(count, B)
        sv = synth.batch_survivors(count, n, k)
        t, _ = O.bench_encode_decode(blocks, n, k, sv, threads, kind)
        passes = max(1, int(round(target_s * share / max(t, 1e-9))))
        for _ in range(passes - 1):
            t2, _ = O.bench_encode_decode(blocks, n, k, sv, threads, kind)
            t += t2
        # weight each class by its share of the batch's bytes
        rate = count * passes * B / t
        total_t += share * float(sizes.sum()) / rate
        total_b += share * float(sizes.sum())
    return {"value": round(total_b / total_t / 2**30, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"C5 mix (N={n},K={k}): per size class {list(C5_SIZES)}, nk8_split_block + XXH64 of every "
                      f"part + nk8_assemble_block from {k} survivors, {threads} pthreads, weighted by the "
                      f"batch's bytes per class, ~{target_s:.0f} s"}


def pcie_rate_ragged(batch, blocks, boff, poff, sizes, ids_np, n, k, pos, ppos):
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


def pmc_traffic(config):
    """Per-launch HBM bytes of the encode kernel from the committed rocprofv3
    PMC summary (tools/pmc.sh: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    FETCH_SIZE halving corrected per MI355X_MICROARCH.md §HBM), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(config)
        return None if entry is None else entry["encode_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def cpu_baseline(S, B, n, k, target_s):
    """The reference's own split + XXH64 + assemble (oracle/_ref), on a
    bounded sample of this workload (at most S stripes, reused across
    passes until ~target_s seconds of CPU time), on this box's host cores."""
    from nkfs_amd import synth
    from oracle import oracle as O
    kind = "reference" if O.ref_lib() is not None else "port"
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    count = int(max(threads, min(S, (256 << 20) // B)))
    blocks = synth.batch_bytes(count, B)
    sv = synth.batch_survivors(count, n, k)
    secs, _ = O.bench_encode_decode(blocks[: max(threads, count // 16)], n, k, sv[: max(threads, count // 16)],
                                    threads, kind)
    per_stripe = secs / max(threads, count // 16)
    passes = max(1, int(round(target_s / max(per_stripe * count, 1e-9))))
    total = 0.0
    for _ in range(passes):
        t, _ = O.bench_encode_decode(blocks, n, k, sv, threads, kind)
        total += t
    done = count * passes
    return {"value": round(done * B / total / 2**30, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"{passes} pass(es) over {count} stripes x {B} B (N={n},K={k}): nk8_split_block + "
                      f"XXH64 of every part + nk8_assemble_block from {k} survivors, {threads} pthreads, "
                      f"{total:.1f} s"}


def pcie_rate(batch, blocks_np, S, B, n, k, ids, avail, device, stream):
    """Host-memory path (nkfs_nk8_encode_host): pinned host blocks -> H2D ->
    fused encode+XXH64 -> D2H of parts and digests, sub-batches pipelined
    on two streams.  User GiB/s; DESIGN.md records it (never the headline)."""
    import torch
    host_in = torch.from_numpy(blocks_np).pin_memory()
    ids_h = ids.cpu().pin_memory()
    out = batch.encode_host(host_in, B, n, k, ids_h)  # warm-up: pinned outputs, pooled streams/scratch
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        batch.encode_host(host_in, B, n, k, ids_h, out=out)
    t1 = time.perf_counter()
    return round(S * B * reps / (t1 - t0) / 2**30, 3)


if __name__ == "__main__":
    main()
