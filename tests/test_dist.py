"""Multi-rank plumbing of bench.py on CPU (gloo, world size 2): weak-scaling
stripe partition, byte-balanced ragged (C5) partition, max-over-ranks timing,
digest all-gather (uneven per-rank counts included) and rank 0's cross-rank
digest check.  The GPU run uses the same functions over RCCL (backend
"nccl") with one process per GPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, w, local = bench.dist_setup("gloo")
    dev = torch.device("cpu")
    first, count = bench.stripe_range(r, 65536)
    strong = bench.strong_range(r, w, 8192)
    t = bench.reduce_max(1.0 + r, dev)
    xs = bench.gather_digest_xor((0xF000_0000_0000_0000 | r), dev)
    # per-part digests of this rank's stripes, as the device would produce
    # them (oracle), all-gathered and checked by rank 0 against regenerated
    # inputs of every rank
    from nkfs_amd import synth
    from oracle import oracle as O
    per, B, n, k = 4, 300, 4, 2
    mine = []
    for s in range(per):
        g = r * per + s
        mine += [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, B), n, k, synth.stripe_ids(g, n))]
    local = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in mine], dtype=torch.int64)

    def expect(rr, s):
        g = rr * per + s
        return [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, B), n, k, synth.stripe_ids(g, n))]

    gathered = bench.gather_digests(local, dev)
    ok = bench.check_rank_digests(gathered, n, expect, samples=per) if r == 0 else None
    bad_local = local.clone()
    if r == 1:  # a wrong digest on rank 1 is caught by rank 0
        bad_local[5] += 1
    bad = bench.gather_digests(bad_local, dev)
    nok = bench.check_rank_digests(bad, n, expect, samples=per) if r == 0 else None
    # C5: byte-balanced ranges of one global ragged batch, uneven stripe
    # counts per rank; each rank's digests of its own range, checked by rank 0
    n5, k5 = 3, 2
    sizes = synth.mixed_sizes(2 * 9, (40, 700, 5000))
    ranges = bench.byte_balanced_ranges(sizes, w)
    lo, hi = ranges[r]
    d5 = []
    for g in range(lo, hi):
        d5 += [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, int(sizes[g])), n5, k5, synth.stripe_ids(g, n5))]
    t5 = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in d5], dtype=torch.int64)

    def expect5(rr, s):
        g = ranges[rr][0] + s
        return [O.xxh64(p) for p in O.encode(synth.stripe_bytes(g, int(sizes[g])), n5, k5, synth.stripe_ids(g, n5))]

    g5 = bench.gather_digests(t5, dev)
    ok5 = bench.check_rank_digests(g5, n5, expect5, samples=100) if r == 0 else None
    counts5 = [len(x) // n5 for x in g5]
    bench.barrier()
    # strong scaling (C3: 8,192 stripes in all): every rank's global stripe
    # indices, all-gathered, must tile [0, 8192) exactly once
    mine_s = torch.arange(strong[0], strong[0] + strong[1], dtype=torch.int64)
    all_s = bench.gather_digests(mine_s, dev)
    tiled = sorted(int(x) for t_ in all_s for x in t_.tolist()) == list(range(8192))
    q.put((r, w, local.numel(), first, count, t, xs, ok, nok, ok5, counts5, ranges, strong, tiled))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for r, (rank, world, nd, first, count, t, xs, ok, nok, ok5, counts5, ranges, strong, tiled) in enumerate(res):
        assert strong == (r * 4096, 4096) and tiled
        assert (rank, world, nd) == (r, 2, 16)
        if r == 0:
            assert ok == 2 and nok == -1 and ok5 == 2
        assert counts5 == [hi - lo for lo, hi in ranges] and ranges[0][0] == 0 and ranges[-1][1] == 18
        assert (first, count) == (r * 65536, 65536)  # disjoint stripe ranges, fixed per-GPU work
        assert t == 2.0                              # max over ranks
        assert xs == [0xF000_0000_0000_0000, 0xF000_0000_0000_0001]


def test_single_rank_defaults(monkeypatch):
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    assert bench.dist_setup("gloo") == (0, 1, 0)
    assert bench.reduce_max(3.5, torch.device("cpu")) == 3.5
    assert bench.gather_digest_xor(7, torch.device("cpu")) == [7]


def test_strong_ranges():
    """C3 strong scaling: the total is split into contiguous,
    disjoint ranges covering it, sizes within one stripe."""
    for total in (8192, 8191, 7, 1):
        for world in (1, 2, 4, 8):
            rs = [bench.strong_range(r, world, total) for r in range(world)]
            assert rs[0][0] == 0 and sum(c for _, c in rs) == total
            assert all(rs[i][0] + rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(c for _, c in rs) - min(c for _, c in rs) <= 1
    assert bench.strong_range(7, 8, 8192) == (7168, 1024)


def test_byte_balanced_ranges():
    """C5 partition: contiguous, disjoint, covering ranges
    whose user bytes differ by at most one stripe's size."""
    from nkfs_amd import synth
    sizes = synth.mixed_sizes(11520 * 4)
    for world in (1, 2, 4, 8):
        ranges = bench.byte_balanced_ranges(sizes, world)
        assert ranges[0][0] == 0 and ranges[-1][1] == len(sizes)
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
        per = [int(sizes[lo:hi].sum()) for lo, hi in ranges]
        assert max(per) - min(per) <= 2 * int(sizes.max())


def _line_worker(rank, world, port, q):
    """One rank of the bench line's bookkeeping at world 2 over gloo: the C3
    strong-scaling workload, this rank's result from stand-in launch times
    (no GPU here: the timings are test inputs, not measurements), the
    per-rank spread collective, rank 0's CPU baseline and the composed line."""
    import argparse
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, w, _ = bench.dist_setup("gloo")
    dev = torch.device("cpu")
    args = argparse.Namespace(no_cpu=False, cpu_seconds=0.02, steps=7, warmup=2)
    first, S, desc = bench.workload("c3", r, w, 0, 8192)
    _, B, n, k, _ = bench.CONFIGS["c3"]
    enc_s, dec_s = 4.4e-3 * S / 8192 * (1 + 0.1 * r), 3.2e-3 * S / 8192
    elapsed = bench.reduce_max(7 * (enc_s + dec_s), dev)
    res = bench.uniform_result("c3", args, r, w, dev, S, B, n, k, desc, 8192, 7, elapsed, enc_s, dec_s, None, None,
                               True, 2 if r == 0 else None, [1, 2])
    line = bench.compose_line(args, r, w, res, {}) if r == 0 else None
    q.put((r, first, S, desc, res["per_rank"], line))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_line_keys():
    """the N > 1 line carries everything the N = 1 line
    does -- roofline (achieved, frac, traffic key), decode roofline, the CPU
    baseline and CPU model on rank 0 at world 2, per-rank encode / decode
    times (max, min) -- and the strong-scaling label states the total split
    over the GPUs, not a per-GPU batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_line_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=150) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (_, f0, s0, d0, pr0, line), (_, f1, s1, d1, pr1, _) = res
    assert (f0, s0, f1, s1) == (0, 4096, 4096, 4096)
    assert "8192 x 1024 KiB stripes in all, split evenly over 2 GPU(s)" in d0 and "per GPU" not in d0
    assert pr0 == pr1 and len(pr0["encode_us"]) == 2
    assert pr0["encode_us_max"] > pr0["encode_us_min"]
    for key in ("metric", "value", "n_gpus", "ms_per_step", "roofline", "decode", "cpu_baseline", "cpu_model",
                "per_rank", "config", "scaling"):
        assert key in line, key
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    roof = line["roofline"]
    assert {"achieved", "peak", "frac", "traffic", "bound", "unit"} <= set(roof)
    assert roof["bytes_per_launch"] == 4096 * (1048576 + 8 * 209716 + 64)
    cb = line["cpu_baseline"]
    assert cb["kind"] in ("reference", "port") and cb["cores"] >= 1 and cb["value"] > 0
    assert line["config"]["stripes_all_gpus"] == 8192
