"""Multi-rank plumbing of bench.py on CPU (gloo, world size 2): weak-scaling
stripe partition, max-over-ranks timing, digest all-gather.  The GPU run uses
the same functions over RCCL (backend "nccl") with one process per GPU."""
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
    gathered = bench.gather_digests(local, dev)
    ok = bench.check_rank_digests(gathered, per, B, n, k, samples=per) if r == 0 else None
    if r == 1:  # a wrong digest on rank 1 is caught by rank 0
        local[5] += 1
    bad = bench.gather_digests(local, dev)
    nok = bench.check_rank_digests(bad, per, B, n, k, samples=per) if r == 0 else None
    bench.barrier()
    q.put((r, w, local.numel(), first, count, t, xs, ok, nok))
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
    for r, (rank, world, nd, first, count, t, xs, ok, nok) in enumerate(res):
        assert (rank, world, nd) == (r, 2, 16)
        if r == 0:
            assert ok == 2 and nok == -1
        assert (first, count) == (r * 65536, 65536)  # disjoint stripe ranges, fixed per-GPU work
        assert t == 2.0                              # max over ranks
        assert xs == [0xF000_0000_0000_0000, 0xF000_0000_0000_0001]


def test_single_rank_defaults(monkeypatch):
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    assert bench.dist_setup("gloo") == (0, 1, 0)
    assert bench.reduce_max(3.5, torch.device("cpu")) == 3.5
    assert bench.gather_digest_xor(7, torch.device("cpu")) == [7]


def test_strong_scaling_partition():
    """--strong-total: a fixed total split evenly, disjoint and covering
    (8,192 x 1 MiB over 1/2/4/8 GPUs); weak by default."""
    assert bench.per_rank_stripes(2048, 0, 8) == 2048
    for world in (1, 2, 4, 8):
        per = bench.per_rank_stripes(2048, 8192, world)
        ranges = [bench.stripe_range(r, per) for r in range(world)]
        covered = [s for first, count in ranges for s in range(first, first + count)]
        assert covered == list(range(8192))
    with pytest.raises(SystemExit):
        bench.per_rank_stripes(2048, 8192, 3)
