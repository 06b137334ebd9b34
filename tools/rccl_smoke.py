"""RCCL (backend "nccl") on the box's one GPU, world size 1: the control
collectives bench.py runs at N > 1 -- barrier on the rank's GPU, MAX
all-reduce, all-gathers of the digest xor, the per-rank spread and padded
digest lists -- executed through bench.py's own helpers on CUDA tensors.
(The 8-GPU run itself is the driver's; this only proves the calls.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    torch.cuda.set_device(0)
    port = int(os.environ.get("NKFS_SMOKE_PORT", "29531"))
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    bench._BARRIER_GPU = 0
    dev = torch.device("cuda", 0)
    bench.barrier()
    assert bench.reduce_max(3.5, dev) == 3.5
    assert bench.gather_digest_xor((1 << 64) - 5, dev) == [(1 << 64) - 5]
    sp = bench.rank_spread(1e-3, 2e-3, dev)
    assert sp["encode_us"] == [1000.0] and sp["decode_us_max"] == 2000.0
    local = torch.arange(40, dtype=torch.int64, device=dev) - 20
    got = bench.gather_digests(local, dev)
    assert len(got) == 1 and torch.equal(got[0], local.cpu())
    bench.barrier()
    dist.destroy_process_group()
    print("rccl smoke ok: barrier(device_ids), all_reduce MAX, all_gather x3 on cuda:0")


if __name__ == "__main__":
    main()
