"""Run one config's encode (and optionally decode) a few times with chosen
struct nkfs_tune fields -- a short, single-purpose process for PMC passes.

    python tools/enc_probe.py c3 enc_kernel=1 [nohash] [dec] [reps=5]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402


def main():
    name = sys.argv[1]
    kv = dict(a.split("=") for a in sys.argv[2:] if "=" in a)
    reps = int(kv.pop("reps", 5))
    flags = {a for a in sys.argv[2:] if "=" not in a}
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    S, B, n, k, _ = CONFIGS[name]
    S = int(kv.pop("stripes", S))
    blocks = batch.synth(S, B)
    ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
    parts = torch.empty((S * n, batch.part_pitch(B, k)), dtype=torch.uint8, device="cuda")
    dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
    ps = batch.part_size(B, k)
    with _lib.tuned(**{a: int(b) for a, b in kv.items()}):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for i in range(reps):
            if i == 1:
                ev[0].record()
            batch.encode(blocks, B, n, k, ids, parts, False if "nohash" in flags else dig)
        ev[1].record()
        torch.cuda.synchronize()
        if reps > 1:
            t = ev[0].elapsed_time(ev[1]) / 1e3 / (reps - 1)
            print(f"{name} S={S} {kv} {sorted(flags)} encode {S * (B + n * ps + 8 * n) / t / 1e9:.0f} GB/s", flush=True)
        if "dec" in flags:
            avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
            out = torch.empty((S, B), dtype=torch.uint8, device="cuda")
            for _ in range(reps):
                batch.decode(parts, n, ids, avail, k, B, out=out)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
