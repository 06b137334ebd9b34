"""Does what ran before the encode change its time?  Per-launch encode time
(HIP events on the launch stream) when preceded by (a) another encode, (b) a
decode (bench.py's step order), (c) a 2 GiB memset of an unrelated buffer.

    python tools/order_probe.py c3 [c2 ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402


def main():
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    for name in sys.argv[1:] or ["c3"]:
        S, B, n, k, _ = CONFIGS[name]
        ps = batch.part_size(B, k)
        blocks = batch.synth(S, B)
        ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
        avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
        parts = torch.empty((S * n, batch.part_pitch(B, k)), dtype=torch.uint8, device="cuda")
        dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
        out = torch.empty((S, B), dtype=torch.uint8, device="cuda")
        junk = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
        work = batch.decode_workspace(S, k, "cuda")
        st = torch.empty(S, dtype=torch.int32, device="cuda")
        enc_b = S * (B + n * ps + 8 * n)
        s = torch.cuda.current_stream()

        def enc():
            batch.encode(blocks, B, n, k, ids, parts, dig)

        def dec():
            batch.decode(parts, n, ids, avail, k, B, out=out, work=work, status=st)

        pre = {"after encode": enc, "after decode": dec, "after 2GiB memset": lambda: junk.fill_(1),
               "after decode+sync": dec}
        for _ in range(2):
            for label, fn in pre.items():
                ts = []
                for _ in range(10):
                    fn()
                    if label.endswith("sync"):
                        torch.cuda.synchronize()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    enc()
                    b.record(s)
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b) / 1e3)
                ts.sort()
                print(f"{name} encode {label:20s} median {ts[5]*1e6:8.1f} us  {enc_b/ts[5]/1e9:7.1f} GB/s  "
                      f"(min {ts[0]*1e6:.1f} max {ts[-1]*1e6:.1f})", flush=True)
        del blocks, parts, out, junk
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
