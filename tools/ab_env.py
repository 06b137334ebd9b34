"""Interleaved A/B of library env knobs in one process (same buffers, same
box): encode and decode GB/s per setting, median of 5 interleaved rounds.

    python tools/ab_env.py NKFS_ENC_G=4,2,1 c2 c3 c4

Every setting's encode output is checked against the first setting's
(parts and digests equal), so a knob cannot win by computing less."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from kbench import timeit  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402


def main():
    knobs = [a for a in sys.argv[1:] if "=" in a]
    cfgs = [a for a in sys.argv[1:] if "=" not in a] or ["c2"]
    settings = [[]]
    for kv in knobs:
        name, vals = kv.split("=", 1)
        settings = [s + [(name, v)] for s in settings for v in vals.split(",")]
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    for name in cfgs:
        if name in CONFIGS:
            S, B, n, k, _ = CONFIGS[name]
        else:  # uniform shape "S:B:n:k", e.g. 3840:1048576:8:5
            S, B, n, k = (int(x) for x in name.split(":"))
        ps = batch.part_size(B, k)
        blocks = batch.synth(S, B)
        ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
        avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
        pitch = batch.part_pitch(B, k)
        parts = torch.empty((S * n, pitch), dtype=torch.uint8, device="cuda")
        dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
        out = torch.empty((S, B), dtype=torch.uint8, device="cuda")
        work = batch.decode_workspace(S, k, "cuda")
        st = torch.empty(S, dtype=torch.int32, device="cuda")
        enc_b = S * (B + n * ps + 8 * n)
        dec_b = S * (k * ps + B + k)
        res = {}
        ref = None
        for rnd in range(5):
            for setting in settings:
                for kk, vv in setting:
                    os.environ[kk] = vv
                te = timeit(lambda: batch.encode(blocks, B, n, k, ids, parts, dig), 10)
                td = timeit(lambda: batch.decode(parts, n, ids, avail, k, B, out=out, work=work, status=st), 10)
                if rnd == 0:
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = (parts[:, :ps].clone(), dig.clone())
                    elif not (torch.equal(ref[0], parts[:, :ps]) and torch.equal(ref[1], dig)):
                        print(f"{name} {setting}: OUTPUT DIFFERS")
                res.setdefault(str(setting), []).append((enc_b / te / 1e9, dec_b / td / 1e9))
                for kk, _ in setting:
                    del os.environ[kk]
        torch.cuda.synchronize()
        ok = torch.equal(out, blocks[:, :B])
        for key, r in res.items():
            e = sorted(x[0] for x in r)
            d = sorted(x[1] for x in r)
            print(f"{name} {key}: encode median {e[2]:.0f} ({e[0]:.0f}-{e[-1]:.0f})  "
                  f"decode median {d[2]:.0f} ({d[0]:.0f}-{d[-1]:.0f})  ok={ok}", flush=True)
        del blocks, parts, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
