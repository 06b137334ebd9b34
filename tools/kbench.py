"""Kernel-level timing of the nkfs device entry points (ablation helper).

    python tools/kbench.py [c2 c3 c4 clu ...]

For each config: encode+hash, encode alone (d_digests = NULL), decode, and
the batched XXH64 of the parts, each averaged over per-launch HIP event
pairs on the launch stream.  A config is a bench.py name or S:B:n:k; kernels
are pinned through struct nkfs_tune (KB_TUNE="enc_kernel=4,dec_kernel=3")."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402


def timeit(fn, reps=20):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] / 1e3


def clusters(count=16384, ch=65536, page=4096):
    """Integrity shapes: whole-cluster sums and 4 KiB page-list dsums."""
    d = batch.synth(count, ch)
    t = timeit(lambda: batch.clu_sum(d))
    print(f"clu  sum x{count}   {t*1e6:9.1f} us {count*ch/t/1e9:7.1f} GB/s")
    exp, _ = batch.clu_sum(d)
    t = timeit(lambda: batch.clu_sum(d, expect=exp))
    print(f"clu  check         {t*1e6:9.1f} us {count*(ch+8)/t/1e9:7.1f} GB/s")
    npg = count * ch // page
    g = torch.Generator().manual_seed(1)
    perm = torch.randperm(npg, generator=g).cuda()
    ptrs = d.data_ptr() + perm.to(torch.int64) * page
    first = torch.arange(count, device="cuda", dtype=torch.int64) * (ch // page)
    lens = torch.full((count,), ch, device="cuda", dtype=torch.int64)
    t = timeit(lambda: batch.pages_dsum(ptrs, first, lens, page))
    print(f"pages dsum scat.   {t*1e6:9.1f} us {count*ch/t/1e9:7.1f} GB/s")


def main():
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    spec = os.environ.get("KB_TUNE", "")
    if spec:
        t = _lib.get_tune()
        for kv in spec.split(","):
            key, val = kv.split("=")
            setattr(t, key, int(val))
        _lib.check(L.nkfs_tune_set(_lib.C.byref(t)), "nkfs_tune_set")
    for name in sys.argv[1:] or ["c2", "c4"]:
        if name == "clu":
            clusters()
            continue
        if name == "cluvar":  # wave count vs power-of-two stride
            for count, ch, pitch in ((16384, 65536, 65536), (16384, 65536, 65536 + 256), (65536, 16384, 16384),
                                     (65536, 16384, 16384 + 256), (131072, 8192, 8192), (4096, 262144, 262144)):
                d = torch.empty((count, pitch), dtype=torch.uint8, device="cuda")
                t = timeit(lambda: batch.clu_sum(d, cluster_size=ch))
                print(f"clu {count:6d} x {ch:6d} pitch {pitch:6d} {t*1e6:9.1f} us {count*ch/t/1e9:7.1f} GB/s")
                del d
            continue
        if ":" in name:  # S:B:n:k
            S, B, n, k = (int(x) for x in name.split(":"))
        else:
            S, B, n, k, _ = CONFIGS[name]
        ps = batch.part_size(B, k)
        blocks = batch.synth(S, B)
        ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
        avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
        parts = torch.empty((S * n, batch.part_pitch(B, k)), dtype=torch.uint8, device="cuda")
        dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
        out = torch.empty((S, B), dtype=torch.uint8, device="cuda")
        work = batch.decode_workspace(S, k, "cuda")
        st = torch.empty(S, dtype=torch.int32, device="cuda")
        enc_b = S * (B + n * ps + 8 * n)
        dec_b = S * (k * ps + B + k)
        t = timeit(lambda: batch.encode(blocks, B, n, k, ids, parts, dig))
        print(f"{name} encode+hash {t*1e6:9.1f} us {enc_b/t/1e9:7.1f} GB/s")
        t = timeit(lambda: batch.encode(blocks, B, n, k, ids, parts, False))
        print(f"{name} encode only {t*1e6:9.1f} us {S*(B+n*ps)/t/1e9:7.1f} GB/s")
        t = timeit(lambda: batch.decode(parts, n, ids, avail, k, B, out=out, work=work, status=st))
        print(f"{name} decode      {t*1e6:9.1f} us {dec_b/t/1e9:7.1f} GB/s")
        off = (torch.arange(S * n, device="cuda", dtype=torch.int64) * parts.stride(0))
        lens = torch.full((S * n,), ps, device="cuda", dtype=torch.int64)
        t = timeit(lambda: batch.xxh64_batch(parts, off, lens))
        print(f"{name} xxh64 parts {t*1e6:9.1f} us {S*n*ps/t/1e9:7.1f} GB/s")
        del blocks, parts, out, dig
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
