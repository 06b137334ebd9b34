"""Interleaved A/B of two builds of libnkfs_crt.so in one process (same
buffers, same box), to separate a code change from box-to-box variance.

    make -C <old checkout>/nkfs_amd/csrc OUTDIR=$PWD/build_ab/old OBJDIR=/tmp/ab_obj
    python tools/ab_lib.py build_ab/old/libnkfs_crt.so [more .so ...] nkfs_amd/lib/libnkfs_crt.so c2 c3 c4
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from kbench import timeit  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402


def load(path):
    L = C.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib._SIGS.items():
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
    _lib.check(L.nkfs_gpu_init(0), path)
    # AB_TUNE="enc_kernel=1,dec_kernel=2": the same struct nkfs_tune fields in every build
    spec = os.environ.get("AB_TUNE", "")
    if spec:
        t = _lib.Tune()
        L.nkfs_tune_get(C.byref(t))
        for kv in spec.split(","):
            key, val = kv.split("=")
            setattr(t, key, int(val))
        _lib.check(L.nkfs_tune_set(C.byref(t)), "nkfs_tune_set")
    return L


def main():
    libs = [(p, load(p)) for p in sys.argv[1:] if p.endswith(".so")]
    batch.gpu_init(0)  # the in-tree build synthesises the inputs
    for name in [a for a in sys.argv[1:] if not a.endswith(".so")]:
        if name in CONFIGS:
            S, B, n, k, _ = CONFIGS[name]
        else:  # S:B:n:k
            S, B, n, k = (int(x) for x in name.split(":"))
        ps = batch.part_size(B, k)
        # layout experiments: AB_PPAD / AB_BPAD bytes added to the part / block pitch
        pitch = batch.part_pitch(B, k) + int(os.environ.get("AB_PPAD", "0"))
        bpitch = B + int(os.environ.get("AB_BPAD", "0"))
        blocks = batch.synth(S, B, pitch=bpitch)
        ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
        avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
        parts = torch.empty((S * n, pitch), dtype=torch.uint8, device="cuda")
        dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
        out = torch.empty((S, B), dtype=torch.uint8, device="cuda")
        work = batch.decode_workspace(S, k, "cuda")
        st = torch.empty(S, dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        enc_b = S * (B + n * ps + 8 * n)
        dec_b = S * (k * ps + B + k)
        res = {}
        for _ in range(5):
            for path, L in libs:
                te = timeit(lambda: L.nkfs_nk8_encode(blocks.data_ptr(), bpitch, B, S, n, k, ids.data_ptr(),
                                                      parts.data_ptr(), pitch, dig.data_ptr(), s), 10)
                td = timeit(lambda: L.nkfs_nk8_decode(parts.data_ptr(), pitch, n, ids.data_ptr(), avail.data_ptr(),
                                                      k, k, B, out.data_ptr(), B, S, work.data_ptr(), st.data_ptr(),
                                                      s), 10)
                res.setdefault(path, []).append((enc_b / te / 1e9, dec_b / td / 1e9))
        torch.cuda.synchronize()
        ok = torch.equal(out, blocks[:, :B])
        # every build's parts and digests against the first build's
        ref = None
        for path, L in libs:
            pp = torch.zeros_like(parts)
            dd = torch.zeros_like(dig)
            _lib.check(L.nkfs_nk8_encode(blocks.data_ptr(), bpitch, B, S, n, k, ids.data_ptr(), pp.data_ptr(), pitch,
                                         dd.data_ptr(), s))
            torch.cuda.synchronize()
            if ref is None:
                ref = (pp[:, :ps], dd)
            elif not (torch.equal(ref[0], pp[:, :ps]) and torch.equal(ref[1], dd)):
                ok = False
                print(f"{name} {path}: parts/digests differ from the first build")
        for path, r in res.items():
            e = sorted(x[0] for x in r)
            d = sorted(x[1] for x in r)
            print(f"{name} {os.path.basename(os.path.dirname(os.path.abspath(path)))}: encode median {e[2]:.0f} "
                  f"({e[0]:.0f}-{e[-1]:.0f})  decode median {d[2]:.0f} ({d[0]:.0f}-{d[-1]:.0f})  ok={ok}")
        del blocks, parts, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
