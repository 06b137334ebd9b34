"""Interleaved A/B of kernel choices / launch shapes (struct nkfs_tune) in one
process on the same buffers: encode and decode per config, each variant
timed in turn, several rounds, median GB/s; outputs of every variant are
checked against the first one (parts, digests, decoded blocks).

    python tools/ab_tune.py c2 c3 c4 -- "enc_kernel=2" "enc_kernel=1,enc_waves_per_cu=8" ...
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


def timeit_evicted(fn, reps, scrub):
    """Median seconds of fn with the caches scrubbed before every rep (the
    bench line's condition: each decode follows an encode that evicted its
    inputs from the 256 MB Infinity Cache).  The scrub
    runs outside the events."""
    s = torch.cuda.current_stream()
    for _ in range(2):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        scrub.add_(1)
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] / 1e3


def parse(spec):
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        out[k] = int(v)
    return out


def main():
    argv = sys.argv[1:]
    cut = argv.index("--")
    names, variants = argv[:cut], [parse(v) for v in argv[cut + 1:]]
    skip_dec = bool(os.environ.get("AB_NODEC"))
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    ev_mb = int(os.environ.get("AB_EVICT", "0") or 0)  # scrub this many MB before every timed launch
    scrub = torch.zeros(ev_mb << 18, dtype=torch.int32, device="cuda") if ev_mb else None

    def tm(fn, reps):
        return timeit_evicted(fn, reps, scrub) if scrub is not None else timeit(fn, reps)
    for name in names:
        if name == "c5":
            ragged(L, variants, rounds)
            continue
        if ":" in name:  # S:B:n:k, e.g. 1024:1048576:8:5 (c3s8)
            S, B, n, k = (int(x) for x in name.split(":"))
        else:
            S, B, n, k, _ = CONFIGS[name]
        ps = batch.part_size(B, k)
        pitch = batch.part_pitch(B, k)
        blocks = batch.synth(S, B)
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

        dptr = 0 if os.environ.get("AB_NOHASH") else dig.data_ptr()

        def enc():
            _lib.check(L.nkfs_nk8_encode(blocks.data_ptr(), blocks.stride(0), B, S, n, k, ids.data_ptr(),
                                         parts.data_ptr(), pitch, dptr, s))

        def dec():
            _lib.check(L.nkfs_nk8_decode(parts.data_ptr(), pitch, n, ids.data_ptr(), avail.data_ptr(), k, k, B,
                                         out.data_ptr(), B, S, work.data_ptr(), st.data_ptr(), s))

        ref = None
        res = {}
        skip_enc = bool(os.environ.get("AB_NOENC"))  # decoder A/B: encode once, time decodes only
        if skip_enc:
            enc()
        for r in range(rounds):
            for vi, v in enumerate(variants):
                with _lib.tuned(**v):
                    te = tm(enc, 10) if not skip_enc else 1.0
                    td = tm(dec, 10) if not skip_dec else 1.0
                    if r == 0:
                        torch.cuda.synchronize()
                        got = (parts[:, :ps].clone(), dig.clone())
                        okd = skip_dec or (bool(torch.equal(out, blocks[:, :B])) and int(st.abs().sum()) == 0)
                        if ref is None:
                            ref = got
                        same = torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
                        res.setdefault(vi, {"ok": same and okd})
                    res.setdefault(vi, {"ok": None})
                res[vi].setdefault("e", []).append(enc_b / te / 1e9)
                res[vi].setdefault("d", []).append(dec_b / td / 1e9)
        if os.environ.get("AB_BOX"):  # this box's own stream for the encode's read:write mix (bench.box_stream)
            from bench import box_stream
            bx = box_stream(blocks, parts, B, n * ps, torch.cuda.current_stream())
            print(f"{name} box stream {bx}", flush=True)
        for vi, v in enumerate(variants):
            e, d = sorted(res[vi]["e"]), sorted(res[vi]["d"])
            print(f"{name} {str(v):60s} enc {e[len(e)//2]:7.0f} ({e[0]:.0f}-{e[-1]:.0f})  "
                  f"dec {d[len(d)//2]:7.0f} ({d[0]:.0f}-{d[-1]:.0f})  ok={res[vi]['ok']}", flush=True)
        del blocks, parts, out, ref
        torch.cuda.empty_cache()


def ragged(L, variants, rounds):
    """C5 mix through the ragged entry points (bench.py's layout)."""
    import numpy as np
    from bench import C5_SIZES
    S, _, n, k, _ = CONFIGS["c5"]
    sizes = synth.mixed_sizes(S, C5_SIZES)
    boff = np.zeros(S, np.int64)
    poff = np.zeros(S, np.int64)
    pos = ppos = 0
    for s_, B in enumerate(sizes.tolist()):
        boff[s_], poff[s_] = pos, ppos
        pos += (B + 255) // 256 * 256
        ppos += n * batch.part_pitch(B, k)
    blocks = torch.randint(0, 256, (pos,), dtype=torch.uint8, device="cuda")
    ids = torch.from_numpy(synth.batch_ids(S, n)).cuda()
    avail = torch.from_numpy(synth.batch_survivors(S, n, k)).cuda()
    sz = torch.from_numpy(sizes.astype(np.int32)).cuda()
    bo = torch.from_numpy(boff).cuda()
    po = torch.from_numpy(poff).cuda()
    parts = torch.empty(ppos, dtype=torch.uint8, device="cuda")
    dig = torch.empty(S * n, dtype=torch.int64, device="cuda")
    out = torch.zeros(pos, dtype=torch.uint8, device="cuda")
    work = batch.decode_workspace(S, k, "cuda")
    st = torch.empty(S, dtype=torch.int32, device="cuda")
    maxB = int(sizes.max())
    ps = [batch.part_size(B, k) for B in sizes.tolist()]
    user = int(sizes.sum())
    enc_b = user + n * sum(ps) + 8 * n * S
    dec_b = k * sum(ps) + user + k * S
    enc = lambda: batch.encode_ragged(blocks, bo, sz, n, k, ids, parts, po, dig, maxB)  # noqa: E731
    dec = lambda: batch.decode_ragged(parts, po, n, ids, avail, k, out, bo, sz, maxB, work=work, status=st)  # noqa: E731
    ref = None
    res = {}
    for r in range(rounds):
        for vi, v in enumerate(variants):
            with _lib.tuned(**v):
                te = timeit(enc, 5)
                td = timeit(dec, 5)
                if r == 0:
                    torch.cuda.synchronize()
                    got = (parts.clone(), dig.clone())
                    okd = bool(torch.equal(out, blocks)) and int(st.abs().sum()) == 0
                    if ref is None:
                        ref = got
                    res.setdefault(vi, {"ok": torch.equal(got[1], ref[1]) and okd})
            res[vi].setdefault("e", []).append(enc_b / te / 1e9)
            res[vi].setdefault("d", []).append(dec_b / td / 1e9)
    for vi, v in enumerate(variants):
        e, d = sorted(res[vi]["e"]), sorted(res[vi]["d"])
        print(f"c5 {str(v):60s} enc {e[len(e)//2]:7.0f} ({e[0]:.0f}-{e[-1]:.0f})  "
              f"dec {d[len(d)//2]:7.0f} ({d[0]:.0f}-{d[-1]:.0f})  ok={res[vi]['ok']}", flush=True)


if __name__ == "__main__":
    main()
