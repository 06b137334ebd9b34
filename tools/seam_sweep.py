"""Dispatch-seam sweep: N8K5 encode+XXH64 and decode over
stripe counts x block sizes that straddle the encoder rules in
nk8_kernels.hip (walk_by_rule: parts of 32-128 KiB on grids beyond 2,048
fused waves; nkfs_fast_encode: the warp-specialised kernel for >= 32 KiB
parts on <= 2,048 fused waves or >= 128 KiB parts; nibble tables beyond
1,536 fused waves) -- every point timed with the automatic choice and with
each family pinned (struct nkfs_tune), median of HIP-event timings, GB/s of
algorithmic bytes; outputs of every family compared with the automatic one.

    python tools/seam_sweep.py [--quick]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from nkfs_amd import _lib, batch, synth  # noqa: E402

ENC = {"auto": {}, "walk": {"enc_kernel": 1}, "fused": {"enc_kernel": 2}, "ws": {"enc_kernel": 3},
       "ws2": {"enc_kernel": 3, "enc_ws_hash_waves": 2}}
DEC = {"auto": {}, "slice": {"dec_kernel": 1}, "wave": {"dec_kernel": 2}}
# SWEEP_ENC=auto,walk,ws2 / SWEEP_DEC= (none) / SWEEP_SHAPES=n8 (N8K5 64 KiB-1 MiB only) narrow a run
if os.environ.get("SWEEP_ENC"):
    ENC = {e: ENC[e] for e in os.environ["SWEEP_ENC"].split(",")}
if "SWEEP_DEC" in os.environ:
    DEC = {d: DEC[d] for d in filter(None, os.environ["SWEEP_DEC"].split(","))}


def main():
    quick = "--quick" in sys.argv
    L = _lib.lib()
    _lib.check(L.nkfs_gpu_init(0))
    shapes = [(8, 5, B, S) for B in (65536, 131072, 262144, 524288, 1048576)
              for S in ((256, 1024, 2048, 4096, 8192, 16384) if not quick else (1024, 4096))]
    if os.environ.get("SWEEP_SHAPES") == "mid":  # the warp-specialised / walk seam below 2,048 stripes
        shapes = [(8, 5, B, S) for B in (20480, 65536, 131072, 262144) for S in (256, 384, 512, 768, 1024, 1536)]
    elif os.environ.get("SWEEP_SHAPES") != "n8":
        shapes += [(4, 2, B, S) for B in (4096, 16384, 65536, 262144) for S in (1024, 8192, 65536)]
        shapes += [(8, 5, B, S) for B in (4096, 20480) for S in (1024, 8192, 65536)]
    rounds = int(os.environ.get("SWEEP_ROUNDS", "3"))
    print(f"{'n':>2} {'k':>2} {'S':>6} {'B':>8} {'ps':>7} {'fused_waves':>11} | encode GB/s: " + " ".join(f"{e:>6}" for e in ENC)
          + " | decode GB/s: " + " ".join(f"{d:>6}" for d in DEC), flush=True)
    for n, k, B, S in shapes:
            if S * B > (16 << 30):
                continue
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

            def enc():
                _lib.check(L.nkfs_nk8_encode(blocks.data_ptr(), B, B, S, n, k, ids.data_ptr(), parts.data_ptr(),
                                             pitch, dig.data_ptr(), s))

            def dec():
                _lib.check(L.nkfs_nk8_decode(parts.data_ptr(), pitch, n, ids.data_ptr(), avail.data_ptr(), k, k, B,
                                             out.data_ptr(), B, S, work.data_ptr(), st.data_ptr(), s))

            reps = 5 if S * B <= (4 << 30) else 3
            # variants interleaved over `rounds` passes, median per variant
            # (the first launches after the buffers are allocated run slow)
            er = {e: [] for e in ENC}
            dr = {d: [] for d in DEC}
            ref, ok = None, True
            for _ in range(rounds):
                for name, tune in ENC.items():
                    with _lib.tuned(**tune):
                        er[name].append(enc_b / timeit(enc, reps) / 1e9)
                        torch.cuda.synchronize()
                        got = dig.clone()
                        ref = got if ref is None else ref
                        ok &= bool(torch.equal(got, ref))
                for name, tune in DEC.items():
                    with _lib.tuned(**tune):
                        dr[name].append(dec_b / timeit(dec, reps) / 1e9)
                        torch.cuda.synchronize()
                        ok &= bool(torch.equal(out, blocks[:, :B])) and int(st.abs().sum()) == 0
            if not DEC:
                dr = {"-": [0.0]}
            er = [sorted(v)[len(v) // 2] for v in er.values()]
            dr = [sorted(v)[len(v) // 2] for v in dr.values()]
            print(f"{n:>2} {k:>2} {S:>6} {B:>8} {ps:>7} {(S + 1) // 2:>11} | " + " ".join(f"{x:6.0f}" for x in er) + " |              "
                  + " ".join(f"{x:6.0f}" for x in dr) + f"  ok={ok}", flush=True)
            del blocks, parts, out, dig, work
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
