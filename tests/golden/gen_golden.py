"""Generate tests/golden/nk8_golden.json from the REFERENCE's own code.

Runs in the build container only (needs /root/reference to build
oracle/_ref/libnkfs_ref.so via oracle/ref/Makefile).  Every expected value
below comes out of the reference's crt/nk8.c (nk8_split_block,
nk8_assemble_block) and crt/xxhash.c (XXH64) called through ctypes; inputs
are regenerated from the seeded stripe synthesiser (nkfs_amd/synth.py), so
the fixture holds only ids, digests and -- for small parts -- the part bytes.

    python tests/golden/gen_golden.py          # everything (new random ids)
    python tests/golden/gen_golden.py c1       # one section only
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from nkfs_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nk8_golden.json")
FULL_BYTES_LIMIT = 2048  # store part bytes verbatim when n*ps <= this

# (block_size, n, k): BASELINE configs C2-C5 shapes + edge cases
# (SURVEY.md §8(c) last rows).
ENCODE_CASES = [
    (4096, 4, 2), (65536, 4, 2), (1048576, 4, 2),           # C2 / C5 N4K2
    (4096, 8, 5), (65536, 8, 5), (262144, 8, 5), (1048576, 8, 5),  # C3/C4/C5
    (1, 2, 2), (2, 2, 2), (3, 2, 2), (1, 3, 3), (2, 4, 3), (3, 5, 3), (4, 5, 3),
    (4, 8, 5), (5, 8, 5), (6, 8, 5), (13, 8, 5), (1000, 7, 3), (4095, 4, 2),
    (65537, 8, 5), (3000, 16, 12), (70000, 255, 254), (253, 255, 254),
    (254, 255, 254), (255, 255, 254), (1, 255, 254), (5000, 32, 20),
    (12345, 10, 4), (777, 17, 16), (4096, 255, 2), (100, 2, 2),
]

ERROR_CASES = [  # (block_size, n, k) that the reference rejects with -EINVAL
    (0, 4, 2), (4096, 4, 1), (4096, 1, 1), (4096, 2, 3), (4096, 256, 2), (4096, 255, 255),
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def c1_section() -> dict:
    """Config 1 user-space half: a 1 MiB + ragged object
    moved in 64 KiB chunks (client/main.c:46); each chunk's payload dsum
    (client/lib/client.c:146-148 == core/upages.c:124-148) and the whole-
    cluster sum of the zero-padded 64 KiB block it lands in (core/dio.c:26-37)."""
    obj_size, chunk = (1 << 20) + 12345, 65536
    obj = synth.stripe_bytes(9000, obj_size)
    dsums, clus = [], []
    for off in range(0, obj_size, chunk):
        piece = obj[off:off + chunk]
        dsums.append(f"{O.ref_xxh64(piece):016x}")
        clu = np.zeros(chunk, np.uint8)
        clu[:piece.size] = piece
        clus.append(f"{O.ref_xxh64(clu):016x}")
    return {"stripe": 9000, "object_size": obj_size, "chunk": chunk, "chunk_dsums": dsums,
            "cluster_sums": clus, "object_sha256": sha(obj)}


def main() -> None:
    R = O.ref_lib()
    assert R is not None, "reference library not built"
    rng = np.random.default_rng(0x6E6B3846)
    enc, dec = [], []
    for ci, (B, n, k) in enumerate(ENCODE_CASES):
        stripe = 1000 + ci
        blk = synth.stripe_bytes(stripe, B)
        ids, parts = O.ref_split(blk, n, k)
        ps = parts.shape[1]
        case = {
            "block_size": B, "n": n, "k": k, "stripe": stripe,
            "input_sha256": sha(blk), "ids": ids.tobytes().hex(), "part_size": ps,
            "part_xxh64": [f"{O.ref_xxh64(parts[i]):016x}" for i in range(n)],
            "parts_sha256": sha(parts),
        }
        if n * ps <= FULL_BYTES_LIMIT:
            case["parts_hex"] = [parts[i].tobytes().hex() for i in range(n)]
        enc.append(case)
        # decode: several survivor orders, some with duplicates / extras
        orders = [list(rng.permutation(n)[:k]) for _ in range(3)]
        orders.append(list(range(n)))                       # all parts, first k used
        orders.append([orders[0][0]] + orders[0])           # duplicate id first
        if n > k:
            orders.append(list(rng.permutation(n)[:k - 1]))  # too few -> -EINVAL
        for order in orders:
            order = [int(x) for x in order]
            err, out = O.ref_assemble([parts[i] for i in order], ids[order], k, B)
            d = {"case": ci, "order": order, "err": int(err)}
            if err == 0:
                d["block_sha256"] = sha(out)
                assert d["block_sha256"] == case["input_sha256"], (B, n, k, order)
            dec.append(d)
    errs = []
    for (B, n, k) in ERROR_CASES:
        blk = synth.stripe_bytes(7, max(B, 1))
        try:
            O.ref_split(blk[:B], n, k)
            code = 0
        except OSError as e:
            code = -e.errno
        errs.append({"block_size": B, "n": n, "k": k, "err": code})
    xx = []
    for L in list(range(0, 72)) + [95, 96, 97, 127, 128, 1000, 2048, 4096, 13108, 52429, 65536, 65537, 209716]:
        for seed in (0, 1, 0x9E3779B185EBCA87):
            data = synth.stripe_bytes(5000 + L, L) if L else np.zeros(0, np.uint8)
            xx.append({"len": L, "stripe": 5000 + L, "seed": f"{seed:x}",
                       "digest": f"{O.ref_xxh64(data, seed):016x}"})
    doc = {
        "generator": "tests/golden/gen_golden.py (reference crt/nk8.c + crt/xxhash.c via oracle/_ref)",
        "synth_seed": f"{synth.SEED:x}",
        "encode": enc, "decode": dec, "split_errors": errs, "xxh64": xx, "c1": c1_section(),
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
    print(f"wrote {OUT}: {len(enc)} encode, {len(dec)} decode, {len(errs)} error, {len(xx)} xxh64 cases")


def refresh(sections: list[str]) -> None:
    """Regenerate only the named sections, keeping the rest of the fixture
    (the encode cases hold ids the reference drew at random)."""
    makers = {"c1": c1_section}
    with open(OUT) as f:
        doc = json.load(f)
    for name in sections:
        doc[name] = makers[name]()
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
    print(f"refreshed {sections} in {OUT}")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        refresh(sys.argv[1:])
    else:
        main()
