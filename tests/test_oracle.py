"""The CPU restatement (oracle/) against the reference's golden vectors.

tests/golden/nk8_golden.json was produced by tests/golden/gen_golden.py from
the reference's own crt/nk8.c + crt/xxhash.c (compiled by oracle/ref/).
These tests pin the oracle before any GPU result is compared with it.
"""
import hashlib

import numpy as np
import pytest
import xxhash

from nkfs_amd import synth
from oracle import oracle as O


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_synth_is_stable(golden):
    for case in golden["encode"][:8]:
        blk = synth.stripe_bytes(case["stripe"], case["block_size"])
        assert sha(blk) == case["input_sha256"]
    # batch and per-stripe generators agree
    b = synth.batch_bytes(5, 1001, first=17)
    for s in range(5):
        assert np.array_equal(b[s], synth.stripe_bytes(17 + s, 1001))


def test_encode_matches_reference_vectors(golden):
    for case in golden["encode"]:
        B, n, k = case["block_size"], case["n"], case["k"]
        blk = synth.stripe_bytes(case["stripe"], B)
        assert sha(blk) == case["input_sha256"]
        ids = np.frombuffer(bytes.fromhex(case["ids"]), dtype=np.uint8)
        parts = O.encode(blk, n, k, ids)
        assert parts.shape == (n, case["part_size"])
        assert sha(parts) == case["parts_sha256"], (B, n, k)
        for i in range(n):
            assert f"{O.xxh64(parts[i]):016x}" == case["part_xxh64"][i]
        if "parts_hex" in case:
            assert [p.tobytes().hex() for p in parts] == case["parts_hex"]


def test_decode_matches_reference_vectors(golden):
    enc = golden["encode"]
    for d in golden["decode"]:
        case = enc[d["case"]]
        B, n, k = case["block_size"], case["n"], case["k"]
        blk = synth.stripe_bytes(case["stripe"], B)
        ids = np.frombuffer(bytes.fromhex(case["ids"]), dtype=np.uint8)
        parts = O.encode(blk, n, k, ids)
        order = d["order"]
        try:
            out = O.decode([parts[i] for i in order], ids[order], k, B)
            err = 0
        except OSError as e:
            err = -e.errno
        assert err == d["err"], (B, n, k, order)
        if err == 0:
            assert sha(out) == d["block_sha256"]


def test_param_errors_match_reference(golden):
    for e in golden["split_errors"]:
        blk = synth.stripe_bytes(7, max(e["block_size"], 1))[: e["block_size"]]
        with pytest.raises(OSError) as ei:
            O.encode(blk, e["n"], e["k"], np.arange(1, e["n"] + 1, dtype=np.uint8) if e["n"] <= 255 else
                     np.ones(e["n"], np.uint8))
        assert -ei.value.errno == e["err"]


def test_xxh64_vectors(golden):
    for v in golden["xxh64"]:
        data = synth.stripe_bytes(v["stripe"], v["len"]) if v["len"] else np.zeros(0, np.uint8)
        seed = int(v["seed"], 16)
        want = int(v["digest"], 16)
        assert O.xxh64(data, seed) == want
        assert xxhash.xxh64_intdigest(data.tobytes(), seed) == want  # independent implementation


def test_c1_chunk_and_cluster_sums(golden):
    """Config 1's user-space sums (client chunk dsum, zero-padded cluster sum)
    as computed by the reference, against the oracle and the xxhash module."""
    c1 = golden["c1"]
    obj = synth.stripe_bytes(c1["stripe"], c1["object_size"])
    assert sha(obj) == c1["object_sha256"]
    ch = c1["chunk"]
    for i, off in enumerate(range(0, obj.size, ch)):
        piece = obj[off:off + ch]
        assert f"{O.xxh64(piece):016x}" == c1["chunk_dsums"][i]
        clu = np.zeros(ch, np.uint8)
        clu[:piece.size] = piece
        assert f"{xxhash.xxh64_intdigest(clu.tobytes()):016x}" == c1["cluster_sums"][i]


def test_gf_table_is_the_aes_field():
    t = O.gf_mul_table()
    assert t[0x57, 0x83] == 0xC1  # FIPS-197 4.2 worked example, poly 0x11B
    assert t[0x57, 0x13] == 0xFE
    # 3 generates the multiplicative group, 2 does not (order 51)
    def order(g):
        x, r = g, 1
        while x != 1:
            x, r = int(t[x, g]), r + 1
        return r
    assert order(3) == 255 and order(2) == 51


@pytest.mark.skipif(O.ref_lib() is None, reason="reference tree not available to build oracle/_ref")
def test_restatement_matches_compiled_reference_random():
    rng = np.random.default_rng(11)
    for _ in range(40):
        k = int(rng.integers(2, 40))
        n = int(rng.integers(k, min(255, k + 30) + 1))
        B = int(rng.integers(1, 20000))
        blk = rng.integers(0, 256, B, dtype=np.uint8)
        ids, parts = O.ref_split(blk, n, k)
        assert np.array_equal(O.encode(blk, n, k, ids), parts)
        sel = rng.permutation(n)[:k]
        err, out = O.ref_assemble([parts[i] for i in sel], ids[sel], k, B)
        assert err == 0 and np.array_equal(out, blk)
        assert np.array_equal(O.decode([parts[i] for i in sel], ids[sel], k, B), blk)
