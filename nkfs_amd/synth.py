"""Synthetic workload definition shared by tests, smoke() and bench.py.

Counter-based splitmix64 (SURVEY.md §8(d) "Inputs"): every byte of every
stripe is a pure function of (seed, stripe index, word index), so the host
(numpy, here) and the device generator (k_synth in
nkfs_amd/csrc/nk8_kernels.hip) produce identical batches without moving
data over PCIe.

    word(seed, s, w) = mix64(seed + GAMMA * ((s << 32) + w + 1))   (mod 2**64)

Stripe s is the little-endian byte image of words 0, 1, ... cut to B bytes.
Part ids follow the reference rule (crt/nk8.c:319-342 with
crt/random.c:15-33): draw v = low byte of the id stream, reject v >= 255,
id = 1 + v, redraw duplicates.  The id stream is the same construction in a
separate domain (seed ^ IDS_DOMAIN).
"""
from __future__ import annotations

import numpy as np

SEED = 0x6E6B3846
GAMMA = 0x9E3779B97F4A7C15
IDS_DOMAIN = 0xA5A5_5A5A_C3C3_3C3C
ERASE_DOMAIN = 0x0F0F_F0F0_1234_4321
SIZE_DOMAIN = 0x5151_1515_7777_0001
M64 = (1 << 64) - 1


def mix64(z):
    """splitmix64 finalizer, vectorised over uint64 arrays (wrapping)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def _stream(seed: int, stripe: int, count: int, first: int = 0) -> np.ndarray:
    ctr = (np.uint64(stripe) << np.uint64(32)) + np.arange(first + 1, first + 1 + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(np.uint64(seed & M64) + np.uint64(GAMMA) * ctr)


def stripe_bytes(stripe: int, block_size: int, seed: int = SEED) -> np.ndarray:
    words = _stream(seed, stripe, (block_size + 7) // 8)
    return words.view(np.uint8)[:block_size].copy()


def batch_bytes(nstripes: int, block_size: int, seed: int = SEED, first: int = 0) -> np.ndarray:
    """[nstripes, block_size] uint8, stripe index offset by `first`."""
    nw = (block_size + 7) // 8
    s = np.arange(first, first + nstripes, dtype=np.uint64)[:, None]
    w = np.arange(1, nw + 1, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        words = mix64(np.uint64(seed & M64) + np.uint64(GAMMA) * ((s << np.uint64(32)) + w))
    return np.ascontiguousarray(words.view(np.uint8)[:, :block_size])


def stripe_ids(stripe: int, n: int, seed: int = SEED) -> np.ndarray:
    """n distinct ids in 1..255 by the reference's rejection rule."""
    ids: list[int] = []
    seen: set[int] = set()
    pos = 0
    while len(ids) < n:
        for v in _stream(seed ^ IDS_DOMAIN, stripe, 256, pos).tolist():
            pos += 1
            v &= 0xFF
            if v >= 255:
                continue
            cand = 1 + v
            if cand not in seen:
                seen.add(cand)
                ids.append(cand)
                if len(ids) == n:
                    break
    return np.array(ids, dtype=np.uint8)


def batch_ids(nstripes: int, n: int, seed: int = SEED, first: int = 0) -> np.ndarray:
    return np.stack([stripe_ids(first + s, n, seed) for s in range(nstripes)]) if nstripes else np.zeros((0, n), np.uint8)


def survivors(stripe: int, n: int, keep: int, seed: int = SEED) -> np.ndarray:
    """`keep` distinct part slots (of n) in a seeded random order: the parts
    left after erasing n-keep (Fisher-Yates on the erase stream)."""
    perm = list(range(n))
    draws = _stream(seed ^ ERASE_DOMAIN, stripe, n)
    for i in range(n - 1, 0, -1):
        j = int(draws[i]) % (i + 1)
        perm[i], perm[j] = perm[j], perm[i]
    return np.array(perm[:keep], dtype=np.uint8)


def batch_survivors(nstripes: int, n: int, keep: int, seed: int = SEED, first: int = 0) -> np.ndarray:
    if not nstripes:
        return np.zeros((0, keep), np.uint8)
    return np.stack([survivors(first + s, n, keep, seed) for s in range(nstripes)])


def mixed_sizes(nstripes: int, choices=(4096, 65536, 1048576), seed: int = SEED) -> np.ndarray:
    """Stripe sizes drawn uniformly from `choices`,
    from a size stream separate from the data stream."""
    draws = _stream(seed ^ SIZE_DOMAIN, 0, nstripes)
    return np.array([choices[int(d) % len(choices)] for d in draws], dtype=np.uint32)
