// xxh64_dev.h -- XXH64 building blocks for CDNA4 kernels.
//
// Same digest as the reference's vendored xxHash (crt/xxhash.c): per 32-byte
// stripe four independent accumulators (:791-810), merge (:849-877), length
// fold (:884), 8/4/1-byte tail (:886-910) and avalanche (:912-916); seed 0
// for csum (crt/csum.c:5).
//
// The four accumulators are the only parallelism XXH64 offers inside one
// message (each round depends on the previous one), so the kernels give
// each accumulator its own lane: lane a of a quad consumes 8-byte words
// a, a+4, a+8, ... of the message.
#pragma once
#include <stdint.h>

namespace nkfs {

constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t XP3 = 0x165667B19E3779F9ull;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ull;

__host__ __device__ inline uint64_t rotl64(uint64_t v, int r) { return (v << r) | (v >> (64 - r)); }

// rotl by 31 as two v_alignbit_b32 on the device (the generic form compiles
// to a 64-bit shift, a shift and an or)
__host__ __device__ inline uint64_t rotl64_31(uint64_t v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
    return (uint64_t(__builtin_amdgcn_alignbit(hi, lo, 1)) << 32) | __builtin_amdgcn_alignbit(lo, hi, 1);
#else
    return rotl64(v, 31);
#endif
}

__host__ __device__ inline uint64_t xxh_round(uint64_t acc, uint64_t w)
{
    return rotl64_31(acc + w * XP2) * XP1;
}

// N rounds over w[0..N) of which the first `valid` count (valid <= 0: none).
// Whole chunks -- every chunk but a message's last -- take the plain chain;
// only a partial chunk pays a compare and two selects per round.
// NKFS_XXH_SELECT=1 forces the select form everywhere (A/B builds).
#ifndef NKFS_XXH_SELECT
#define NKFS_XXH_SELECT 0
#endif
template <int N>
__device__ inline uint64_t xxh_rounds(uint64_t acc, const uint64_t (&w)[N], int valid)
{
    if (!NKFS_XXH_SELECT && valid >= N) {
#pragma unroll
        for (int r = 0; r < N; ++r)
            acc = xxh_round(acc, w[r]);
    } else {
#pragma unroll
        for (int r = 0; r < N; ++r) {
            const uint64_t nx = xxh_round(acc, w[r]);
            acc = r < valid ? nx : acc;
        }
    }
    return acc;
}

// Initial value of accumulator a (0..3) for a seed (xxhash.c:566-577).
__host__ __device__ inline uint64_t xxh_acc_init(int a, uint64_t seed)
{
    return a == 0 ? seed + XP1 + XP2 : a == 1 ? seed + XP2 : a == 2 ? seed : seed - XP1;
}

__host__ __device__ inline uint64_t xxh_merge(uint64_t h, uint64_t v)
{
    return (h ^ xxh_round(0, v)) * XP1 + XP4;
}

__host__ __device__ inline uint64_t xxh_converge(uint64_t v1, uint64_t v2, uint64_t v3, uint64_t v4)
{
    uint64_t h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh_merge(h, v1);
    h = xxh_merge(h, v2);
    h = xxh_merge(h, v3);
    return xxh_merge(h, v4);
}

__host__ __device__ inline uint64_t xxh_avalanche(uint64_t h)
{
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

// Tail bytes (< 32) after the stripes; p is 8-byte aligned (device buffers
// are laid out so).  Ends with the avalanche.
__device__ inline uint64_t xxh_tail(uint64_t h, const uint8_t *p, uint32_t left)
{
    while (left >= 8) {
        uint64_t w = *reinterpret_cast<const uint64_t *>(p);
        h = rotl64(h ^ xxh_round(0, w), 27) * XP1 + XP4;
        p += 8;
        left -= 8;
    }
    if (left >= 4) {
        uint32_t w = *reinterpret_cast<const uint32_t *>(p);
        h = rotl64(h ^ (uint64_t(w) * XP1), 23) * XP2 + XP3;
        p += 4;
        left -= 4;
    }
    while (left--) {
        h = rotl64(h ^ (uint64_t(*p++) * XP5), 11) * XP1;
    }
    return xxh_avalanche(h);
}

// Same as xxh_tail for a tail held in registers (little-endian bytes of
// w[0..3]; `left` < 32 valid bytes).
__device__ inline uint64_t xxh_tail_regs(uint64_t h, const uint64_t w[4], uint32_t left)
{
    int i = 0;
    for (; left >= 8; left -= 8, ++i)
        h = rotl64(h ^ xxh_round(0, w[i]), 27) * XP1 + XP4;
    uint64_t r = i < 4 ? w[i] : 0;
    if (left >= 4) {
        h = rotl64(h ^ (uint64_t(uint32_t(r)) * XP1), 23) * XP2 + XP3;
        r >>= 32;
        left -= 4;
    }
    for (; left; --left, r >>= 8)
        h = rotl64(h ^ (uint64_t(r & 0xFF) * XP5), 11) * XP1;
    return xxh_avalanche(h);
}

}  // namespace nkfs
