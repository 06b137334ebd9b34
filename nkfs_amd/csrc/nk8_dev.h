// nk8_dev.h -- device helpers shared by the fused N-K kernels (nk8_fast.hip,
// nk8_ws.hip): packed GF(2^8) product tables, byte transposes, 16-byte
// stores and per-stripe geometry.  Reference arithmetic: crt/nk8.c:54-74
// (GF(2^8)/0x11B products), crt/nk8.c:311-317 (part size).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf256.h"
#include "nkfs_internal.h"

namespace nkfs {
namespace dev {

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;


__device__ inline u32 part_size_of(u32 B, int k) { return B / u32(k) + ((B % u32(k)) ? 1u : 0u); }

// per-byte GF product of two packed words (a_i * b_i for each byte i)
__device__ inline u32 gf_mul_packed(u32 a, u32 b)
{
    u32 r = 0;
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        const u32 mask = ((b >> bit) & 0x01010101u) * 0xFFu;
        r ^= a & mask;
        a = gf_xtime4(a);
    }
    return r;
}

// Fill a 256-entry packed product table T[x] = XOR_{bit b of x} basis[b]
// (multiplication by a constant is GF(2)-linear) with the LP lanes of one
// stripe: lane li owns entries x = li + LP*j, walks j in Gray-code order and
// pays one XOR per entry and word; consecutive lanes write consecutive
// entries, so the LDS stores are conflict-free.
template <int W, int LP>
__device__ inline void build_table(u8 *t, const u32 (&basis)[8][W], int li)
{
    constexpr int LB = LP == 16 ? 4 : LP == 32 ? 5 : 6;
    static_assert(LP == 16 || LP == 32 || LP == 64, "lanes per stripe");
    u32 hv[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
        u32 e = 0;
#pragma unroll
        for (int b = 0; b < LB; ++b)
            e ^= basis[b][w] & (0u - ((u32(li) >> b) & 1u));
        hv[w] = e;
    }
#pragma unroll
    for (int j = 0; j < 256 / LP; ++j) {
        if (j) {
            const int bit = __builtin_ctz(j);
#pragma unroll
            for (int w = 0; w < W; ++w)
                hv[w] ^= basis[LB + bit][w];
        }
        const int x = li + LP * (j ^ (j >> 1));
        if constexpr (W == 2)
            *reinterpret_cast<uint2 *>(t + x * 8) = make_uint2(hv[0], hv[1]);
        else
            *reinterpret_cast<u32 *>(t + x * 4) = hv[0];
    }
}

// Packed 16-byte table T[x] = XOR_{bit b of x} basis[b] for one 64-lane wave
// (lane li owns x = li + 64 j, Gray-code order: one XOR per entry and word).
__device__ inline void build_table16(u8 *t, const u32 (&basis)[8][4], int li)
{
    u32 hv[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        u32 e = 0;
#pragma unroll
        for (int b = 0; b < 6; ++b)
            e ^= basis[b][w] & (0u - ((u32(li) >> b) & 1u));
        hv[w] = e;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j) {
            const int bit = __builtin_ctz(j);
#pragma unroll
            for (int w = 0; w < 4; ++w)
                hv[w] ^= basis[6 + bit][w];
        }
        const int x = li + 64 * (j ^ (j >> 1));
        *reinterpret_cast<uint4 *>(t + x * 16) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
    }
}

// basis[b] = packed coefficient row * 2^b (b = 0..7)
template <int W>
__device__ inline void make_basis(u32 (&basis)[8][W], const u32 (&row)[W])
{
#pragma unroll
    for (int w = 0; w < W; ++w) {
        u32 x = row[w];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            basis[b][w] = x;
            x = gf_xtime4(x);
        }
    }
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// 16-byte store, plain or non-temporal (global_store_dwordx4 ... nt): the
// parts/blocks are written once and not read again by this kernel
__device__ inline void store16(void *p, u32 a, u32 b, u32 c, u32 d, bool nt)
{
    const v4u v = {a, b, c, d};
    if (nt)
        __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(p));
    else
        *reinterpret_cast<v4u *>(p) = v;
}

// Output dword q (bytes 4q..4q+3) of 4 consecutive K-byte rows, each row
// held in W dwords of `row` (row r, byte m at row[r*W + m/4] byte m%4).
// The <= 3 distinct source dwords are merged with one or two v_perm_b32.
template <int K, int W>
__device__ __forceinline__ u32 pack_dword(const u32 *row, int q)
{
    int src[4], byt[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int p = 4 * q + b, r = p / K, m = p % K;
        src[b] = r * W + (m >> 2);
        byt[b] = m & 3;
    }
    // distinct sources in first-use order
    int d0 = src[0], d1 = -1, d2 = -1;
#pragma unroll
    for (int b = 1; b < 4; ++b) {
        if (src[b] != d0 && d1 < 0)
            d1 = src[b];
        else if (src[b] != d0 && src[b] != d1 && d2 < 0)
            d2 = src[b];
    }
    u32 sel = 0;
    if (d1 < 0) {
#pragma unroll
        for (int b = 0; b < 4; ++b)
            sel |= u32(byt[b]) << (8 * b);
        return __builtin_amdgcn_perm(row[d0], row[d0], sel);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b)
        sel |= u32(src[b] == d0 ? byt[b] : 4 + byt[b]) << (8 * b);
    const u32 t = __builtin_amdgcn_perm(row[d1], row[d0], sel);
    if (d2 < 0)
        return t;
    u32 sel2 = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
        sel2 |= u32(src[b] == d2 ? 4 + byt[b] : b) << (8 * b);
    return __builtin_amdgcn_perm(row[d2], t, sel2);
}

// 4x4 byte transpose: in[r] byte c -> out[c] byte r
__device__ inline void transpose4(u32 a, u32 b, u32 c, u32 d, u32 &o0, u32 &o1, u32 &o2, u32 &o3)
{
    // v_perm_b32(S0, S1, sel): selector 0-3 -> S1 bytes, 4-7 -> S0 bytes
    const u32 t0 = __builtin_amdgcn_perm(b, a, 0x05010400u);  // a0 b0 a1 b1
    const u32 t1 = __builtin_amdgcn_perm(b, a, 0x07030602u);  // a2 b2 a3 b3
    const u32 t2 = __builtin_amdgcn_perm(d, c, 0x05010400u);  // c0 d0 c1 d1
    const u32 t3 = __builtin_amdgcn_perm(d, c, 0x07030602u);  // c2 d2 c3 d3
    o0 = __builtin_amdgcn_perm(t2, t0, 0x05040100u);         // a0 b0 c0 d0
    o1 = __builtin_amdgcn_perm(t2, t0, 0x07060302u);         // a1 b1 c1 d1
    o2 = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
    o3 = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
}

__device__ inline u64 shfl64(u64 v, int src)
{
    u32 lo = __shfl(u32(v), src, 64);
    u32 hi = __shfl(u32(v >> 32), src, 64);
    return (u64(hi) << 32) | lo;
}

// Run decoder workspace layout (nk8_walk.hip, k_run_plan / k_decode_run)
__host__ __device__ inline u32 run_plan_stride(int k) { return (u32(k + k * k) + 3u) & ~3u; }
__host__ __device__ inline u64 run_loc_off(u32 nstripes, int k)
{
    return (u64(nstripes) * run_plan_stride(k) + 15u) & ~u64(15);
}
__host__ __device__ inline u64 run_gsum_off(u32 nstripes, int k)
{
    return (run_loc_off(nstripes, k) + u64(nstripes) * 4u + 15u) & ~u64(15);
}


struct Stripe {
    const u8 *blk;
    u8 *parts;
    u64 pitch;
    u32 B;
    u32 ps;
};

__device__ inline Stripe stripe_at(const nkfs_geom &g, u32 s)
{
    Stripe v;
    if (g.block_sizes) {
        v.B = g.block_sizes[s];
        v.blk = g.blocks + g.block_off[s];
        v.parts = g.parts + g.part_off[s];
        v.ps = part_size_of(v.B, g.k);
        v.pitch = (u64(v.ps) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
    } else {
        v.B = g.block_size;
        v.blk = g.blocks + u64(s) * g.block_pitch;
        v.parts = g.parts + u64(s) * u64(g.n) * g.part_pitch;
        v.ps = part_size_of(v.B, g.k);
        v.pitch = g.part_pitch;
    }
    return v;
}

// Stripe behind wave slot `slot` (g.order applied) and whether this launch
// processes it: the slot is in range and the stripe's part size lies in the
// launch's window [part_min, part_max) (0 = unbounded).
__device__ inline bool slot_live(const nkfs_geom &g, u32 slot, u32 &s)
{
    s = slot;
    if (slot >= g.nstripes)
        return false;
    if (g.order)
        s = g.order[slot];
    if (!g.part_min && !g.part_max)
        return true;
    const u32 ps = part_size_of(g.block_sizes ? g.block_sizes[s] : g.block_size, g.k);
    return ps >= g.part_min && (!g.part_max || ps < g.part_max);
}

}  // namespace dev
}  // namespace nkfs
