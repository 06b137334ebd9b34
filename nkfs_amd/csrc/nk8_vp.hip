// nk8_vp.hip -- N-K encode for k > 8 on the vector ALU: GF(2^8) products by
// v_perm_b32 from 2-bit product tables held in scalar registers.
//
// Reference arithmetic: crt/nk8.c:403-420 -- part_i[j] = XOR_m x_i^m
// d[j*k+m], d zero past block_size (:393-398); XXH64 of every part
// (crt/csum.c, crt/xxhash.c:791-916).
//
// The LDS-table encoders (k_encode_bign, k_encode_big) spend one
// random-index ds_read_b128 per (row, column, 16 parts).  The 16 lanes of a
// b128 lane group pick their bank slots at random (~3 passes instead of 1),
// and W2 (N48K32) runs LDS-bound at ~28 CU cycles per row.
//
// Multiplication by a constant c is GF(2)-linear, so
//     c a = T0[a & 3] ^ T1[(a >> 2) & 3] ^ T2[(a >> 4) & 3] ^ T3[a >> 6]
// with four 4-entry tables T_i[j] = c (j << 2i), one dword each.  v_perm_b32
// with both sources T_i and selector bytes (a >> 2i) & 3 looks up four bytes
// at once.  A lane holds one dword per column -- the column's bytes of its 4
// rows -- so a coefficient (part p, column m) costs 4 v_perm + 2 three-input
// XORs per 4 rows: 1.5 VALU instructions per byte product.  The tables are
// uniform: scalar registers (the same SGPR as both sources counts once
// against the constant bus), loaded with s_load from a per-(stripe, part
// group, column) layout that k_vp_tables writes before the encode (16 bytes
// per coefficient, read through the constant address space so the loads are
// scalar).  No LDS tables: the LDS holds only the hash wave's progress
// counters, and the accumulator of part p for a lane's 4 rows is directly
// the dword it stores (no output transpose).
//
// Persistent: one workgroup of 16 waves per CU walks units = (stripe, group
// of 16 parts) b, b + grid, ...; units u, u + 8, u + 16 are one stripe's
// part groups on one XCD (workgroup b runs on XCD b mod 8).  Waves 0..14
// encode slices of 3,840 rows (a lane owns 4 consecutive rows); wave 15
// folds every part's XXH64 from the L2 once all 15 progress counts pass a
// slice (the hash wave of k_encode_bign, nk8_bign.hip).
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include <type_traits>

#include "nk8_dev.h"
#include "nkfs_internal.h"
#include "runtime.h"
#include "scratch.h"
#include "xxh64_dev.h"

using namespace nkfs;
using namespace nkfs::dev;

namespace {

typedef unsigned int v2u __attribute__((ext_vector_type(2)));

constexpr int VP_WAVES = 16, VP_EW = 15, VP_P = 16;
constexpr u32 VP_ROWS = 64u * VP_EW * 4u;     // 3,840 rows (120 XXH64 rounds) per slice
constexpr u64 VP_TAB_BUDGET = 32ull << 20;    // table bytes per launch window

__device__ __forceinline__ u32 vxor3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// unit u -> window stripe (>= the window's count: none) and part group
__device__ __forceinline__ u32 vp_stripe(u32 u, u32 ngroups, u32 &grp)
{
    const u32 loc = u >> 3;
    grp = loc % ngroups;
    return (loc / ngroups) * 8 + (u & 7);
}

// Tables of a window of stripes [s0, s0 + nstr): thread (unit, column m,
// part e of the unit) writes the four 2-bit tables of c = x_{p0+e}^m
// (crt/nk8.c:404-406: the generator row of part p is its id's powers),
// 0 for parts past n.  Layout: ((unit * k + m) * 16 + e) uint4.
__global__ __launch_bounds__(256) void k_vp_tables(nkfs_geom g, const u8 *ids, u32 s0, u32 nstr, u32 ngroups,
                                                   uint4 *tab)
{
    const u64 t = u64(blockIdx.x) * 256u + threadIdx.x;
    const u32 k = u32(g.k);
    const u64 um = t >> 4;
    const u32 e = u32(t & 15u), m = u32(um % k);
    const u64 ul = um / k;
    if (ul >= u64(nstr) * ngroups)
        return;
    const u32 sl = u32(ul / ngroups), grp = u32(ul % ngroups);
    const int p = int(grp) * VP_P + int(e);
    u32 c = 0;
    if (p < g.n) {
        u32 x = ids[u64(s0 + sl) * u64(g.n) + u64(p)];
        c = 1;
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            if ((m >> bit) & 1)
                c = gf_mul_packed(c, x);
            x = gf_mul_packed(x, x);
        }
    }
    u32 b[8];
    b[0] = c;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        b[i] = gf_xtime4(b[i - 1]);
    u32 T[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        T[i] = (b[2 * i] << 8) | (b[2 * i + 1] << 16) | ((b[2 * i] ^ b[2 * i + 1]) << 24);
    tab[t] = make_uint4(T[0], T[1], T[2], T[3]);
}

typedef unsigned int v16u __attribute__((ext_vector_type(16)));

// The tables of 8 coefficients (128 B at base + off): two s_load_dwordx16
// issued by hand, with no wait.  Scalar loads return out of order, so the
// compiler's own schedule waits lgkmcnt(0) one or two coefficients after
// each load (the SMEM latency exposed ~130 times per row quad: 50 % of wave
// time waiting, profiles/r06/sq_vp_summary.txt); here batch b + 1 is in
// flight under batch b's 48 VALU instructions, and vp_wait ties the wait to
// the registers so no use can be scheduled above it.
// base advances by one batch per load through an opaque register update:
// the compiler cannot precompute the 2k batch addresses of a row quad
// (hoisted, they spilled ~180 SGPRs)
__device__ __forceinline__ void vp_next(u64 &base)
{
    base += 128u;
    asm volatile("" : "+s"(base));
}
__device__ __forceinline__ void vp_sload(v16u &a, v16u &b, u64 base)
{
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40" : "=&s"(a), "=&s"(b) : "s"(base));
}
__device__ __forceinline__ void vp_wait(v16u &a, v16u &b)
{
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(a), "+s"(b));
}

// acc[e0 + e] ^= c_e * col for 8 parts: T = their tables (uniform, 4
// dwords each), s = the column's selectors
__device__ __forceinline__ void vp_apply8(u32 *acc, const v16u &ta, const v16u &tb, const u32 (&s)[4])
{
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const u32 t0 = e < 4 ? ta[4 * e] : tb[4 * (e - 4)];
        const u32 t1 = e < 4 ? ta[4 * e + 1] : tb[4 * (e - 4) + 1];
        const u32 t2 = e < 4 ? ta[4 * e + 2] : tb[4 * (e - 4) + 2];
        const u32 t3 = e < 4 ? ta[4 * e + 3] : tb[4 * (e - 4) + 3];
        acc[e] = vxor3(acc[e], __builtin_amdgcn_perm(t0, t0, s[0]), __builtin_amdgcn_perm(t1, t1, s[1]));
        acc[e] = vxor3(acc[e], __builtin_amdgcn_perm(t2, t2, s[2]), __builtin_amdgcn_perm(t3, t3, s[3]));
    }
}

__device__ __forceinline__ void vp_sel(u32 a, u32 (&s)[4])
{
    s[0] = a & 0x03030303u;
    s[1] = (a >> 2) & 0x03030303u;
    s[2] = (a >> 4) & 0x03030303u;
    s[3] = (a >> 6) & 0x03030303u;
}

// KC != 0: k == KC, k % 4 == 0 and the block dword aligned: a lane's 4 rows
// are 4k contiguous bytes in k/4 16-byte loads; KC == 0: any k, per row and
// 16-column chunk a 16 + 4-byte load aligned by v_alignbyte (chunk c + 1's
// loads in flight under chunk c's products)
template <bool HASH, int KC>
__global__ __launch_bounds__(64 * VP_WAVES, 1) void k_encode_vp(nkfs_geom g, u64 tab_addr, u64 *digests, u32 s0,
                                                                 u32 nstr, u32 ngroups, u32 nunits)
{
    __shared__ u32 done[VP_WAVES];  // slices stored so far, per encoder wave
    const int n = g.n, k = KC ? KC : g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nch = (k + 15) >> 4;
    if (tid < VP_WAVES)
        done[tid] = 0;
    __syncthreads();

    if (wave < VP_EW) {
        u32 seq = 0;
#pragma unroll 1
        for (u32 u = blockIdx.x; u < nunits; u += gridDim.x) {
            u32 grp;
            const u32 sw = vp_stripe(u, ngroups, grp);
            if (sw >= nstr)
                continue;  // the whole workgroup
            const Stripe v = stripe_at(g, s0 + sw);
            const int p0 = int(grp) * VP_P, np = min(VP_P, n - p0);
            const u64 ut = tab_addr + (u64(sw) * ngroups + grp) * u64(k) * (VP_P * 16u);
            // the block through a buffer resource based at the dword below
            // it: loads are dword aligned and anything past B reads 0 (the
            // bytes past B inside its last dword are masked in the last slice)
            const u32 mis = u32(reinterpret_cast<uintptr_t>(v.blk) & 3u);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<u8 *>(v.blk - mis), (short)0, int((v.B + mis + 3u) & ~3u), 0x00020000);
            const u32 nsl = (v.ps + VP_ROWS - 1) / VP_ROWS;
            const u32 rl = u32(wave * 64 + lane) * 4u;
            u32 rw[KC ? KC : 1];
            u32 raw[2][4][5];
            auto load_kc = [&](u32 r0) {
                if constexpr (KC != 0) {
#pragma unroll
                    for (int i = 0; i < KC / 4; ++i) {
                        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, r0 * u32(KC) + 16u * u32(i), 0, 0);
                        rw[4 * i] = x.x;
                        rw[4 * i + 1] = x.y;
                        rw[4 * i + 2] = x.z;
                        rw[4 * i + 3] = x.w;
                    }
                }
            };
            auto load_ch = [&](u32 (&x)[4][5], u32 r0, int c) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const u32 a = ((r0 + u32(q)) * u32(k) + 16u * u32(c) + mis) & ~3u;
                    const v4u y = __builtin_amdgcn_raw_buffer_load_b128(rs, a, 0, 0);
                    x[q][0] = y.x;
                    x[q][1] = y.y;
                    x[q][2] = y.z;
                    x[q][3] = y.w;
                    x[q][4] = __builtin_amdgcn_raw_buffer_load_b32(rs, a + 16u, 0, 0);
                }
            };
            if constexpr (KC != 0)
                load_kc(rl);
            else
                load_ch(raw[0], rl, 0);
#pragma unroll 1
            for (u32 sl = 0; sl < nsl; ++sl) {
                const u32 r0 = sl * VP_ROWS + rl;
                const bool last = sl + 1 == nsl;
                u32 acc[VP_P];
#pragma unroll
                for (int e = 0; e < VP_P; ++e)
                    acc[e] = 0;
                // the tables of column 0, parts 0..7 (batches alternate
                // between tc and tn)
                v16u tc0, tc1, tn0, tn1;
                u64 tb = ut;
                vp_sload(tc0, tc1, tb);
                vp_wait(tc0, tc1);
                // one 16-column chunk: d[q][w] = row q's bytes of columns
                // 16c + 4w .. + 3, transposed to one dword per column
                auto chunk = [&](const u32 (&x)[4][5], int c) {
                    u32 d[4][4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const u32 pos = (r0 + u32(q)) * u32(k) + 16u * u32(c);
                        if constexpr (KC != 0) {
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                d[q][w] = 4 * c + w < KC / 4 ? rw[q * (KC / 4) + 4 * c + w] : 0u;
                        } else {
                            const u32 sh = (pos + mis) & 3u;
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                d[q][w] = __builtin_amdgcn_alignbyte(x[q][w + 1], x[q][w], sh);
                        }
                        if (last) {
                            // bytes at or past B are zero (the reference
                            // zero-pads its tail row)
                            const u32 valid = v.B > pos ? min(v.B - pos, 16u) : 0u;
#pragma unroll
                            for (int w = 0; w < 4; ++w) {
                                const u32 keep = valid > u32(4 * w) ? min(valid - u32(4 * w), 4u) : 0u;
                                d[q][w] &= u32((u64(1) << (8 * keep)) - 1u);
                            }
                        }
                    }
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        u32 col[4];
                        transpose4(d[0][w], d[1][w], d[2][w], d[3][w], col[0], col[1], col[2], col[3]);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int m = 16 * c + 4 * w + i;
                            if (m >= k)
                                break;  // uniform
                            u32 sv[4];
                            vp_sel(col[i], sv);
                            // batch 2m: parts 0..7 (in flight), 2m + 1: 8..15
                            vp_next(tb);
                            vp_sload(tn0, tn1, tb);
                            vp_apply8(acc, tc0, tc1, sv);
                            vp_wait(tn0, tn1);
                            if (m + 1 < k)
                                {
                                vp_next(tb);
                                vp_sload(tc0, tc1, tb);
                            }
                            vp_apply8(acc + 8, tn0, tn1, sv);
                            if (m + 1 < k)
                                vp_wait(tc0, tc1);
                        }
                    }
                };
                if constexpr (KC != 0) {
#pragma unroll
                    for (int c = 0; c < (KC + 15) / 16; ++c)
                        chunk(raw[0], c);
                } else {
                    // chunks in pairs: chunk c + 1's loads in flight under
                    // chunk c's products (static buffer indices: no scratch)
#pragma unroll 1
                    for (int c = 0; c < nch; c += 2) {
                        if (c + 1 < nch)
                            load_ch(raw[1], r0, c + 1);
                        chunk(raw[0], c);
                        if (c + 1 < nch) {
                            if (c + 2 < nch)
                                load_ch(raw[0], r0, c + 2);
                            chunk(raw[1], c + 1);
                        }
                    }
                }
                if (r0 < v.ps) {
#pragma unroll
                    for (int e = 0; e < VP_P; ++e) {
                        if (e >= np)
                            break;
                        u8 *dst = v.parts + u64(p0 + e) * v.pitch + r0;
                        if (r0 + 4u <= v.ps) {
                            *reinterpret_cast<u32 *>(dst) = acc[e];
                        } else {
                            for (u32 cb = 0; cb < 4 && r0 + cb < v.ps; ++cb)
                                dst[cb] = u8(acc[e] >> (8 * cb));
                        }
                    }
                }
                // the next slice's loads after the stores; the progress count
                // waits for the stores only (the loads stay in flight)
                if constexpr (HASH) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (!last) {
                        if constexpr (KC != 0) {
                            load_kc(r0 + VP_ROWS);
                            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KC / 4) : "memory");
                        } else {
                            load_ch(raw[0], r0 + VP_ROWS, 0);
                            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                        }
                    } else {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    ++seq;
                    if (lane == 0)
                        __hip_atomic_store(&done[wave], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else if (!last) {
                    if constexpr (KC != 0)
                        load_kc(r0 + VP_ROWS);
                    else
                        load_ch(raw[0], r0 + VP_ROWS, 0);
                }
            }
        }
    } else if constexpr (HASH) {
        // lane 4e + a: XXH64 accumulator a of part p0 + e
        const int e = lane >> 2, a = lane & 3;
        u32 seq = 0;
#pragma unroll 1
        for (u32 u = blockIdx.x; u < nunits; u += gridDim.x) {
            u32 grp;
            const u32 sw = vp_stripe(u, ngroups, grp);
            if (sw >= nstr)
                continue;
            const u32 s = s0 + sw;
            const Stripe v = stripe_at(g, s);
            const int p0 = int(grp) * VP_P, np = min(VP_P, n - p0);
            const u32 nsl = (v.ps + VP_ROWS - 1) / VP_ROWS;
            const u32 nst = v.ps >> 5;  // whole 32-byte stripes of every part
            // the group's parts through one buffer resource (the launcher
            // checks n * pitch < 2^31); loads bypass the CU's L1 (sc0)
            const __amdgpu_buffer_rsrc_t pr =
                __builtin_amdgcn_make_buffer_rsrc(v.parts, (short)0, int(u64(n) * v.pitch), 0x00020000);
            const u32 pbase = u32(u64(p0 + min(e, np - 1)) * v.pitch);
            u64 hacc = xxh_acc_init(a, 0);
#pragma unroll 1
            for (u32 sl = 0; sl < nsl; ++sl) {
                ++seq;
                for (;;) {
                    const u32 dv = lane < VP_EW ? __hip_atomic_load(&done[lane], __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP)
                                                : 0xFFFFFFFFu;
                    if (!__ballot(dv < seq))
                        break;
                    __builtin_amdgcn_s_sleep(8);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const u32 rb = sl * (VP_ROWS / 32u);
                const int re = int(min(rb + VP_ROWS / 32u, nst));
                // a ring of 4 x 8 rounds: three batches' loads in flight
                // while one is folded; loads past the slice's rounds re-read
                // its last round (rows of the next slice are not stored yet)
                const u32 rlast = re > int(rb) ? u32(re) - 1u : rb;
                auto ld = [&](uint64_t (&w)[8], u32 r) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const u32 ri = min(r + u32(i), rlast);
                        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(pr, pbase + 32u * ri + 8u * u32(a), 0, 1);
                        w[i] = (u64(x.y) << 32) | x.x;
                    }
                };
                uint64_t w0[8], w1[8], w2[8], w3[8];
                ld(w0, rb);
                ld(w1, rb + 8);
                ld(w2, rb + 16);
#pragma unroll 1
                for (int r = int(rb); r < re; r += 32) {
                    ld(w3, u32(r) + 24);
                    hacc = xxh_rounds<8>(hacc, w0, re - r);
                    ld(w0, u32(r) + 32);
                    hacc = xxh_rounds<8>(hacc, w1, re - r - 8);
                    ld(w1, u32(r) + 40);
                    hacc = xxh_rounds<8>(hacc, w2, re - r - 16);
                    ld(w2, u32(r) + 48);
                    hacc = xxh_rounds<8>(hacc, w3, re - r - 24);
                }
            }
            // every slice is stored: the tail (ps & 31 bytes after the last
            // whole stripe), converge, length, avalanche
            uint64_t tw[4] = {0, 0, 0, 0};
            if (v.ps & 31) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const v2u x = __builtin_amdgcn_raw_buffer_load_b64(pr, pbase + 32u * nst + 8u * u32(i), 0, 1);
                    tw[i] = (u64(x.y) << 32) | x.x;
                }
            }
            const int base = lane & ~3;
            const u64 v1 = shfl64(hacc, base), v2 = shfl64(hacc, base + 1);
            const u64 v3 = shfl64(hacc, base + 2), v4 = shfl64(hacc, base + 3);
            if (a == 0 && e < np) {
                u64 h = v.ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
                h += v.ps;
                digests[u64(s) * u64(n) + u64(p0 + e)] = xxh_tail_regs(h, tw, v.ps & 31);
            }
        }
    }
}

}  // namespace

// Encode a uniform or ragged batch (2 <= k <= 254) on k_encode_vp, XXH64 of
// every part into digests when non-null.  Stripes go in windows whose
// coefficient tables fit VP_TAB_BUDGET (k_vp_tables, then the encode, in
// stream order).  -ENOSYS when the shape is outside what it handles or no
// table scratch is to be had (the caller takes another encoder).
extern "C" int nkfs_vp_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, hipStream_t st)
{
    const int k = g->k, n = g->n;
    if (k < 2 || k > 254 || n < k || n > 255 || g->part_min || g->part_max || g->order)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    // 4-byte aligned parts and pitch (dword stores); block offsets (rows +
    // one slice) and a stripe's part span inside 31 bits
    const u64 ps_max = (u64(g->block_size) + u64(k) - 1) / u64(k);  // ragged: block_size = the largest
    const u64 pitch_max = g->block_sizes ? (ps_max + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1) : g->part_pitch;
    if (((reinterpret_cast<uintptr_t>(g->parts) | (g->block_sizes ? 0 : g->part_pitch)) & 3) ||
        (ps_max + VP_ROWS) * u64(k) + 64 > 0x7FFFFFFFull || u64(n) * pitch_max > 0x7FFFFFFFull)
        return -ENOSYS;
    const u32 ngroups = u32((n + VP_P - 1) / VP_P);
    const u64 per_stripe = u64(ngroups) * u64(k) * VP_P * 16u;
    // a window: a multiple of 8 stripes whose tables fit the budget
    u64 win = VP_TAB_BUDGET / per_stripe / 8 * 8;
    if (!win)
        win = 8;
    if (win > g->nstripes)
        win = (u64(g->nstripes) + 7) / 8 * 8;
    Scratch sc;
    uint4 *tab = static_cast<uint4 *>(sc.take(g, win * per_stripe, st));
    if (!tab)
        return -ENOSYS;
    const u64 cus = u64(nkfs_cu_count()) / 8 * 8;
    // k % 4 == 0 with dword-aligned blocks (uniform batches): a lane's 4
    // rows in k/4 contiguous 16-byte loads (k-specialised kernels)
    const bool kc = !g->block_sizes && ((reinterpret_cast<uintptr_t>(g->blocks) | g->block_pitch) & 3) == 0;
    const int kk = kc && (k == 20 || k == 24 || k == 28 || k == 32) ? k : 0;
    int rc = 0;
    for (u64 s0 = 0; s0 < g->nstripes && !rc; s0 += win) {
        const u32 nstr = u32(std::min<u64>(win, g->nstripes - s0));
        const u64 nunits = (u64(nstr) + 7) / 8 * 8 * ngroups;
        const u64 threads = u64(nstr) * ngroups * u64(k) * VP_P;
        hipLaunchKernelGGL(k_vp_tables, dim3(u32((threads + 255) / 256)), dim3(256), 0, st, *g, ids, u32(s0), nstr,
                           ngroups, tab);
        const u32 grid = u32(nunits < cus || !cus ? nunits : cus);
        auto go = [&](auto hash, auto kcon) {
            hipLaunchKernelGGL((k_encode_vp<decltype(hash)::value, decltype(kcon)::value>), dim3(grid),
                               dim3(64 * VP_WAVES), 0, st, *g, u64(reinterpret_cast<uintptr_t>(tab)), digests,
                               u32(s0), nstr, ngroups, u32(nunits));
        };
        auto pick = [&](auto hash) {
            switch (kk) {
            case 20: go(hash, std::integral_constant<int, 20>{}); break;
            case 24: go(hash, std::integral_constant<int, 24>{}); break;
            case 28: go(hash, std::integral_constant<int, 28>{}); break;
            case 32: go(hash, std::integral_constant<int, 32>{}); break;
            default: go(hash, std::integral_constant<int, 0>{});
            }
        };
        if (digests)
            pick(std::true_type{});
        else
            pick(std::false_type{});
        rc = hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    const int e = sc.finish();
    return rc ? rc : e;
}
