// nk8_ws.hip -- warp-specialised fused encode + XXH64 for n <= 8, k <= 8.
//
// Reference: crt/nk8.c:403-420 (part_i[j] = XOR_m ids[i]^m * d[j*k+m]) and
// crt/xxhash.c:358-496 (XXH64, seed 0 as crt/csum.c:5), per part.
//
// XXH64 of one part is a serial chain per accumulator, so a batch has exactly
// 4 * n chains per stripe and a hash wave is only fully used when it owns
// 64 of them: S = 16 / E stripes (E = 4 packed bytes for n <= 4, 8 for
// n <= 8).  k_encode_fast puts those S stripes in ONE wave that both encodes
// and hashes; its HBM accesses are then S short segments per instruction
// and one wave streams S whole stripes, which leaves big stripes (few waves
// in the grid) latency-bound.  Here a workgroup = NE encoder waves + 1 hash
// wave over the same S stripes:
//   * encoder wave e works on stripe e % S, rows sub*1024 .. of every chunk
//     (sub = e / S, NE / S waves per stripe): 64 lanes x 16 rows, so every
//     global load and store instruction covers one contiguous 1 KiB run of
//     one stripe or part;
//   * encoded parts go to HBM and to a double-buffered LDS exchange;
//   * the hash wave (lane = stripe, part, accumulator) folds chunk c-1 from
//     LDS while the encoders produce chunk c; one barrier per chunk.
// HW = 2 hash waves own S = 2 * 16 / E stripes (n > 4: four stripes of 1,024
// rows per chunk instead of two of 2,048).  One XXH64 round is ~35 ns of
// dependent 64-bit multiplies, so a hash wave folds at most ~14.5 GB/s:
// with one per CU that is ~3.7 TB/s of parts, i.e. a ~6 TB/s ceiling on the
// N8K5 encode (61 % of its bytes are hashed) that a fast box's HBM reaches
// (tools/xxh_rate.hip).
// Packed product tables T_m[x] = (ids_0^m * x, ..., ids_{n-1}^m * x),
// m = 1..k-1, are built per stripe in LDS exactly as in k_encode_fast.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>

#include "nk8_dev.h"
#include "nkfs_internal.h"
#include "xxh64_dev.h"

using namespace nkfs;
using namespace nkfs::dev;

// SB: single-buffered exchange (the hash wave copies its words to registers
// between two barriers per chunk) -- half the LDS, so more workgroups per CU
// NKFS_WS_HPRIO (experiment builds): the hash waves' s_setprio level
#ifndef NKFS_WS_HPRIO
#define NKFS_WS_HPRIO 0
#endif
template <int K, int E, int NE, bool SB, int PF, int HW>
__global__ __launch_bounds__(64 * (NE + HW)) void k_encode_ws(nkfs_geom g, const u8 *ids, u64 *digests, bool nt)
{
    constexpr int SPH = 16 / E;     // stripes per hash wave: 4 accumulators x E parts x SPH = 64 chains
    constexpr int S = HW * SPH;     // stripes per workgroup
    constexpr int WPS = NE / S;     // encoder waves per stripe
    static_assert(NE % S == 0 && WPS >= 1, "encoder waves per stripe");
    constexpr int CR = WPS * 1024;  // rows per stripe per chunk
    constexpr int SP = CR + 32;     // exchange bytes per part (+32: hash reads spread over all banks, tail room)
    constexpr int TB = 256 * E;     // bytes per packed table
    constexpr int W = E / 4;        // dwords per packed entry
    constexpr int RPC = CR / 32;    // XXH64 rounds per chain per chunk
    __shared__ __attribute__((aligned(16))) u8 tbl[S * (K - 1) * TB];
    __shared__ __attribute__((aligned(16))) u8 xbuf[SB ? 1 : 2][S * E * SP];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool hasher = wave >= NE;
    const int n = g.n;

    // chunks the workgroup iterates: the largest of its stripes' (ragged)
    u32 nch = 0;
    bool any = false;
#pragma unroll
    for (int j = 0; j < S; ++j) {
        u32 sj;
        if (slot_live(g, blockIdx.x * S + j, sj)) {
            const u32 psj = part_size_of(g.block_sizes ? g.block_sizes[sj] : g.block_size, K);
            nch = max(nch, (psj + CR - 1) / CR);
            any = true;
        }
    }
    if (!any)
        return;  // the same for every wave of the workgroup: its stripes belong to another launch

    if (!hasher) {
        // ------------------------------------------------------ encoder wave
        const int gs = wave % S, sub = wave / S;
        u32 s;
        const bool live = slot_live(g, blockIdx.x * S + gs, s);
        Stripe v{};
        if (live)
            v = stripe_at(g, s);
        const bool aligned =
            ((reinterpret_cast<uintptr_t>(v.blk) | reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 15) == 0;
        // PF register sets of chunk loads rotate: chunk c encodes from set
        // c % PF and, once encoded, that set takes the loads of chunk c + PF,
        // so with PF = 2 the next chunk's loads are in flight through this
        // chunk's lookups as well as its stores (PF = 1: only its stores)
        u32 d[PF][4 * K];
        auto load_task = [&](u32 (&x)[4 * K], u32 r0) {
            const u64 off = u64(r0) * K;
            if (aligned && off + 16 * K <= v.B) {
                const uint4 *src = reinterpret_cast<const uint4 *>(v.blk + off);
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    const uint4 t = src[q];
                    x[4 * q] = t.x;
                    x[4 * q + 1] = t.y;
                    x[4 * q + 2] = t.z;
                    x[4 * q + 3] = t.w;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4 * K; ++q) {
                    u32 y = 0;
                    for (int b = 0; b < 4; ++b) {
                        const u64 p = off + 4 * q + b;
                        if (p < v.B)
                            y |= u32(v.blk[p]) << (8 * b);
                    }
                    x[q] = y;
                }
            }
        };
        const u32 rbase = sub * 1024 + 16 * lane;  // this lane's first row in every chunk
        // first chunks requested before the table build
#pragma unroll
        for (int p = 0; p < PF; ++p)
            if (live && rbase + u32(p) * CR < v.ps)
                load_task(d[p], rbase + u32(p) * CR);

        // tables of stripe gs, split over its WPS encoder waves
        u32 coef[W], idw[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            u32 x = 0;
            if (live)
                for (int b = 0; b < 4; ++b)
                    if (4 * w + b < n)
                        x |= u32(ids[u64(s) * n + 4 * w + b]) << (8 * b);
            idw[w] = x;
            coef[w] = x;
        }
        u8 *mytbl = tbl + gs * (K - 1) * TB;
#pragma unroll
        for (int m = 1; m < K; ++m) {
            if ((m - 1) % WPS == sub) {
                u32 basis[8][W];
                make_basis<W>(basis, coef);
                build_table<W, 64>(mytbl + (m - 1) * TB, basis, lane);
            }
#pragma unroll
            for (int w = 0; w < W; ++w)
                coef[w] = gf_mul_packed(coef[w], idw[w]);
        }
        __syncthreads();

        auto chunk = [&](u32 (&x)[4 * K], u32 c) {
            const u32 r0 = c * CR + rbase;
            if (live && r0 < v.ps) {
                // 16 rows in four groups of 4: lookups + XOR, then the group's
                // 4 x E bytes are transposed into 4 bytes of each part
                u32 out[E][4];
                u32 tdep = 0;  // 0 at run time; chains each group's lookups behind the previous group
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    u32 row[4][W];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int p0 = (4 * q + rr) * K;
                        const u32 rep = __builtin_amdgcn_perm(0u, x[p0 >> 2], 0x01010101u * u32(p0 & 3));
#pragma unroll
                        for (int w = 0; w < W; ++w)
                            row[rr][w] = rep;
#pragma unroll
                        for (int m = 1; m < K; ++m) {
                            const int p = p0 + m;
                            const u32 byte = (x[p >> 2] >> (8 * (p & 3))) & 0xFFu;
                            const u8 *e = mytbl + tdep + (m - 1) * TB + byte * E;
                            if constexpr (E == 8) {
                                const uint2 t = *reinterpret_cast<const uint2 *>(e);
                                row[rr][0] ^= t.x;
                                row[rr][1] ^= t.y;
                            } else {
                                row[rr][0] ^= *reinterpret_cast<const u32 *>(e);
                            }
                        }
                    }
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        transpose4(row[0][w], row[1][w], row[2][w], row[3][w], out[4 * w][q], out[4 * w + 1][q],
                                   out[4 * w + 2][q], out[4 * w + 3][q]);
                    // the next group's lookup addresses depend (opaquely) on this
                    // group's result, so they are not all hoisted up front: that
                    // would hold 16 x (K-1) x W lookup results in VGPRs at once
                    if constexpr (K * W > 8)
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(out[0][q]));
                }
                if (r0 + PF * CR < v.ps)
                    load_task(x, r0 + PF * CR);  // chunk c + PF's rows, in flight under what follows
                u8 *xb = xbuf[SB ? 0 : (c & 1)] + gs * E * SP + sub * 1024 + 16 * lane;
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    if (i < n) {
                        u8 *dst = v.parts + u64(i) * v.pitch + r0;
                        if (aligned) {
                            store16(dst, out[i][0], out[i][1], out[i][2], out[i][3], nt);
                        } else {
                            for (int b = 0; b < 16 && r0 + b < v.ps; ++b)
                                dst[b] = u8(out[i][b >> 2] >> (8 * (b & 3)));
                        }
                        *reinterpret_cast<uint4 *>(xb + i * SP) = make_uint4(out[i][0], out[i][1], out[i][2], out[i][3]);
                    }
                }
            }
            __syncthreads();
            if constexpr (SB)
                __syncthreads();  // the hash wave has copied the chunk
        };
        for (u32 c = 0; c < nch; c += PF) {
            chunk(d[0], c);
            if constexpr (PF == 2)
                if (c + 1 < nch)
                    chunk(d[PF - 1], c + 1);
        }
        return;
    }

    // ------------------------------------------------------------ hash wave
    if (NKFS_WS_HPRIO)
        __builtin_amdgcn_s_setprio(NKFS_WS_HPRIO);
    constexpr int LPS = 64 / SPH;  // hash lanes per stripe (4 x E)
    const int hs = (wave - NE) * SPH + lane / LPS, hli = lane % LPS;
    const int hi = hli >> 2, ha = hli & 3;
    u32 s;
    const bool live = slot_live(g, blockIdx.x * S + hs, s);
    u32 ps = 0;
    if (live)
        ps = part_size_of(g.block_sizes ? g.block_sizes[s] : g.block_size, K);
    const bool hlane = live && hi < n;
    const u32 nst = ps >> 5;                 // whole 32-byte stripes of the part
    const u32 own = (ps + CR - 1) / CR;      // this stripe's chunks
    u64 acc = xxh_acc_init(ha, 0);
    const int xoff = (hs * E + hi) * SP + 8 * ha;
    auto fold = [&](u32 c) {
        const u8 *src = xbuf[SB ? 0 : (c & 1)] + xoff;
        const int left = int(nst) - int(c * RPC);
        if (left >= RPC) {
#pragma unroll 8
            for (int r = 0; r < RPC; ++r)
                acc = xxh_round(acc, *reinterpret_cast<const u64 *>(src + 32 * r));
        } else {
            for (int r = 0; r < left; ++r)
                acc = xxh_round(acc, *reinterpret_cast<const u64 *>(src + 32 * r));
        }
    };
    __syncthreads();  // tables built (the encoders' first barrier)
    if constexpr (SB) {
        static_assert(RPC <= 32, "hash words staged in registers");
        for (u32 c = 0; c < nch; ++c) {
            __syncthreads();  // chunk c is in the exchange
            u64 hw[RPC];
            int hv = 0;
            if (hlane && c < own) {
                const u8 *src = xbuf[0] + xoff;
                const int left = int(nst) - int(c * RPC);
                hv = left < 0 ? 0 : (left > RPC ? RPC : left);
#pragma unroll
                for (int r = 0; r < RPC; ++r)
                    hw[r] = *reinterpret_cast<const u64 *>(src + 32 * r);
            }
            __syncthreads();  // the encoders may overwrite it now
            if (hv == RPC) {
#pragma unroll
                for (int r = 0; r < RPC; ++r)
                    acc = xxh_round(acc, hw[r]);
            } else {
#pragma unroll
                for (int r = 0; r < RPC; ++r) {
                    const u64 nx = xxh_round(acc, hw[r]);
                    acc = r < hv ? nx : acc;
                }
            }
        }
    } else {
        for (u32 c = 0; c < nch; ++c) {
            if (hlane && c >= 1 && c - 1 < own)
                fold(c - 1);
            __syncthreads();
        }
        if (hlane && nch >= 1 && nch - 1 < own)
            fold(nch - 1);
    }

    const int base = lane & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    if (hlane && ha == 0) {
        u64 h = ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
        h += ps;
        u64 tw[4] = {0, 0, 0, 0};
        const u32 left = ps & 31;
        if (left) {
            // the tail sits in this stripe's last chunk, untouched since
            const u32 toff = nst * 32 - (own - 1) * CR;
            const u64 *src = reinterpret_cast<const u64 *>(xbuf[SB ? 0 : ((own - 1) & 1)] + (hs * E + hi) * SP + toff);
#pragma unroll
            for (int w = 0; w < 4; ++w)
                tw[w] = src[w];
        }
        digests[u64(s) * n + hi] = xxh_tail_regs(h, tw, left);
    }
}

template <int E, int NE, bool SB, int PF, int HW = 1>
static int launch_ws(int k, hipStream_t st, const nkfs_geom &g, const uint8_t *ids, uint64_t *dig, bool nt)
{
    constexpr int S = HW * 16 / E;
    const dim3 grid((g.nstripes + S - 1) / S), block(64 * (NE + HW));
    switch (k) {
#define NKFS_K(KK)                                                                         \
    case KK:                                                                               \
        hipLaunchKernelGGL((k_encode_ws<KK, E, NE, SB, PF, HW>), grid, block, 0, st, g, ids, dig, nt); \
        return 0;
        NKFS_K(2)
        NKFS_K(3)
        NKFS_K(4)
        NKFS_K(5)
        NKFS_K(6)
        NKFS_K(7)
        NKFS_K(8)
#undef NKFS_K
    default:
        return -ENOSYS;
    }
}

// Fused encode + XXH64 of a uniform or ragged batch (n <= 8, k <= 8) with the
// warp-specialised kernel; ne = encoder waves per workgroup (E = 4: 4 or 8;
// E = 8: 2 or 4).  -ENOSYS outside that range.
extern "C" int nkfs_ws_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, int ne, bool nt,
                              hipStream_t st)
{
    if (g->n > 8 || g->k > 8 || !digests)
        return -ENOSYS;
    int rc;
    // chunks of loads in flight per encoder wave (struct nkfs_tune.enc_ws_prefetch)
    // n > 4: struct nkfs_tune.enc_ws_hash_waves picks one or two hash waves
    // per workgroup (0: nkfs_ws_auto_hash_waves -- two where the grid of
    // four-stripe workgroups ends no later: N8K5 768 x 64 KiB 3,445 / 2,474,
    // 8,192 x 512 KiB +1-4 %, 512 x 128 KiB 2,958 / 3,713; seam_mid.txt);
    // n > 4: struct nkfs_tune.enc_ws_waves overrides the caller's 4 encoder
    // waves with 6 (three per stripe, 3,072-row chunks: the exchange then
    // holds 99 KiB and the workgroup 7 waves, one per CU as before, with half
    // as many loads again in flight)
    const nkfs_tune t = nkfs_tune_now();
    const int pf = t.enc_ws_prefetch;
    if (g->n > 4 && ne == 4 && t.enc_ws_waves == 6)
        ne = 6;
    if (g->n <= 4)
        rc = ne == 8 ? launch_ws<4, 8, false, 1>(g->k, st, *g, ids, digests, nt)
                     : launch_ws<4, 4, false, 1>(g->k, st, *g, ids, digests, nt);
    else if (ne == 4 && (t.enc_ws_hash_waves == 2 || (!t.enc_ws_hash_waves && nkfs_ws_auto_hash_waves(g->nstripes) == 2)))
        rc = pf >= 2 ? launch_ws<8, 4, false, 2, 2>(g->k, st, *g, ids, digests, nt)
                     : launch_ws<8, 4, false, 1, 2>(g->k, st, *g, ids, digests, nt);
    else if (ne == 6)
        rc = pf >= 2 ? launch_ws<8, 6, false, 2>(g->k, st, *g, ids, digests, nt)
                     : launch_ws<8, 6, false, 1>(g->k, st, *g, ids, digests, nt);
    else if (pf >= 2)
        rc = ne == 4 ? launch_ws<8, 4, false, 2>(g->k, st, *g, ids, digests, nt)
                     : launch_ws<8, 2, false, 2>(g->k, st, *g, ids, digests, nt);
    else
        rc = ne == 4 ? launch_ws<8, 4, false, 1>(g->k, st, *g, ids, digests, nt)
                     : launch_ws<8, 2, false, 1>(g->k, st, *g, ids, digests, nt);
    if (rc)
        return rc;
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
