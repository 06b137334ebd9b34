// nk8_fast.hip -- streaming fast path of the nkfs N-K encode for n <= 8:
// encode fused with XXH64 of every part, one pass over HBM.
//
// Reference: crt/nk8.c:403-420 (part_i[j] = XOR_m ids[i]^m * d[j*k+m]) and
// crt/xxhash.c:358-496 (XXH64, seed 0 as crt/csum.c:5), per part.
//
// Shape of one workgroup = one wave (64 lanes) = G stripes in lock step:
//   E = 4 (n <= 4): G = 4 stripes, 16 lanes per stripe, chunk R = 256 rows
//   E = 8 (n <= 8): G = 2 stripes, 32 lanes per stripe, chunk R = 512 rows
// so that 4 lanes x n parts x G stripes <= 64 hash chains fill the wave: XXH64
// of one part is serial, its only parallelism being its four accumulators,
// so every lane owns one (stripe, part, accumulator) chain for the whole
// stripe and the chunk loop feeds it 8-byte words in order.
//
// Per chunk each lane encodes 16 consecutive rows of its stripe (16*k input
// bytes: k x 16-byte loads, coalesced across lanes):
//   row r -> E packed bytes  = rep(d[r*k]) ^ XOR_{m>=1} T_m[d[r*k+m]]
// where T_m[x] = (ids[0]^m * x, ..., ids[n-1]^m * x) is a per-stripe packed
// product table in LDS (built from eight basis products: multiplication by a
// constant is GF(2)-linear), so one LDS lookup yields the term for all n parts
// and column m = 0 (coefficient 1) needs no lookup at all.  A byte transpose
// (v_perm) turns 16 rows x E bytes into 16 bytes per part, which go to HBM
// (one 16-byte store per part) and to an LDS exchange buffer from which the
// hash lanes take their words.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/nkfs_gpu.h"
#include "nk8_dev.h"
#include "gf256.h"
#include "nkfs_internal.h"
#include "xxh64_dev.h"

using namespace nkfs;
typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

using namespace nkfs::dev;

// P = chunks of rows in flight per lane (prefetch depth, rotating register
// slots): grids with few waves per SIMD (big stripes) cannot hide HBM
// latency behind other waves, so each wave keeps more of its own loads out.
//
// NIB: nibble tables.  Multiplication by a constant is GF(2)-linear, so
// T_m[x] = L_m[x & 15] ^ H_m[x >> 4] with 16-entry tables L_m[v] = T_m[v],
// H_m[v] = T_m[v << 4]: two lookups per byte instead of one, but a
// half-table's 16 entries sit in distinct LDS banks (same entry =
// broadcast), so lookups never conflict, and the tables take 32 entries per
// m instead of 256.  Stripes that share a 32-lane LDS group are offset by
// half a bank row so their halves use disjoint banks.
template <int K, int E, int P, bool HASH, bool NIB>
__global__ __launch_bounds__(64) void k_encode_fast(nkfs_geom g, const u8 *ids, u64 *digests, bool nt)
{
    constexpr int G = E == 4 ? 4 : 2;   // stripes per wave
    constexpr int LP = 64 / G;          // lanes per stripe
    constexpr int R = 16 * LP;          // rows per stripe per chunk
    constexpr int SP = R + 32;          // LDS bytes per part in the exchange buffer (bank spread)
    constexpr int TB = (NIB ? 32 : 256) * E;  // bytes per packed table (per m)
    constexpr int TS = (K - 1) * TB + (NIB ? 16 * E : 0);  // bytes per stripe (+ bank offset room)
    constexpr int W = E / 4;            // dwords per packed entry
    __shared__ __attribute__((aligned(16))) u8 tbl[G * TS];
    __shared__ __attribute__((aligned(16))) u8 xbuf[G * E * SP];

    const int lane = threadIdx.x;
    const int gi = lane / LP;
    const int li = lane % LP;
    const int n = g.n;
    u32 s;
    const bool live = slot_live(g, blockIdx.x * G + gi, s);
    if (!__any(live))
        return;  // every stripe of this wave belongs to the other launch of a split batch
    Stripe v{};
    if (live)
        v = stripe_at(g, s);

    // ---- hash chain of this lane: part hi, accumulator ha
    const int hi = li >> 2, ha = li & 3;
    const bool hlane = HASH && live && hi < n;
    u64 acc = xxh_acc_init(ha, 0);
    const u32 nst = v.ps >> 5;  // whole 32-byte stripes of each part
    const u32 nchunks = live ? (v.ps + R - 1) / R : 0;
    const bool aligned = ((reinterpret_cast<uintptr_t>(v.blk) | reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 15) == 0;

    u32 dq[P][4 * K];
    auto load_task = [&](u32 (&d)[4 * K], u32 r0) {
        const u64 off = u64(r0) * K;
        if (aligned && off + 16 * K <= v.B) {
            const uint4 *src = reinterpret_cast<const uint4 *>(v.blk + off);
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const uint4 t = src[q];
                d[4 * q] = t.x;
                d[4 * q + 1] = t.y;
                d[4 * q + 2] = t.z;
                d[4 * q + 3] = t.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4 * K; ++q) {
                u32 x = 0;
                for (int b = 0; b < 4; ++b) {
                    const u64 p = off + 4 * q + b;
                    if (p < v.B)
                        x |= u32(v.blk[p]) << (8 * b);
                }
                d[q] = x;
            }
        }
    };
    // the first P chunks' rows are requested before the tables are built: the
    // HBM latency hides under the table build instead of following it
#pragma unroll
    for (int p = 0; p < P; ++p)
        if (u32(p) < nchunks && p * R + 16 * li < v.ps)
            load_task(dq[p], p * R + 16 * li);

    // ---- packed product tables T_m, m = 1..K-1, for this lane's stripe
    u32 coef[W];  // packed ids[i]^m
    u32 idw[W];
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
    u8 *mytbl = tbl + gi * TS + (NIB ? (gi & 1) * 16 * E : 0);
#pragma unroll
    for (int m = 1; m < K; ++m) {
        u32 basis[8][W];
        make_basis<W>(basis, coef);
        if constexpr (NIB) {
            // entry e: half h = e >> 4 (low / high nibble), value v = e & 15
#pragma unroll
            for (int e0 = 0; e0 < 32; e0 += LP) {
                const int e = e0 + li;
                if (e < 32) {
                    const int v = e & 15, h = e >> 4;
                    u32 val[W];
#pragma unroll
                    for (int w = 0; w < W; ++w) {
                        u32 x = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            x ^= basis[4 * h + b][w] & (0u - u32((v >> b) & 1));
                        val[w] = x;
                    }
                    u8 *dst = mytbl + (m - 1) * TB + e * E;
                    if constexpr (W == 2)
                        *reinterpret_cast<uint2 *>(dst) = make_uint2(val[0], val[1]);
                    else
                        *reinterpret_cast<u32 *>(dst) = val[0];
                }
            }
        } else {
            build_table<W, LP>(mytbl + (m - 1) * TB, basis, li);
        }
#pragma unroll
        for (int w = 0; w < W; ++w)
            coef[w] = gf_mul_packed(coef[w], idw[w]);
    }
    __syncthreads();

    // Software pipeline: step c encodes chunk c while the hash lanes run the
    // XXH64 rounds of chunk c-1 from registers (hw[]), so the serial multiply
    // chain overlaps the table lookups instead of following them.
    constexpr int RPC = R / 32;  // rounds per chain per chunk
    u64 hw[RPC];
    int hvalid = 0;              // rounds pending in hw[]
    auto step = [&](u32 (&d)[4 * K], u32 c) {
        const u32 r0 = c * R + 16 * li;
        const bool act = c < nchunks && r0 < v.ps;
        u32 row[16][W];
        if (act) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int p0 = r * K;
                const u32 rep = __builtin_amdgcn_perm(0u, d[p0 >> 2], 0x01010101u * u32(p0 & 3));
#pragma unroll
                for (int w = 0; w < W; ++w)
                    row[r][w] = rep;
#pragma unroll
                for (int m = 1; m < K; ++m) {
                    const int p = p0 + m;
                    const u32 byte = (d[p >> 2] >> (8 * (p & 3))) & 0xFFu;
                    if constexpr (NIB) {
                        const u8 *e0 = mytbl + (m - 1) * TB + (byte & 15u) * E;
                        const u8 *e1 = mytbl + (m - 1) * TB + (16u + (byte >> 4)) * E;
                        if constexpr (E == 8) {
                            const uint2 t0 = *reinterpret_cast<const uint2 *>(e0);
                            const uint2 t1 = *reinterpret_cast<const uint2 *>(e1);
                            row[r][0] ^= t0.x ^ t1.x;
                            row[r][1] ^= t0.y ^ t1.y;
                        } else {
                            row[r][0] ^= *reinterpret_cast<const u32 *>(e0) ^ *reinterpret_cast<const u32 *>(e1);
                        }
                    } else {
                        const u8 *e = mytbl + (m - 1) * TB + byte * E;
                        if constexpr (E == 8) {
                            const uint2 t = *reinterpret_cast<const uint2 *>(e);
                            row[r][0] ^= t.x;
                            row[r][1] ^= t.y;
                        } else {
                            row[r][0] ^= *reinterpret_cast<const u32 *>(e);
                        }
                    }
                }
            }
        }
        if constexpr (HASH) {
#pragma unroll
            for (int rr = 0; rr < RPC; ++rr) {
                const u64 nxt = xxh_round(acc, hw[rr]);
                acc = rr < hvalid ? nxt : acc;
            }
        }
        if (act) {
            // this slot's rows are consumed: refill it with chunk c+P while
            // this chunk is stored
            if (c + P < nchunks && r0 + P * R < v.ps)
                load_task(d, r0 + P * R);
            // rows -> parts: out[i][q] = bytes of part i for rows 4q..4q+3
            u32 out[E][4];
#pragma unroll
            for (int w = 0; w < W; ++w)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    transpose4(row[4 * q][w], row[4 * q + 1][w], row[4 * q + 2][w], row[4 * q + 3][w],
                               out[4 * w][q], out[4 * w + 1][q], out[4 * w + 2][q], out[4 * w + 3][q]);
#pragma unroll
            for (int i = 0; i < E; ++i) {
                if (i < n) {
                    const uint4 val = make_uint4(out[i][0], out[i][1], out[i][2], out[i][3]);
                    u8 *dst = v.parts + u64(i) * v.pitch + r0;
                    if (aligned) {
                        store16(dst, val.x, val.y, val.z, val.w, nt);
                    } else {
                        for (int b = 0; b < 16 && r0 + b < v.ps; ++b)
                            dst[b] = u8(out[i][b >> 2] >> (8 * (b & 3)));
                    }
                    if constexpr (HASH)
                        *reinterpret_cast<uint4 *>(xbuf + (gi * E + i) * SP + 16 * li) = val;
                }
            }
        }
        if constexpr (HASH) {
            __syncthreads();
            hvalid = 0;
            if (hlane && c < nchunks) {
                const u8 *src = xbuf + (gi * E + hi) * SP + 8 * ha;
                const int left = int(nst) - int(c * RPC);
                hvalid = left < 0 ? 0 : (left > RPC ? RPC : left);
#pragma unroll
                for (int rr = 0; rr < RPC; ++rr)
                    hw[rr] = *reinterpret_cast<const u64 *>(src + 32 * rr);
            }
            __syncthreads();
        }
    };
    // with HASH one step past the last chunk folds its words; steps past a
    // stripe's end are no-ops, so the P-unrolled body needs no exit inside
    const u32 last = HASH ? nchunks : (nchunks ? nchunks - 1 : 0);
    for (u32 c = 0; __any(nchunks && c <= last); c += P) {
#pragma unroll
        for (int p = 0; p < P; ++p)
            step(dq[p], c + p);
    }

    if constexpr (HASH) {
        const int base = lane & ~3;
        const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
        const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
        if (hlane && ha == 0) {
            u64 h = v.ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
            h += v.ps;
            u64 tw[4] = {0, 0, 0, 0};
            const u32 left = v.ps & 31;
            if (left) {
                // the tail sits in the last chunk's exchange buffer
                const u32 toff = nst * 32 - (nchunks - 1) * R;
                const u64 *src = reinterpret_cast<const u64 *>(xbuf + (gi * E + hi) * SP + toff);
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    tw[w] = src[w];
            }
            digests[u64(s) * n + hi] = xxh_tail_regs(h, tw, left);
        }
    }
}

// Dynamic LDS request that caps a one-wave-workgroup kernel at `target`
// resident waves per CU (0 = no cap): the LDS a CU has divided by the target,
// less the kernel's static LDS.
static size_t lds_cap_pad(const void *kern, int target)
{
    if (target <= 0)
        return 0;
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, kern) != hipSuccess)
        return 0;
    if (target < 3)
        target = 3;  // keeps the request under the 64 KiB dynamic default
    const size_t per = size_t(160 * 1024) / size_t(target);
    return per > a.sharedSizeBytes ? per - a.sharedSizeBytes : 0;
}

template <int E, bool HASH, bool NIB>
static int launch_k(int k, hipStream_t st, const nkfs_geom &g, const u8 *ids, u64 *dig)
{
    constexpr int G = E == 4 ? 4 : 2;
    const dim3 grid((g.nstripes + G - 1) / G);
    const int cap = nkfs_tune_now().enc_fused_waves_per_cu;
    switch (k) {
#define NKFS_K(KK)                                                                                      \
    case KK:                                                                                            \
        hipLaunchKernelGGL((k_encode_fast<KK, E, 1, HASH, NIB>), grid, dim3(64),                        \
                           lds_cap_pad(reinterpret_cast<const void *>(&k_encode_fast<KK, E, 1, HASH, NIB>), cap), \
                           st, g, ids, dig, false);                                                      \
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

extern "C" int nkfs_ws_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, int ne, bool nt,
                              hipStream_t st);

// Fused encoder family for n <= 8, k <= 8.  rules != 0: the measured shape
// rules pick the fused or the warp-specialised kernel; rules == 0: the fused
// kernel only.  nib: -1 by rule, 0 / 1 forced (struct nkfs_tune).  Returns
// -ENOSYS outside the fast path (the caller then uses the generic kernels).
extern "C" int nkfs_fast_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, int rules, int nib,
                                hipStream_t st)
{
    if (g->n > 8 || g->k > 8)
        return -ENOSYS;
    const int E = g->n <= 4 ? 4 : 8;
    // n <= 8 grids of at most two waves per SIMD of big stripes (e.g. C3:
    // 2,048 x 1 MiB) are issue-bound in the fused kernel; there the
    // warp-specialised kernel (4 encoder waves + 1 hash wave per 2 stripes)
    // wins: N8K5 1 MiB x 3,840: fused 3.60 / nibble 4.60 / warp-specialised
    // 4.90 TB/s, x 4,096: 3.84 / 4.76 / 5.06 (profiles/r01/ab_ws_shapes.txt).
    // Ragged batches (sizes only on the device) keep the fused kernel.
    const u32 fused_waves = (g->nstripes + (E == 4 ? 3u : 1u)) / (E == 4 ? 4u : 2u);
    const u32 ps = g->block_sizes ? 0u : (g->block_size + u32(g->k) - 1) / u32(g->k);
    // n > 4: parts of 8 KiB and up that the walk rule (walk_by_rule,
    // nk8_kernels.hip) left here -- parts of 64 KiB and up, or grids too small
    // for the walk encoder -- take the warp-specialised kernel: 256 x 64 KiB
    // N8K5 ws 1,402 / walk 1,036 / fused 598 GB/s, C3 8,192 x 1 MiB ws 5,215
    // / fused 5,023 (profiles/r03/seam_sweep_box1.txt).  n <= 4: parts of 8
    // KiB and up, or at most 1,024 stripes: N4K2 65,536 x 16 KiB ws 5,816 /
    // fused 4,960, 1,024 x 64 KiB 4,206 / 1,616, 1,024 x 4 KiB 1,336 / 911;
    // C2 (65,536 x 4 KiB) stays fused 5,237 / ws 4,332 (seam_sweep_box2.txt).
    // Round 4: n > 4 from 4 KiB parts on <= 1,024 stripes as well (walk_by_rule).
    if (rules && digests &&
        (ps >= 8192 || (E == 4 && !g->block_sizes && g->nstripes <= 1024) ||
         (E == 8 && ps >= 4096 && g->nstripes <= 1024)))
        return nkfs_ws_encode(g, ids, digests, 4, false, st);
    // Nibble tables free LDS (N8K5: 25 -> 11 KB per wave, the occupancy
    // limit) at twice the lookups: a win where the grid offers more waves
    // than 25 KB tables let reside (C4 encode +3.2 %), a loss where one wave
    // per SIMD is issue-bound (C3 -15 %) or LDS never limited (n <= 4: -2 %)
    // -- profiles/r01/ab_nibble_tables.txt.  The 25 KB form lets 6 waves
    // reside per CU (1,536 on the chip), so nibble tables take every grid
    // beyond that.
    const bool nb = nib < 0 ? E == 8 && fused_waves > 1536 : nib != 0;
    const int rc = E == 4 ? (digests ? launch_k<4, true, false>(g->k, st, *g, ids, digests)
                                     : launch_k<4, false, false>(g->k, st, *g, ids, digests))
                          : nb ? (digests ? launch_k<8, true, true>(g->k, st, *g, ids, digests)
                                          : launch_k<8, false, true>(g->k, st, *g, ids, digests))
                               : (digests ? launch_k<8, true, false>(g->k, st, *g, ids, digests)
                                          : launch_k<8, false, false>(g->k, st, *g, ids, digests));
    if (rc)
        return rc;
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// ------------------------------------------------------------------ decode
//
// One wave = G stripes (G = 1 as launched; the kernel also takes G = 2, 4),
// k <= 8 (crt/nk8.c:446-599):
//  1. lane 0 of each stripe picks the first k offered parts with distinct ids
//     (crt/nk8.c:512-537) and forms M(t) = prod_c (t + x_c);
//  2. lane c < k of the stripe computes row c of W = V^-1 for V[m][c] = x_c^m
//     in closed form (Lagrange basis: W[c][m] = [t^m] M(t)/(t + x_c) divided
//     by M'(x_c)), the unique inverse the reference's Gauss-Jordan produces;
//  3. packed tables U_c[x] = (W[c][0]*x, ..., W[c][k-1]*x) go to LDS;
//  4. every lane rebuilds 16 rows per step: one 16-byte load from each of the
//     k parts, k*16 lookups, rows packed back to k*16 contiguous bytes:
//       block[j*k + m] = XOR_c part_c[j] * W[c][m]      (crt/nk8.c:552-582)
//     with the next step's loads issued before this step's stores.
namespace {

// bit-serial GF(2^8)/0x11B product in registers (no tables needed)
__device__ inline u32 gfm(u32 a, u32 b)
{
    u32 r = 0;
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        r ^= a & (0u - ((b >> bit) & 1u));
        a = ((a << 1) ^ (0x11Bu & (0u - ((a >> 7) & 1u)))) & 0xFFu;
    }
    return r;
}

}  // namespace

// U = 16-row units per lane per step (one-shot steps for short stripes: a
// 4 KiB N4K2 stripe is a single step of 2 x 1024 rows at U = 2)
// NKFS_DEC_FAST_WPE: waves per SIMD requested for the non-verifying form
// (0: the compiler's choice -- 102 SGPRs, 7 waves per SIMD for k = 2)
#ifndef NKFS_DEC_FAST_WPE
#define NKFS_DEC_FAST_WPE 0
#endif
template <int K, int E, int G, int U, bool VERIFY>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(VERIFY || !NKFS_DEC_FAST_WPE ? 1 : NKFS_DEC_FAST_WPE))) void k_decode_fast(nkfs_geom g, int n_slots, const u8 *ids, const u8 *avail,
                                                    int navail, int32_t *status, const u8 *inv, bool nt, int slices,
                                                    const u64 *expect, u64 *badmask)
{
    constexpr int LP = 64 / G;
    constexpr int R = 16 * LP;  // rows per unit (one 16-row block per lane)
    constexpr int RS = R * U;   // rows per stripe per step
    static_assert(!VERIFY || U == 1, "the verifying form hashes one unit per step");
    constexpr int W = E / 4;
    constexpr int TB = 256 * E;
    constexpr int SPX = R + 32;  // verify exchange buffer bytes per part
    static_assert(!VERIFY || 4 * K <= LP, "one hash chain per lane");
    __shared__ __attribute__((aligned(16))) u8 tbl[G * K * TB];
    __shared__ __attribute__((aligned(16))) u8 xbuf[VERIFY ? G * K * SPX : 16];
    __shared__ u8 slot[G][K], M[G][K + 1], xs[G][K], wrow[G][K][K];
    __shared__ u8 cand_id[G][LP], cand_slot[G][LP];
    __shared__ u32 inv4[64];  // GF inverses, 4 per word
    __shared__ int have[G];

    const int lane = threadIdx.x;
    const int gi = lane / LP, li = lane % LP;
    // blockIdx.x = group * slices + slice: long stripes are split into row
    // slices on separate waves (decode rows are independent)
    const u32 grp = blockIdx.x / u32(slices), slice = blockIdx.x % u32(slices);
    const u32 slot_ = grp * G + gi;
    const bool live = slot_ < g.nstripes;
    const u32 s = live && g.order ? g.order[slot_] : slot_;
    inv4[lane] = reinterpret_cast<const u32 *>(inv)[lane];
    // the first LP offered parts and their ids, loaded in parallel
    const u8 *sid = ids + u64(s) * n_slots;
    const u8 *sav = avail + u64(s) * navail;
    if (live && li < navail) {
        const u8 sl = sav[li];
        cand_slot[gi][li] = sl;
        cand_id[gi][li] = sid[sl];
    }
    __syncthreads();

    // The first K offered slots are the selection unless an id repeats
    // among them (crt/nk8.c:512-537): request the first step's rows from
    // them now, so the HBM latency hides under the selection, the inverse
    // and the table build; a changed selection reloads below.
    // geometry of this stripe: uniform, or ragged as nkfs_nk8_encode_ragged
    // lays it out (part pitch = part size rounded to NKFS_PART_ALIGN)
    u32 B = g.block_size;
    u64 ppitch = g.part_pitch;
    const u8 *pbase = g.parts + u64(s) * n_slots * g.part_pitch;
    u8 *out = const_cast<u8 *>(g.blocks) + u64(s) * g.block_pitch;
    if (g.block_sizes) {
        B = live ? g.block_sizes[s] : 0u;
        ppitch = (u64(part_size_of(B, K)) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
        pbase = live ? g.parts + g.part_off[s] : g.parts;
        out = live ? const_cast<u8 *>(g.blocks) + g.block_off[s] : out;
    }
    const u32 ps = part_size_of(B, K);
    const u32 steps = (ps + RS - 1) / RS, per = VERIFY ? steps : (steps + slices - 1) / slices;
    const u32 rend = VERIFY ? ps : min(ps, (slice + 1) * per * RS);
    const u32 rfirst = (VERIFY ? 0u : slice * per * RS) + 16 * li;
    u8 spec[K];
    const u8 *src[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        spec[c] = (c < navail && c < LP) ? cand_slot[gi][c] : 0;
        src[c] = pbase + spec[c] * ppitch;
    }
    u32 pv[U][K][4];
    auto load_step = [&](u32 r0) {  // caller checks r0 < rend; later units check themselves
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u && r0 + u * R >= rend)
                continue;
#pragma unroll
            for (int c = 0; c < K; ++c) {
                const uint4 t = *reinterpret_cast<const uint4 *>(src[c] + r0 + u * R);  // pitch >= round16(ps)
                pv[u][c][0] = t.x;
                pv[u][c][1] = t.y;
                pv[u][c][2] = t.z;
                pv[u][c][3] = t.w;
            }
        }
    };
    if (live && navail >= K && rfirst < rend)
        load_step(rfirst);

    // first K distinct ids in offered order (crt/nk8.c:512-537)
    if (navail <= LP) {
        // lane-parallel: candidate li is taken when no earlier candidate has
        // its id and fewer than K earlier candidates were taken
        const bool cand = live && li < navail;
        const u8 myid = cand ? cand_id[gi][li] : 0;
        bool dup = false;
        for (int j = 0; cand && j < li; ++j)
            dup |= cand_id[gi][j] == myid;
        const bool first = cand && !dup;
        const u64 gmask = LP == 64 ? ~0ull : (((1ull << LP) - 1) << (gi * LP));
        const u64 taken = u64(__ballot(first)) & gmask;
        const int rank = __popcll(taken & ((1ull << lane) - 1));
        if (first && rank < K) {
            xs[gi][rank] = myid;
            slot[gi][rank] = cand_slot[gi][li];
        }
        if (li == 0) {
            const int h = min(K, __popcll(taken));
            have[gi] = h;
            if (live && status && slice == 0)
                status[s] = h < K ? -EINVAL : 0;
            if (live && VERIFY && badmask)
                badmask[s] = 0;
        }
    } else if (li == 0) {
        int h = 0;
        if (live) {
            for (int c = 0; c < navail && h < K; ++c) {
                u8 sl, id;
                if (c < LP) {
                    sl = cand_slot[gi][c];
                    id = cand_id[gi][c];
                } else {
                    sl = sav[c];
                    id = sid[sl];
                }
                bool dup = false;
                for (int d = 0; d < h; ++d)
                    dup |= xs[gi][d] == id;
                if (dup)
                    continue;
                xs[gi][h] = id;
                slot[gi][h] = sl;
                ++h;
            }
            if (status && slice == 0)
                status[s] = h < K ? -EINVAL : 0;
            if (VERIFY && badmask)
                badmask[s] = 0;
        }
        have[gi] = h;
    }
    __syncthreads();
    // M(t) = prod_c (t + x_c), by lane 0 of the stripe
    if (li == 0 && have[gi] == K) {
        u32 m[K + 1];
        m[0] = 1;
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const u32 x = xs[gi][c];
            m[c + 1] = m[c];
#pragma unroll
            for (int i = c; i >= 1; --i)
                m[i] = m[i - 1] ^ gfm(x, m[i]);
            m[0] = gfm(x, m[0]);
        }
#pragma unroll
        for (int i = 0; i <= K; ++i)
            M[gi][i] = u8(m[i]);
    }
    __syncthreads();
    const bool ok = have[gi] == K;
    if (ok && li < K) {
        const u32 xc = xs[gi][li];
        u32 q[K];
        u32 acc = M[gi][K];
        q[K - 1] = acc;
#pragma unroll
        for (int i = K - 1; i >= 1; --i) {
            acc = M[gi][i] ^ gfm(xc, acc);
            q[i - 1] = acc;
        }
        u32 d = 0;
#pragma unroll
        for (int i = K - 1; i >= 0; --i)
            d = gfm(d, xc) ^ q[i];
        const u32 dinv = (inv4[d >> 2] >> (8 * (d & 3))) & 0xFFu;
#pragma unroll
        for (int i = 0; i < K; ++i)
            wrow[gi][li][i] = u8(gfm(q[i], dinv));
    }
    __syncthreads();
    u8 *mytbl = tbl + gi * K * TB;
    if (ok) {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            u32 rw[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                u32 x = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (4 * w + b < K)
                        x |= u32(wrow[gi][c][4 * w + b]) << (8 * b);
                rw[w] = x;
            }
            u32 basis[8][W];
            make_basis<W>(basis, rw);
            build_table<W, LP>(mytbl + c * TB, basis, li);
        }
    }
    __syncthreads();
    if (!ok)
        return;

    bool respec = false;
#pragma unroll
    for (int c = 0; c < K; ++c) {
        respec |= slot[gi][c] != spec[c];
        src[c] = pbase + slot[gi][c] * ppitch;
    }
    if (respec && rfirst < rend)
        load_step(rfirst);
    const bool aligned = ((reinterpret_cast<uintptr_t>(out) | (g.block_sizes ? 0 : g.block_pitch)) & 15) == 0;
    auto rebuild = [&](u32 (&o)[4 * K], int u) {
        // 16 rows in four groups of 4: lookups, XOR, then the group's 4*K
        // bytes are packed into K output dwords with v_perm (<= 2 per dword).
        // Each group's table addresses depend (opaquely, tdep == 0) on the
        // previous group's result: hoisting all 16*K lookups ahead would hold
        // them in VGPRs at once (205 VGPRs at K = 5, 2 waves per SIMD)
        u32 tdep = 0;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            u32 row[4 * W];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int r = 4 * gq + rr;
#pragma unroll
                for (int w = 0; w < W; ++w)
                    row[rr * W + w] = 0;
#pragma unroll
                for (int c = 0; c < K; ++c) {
                    const u32 byte = (pv[u][c][r >> 2] >> (8 * (r & 3))) & 0xFFu;
                    const u8 *e = mytbl + tdep + c * TB + byte * E;
                    if constexpr (E == 8) {
                        const uint2 t = *reinterpret_cast<const uint2 *>(e);
                        row[rr * W] ^= t.x;
                        row[rr * W + 1] ^= t.y;
                    } else {
                        row[rr * W] ^= *reinterpret_cast<const u32 *>(e);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < K; ++q)
                o[gq * K + q] = pack_dword<K, W>(row, q);
            if constexpr (K * W > 8)
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(o[gq * K]));
        }
    };
    auto emit = [&](const u32 (&o)[4 * K], u32 r0) {
        const u64 off = u64(r0) * K;
        if (aligned && off + 16 * K <= B) {
            uint4 *dst = reinterpret_cast<uint4 *>(out + off);
#pragma unroll
            for (int q = 0; q < K; ++q)
                store16(dst + q, o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3], nt);
        } else {
#pragma unroll
            for (int q = 0; q < 4 * K; ++q)
                for (int b = 0; b < 4; ++b)
                    if (off + 4 * q + b < B)
                        out[off + 4 * q + b] = u8(o[q] >> (8 * b));
        }
    };

    if constexpr (!VERIFY) {
        for (u32 r0 = rfirst; r0 < rend; r0 += RS) {
            u32 o[U][4 * K];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (!u || r0 + u * R < rend)
                    rebuild(o[u], u);
            if (r0 + RS < rend)
                load_step(r0 + RS);  // prefetch the next step under this one's stores
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (!u || r0 + u * R < rend)
                    emit(o[u], r0 + u * R);
        }
    } else {
        // Integrity-checked decode: the k parts read for the rebuild are also
        // hashed (XXH64, seed 0) and compared with their stored digests, as
        // the core checks every block it reads (core/inode.c:561-575).  One
        // lane per (part, accumulator); words reach the hash lanes through
        // LDS and the rounds of step t-1 run beside the lookups of step t.
        constexpr int RPC = R / 32;
        const int hc = li >> 2, ha = li & 3;
        const bool hlane = li < 4 * K;
        const u32 nst = ps >> 5;
        u64 acc = xxh_acc_init(ha, 0);
        u64 hw[RPC];
        int hvalid = 0;
        for (u32 t = 0; t <= steps; ++t) {
            const u32 r0 = t * R + 16 * li;
            const bool act = t < steps && r0 < ps;
            u32 o[4 * K];
            if (act)
                rebuild(o, 0);
#pragma unroll
            for (int r = 0; r < RPC; ++r) {
                const u64 nxt = xxh_round(acc, hw[r]);
                acc = r < hvalid ? nxt : acc;
            }
            if (act) {
#pragma unroll
                for (int c = 0; c < K; ++c)
                    *reinterpret_cast<uint4 *>(xbuf + (gi * K + c) * SPX + 16 * li) =
                        make_uint4(pv[0][c][0], pv[0][c][1], pv[0][c][2], pv[0][c][3]);
                if (r0 + R < ps)
                    load_step(r0 + R);
                emit(o, r0);
            }
            __syncthreads();
            hvalid = 0;
            if (hlane && t < steps) {
                const u8 *hsrc = xbuf + (gi * K + hc) * SPX + 8 * ha;
                const int left = int(nst) - int(t * RPC);
                hvalid = left < 0 ? 0 : (left > RPC ? RPC : left);
#pragma unroll
                for (int r = 0; r < RPC; ++r)
                    hw[r] = *reinterpret_cast<const u64 *>(hsrc + 32 * r);
            }
            __syncthreads();
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
                const u32 toff = nst * 32 - (steps - 1) * R;
                const u64 *tp = reinterpret_cast<const u64 *>(xbuf + (gi * K + hc) * SPX + toff);
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    tw[w] = tp[w];
            }
            const u8 sl = slot[gi][hc];
            if (xxh_tail_regs(h, tw, left) != expect[u64(s) * n_slots + sl]) {
                if (badmask)
                    atomicOr(reinterpret_cast<unsigned long long *>(badmask + s), 1ull << (sl < 63 ? sl : 63));
                if (status)
                    status[s] = -EIO;
            }
        }
    }
}

extern "C" int nkfs_fast_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                                int navail, int32_t *status, const void *gf, hipStream_t st,
                                const uint64_t *expect, uint64_t *badmask)
{
    if (g->k > 8 || (g->part_pitch & 15) ||
        (reinterpret_cast<uintptr_t>(g->parts) & 15))
        return -ENOSYS;
    // one stripe per wave: for k 5..8 it halves the E=8 tables and lifts
    // occupancy (C3 decode 3.27 -> 4.03 TB/s over two stripes per wave); for
    // k <= 4 the wave then streams one stripe's parts in 1 KiB runs (C2
    // decode 4.48 -> 5.08 TB/s over four stripes per wave, tools/ab_lib.py).
    const GfTables *t = (const GfTables *)gf;
    const bool nt = false;
    const bool verify = expect != nullptr;
    const int G = 1;
    const u32 groups = (g->nstripes + G - 1) / G;
    // enough waves to fill the chip (>= 4 per SIMD), never a slice under 4
    // steps; the verifying form hashes each part in order: one slice
    const u32 ps = g->block_size / u32(g->k) + (g->block_size % u32(g->k) ? 1u : 0u);
    // two 16-row units per lane per step (one-shot 4 KiB N4K2 stripes, half
    // the steps of long ones): decode +3 % (C2), +9 % (C3), +6 % (C4) in
    // one-process A/B (profiles/r01/ab_decode_units.txt); NKFS_DEC_U=1 = old
    const int U = verify ? 1 : 2;
    const u32 R = 16u * (64u / u32(G)) * u32(U);
    const u32 steps = (ps + R - 1) / R;
    u32 slices = 1;
    const u32 target = 4096;
    while (!verify && groups * slices < target && steps / (slices * 2) >= 4)
        slices *= 2;
    const dim3 grid(groups * slices);
    const int cap = nkfs_tune_now().dec_wave_waves_per_cu;
#define NKFS_DK(KK, EE, GG)                                                                                       \
    do {                                                                                                          \
        if (verify)                                                                                               \
            hipLaunchKernelGGL((k_decode_fast<KK, EE, GG, 1, true>), grid, dim3(64),                               \
                               lds_cap_pad(reinterpret_cast<const void *>(&k_decode_fast<KK, EE, GG, 1, true>), cap), \
                               st, *g, n_slots, ids, avail, navail, status, t->inv, nt, int(slices), expect,      \
                               badmask);                                                                          \
        else                                                                                                      \
            hipLaunchKernelGGL((k_decode_fast<KK, EE, GG, 2, false>), grid, dim3(64),                              \
                               lds_cap_pad(reinterpret_cast<const void *>(&k_decode_fast<KK, EE, GG, 2, false>), cap), \
                               st, *g, n_slots, ids, avail, navail, status, t->inv, nt, int(slices), expect,      \
                               badmask);                                                                          \
    } while (0)
    switch (g->k) {
    case 2: NKFS_DK(2, 4, 1); break;
    case 3: NKFS_DK(3, 4, 1); break;
    case 4: NKFS_DK(4, 4, 1); break;
    case 5: NKFS_DK(5, 8, 1); break;
    case 6: NKFS_DK(6, 8, 1); break;
    case 7: NKFS_DK(7, 8, 1); break;
    case 8: NKFS_DK(8, 8, 1); break;
#undef NKFS_DK
    default:
        return -ENOSYS;
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
