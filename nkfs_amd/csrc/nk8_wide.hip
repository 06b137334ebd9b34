// nk8_wide.hip -- the shapes the fused kernels do not take: encode with
// n > 8 parts (up to 255) and 2 <= k <= 16, or a handful of big stripes (one
// nk8_split_block call); decode with 8 < k <= 16.
//
// Reference: crt/nk8.c:403-420 -- part_i[j] = XOR_m ids[i]^m * d[j*k + m],
// d zero past block_size (:393-398); crt/nk8.c:552-582 -- block[j*k + m] =
// XOR_c part_c[j] * W[c][m], W the inverse of the survivors' Vandermonde rows.
//
// Parts are taken eight at a time (a "part group"): for a stripe and group,
// the packed tables T_m[x] = (ids_{8g}^m x, ..., ids_{8g+7}^m x), m = 1..k-1,
// give one row's term for eight parts per ds_read_b64, exactly as in the
// fused kernels; k-1 lookups + XORs per row and group.  A workgroup (4
// waves) owns one (stripe, two groups, row slice): it builds the groups'
// tables once in LDS, then every lane encodes 16 rows per step (k 16-byte
// loads of its contiguous 16k bytes, read once for 16 parts; 16 bytes of
// each part out, one contiguous 1 KiB run per store instruction).  With
// more than 16 parts the group pairs of a stripe read the same block, so
// they are placed on the same XCD (MI355X hands workgroup b to XCD b mod 8)
// and share its L2.  Big stripes are cut into row slices
// so that a few stripes still fill the chip.  XXH64 of the parts runs
// afterwards as the batched message hash (k_xxh64_fast), since one part's
// chain is serial over all of its rows.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nk8_dev.h"
#include "xxh64_dev.h"

using namespace nkfs;
using namespace nkfs::dev;

namespace {

constexpr int WIDE_MAX_K = 16;
constexpr u32 STEP_ROWS = 4 * 1024;  // rows a workgroup encodes per step

template <int K, int NG>
__global__ __launch_bounds__(256) void k_encode_wide(nkfs_geom g, const u8 *ids, u32 ngroups, u32 nslices,
                                                     u32 slice_rows)
{
    constexpr int TB = 256 * 8;  // bytes per packed table
    __shared__ __attribute__((aligned(16))) u8 tbl[NG][(K - 1) * TB];

    // block -> (stripe, NG consecutive groups, slice); the group sets and
    // slices of stripe s all land on XCD s mod 8
    const u32 b = blockIdx.x;
    const u32 loc = b >> 3;
    const u32 slice = loc % nslices;
    const u32 gset = (loc / nslices) % ngroups;
    const u32 s = (loc / nslices / ngroups) * 8 + (b & 7);
    if (s >= g.nstripes)
        return;  // the whole workgroup: no barrier is skipped by part of it
    const Stripe v = stripe_at(g, s);
    const u32 r_begin = slice * slice_rows;
    if (r_begin >= v.ps)
        return;
    const u32 r_end = min(v.ps, r_begin + slice_rows);
    const int n = g.n;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int i0[NG], ne[NG];
#pragma unroll
    for (int h = 0; h < NG; ++h) {
        i0[h] = (int(gset) * NG + h) * 8;
        ne[h] = max(0, min(8, n - i0[h]));
    }

    // tables of parts i0..i0+7 of each group (coefficient 0 past n: those
    // entries are 0 and nothing is stored for them); wave w builds T_m for
    // m-1 = w mod 4
#pragma unroll
    for (int h = 0; h < NG; ++h) {
        u32 idw[2] = {0, 0};
        for (int e = 0; e < ne[h]; ++e)
            idw[e >> 2] |= u32(ids[u64(s) * u64(n) + u64(i0[h] + e)]) << (8 * (e & 3));
        u32 coef[2] = {idw[0], idw[1]};
#pragma unroll
        for (int m = 1; m < K; ++m) {
            if ((m - 1) % 4 == wave) {
                u32 basis[8][2];
                make_basis<2>(basis, coef);
                build_table<2, 64>(tbl[h] + (m - 1) * TB, basis, lane);
            }
            coef[0] = gf_mul_packed(coef[0], idw[0]);
            coef[1] = gf_mul_packed(coef[1], idw[1]);
        }
    }
    __syncthreads();

    const bool aligned =
        ((reinterpret_cast<uintptr_t>(v.blk) | reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 15) == 0;
    for (u32 r0 = r_begin + u32(wave) * 1024u + 16u * u32(lane); r0 < r_end; r0 += STEP_ROWS) {
        // 16 rows = 16k bytes of the block (zero past B), read once for all
        // NG groups
        u32 d[4 * K];
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
                for (int c = 0; c < 4; ++c) {
                    const u64 p = off + 4 * q + c;
                    if (p < v.B)
                        x |= u32(v.blk[p]) << (8 * c);
                }
                d[q] = x;
            }
        }
        u32 tdep = 0;  // 0 at run time; orders each row group's lookups after the previous one
#pragma unroll
        for (int h = 0; h < NG; ++h) {
            // four groups of 4 rows: lookups + XOR, then 4 rows x 8 bytes
            // are transposed into 4 bytes of each of the 8 parts
            u32 out[8][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                u32 row[4][2];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int p0 = (4 * q + rr) * K;
                    const u32 rep = __builtin_amdgcn_perm(0u, d[p0 >> 2], 0x01010101u * u32(p0 & 3));
                    row[rr][0] = rep;
                    row[rr][1] = rep;
#pragma unroll
                    for (int m = 1; m < K; ++m) {
                        const int p = p0 + m;
                        // (| tdep: no common subexpression across groups,
                        // which would keep 16 (k-1) extracted bytes live)
                        const u32 byte = ((d[p >> 2] | tdep) >> (8 * (p & 3))) & 0xFFu;
                        const uint2 t = *reinterpret_cast<const uint2 *>(tbl[h] + tdep + (m - 1) * TB + byte * 8);
                        row[rr][0] ^= t.x;
                        row[rr][1] ^= t.y;
                    }
                }
#pragma unroll
                for (int w = 0; w < 2; ++w)
                    transpose4(row[0][w], row[1][w], row[2][w], row[3][w], out[4 * w][q], out[4 * w + 1][q],
                               out[4 * w + 2][q], out[4 * w + 3][q]);
                // without this the compiler hoists all 16 rows' lookups up
                // front and holds 32 (k-1) results in VGPRs
                if constexpr (K > 4)
                    asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(out[0][q]));
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i < ne[h]) {
                    u8 *dst = v.parts + u64(i0[h] + i) * v.pitch + r0;
                    if (aligned && r0 + 16 <= v.ps) {
                        store16(dst, out[i][0], out[i][1], out[i][2], out[i][3], false);
                    } else {
                        for (int c = 0; c < 16 && r0 + c < v.ps; ++c)
                            dst[c] = u8(out[i][c >> 2] >> (8 * (c & 3)));
                    }
                }
            }
        }
    }
}

// Fused encode + XXH64 for the part-group shapes (2 <= k <= 16, any n):
// a workgroup = (stripe, group of 16 parts) walks the stripe's rows in
// order with NE encoder waves and one hash wave.  Encoder lane = 4
// consecutive rows per chunk (k dwords of the block; CR = 256 NE rows per
// chunk): the packed tables T_m[x] = (x_{16g}^m x, ..., x_{16g+15}^m x),
// 16-byte entries, give a row's term for all 16 parts per ds_read_b128;
// 4 rows x 16 parts are transposed into one dword of 4 rows per part, stored
// to HBM (a wave writes 256 contiguous bytes of a part per instruction) and
// into an LDS exchange.  The hash wave (lane = 4 part + a) copies chunk c's
// words to registers and folds them while the encoders produce chunk c+1
// (two barriers per chunk): XXH64 is serial over a
// part's rows (crt/xxhash.c:791-810), so a stripe must be walked in order by
// one workgroup, and the parts are never read back (the two-pass form
// re-read them: W1 PMC traffic 1.57x).  The group workgroups of a stripe
// sit on one XCD (b mod 8) and share its block's lines in L2.
// PF: chunks of block loads in flight per encoder lane (1: the next chunk's
// loads issue after this chunk's lookups; 2: two register sets rotate, so
// a chunk's loads have two chunk periods to arrive).
// NKFS_WW_HPRIO (experiment builds): the hash wave's s_setprio level
#ifndef NKFS_WW_HPRIO
#define NKFS_WW_HPRIO 0
#endif
template <int K, int NE, int PF>
__global__ __launch_bounds__(64 * (NE + 1), 2) void k_encode_wide_ws(nkfs_geom g, const u8 *ids, u64 *digests,
                                                                  u32 ngroups)
{
    constexpr int CR = 256 * NE;   // rows per chunk
    constexpr int SP = CR + 32;    // exchange bytes per part (+32: the hash lanes' reads spread over the banks)
    constexpr int TB = 256 * 16;   // bytes per packed table
    constexpr int RPC = CR / 32;   // XXH64 rounds per chain per chunk
    __shared__ __attribute__((aligned(16))) u8 tbl[(K - 1) * TB];
    // single-buffered exchange: two barriers per chunk (the hash wave copies
    // its words to registers between them); double-buffered, a workgroup
    // needs 79 KiB at k = 12 and the CU keeps only one resident
    __shared__ __attribute__((aligned(16))) u8 xbuf[16 * SP];

    const u32 b = blockIdx.x;
    const u32 grp = (b >> 3) % ngroups;
    const u32 s = (b >> 3) / ngroups * 8 + (b & 7);
    if (s >= g.nstripes)
        return;  // the whole workgroup
    const Stripe v = stripe_at(g, s);
    const int n = g.n;
    const int p0 = int(grp) * 16, np = min(16, n - p0);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const u32 nch = (v.ps + CR - 1) / CR;
    if (!nch)
        return;

    if (wave < NE) {
        // ------------------------------------------------------ encoder wave
        const u32 rbase = u32(wave) * 256u + 4u * u32(lane);  // this lane's first row in every chunk
        const bool aligned =
            ((reinterpret_cast<uintptr_t>(v.blk) | reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 15) == 0;
        u32 d[PF][K];  // 4 rows x K bytes per register set
        auto load_task = [&](u32 (&x)[K], u32 r0) {
            const u64 off = u64(r0) * K;
            if (aligned && off + 4 * K <= v.B) {
                const u32 *src = reinterpret_cast<const u32 *>(v.blk + off);
#pragma unroll
                for (int q = 0; q < K; ++q)
                    x[q] = src[q];
            } else {
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    u32 y = 0;
                    for (int e = 0; e < 4; ++e) {
                        const u64 p = off + 4 * q + e;
                        if (p < v.B)
                            y |= u32(v.blk[p]) << (8 * e);
                    }
                    x[q] = y;
                }
            }
        };
#pragma unroll
        for (int p = 0; p < PF; ++p)  // first chunks requested before the table build
            if (rbase + u32(p) * CR < v.ps)
                load_task(d[p], rbase + u32(p) * CR);
        // tables T_m, m = 1..K-1, of the group's parts, split over the
        // encoder waves (coefficient 0 past n: nothing is stored for those)
        u32 idw[4] = {0, 0, 0, 0};
        for (int e = 0; e < np; ++e)
            idw[e >> 2] |= u32(ids[u64(s) * u64(n) + u64(p0 + e)]) << (8 * (e & 3));
        u32 coef[4] = {idw[0], idw[1], idw[2], idw[3]};
#pragma unroll 1
        for (int m = 1; m < K; ++m) {
            if ((m - 1) % NE == wave) {
                u32 basis[8][4];
                make_basis<4>(basis, coef);
                build_table16(tbl + (m - 1) * TB, basis, lane);
            }
#pragma unroll
            for (int w = 0; w < 4; ++w)
                coef[w] = gf_mul_packed(coef[w], idw[w]);
        }
        __syncthreads();

        auto chunk = [&](u32 (&d)[K], u32 c) {
            const u32 r0 = c * CR + rbase;
            if (r0 < v.ps) {
                // rows r0..r0+3: the m = 0 term is the byte itself (x^0 = 1)
                u32 rows[4][4];
                u32 tdep = 0;  // 0 at run time: one row's lookups in flight at a time
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int pb = rr * K;
                    const u32 rep = __builtin_amdgcn_perm(0u, d[pb >> 2], 0x01010101u * u32(pb & 3));
                    uint4 e = make_uint4(rep, rep, rep, rep);
#pragma unroll
                    for (int m = 1; m < K; ++m) {
                        const int p = pb + m;
                        const u32 byte = (d[p >> 2] >> (8 * (p & 3))) & 0xFFu;
                        const uint4 t = *reinterpret_cast<const uint4 *>(tbl + tdep + (m - 1) * TB + byte * 16);
                        e.x ^= t.x;
                        e.y ^= t.y;
                        e.z ^= t.z;
                        e.w ^= t.w;
                    }
                    rows[rr][0] = e.x;
                    rows[rr][1] = e.y;
                    rows[rr][2] = e.z;
                    rows[rr][3] = e.w;
                    asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(e.x), "v"(e.y), "v"(e.z), "v"(e.w));
                }
                if (r0 + PF * CR < v.ps)
                    load_task(d, r0 + PF * CR);  // chunk c + PF's rows in flight under what follows
                // 4 rows x 16 parts -> 16 parts x 4 rows (one dword each)
                u32 out[16];
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    transpose4(rows[0][w], rows[1][w], rows[2][w], rows[3][w], out[4 * w], out[4 * w + 1],
                               out[4 * w + 2], out[4 * w + 3]);
                u8 *xb = xbuf + rbase;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (i < np) {
                        u8 *dst = v.parts + u64(p0 + i) * v.pitch + r0;
                        if (aligned && r0 + 4 <= v.ps) {
                            *reinterpret_cast<u32 *>(dst) = out[i];
                        } else {
                            for (u32 e = 0; e < 4 && r0 + e < v.ps; ++e)
                                dst[e] = u8(out[i] >> (8 * e));
                        }
                        *reinterpret_cast<u32 *>(xb + i * SP) = out[i];
                    }
                }
            }
            __syncthreads();  // chunk c is in the exchange
            __syncthreads();  // the hash wave has copied it
        };
        for (u32 c = 0; c < nch; c += PF) {
            chunk(d[0], c);
            if constexpr (PF == 2)
                if (c + 1 < nch)
                    chunk(d[PF - 1], c + 1);
        }
        return;
    }

    // ---------------------------------------------------------------- hash wave
    if (NKFS_WW_HPRIO)
        __builtin_amdgcn_s_setprio(NKFS_WW_HPRIO);
    const int hi = lane >> 2, ha = lane & 3;  // part p0 + hi, accumulator ha
    const bool hlane = hi < np;
    const u32 nst = v.ps >> 5;  // whole 32-byte stripes of every part
    u64 acc = xxh_acc_init(ha, 0);
    const int xoff = hi * SP + 8 * ha;
    static_assert(RPC <= 32, "hash words staged in registers");
    __syncthreads();  // tables built
    u64 tw[4] = {0, 0, 0, 0};  // the tail words of the last chunk (read before it is overwritten)
    const u32 left = v.ps & 31;
    for (u32 c = 0; c < nch; ++c) {
        __syncthreads();  // chunk c is in the exchange
        u64 hw[RPC];
        int hv = 0;
        if (hlane) {
            const u8 *src = xbuf + xoff;
            const int lft = int(nst) - int(c * RPC);
            hv = lft < 0 ? 0 : (lft > RPC ? RPC : lft);
#pragma unroll
            for (int r = 0; r < RPC; ++r)
                hw[r] = *reinterpret_cast<const u64 *>(src + 32 * r);
            if (c == nch - 1 && left) {
                const u8 *t = xbuf + hi * SP + (nst * 32 - c * CR);
#pragma unroll
                for (u32 e = 0; e < 32; ++e)
                    if (e < left)
                        tw[e >> 3] |= u64(t[e]) << (8 * (e & 7));
            }
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
    const int base = lane & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    if (hlane && ha == 0) {
        u64 h = v.ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
        h += v.ps;
        digests[u64(s) * u64(n) + u64(p0 + hi)] = xxh_tail_regs(h, tw, left);
    }
}

// Decode, 2 <= k <= 16: one workgroup (4 waves) per (stripe, row slice).
// Survivor c's table U_c[x] = (W[c][0] x, ..., W[c][15] x) packs the
// products for all k output bytes of a row, so a row costs k ds_read_b128 +
// XORs.  A wave rebuilds 1,024 rows per step in four runs of 256 rows: lane
// l takes rows 4l..4l+3 of a run (one dword of each survivor part; the
// step's 4k loads are issued up front), packs them to 4k block bytes, and
// the run's 256k contiguous bytes go through a per-wave LDS stage so that
// every store instruction writes one contiguous 1 KiB run (direct stores
// from the lanes would stride 4k bytes apart: PMC showed 2x the write
// traffic for the 16k-byte stride of a 16-rows-per-lane form).  The
// selection and W come from k_decode_prep (work: k slot numbers, then W
// row-major).
template <int K>
__global__ __launch_bounds__(256) void k_decode_wide(nkfs_geom g, const u8 *work, const int32_t *status,
                                                     u32 nslices, u32 slice_rows)
{
    constexpr int TB = 256 * 16;   // bytes per packed table
    constexpr int SB = 256 * K;    // stage bytes per wave: one run of 256 rows
    constexpr int NST = (SB + 1023) / 1024;  // 1 KiB store instructions per run
    __shared__ __attribute__((aligned(16))) u8 tbl[K * TB];
    __shared__ __attribute__((aligned(16))) u8 stage[4][SB];
    const u32 b = blockIdx.x;
    const u32 slice = (b >> 3) % nslices;
    const u32 s = (b >> 3) / nslices * 8 + (b & 7);
    if (s >= g.nstripes || (status && status[s]))
        return;
    const Stripe v = stripe_at(g, s);  // g.blocks = the output, g.n = slots per stripe
    const u32 r_begin = slice * slice_rows;
    if (r_begin >= v.ps)
        return;
    const u32 r_end = min(v.ps, r_begin + slice_rows);
    const u8 *wk = work + u64(s) * u64(K + K * K);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (c % 4 == wave) {
            u32 row[4] = {0, 0, 0, 0};
            for (int m = 0; m < K; ++m)
                row[m >> 2] |= u32(wk[K + c * K + m]) << (8 * (m & 3));
            u32 basis[8][4];
            make_basis<4>(basis, row);
            build_table16(tbl + c * TB, basis, lane);
        }
    }
    const u8 *src[K];
#pragma unroll
    for (int c = 0; c < K; ++c)
        src[c] = v.parts + u64(wk[c]) * v.pitch;
    __syncthreads();

    u8 *out = const_cast<u8 *>(v.blk);
    u8 *stg = stage[wave];
    const bool pal = ((reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 3) == 0;
    const bool oal = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    // wave-uniform loop: a middle slice holds whole steps (slice_rows is a
    // multiple of 4,096), so rows past r_end exist only past ps, whose bytes
    // lie past B and are never stored
    for (u32 rw = r_begin + u32(wave) * 1024u; rw < r_end; rw += STEP_ROWS) {
        u32 p[4][K];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32 r0 = rw + 256u * q + 4u * lane;
#pragma unroll
            for (int c = 0; c < K; ++c) {
                if (pal && r0 + 4 <= v.ps) {
                    p[q][c] = *reinterpret_cast<const u32 *>(src[c] + r0);
                } else {
                    u32 x = 0;
                    for (int e = 0; e < 4; ++e)
                        if (r0 + e < v.ps)
                            x |= u32(src[c][r0 + e]) << (8 * e);
                    p[q][c] = x;
                }
            }
        }
        u32 tdep = 0;  // 0 at run time; orders each run's lookups after the previous run
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            u32 row[4][4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    row[rr][w] = 0;
#pragma unroll
                for (int c = 0; c < K; ++c) {
                    const u32 x = (p[q][c] >> (8 * rr)) & 0xFFu;
                    const uint4 t = *reinterpret_cast<const uint4 *>(tbl + tdep + c * TB + x * 16);
                    row[rr][0] ^= t.x;
                    row[rr][1] ^= t.y;
                    row[rr][2] ^= t.z;
                    row[rr][3] ^= t.w;
                }
            }
            // rows rw + 256q + 4l .. +3 = run bytes [4K l, 4K l + 4K)
#pragma unroll
            for (int d = 0; d < K; ++d)
                *reinterpret_cast<u32 *>(stg + 4 * K * lane + 4 * d) = pack_dword<K, 4>(&row[0][0], d);
            __builtin_amdgcn_wave_barrier();
            const u64 base = u64(rw + 256u * q) * K;
#pragma unroll
            for (int j = 0; j < NST; ++j) {
                const u32 bo = 1024u * j + 16u * lane;
                if (bo < u32(SB)) {
                    const uint4 t = *reinterpret_cast<const uint4 *>(stg + bo);
                    const u64 off = base + bo;
                    if (oal && off + 16 <= v.B) {
                        store16(out + off, t.x, t.y, t.z, t.w, false);
                    } else if (off < v.B) {
                        const u32 tw[4] = {t.x, t.y, t.z, t.w};
                        for (int e = 0; e < 16 && off + e < v.B; ++e)
                            out[off + e] = u8(tw[e >> 2] >> (8 * (e & 3)));
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(row[0][0]));
        }
    }
}

// row slices so that the grid has about `min_wgs` workgroups (never a slice
// below one step): returns slices, sets *rows
u64 slices_for(u64 base, u32 ps_max, int cus, u64 *rows)
{
    const u64 steps = (u64(ps_max) + STEP_ROWS - 1) / STEP_ROWS;  // >= 1
    const u64 min_wgs = u64(cus > 0 ? cus : 256) * 8;
    u64 ns = (min_wgs + base - 1) / base;
    ns = ns > steps ? steps : ns < 1 ? 1 : ns;
    *rows = (steps + ns - 1) / ns * STEP_ROWS;
    ns = (u64(ps_max) + *rows - 1) / *rows;
    return ns < 1 ? 1 : ns;
}

}  // namespace

// Encode (no hash) a uniform or ragged batch with 2 <= k <= 16, any n <= 255.
// Workgroups: ceil(nstripes / 8) * 8 stripes x ceil(n / 16) group pairs x row
// slices, the slices chosen so that the grid has at least `min_wgs`
// workgroups when the stripes are big enough to be cut.  -ENOSYS for k > 16.
extern "C" int nkfs_wide_encode(const nkfs_geom *g, const uint8_t *ids, int cus, hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > WIDE_MAX_K || g->n < k || g->n > 255)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    // part groups of 8; a workgroup takes two groups (one read of the block
    // for 16 parts) when n > 8 and the pair's tables and registers still
    // leave 3 waves per SIMD (k <= 14; profiles/r02/wide_kbench.txt: N16K12
    // encode 4.61 -> 4.78 TB/s, N20K16 at 2 waves per SIMD 3.57 -> 3.11)
    const int NG = g->n > 8 && k <= 14 ? 2 : 1;
    const u64 ngroups = (u64(g->n + 7) / 8 + NG - 1) / NG;
    const u64 base = (u64(g->nstripes) + 7) / 8 * 8 * ngroups;
    u64 slice_rows = 0;
    const u64 nslices = slices_for(base, ps_max, cus, &slice_rows);
    const u64 grid = base * nslices;
    if (grid > 0x7FFFFFFFull || slice_rows > 0xFFFFFFFFull)
        return -EINVAL;
    const dim3 gd = dim3(u32(grid)), bd = dim3(256);
    switch (k) {
#define NKFS_K(KK)                                                                                       \
    case KK:                                                                                             \
        if (NG == 2)                                                                                     \
            hipLaunchKernelGGL((k_encode_wide<KK, 2>), gd, bd, 0, st, *g, ids, u32(ngroups), u32(nslices), \
                               u32(slice_rows));                                                         \
        else                                                                                             \
            hipLaunchKernelGGL((k_encode_wide<KK, 1>), gd, bd, 0, st, *g, ids, u32(ngroups), u32(nslices), \
                               u32(slice_rows));                                                         \
        break;
        NKFS_K(2)
        NKFS_K(3)
        NKFS_K(4)
        NKFS_K(5)
        NKFS_K(6)
        NKFS_K(7)
        NKFS_K(8)
        NKFS_K(9)
        NKFS_K(10)
        NKFS_K(11)
        NKFS_K(12)
        NKFS_K(13)
        NKFS_K(14)
        NKFS_K(15)
        NKFS_K(16)
#undef NKFS_K
    default:
        return -ENOSYS;
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Fused encode + XXH64 of every part, 2 <= k <= 16, any n <= 255: one
// workgroup per (stripe, group of 16 parts) walking the stripe in order.
// For batches that fill the chip (the caller decides); -ENOSYS outside the
// shapes.
extern "C" int nkfs_wide_ws_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > WIDE_MAX_K || g->n < k || g->n > 255 || !digests)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    const u64 ngroups = (u64(g->n) + 15) / 16;
    const u64 grid = (u64(g->nstripes) + 7) / 8 * 8 * ngroups;
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    const dim3 gd = dim3(u32(grid));
    // chunks of loads in flight per encoder lane: struct nkfs_tune.enc_ws_prefetch
    const int pf = nkfs_tune_now().enc_ws_prefetch;
    switch (k) {
#define NKFS_K(KK, NE)                                                                                    \
    case KK:                                                                                              \
        if (pf >= 2)                                                                                      \
            hipLaunchKernelGGL((k_encode_wide_ws<KK, NE, 2>), gd, dim3(64 * (NE + 1)), 0, st, *g, ids, digests, \
                               u32(ngroups));                                                             \
        else                                                                                              \
            hipLaunchKernelGGL((k_encode_wide_ws<KK, NE, 1>), gd, dim3(64 * (NE + 1)), 0, st, *g, ids, digests, \
                               u32(ngroups));                                                             \
        break;
        // three encoder waves + the hash wave = 256 threads: a 320-thread
        // workgroup (four encoder waves) stayed alone on its CU (SQ: ~5
        // resident waves per CU) whatever its LDS and VGPRs
        NKFS_K(2, 3)
        NKFS_K(3, 3)
        NKFS_K(4, 3)
        NKFS_K(5, 3)
        NKFS_K(6, 3)
        NKFS_K(7, 3)
        NKFS_K(8, 3)
        NKFS_K(9, 3)
        NKFS_K(10, 3)
        NKFS_K(11, 3)
        NKFS_K(12, 3)
        NKFS_K(13, 3)
        NKFS_K(14, 3)
        NKFS_K(15, 3)
        NKFS_K(16, 3)
#undef NKFS_K
    default:
        return -ENOSYS;
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Decode a uniform or ragged batch with 2 <= k <= 16 from the plan
// k_decode_prep left in `work` (stripes with status != 0 are skipped).
extern "C" int nkfs_wide_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, int cus,
                                hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > WIDE_MAX_K)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    const u64 base = (u64(g->nstripes) + 7) / 8 * 8;
    u64 slice_rows = 0;
    const u64 nslices = slices_for(base, ps_max, cus, &slice_rows);
    const u64 grid = base * nslices;
    if (grid > 0x7FFFFFFFull || slice_rows > 0xFFFFFFFFull)
        return -EINVAL;
    const dim3 gd = dim3(u32(grid)), bd = dim3(256);
    switch (k) {
#define NKFS_K(KK)                                                                                       \
    case KK:                                                                                             \
        hipLaunchKernelGGL(k_decode_wide<KK>, gd, bd, 0, st, *g, work, status, u32(nslices), u32(slice_rows)); \
        break;
        NKFS_K(2)
        NKFS_K(3)
        NKFS_K(4)
        NKFS_K(5)
        NKFS_K(6)
        NKFS_K(7)
        NKFS_K(8)
        NKFS_K(9)
        NKFS_K(10)
        NKFS_K(11)
        NKFS_K(12)
        NKFS_K(13)
        NKFS_K(14)
        NKFS_K(15)
        NKFS_K(16)
#undef NKFS_K
    default:
        return -ENOSYS;
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
