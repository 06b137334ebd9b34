// nk8_bign.hip -- decode for k > 8 with replicated product tables: every
// lookup of a wave lands in its own LDS bank slot.
//
// Reference arithmetic: crt/nk8.c:552-582 -- block[j*k+m] = XOR_c part_c[j]
// W[c][m], W the inverse of the first k distinct survivors' Vandermonde rows
// (k_decode_prep leaves the selection and W in `work`).
//
// k_decode_big / k_decode_wide look up packed 16-byte products U_c[x] =
// (W[c][m0] x, ..., W[c][m0+15] x) with one ds_read_b128 per (row, survivor).
// The index x is a data byte, so the 16 lanes of a b128 lane group pick
// their 16-byte slots of a bank row at random: 3.07 passes per group on
// average instead of 1 (the expected fullest of 16 random bins), and the
// kernels are bound by LDS cycles (profiles/r03/sq_w2_summary.txt: LDS
// active 86 % with an 85 % conflict share).  Here the tables are laid out so
// that lane l's entries always sit in bank slot l & 15 (MODE 2) or in one of
// two slot sets by lane parity (MODE 1):
//
//  MODE 2  nibble tables, 16 replicas: U_c[x] = L_c[x & 15] ^ H_c[x >> 4];
//          L_c[v] at c*4096 + v*256 + slot, H_c[v] at 64 KiB + v*4096 +
//          c*256 + slot (slot = 16*(lane & 15)).  Both addresses come from
//          one v_perm (byte q of the survivors' dword next to the slot byte)
//          and one AND / AND-OR; two conflict-free lookups (8 LDS cycles per
//          wave for 16 products x 64 rows) instead of one random one (~12).
//  MODE 1  byte tables, 2 replicas: U_c[x] at c*8192 + x*32 + 16*(lane & 1)
//          (v_perm + shift); 8 lanes per slot set: 2.6 passes per group.
//  MODE 0  byte tables, 1 copy (64 KiB), the same loop: the A/B baseline.
//
// Workgroup = (stripe, group of 16 output columns, slice of 2,048*T rows), 8
// waves; lane = 4 consecutive rows: one dword of each of a chunk's 16
// survivor parts (coalesced, 256 B per wave instruction) feeds its 4 rows
// directly (v_perm picks the row's byte), so no LDS stage is needed.  The
// groups of a (stripe, slice) run back to back on one XCD (workgroup b on XCD
// b mod 8), so the rows' output lines complete in its L2.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nk8_dev.h"
#include "nkfs_internal.h"

using namespace nkfs;
using namespace nkfs::dev;

namespace {

constexpr int BN_T = 4;                        // row quads per lane per slice
constexpr int BN_WAVES = 8;
constexpr u32 BN_ROWS = 64u * BN_WAVES * 4u * BN_T;   // rows per workgroup slice (8,192)

template <int MODE>
struct BnLayout {
    static constexpr u32 bytes = MODE == 0 ? 65536u : 131072u;
};

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); the compiler
// emits two v_xor_b32 for it
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ u32 load4_any(const u8 *p, u32 left)
{
    u32 w = 0;
#pragma unroll
    for (u32 e = 0; e < 4; ++e) {
        const u32 b = p[e < left ? e : left - 1];
        w |= (e < left ? b : 0u) << (8 * e);
    }
    return w;
}

template <int MODE, bool PAL>
__global__ __launch_bounds__(64 * BN_WAVES, 1) void k_decode_bign(nkfs_geom g, const u8 *work, const int32_t *status,
                                                                 u32 ngroups, u32 nslices)
{
    __shared__ __attribute__((aligned(16))) u8 tbl[BnLayout<MODE>::bytes];
    const u32 b = blockIdx.x;
    const u32 loc = b >> 3;
    const u32 h = loc % ngroups;
    const u32 slice = (loc / ngroups) % nslices;
    const u32 s = (loc / ngroups / nslices) * 8 + (b & 7);
    if (s >= g.nstripes || (status && status[s]))
        return;  // the whole workgroup
    const Stripe v = stripe_at(g, s);  // g.blocks = the output, g.n = slots per stripe
    const u32 r_begin = slice * BN_ROWS;
    if (r_begin >= v.ps)
        return;
    const int k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const u8 *wk = work + u64(s) * u64(k + k * k);

    // the slot byte of this lane's table entries
    // (MODE 2: byte 2 = 1 puts the high-nibble tables' addresses at 64 KiB)
    const u32 slotv = MODE == 2 ? 0x10000u | u32(lane & 15) * 16u : MODE == 1 ? u32(lane & 1) * 128u : 0u;

    uint4 acc[BN_T][4];
#pragma unroll
    for (int t = 0; t < BN_T; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[t][q] = make_uint4(0, 0, 0, 0);

    const int nch = (k + 15) / 16;
    for (int cc = 0; cc < nch; ++cc) {
        __syncthreads();  // the previous chunk's lookups are done
        // ---- tables of survivors 16cc .. 16cc+15 for output columns 16h ..
        if constexpr (MODE == 2) {
            // 32 (kind, column) pairs x 4 wave writes of 4 value rows x 16
            // replicas; wave w takes pairs w, w + 8, w + 16, w + 24
#pragma unroll 1
            for (int pi = wave; pi < 32; pi += BN_WAVES) {
                const int kind = pi >> 4, j = pi & 15, c = 16 * cc + j;
                u32 row[4] = {0, 0, 0, 0};
                if (c < k)
                    for (int e = 0; e < 16; ++e) {
                        const int m = 16 * int(h) + e;
                        if (m < k)
                            row[e >> 2] |= u32(wk[k + c * k + m]) << (8 * (e & 3));
                    }
                u32 basis[8][4];
                make_basis<4>(basis, row);
#pragma unroll
                for (int it = 0; it < 4; ++it) {
                    const int vv = 4 * it + (lane >> 4);
                    u32 e4[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb)
                        if ((vv >> bb) & 1)
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                e4[w] ^= basis[4 * kind + bb][w];
                    const u32 addr = kind == 0 ? u32(j) * 4096u + u32(vv) * 256u + u32(lane & 15) * 16u
                                               : 65536u + u32(vv) * 4096u + u32(j) * 256u + u32(lane & 15) * 16u;
                    *reinterpret_cast<uint4 *>(tbl + addr) = make_uint4(e4[0], e4[1], e4[2], e4[3]);
                }
            }
        } else {
            // byte tables: column j, entries x = 32 m + (lane >> (MODE)) ...;
            // MODE 1: replica lane & 1, 32 entries per wave write; MODE 0:
            // 64 entries per wave write
            constexpr int EPW = MODE == 1 ? 32 : 64;  // entries per wave write
            constexpr int NW = 256 / EPW;             // wave writes per column
#pragma unroll 1
            for (int j = wave; j < 16; j += BN_WAVES) {
                const int c = 16 * cc + j;
                u32 row[4] = {0, 0, 0, 0};
                if (c < k)
                    for (int e = 0; e < 16; ++e) {
                        const int m = 16 * int(h) + e;
                        if (m < k)
                            row[e >> 2] |= u32(wk[k + c * k + m]) << (8 * (e & 3));
                    }
                u32 basis[8][4];
                make_basis<4>(basis, row);
                const int x0 = MODE == 1 ? (lane >> 1) : lane;
                constexpr int LB = MODE == 1 ? 5 : 6;  // low bits fixed per lane
                u32 hv[4] = {0, 0, 0, 0};
#pragma unroll
                for (int bb = 0; bb < LB; ++bb)
                    if ((x0 >> bb) & 1)
#pragma unroll
                        for (int w = 0; w < 4; ++w)
                            hv[w] ^= basis[bb][w];
#pragma unroll
                for (int mi = 0; mi < NW; ++mi) {
                    if (mi) {
                        const int bit = __builtin_ctz(mi);
#pragma unroll
                        for (int w = 0; w < 4; ++w)
                            hv[w] ^= basis[LB + bit][w];
                    }
                    const int x = x0 + EPW * (mi ^ (mi >> 1));
                    const u32 addr = MODE == 1 ? u32(j) * 8192u + u32(x) * 32u + u32(lane & 1) * 16u
                                               : u32(j) * 4096u + u32(x) * 16u;
                    *reinterpret_cast<uint4 *>(tbl + addr) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
                }
            }
        }
        __syncthreads();

        // ---- survivor part bases of the chunk (zero table past k)
        const u8 *src[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int c = 16 * cc + j;
            src[j] = v.parts + (c < k ? u64(wk[c]) * v.pitch : 0);
        }
        auto load = [&](u32 (&d)[16], int t) {
            const u32 r4 = r_begin + (u32(t) * 64u * BN_WAVES + u32(tid)) * 4u;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const bool ok = 16 * cc + j < k && r4 < v.ps;
                if constexpr (PAL)
                    d[j] = ok ? *reinterpret_cast<const u32 *>(src[j] + r4) : 0u;
                else
                    d[j] = ok ? load4_any(src[j] + r4, v.ps - r4) : 0u;
            }
        };
        // quad t's dwords in dc, quad t+1's loads in flight in dn; the
        // quads' accumulators rotate by one per quad (back in order after
        // BN_T), so the loop is not unrolled and every index stays static
        u32 dc[16], dn[16];
        load(dc, 0);
#pragma unroll 1
        for (int t = 0; t < BN_T; ++t) {
            if (t + 1 < BN_T)
                load(dn, t + 1);
            // tdep (0 at run time) chains each survivor's lookups behind the
            // previous survivor's XORs: unchained, the compiler hoists all
            // 64 (128) lookups of a quad and spills
            u32 tdep = 0;
            uint4 a4[4] = {acc[0][0], acc[0][1], acc[0][2], acc[0][3]};
            if constexpr (MODE == 2) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const u32 sv = slotv + tdep;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        // P = 1 << 16 | (byte q of the survivor dword) << 8 | slot
                        const u32 P = __builtin_amdgcn_perm(dc[j], sv, 0x0C020000u | (u32(4 + q) << 8));
                        const uint4 a = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + (P & 0x0FFFu));
                        const uint4 c2 = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 256u + (P & 0x1F0FFu));
                        a4[q].x = xor3(a4[q].x, a.x, c2.x);
                        a4[q].y = xor3(a4[q].y, a.y, c2.y);
                        a4[q].z = xor3(a4[q].z, a.z, c2.z);
                        a4[q].w = xor3(a4[q].w, a.w, c2.w);
                    }
                    asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
                }
            } else {
                // survivors in pairs: one three-input XOR per word folds both lookups
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    const u32 sv = slotv + tdep;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const u32 sel = 0x0C0C0000u | (u32(4 + q) << 8);
                        const u32 P0 = __builtin_amdgcn_perm(dc[j], sv, sel), P1 = __builtin_amdgcn_perm(dc[j + 1], sv, sel);
                        constexpr u32 CS = MODE == 1 ? 8192u : 4096u;  // column stride
                        constexpr int SH = MODE == 1 ? 3 : 4;          // x << 8 -> x * 32 (+ replica) / x * 16
                        const uint4 a = *reinterpret_cast<const uint4 *>(tbl + u32(j) * CS + (P0 >> SH));
                        const uint4 c2 = *reinterpret_cast<const uint4 *>(tbl + u32(j + 1) * CS + (P1 >> SH));
                        a4[q].x = xor3(a4[q].x, a.x, c2.x);
                        a4[q].y = xor3(a4[q].y, a.y, c2.y);
                        a4[q].z = xor3(a4[q].z, a.z, c2.z);
                        a4[q].w = xor3(a4[q].w, a.w, c2.w);
                    }
                    asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
                }
            }
#pragma unroll
            for (int i = 0; i + 1 < BN_T; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[i][q] = acc[i + 1][q];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                acc[BN_T - 1][q] = a4[q];
#pragma unroll
            for (int j = 0; j < 16; ++j)
                dc[j] = dn[j];
        }
    }

    // row r's bytes 16h..16h+15 at r*k + 16h (fewer in the last group;
    // nothing at or past B)
    u8 *out = const_cast<u8 *>(v.blk);
    const uintptr_t oa = reinterpret_cast<uintptr_t>(out);
#pragma unroll
    for (int t = 0; t < BN_T; ++t) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32 r = r_begin + (u32(t) * 64u * BN_WAVES + u32(tid)) * 4u + u32(q);
            if (r >= v.ps)
                continue;
            const u64 rb = u64(r) * u64(k);
            const u64 off = rb + 16u * h;
            const u32 tw[4] = {acc[t][q].x, acc[t][q].y, acc[t][q].z, acc[t][q].w};
            const u64 lim = min(u64(v.B), rb + u64(k));  // this row's bytes
            if (off + 16 <= lim && ((oa + off) & 15) == 0) {
                store16(out + off, tw[0], tw[1], tw[2], tw[3], false);
            } else if (off + 16 <= lim && ((oa + off) & 3) == 0) {
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    *reinterpret_cast<u32 *>(out + off + 4 * w) = tw[w];
            } else {
#pragma unroll
                for (u32 c = 0; c < 16; ++c)
                    if (off + c < lim)
                        out[off + c] = u8(tw[c >> 2] >> (8 * (c & 3)));
            }
        }
    }
}

template <int MODE>
int launch_bign(const nkfs_geom *g, const uint8_t *work, const int32_t *status, u32 ngroups, u32 nslices, u64 grid,
                bool pal, hipStream_t st)
{
    if (pal)
        hipLaunchKernelGGL((k_decode_bign<MODE, true>), dim3(u32(grid)), dim3(64 * BN_WAVES), 0, st, *g, work, status,
                           ngroups, nslices);
    else
        hipLaunchKernelGGL((k_decode_bign<MODE, false>), dim3(u32(grid)), dim3(64 * BN_WAVES), 0, st, *g, work,
                           status, ngroups, nslices);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // namespace

// Decode a uniform or ragged batch with 2 <= k <= 254 from the plan
// k_decode_prep left in `work` (stripes with status != 0 are skipped), with
// table layout `mode` (0 byte, 1 byte x 2 replicas, 2 nibble x 16 replicas).
extern "C" int nkfs_bign_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, int mode,
                                hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > 254 || mode < 0 || mode > 2)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    if (u64(g->block_size) + 64u > 0x7FFFFFFFull)
        return -ENOSYS;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    const u64 ngroups = (u64(k) + 15) / 16;
    const u64 nslices = (u64(ps_max) + BN_ROWS - 1) / BN_ROWS;
    const u64 grid = (u64(g->nstripes) + 7) / 8 * 8 * ngroups * (nslices ? nslices : 1);
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    // dword survivor loads: uniform batches with 4-byte aligned parts and pitch
    const bool pal = !g->block_sizes && ((reinterpret_cast<uintptr_t>(g->parts) | g->part_pitch) & 3) == 0;
    const u32 ng = u32(ngroups), ns = u32(nslices ? nslices : 1);
    switch (mode) {
    case 0: return launch_bign<0>(g, work, status, ng, ns, grid, pal, st);
    case 1: return launch_bign<1>(g, work, status, ng, ns, grid, pal, st);
    default: return launch_bign<2>(g, work, status, ng, ns, grid, pal, st);
    }
}
