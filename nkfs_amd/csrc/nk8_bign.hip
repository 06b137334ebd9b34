// nk8_bign.hip -- decode for k > 8 without an LDS stage and with product
// tables whose lookups stay in their lanes' own bank slots.
//
// Reference arithmetic: crt/nk8.c:552-582 -- block[j*k+m] = XOR_c part_c[j]
// W[c][m], W the inverse of the first k distinct survivors' Vandermonde rows
// (k_decode_prep leaves the selection and W in `work`).
//
// k_decode_big / k_decode_wide look up packed 16-byte products U_c[x] =
// (W[c][m0] x, ..., W[c][m0+15] x) with one ds_read_b128 per (row, survivor)
// from a survivor stage in LDS.  The index x is a data byte, so the 16 lanes
// of a b128 lane group pick their 16-byte bank slots at random: 3.07 passes
// per group on average instead of 1 (the expected fullest of 16 random
// bins), and those kernels are bound by LDS cycles (profiles/r03/
// sq_w2_summary.txt: LDS active 86 % with an 85 % conflict share).
//
// Here a lane owns 4 consecutive rows: one dword of each of a chunk's CW
// survivor parts (coalesced buffer loads, 256 B per wave instruction) feeds
// its 4 rows directly -- v_perm places the row's byte next to the lane's
// slot byte, so the LDS address needs no shift or add.  Table layouts
// (struct nkfs_tune.dec_bign):
//
//  0  byte tables: U_c[x] at c*4096 + x*16 (64 KiB, CW = 16): random slots.
//  1  nibble tables, 16 replicas: U_c[x] = L_c[x & 15] ^ H_c[x >> 4], each
//     entry stored once per bank slot, lane l reading slot l & 15: every
//     lookup conflict-free (two per product instead of one random).
//     L_c[v] at c*4096 + v*256 + slot, H_c[v] 64 KiB higher (CW = 16, 128
//     KiB: one workgroup per CU).
//  2  the same nibble tables for CW = 8 survivors per chunk (64 KiB): two
//     workgroups per CU, H_c at 32 KiB.
//
// Workgroup = (stripe, group of 16 output columns, slice of ROWS rows);
// chunks of CW survivors: table build, then every row quad of the slice.
// The groups of a (stripe, slice) run back to back on one XCD (workgroup b
// on XCD b mod 8), so the rows' output lines complete in its L2.  For k <=
// 16 (one group) with k % 4 == 0 a row quad is 4k contiguous output bytes,
// written with dword stores.
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

// launch shape per table layout: survivors per chunk, table bytes, waves
// per workgroup, row quads per lane per slice and workgroups per CU
template <int MODE>
struct BnShape {
    static constexpr int CW = MODE == 2 ? 8 : 16;
    static constexpr u32 TBYTES = MODE == 1 ? 131072u : 65536u;
    static constexpr int WAVES = MODE == 1 ? 16 : 8;
    static constexpr int T = 2;
    static constexpr int PER_CU = MODE == 1 ? 1 : 2;
    static constexpr u32 ROWS = 64u * WAVES * 4u * T;   // 8,192 / 4,096 rows per slice
    static constexpr u32 HI = MODE == 2 ? 32768u : 0u;  // H_c offset by immediate (MODE 1: by the slot word)
};

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a release
// fence over all memory and waits for every load in flight (vmcnt(0)),
// which would drain the survivor prefetch at every table build.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); the compiler
// emits two v_xor_b32 for it
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// mask ? a : b per bit in one v_bitop3_b32 (operand truth tables S0 0xF0,
// S1 0xCC, S2 0xAA: (S2 & S0) | (~S2 & S1) = 0xE4); the compiler turns the
// C form into a v_cndmask on an SGPR lane mask (half rate)
__device__ __forceinline__ u32 mux3(u32 mask, u32 a, u32 b)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xE4" : "=v"(r) : "v"(a), "v"(b), "v"(mask));
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

// ONE: k <= CW, a single chunk: the workgroup builds its tables once and
// walks slices wi, wi + nwg, ... of its stripe (the next slice's first
// survivor loads in flight under the current one's last quad); otherwise
// one slice per workgroup (nwg = nslices), tables rebuilt per chunk.
template <int MODE, bool PAL, bool ONE>
__global__ __launch_bounds__(64 * BnShape<MODE>::WAVES, BnShape<MODE>::PER_CU) void k_decode_bign(
    nkfs_geom g, const u8 *work, const int32_t *status, u32 ngroups, u32 nslices, u32 nwg)
{
    using SH = BnShape<MODE>;
    constexpr int CW = SH::CW, WAVES = SH::WAVES, T = SH::T, NT = 64 * WAVES;
    constexpr bool NIB = MODE == 1 || MODE == 2;
    // MODE 4: byte tables in the diagonal layout -- entry x of survivor j at
    // x * 256 + j * 16, the chunk's 16 tables in the 16 bank slots of each x
    // row -- and lane l walks the survivors from (l & 15): the 16 lanes of a
    // b128 lane group read 16 distinct slots (MODE 0: random slots, ~3
    // passes per group)
    constexpr bool DIAG = MODE == 4;
    __shared__ __attribute__((aligned(16))) u8 tbl[SH::TBYTES];
    __shared__ __attribute__((aligned(16))) u32 wq[CW][4];  // a chunk's W rows, columns 16h ..
    __shared__ u32 wslot[CW];                               // a chunk's survivor slots

    const u32 b = blockIdx.x;
    const u32 loc = b >> 3;
    const u32 h = loc % ngroups;
    const u32 wi = (loc / ngroups) % nwg;
    const u32 s = (loc / ngroups / nwg) * 8 + (b & 7);
    if (s >= g.nstripes || (status && status[s]))
        return;  // the whole workgroup
    const Stripe v = stripe_at(g, s);  // g.blocks = the output, g.n = slots per stripe
    if (wi * SH::ROWS >= v.ps)
        return;
    const int k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const u8 *wk = work + u64(s) * u64(k + k * k);

    // the lane's slot byte (byte 0 of every table address); MODE 1 puts the
    // H tables 64 KiB up through byte 2 of the high lookups' slot word
    const u32 slot_lo = NIB ? u32(lane & 15) * 16u : 0u;
    const u32 slot_hi = slot_lo | (MODE == 1 ? 0x10000u : 0u);
    // DIAG: byte i of dslot[g] = the slot ((4 g + i + (lane & 15)) & 15) * 16
    u32 dslot[4];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
        u32 x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            x |= (((u32(4 * gq + i) + u32(lane & 15)) & 15u) << 4) << (8 * i);
        dslot[gq] = x;
    }

    uint4 acc[T][4];

    // CW*16 + CW bytes per chunk: item i < CW*16 is byte (i & 15) of chunk
    // row i >> 4 of W (columns 16h ..), the next CW the survivor slot
    // numbers (0 past k); thread tid fetches items tid and tid + NT one
    // chunk ahead, so a table build never waits for HBM.  The raw bytes and
    // their liveness are kept apart, so the loads stay in flight until the
    // next chunk's LDS write uses them.
    constexpr int NW = CW * 16, NI = NW + CW;
    auto wsrc = [&](int cc, int i, bool &live) -> const u8 * {
        if (i >= NW) {
            const int c = CW * cc + (i - NW);
            live = i < NI && c < k;
            return wk + (live ? c : 0);
        }
        const int c = CW * cc + (i >> 4), m = 16 * int(h) + (i & 15);
        live = c < k && m < k;
        return wk + k + (live ? c * k + m : 0);  // clamped: no branch
    };
    bool wl0, wl1 = false;
    u8 wr0 = *wsrc(0, tid, wl0), wr1 = 0;
    if (tid + NT < NI)
        wr1 = *wsrc(0, tid + NT, wl1);
    auto wput = [&](int i, u32 wv) {
        if (i < NW)
            reinterpret_cast<u8 *>(wq)[i] = u8(wv);
        else if (i < NI)
            wslot[i - NW] = wv;
    };

    // survivor loads through one buffer resource over the stripe's slots
    // (PAL; the launcher checks n * pitch < 2^31): offset = slot * pitch +
    // row, no branch; rows past a part read its neighbour (rows never
    // stored) or 0 past the slots, survivors past k read slot 0's part into
    // a zero table.  Without PAL (ragged batches, unaligned parts): byte
    // loads, clamped.
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u8 *>(v.parts), (short)0, int(u64(g.n) * v.pitch), 0x00020000);

    const int nch = ONE ? 1 : (k + CW - 1) / CW;
    u32 d0[CW], d1[CW];
    u32 soff[CW];
    auto load = [&](u32 (&d)[CW], u32 rb, int t, int cc) {
        const u32 r4 = rb + (u32(t) * u32(NT) + u32(tid)) * 4u;
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            if constexpr (PAL) {
                d[j] = __builtin_amdgcn_raw_buffer_load_b32(prs, soff[j] + r4, 0, 0);
            } else {
                const bool ok = CW * cc + j < k && r4 < v.ps;
                d[j] = ok ? load4_any(v.parts + soff[j] + r4, v.ps - r4) : 0u;
            }
        }
    };
    for (u32 slice = wi;; slice += nwg) {
    const u32 r_begin = slice * SH::ROWS;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[t][q] = make_uint4(0, 0, 0, 0);
    const u32 next = slice + nwg;
    const bool more = ONE && next * SH::ROWS < v.ps;
    for (int cc = 0; cc < nch; ++cc) {
      if (!ONE || slice == wi) {
        lds_barrier();  // the previous chunk's lookups are done
        wput(tid, wl0 ? u32(wr0) : 0u);
        if (tid + NT < NI)
            wput(tid + NT, wl1 ? u32(wr1) : 0u);
        if (cc + 1 < nch) {
            wr0 = *wsrc(cc + 1, tid, wl0);
            if (tid + NT < NI)
                wr1 = *wsrc(cc + 1, tid + NT, wl1);
        }
        lds_barrier();

#pragma unroll
        for (int j = 0; j < CW; ++j)
            soff[j] = CW * cc + j < k ? u32(u64(wslot[j]) * v.pitch) : 0u;
        // the first quad's survivor loads fly while the tables are built
        load(d0, r_begin, 0, cc);

        // ---- tables of the chunk's survivors for output columns 16h ..
        if constexpr (NIB) {
            // (kind, column) pairs x 4 wave writes of 4 value rows x 16
            // replicas: lane l writes value 4 it + l / 16 into slot l & 15
#pragma unroll 1
            for (int pi = wave; pi < 2 * CW; pi += WAVES) {
                const int kind = pi / CW, j = pi % CW;  // wave-uniform
                // basis of the kind's nibble: row * 2^(4 kind + b), b < 4
                u32 bs[4][4];
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    u32 x = wq[j][w];
                    if (kind)
                        x = gf_xtime4(gf_xtime4(gf_xtime4(gf_xtime4(x))));
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb) {
                        bs[bb][w] = x;
                        x = gf_xtime4(x);
                    }
                }
                const u32 base = u32(j) * 4096u + (kind ? (MODE == 1 ? 65536u : SH::HI) : 0u);
#pragma unroll
                for (int it = 0; it < 4; ++it) {
                    const u32 vv = u32(4 * it) + u32(lane >> 4);
                    u32 e4[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb) {
                        const u32 msk = 0u - ((vv >> bb) & 1u);  // branch-free select of the bit's basis
#pragma unroll
                        for (int w = 0; w < 4; ++w)
                            e4[w] ^= bs[bb][w] & msk;
                    }
                    *reinterpret_cast<uint4 *>(tbl + base + vv * 256u + u32(lane & 15) * 16u) =
                        make_uint4(e4[0], e4[1], e4[2], e4[3]);
                }
            }
        } else if constexpr (DIAG) {
            // lane l builds table j = l & 15, entries x = (l >> 4) + 4 i + 32
            // wave (Gray-code walk over i < 8): the 8 lanes of a ds_write_b128
            // group write 8 slots of one x row (no conflict)
            static_assert(WAVES == 8 && CW == 16, "diagonal build: 8 waves x 32 entries per table");
            const int j = lane & 15, xl = lane >> 4;
            const u32 row[4] = {wq[j][0], wq[j][1], wq[j][2], wq[j][3]};
            u32 basis[8][4];
            make_basis<4>(basis, row);
            u32 hv[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                u32 e = 0;
#pragma unroll
                for (int bb = 0; bb < 2; ++bb)
                    e ^= basis[bb][w] & (0u - ((u32(xl) >> bb) & 1u));
#pragma unroll
                for (int bb = 0; bb < 3; ++bb)
                    e ^= basis[5 + bb][w] & (0u - ((u32(wave) >> bb) & 1u));
                hv[w] = e;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i) {
                    const int bit = __builtin_ctz(i);
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        hv[w] ^= basis[2 + bit][w];
                }
                const u32 x = u32(xl) + 4u * u32(i ^ (i >> 1)) + 32u * u32(wave);
                *reinterpret_cast<uint4 *>(tbl + x * 256u + u32(j) * 16u) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            }
        } else {
            // byte tables: column j, entries x = lane + 64 m (Gray-code walk
            // over the two high bits, one XOR per entry)
#pragma unroll 1
            for (int j = wave; j < CW; j += WAVES) {
                const u32 row[4] = {wq[j][0], wq[j][1], wq[j][2], wq[j][3]};
                u32 basis[8][4];
                make_basis<4>(basis, row);
                u32 hv[4] = {0, 0, 0, 0};
#pragma unroll
                for (int bb = 0; bb < 6; ++bb) {
                    const u32 msk = 0u - ((u32(lane) >> bb) & 1u);
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        hv[w] ^= basis[bb][w] & msk;
                }
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    if (mi) {
                        const int bit = __builtin_ctz(mi);
#pragma unroll
                        for (int w = 0; w < 4; ++w)
                            hv[w] ^= basis[6 + bit][w];
                    }
                    const int x = lane + 64 * (mi ^ (mi >> 1));
                    *reinterpret_cast<uint4 *>(tbl + u32(j) * 4096u + u32(x) * 16u) =
                        make_uint4(hv[0], hv[1], hv[2], hv[3]);
                }
            }
        }
        lds_barrier();
      }

        // one row quad: the CW survivors' products into a4[q] (row 4i + q);
        // tdep (0 at run time) links groups of 16 lookups, so the compiler
        // keeps 16 in flight instead of hoisting all of them (spills)
        auto quad = [&](const u32 (&d)[CW], uint4 (&a4)[4], int cc) {
            u32 tdep = 0;
            if constexpr (NIB) {
#pragma unroll
                for (int j = 0; j < CW; ++j) {
                    if (CW * cc + j >= k)
                        break;  // survivors past k (uniform): their tables are zero
                    const u32 dl = d[j] & 0x0F0F0F0Fu, dh = (d[j] >> 4) & 0x0F0F0F0Fu;
                    const u32 sl = slot_lo + tdep, sh = slot_hi + tdep;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        // (nibble of row q's byte) << 8 | slot byte (| 1 << 16)
                        const u32 sel = 0x0C020000u | (u32(4 + q) << 8);
                        const u32 Pl = __builtin_amdgcn_perm(dl, sl, sel), Ph = __builtin_amdgcn_perm(dh, sh, sel);
                        const uint4 a = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + Pl);
                        const uint4 c2 = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + SH::HI + Ph);
                        a4[q].x = xor3(a4[q].x, a.x, c2.x);
                        a4[q].y = xor3(a4[q].y, a.y, c2.y);
                        a4[q].z = xor3(a4[q].z, a.z, c2.z);
                        a4[q].w = xor3(a4[q].w, a.w, c2.w);
                    }
                    if (j & 1)
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
                }
            } else if constexpr (DIAG) {
                // dd[t] = d[(t + r) & 15]: four mux stages by the bits of r
                u32 dd[CW];
#pragma unroll
                for (int t = 0; t < CW; ++t)
                    dd[t] = d[t];
#pragma unroll
                for (int st2 = 3; st2 >= 0; --st2) {
                    const u32 mk = (u32(lane) >> st2) & 1u ? ~0u : 0u;
                    u32 nx[CW];
#pragma unroll
                    for (int t = 0; t < CW; ++t)
                        nx[t] = mux3(mk, dd[(t + (1 << st2)) & 15], dd[t]);
#pragma unroll
                    for (int t = 0; t < CW; ++t)
                        dd[t] = nx[t];
                }
                // every step (survivors past k meet zero tables)
#pragma unroll
                for (int t = 0; t < CW; t += 2) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        // byte 0: the slot of survivor (t + r) & 15, byte 1: row q's byte
                        const u32 s0 = 0x0C0C0004u | (u32(q) << 8) | u32(t & 3);
                        const u32 s1 = 0x0C0C0004u | (u32(q) << 8) | u32((t + 1) & 3);
                        const u32 P0 = __builtin_amdgcn_perm(dslot[t >> 2], dd[t], s0) + tdep;
                        const u32 P1 = __builtin_amdgcn_perm(dslot[(t + 1) >> 2], dd[t + 1], s1) + tdep;
                        const uint4 a = *reinterpret_cast<const uint4 *>(tbl + P0);
                        const uint4 c2 = *reinterpret_cast<const uint4 *>(tbl + P1);
                        a4[q].x = xor3(a4[q].x, a.x, c2.x);
                        a4[q].y = xor3(a4[q].y, a.y, c2.y);
                        a4[q].z = xor3(a4[q].z, a.z, c2.z);
                        a4[q].w = xor3(a4[q].w, a.w, c2.w);
                    }
                    if (t & 2)
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
                }
            } else {
                // survivors in pairs: one three-input XOR per word folds both
#pragma unroll
                for (int j = 0; j < CW; j += 2) {
                    if (CW * cc + j >= k)
                        break;  // survivors past k (uniform): their tables are zero
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        // (row q's byte) << 4: the 16-byte entry of the table
                        const u32 sel = 0x0C0C0C00u | u32(4 + q);
                        const u32 P0 = (__builtin_amdgcn_perm(d[j], 0u, sel) << 4) + tdep;
                        const u32 P1 = (__builtin_amdgcn_perm(d[j + 1], 0u, sel) << 4) + tdep;
                        const uint4 a = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + P0);
                        const uint4 c2 = *reinterpret_cast<const uint4 *>(tbl + u32(j + 1) * 4096u + P1);
                        a4[q].x = xor3(a4[q].x, a.x, c2.x);
                        a4[q].y = xor3(a4[q].y, a.y, c2.y);
                        a4[q].z = xor3(a4[q].z, a.z, c2.z);
                        a4[q].w = xor3(a4[q].w, a.w, c2.w);
                    }
                    if (j & 2)
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
                }
            }
        };
        // two named buffers of survivor dwords (quad 0 in one, quad 1's
        // loads in flight in the other: the compiler's wait covers only the
        // loads a quad consumes)
        static_assert(T == 2, "one pass of two quads per chunk");
        load(d1, r_begin, 1, cc);
        quad(d0, acc[0], cc);
        if constexpr (ONE)  // the next slice's first quad (its rows, or these again past the end)
            load(d0, more ? next * SH::ROWS : r_begin, 0, cc);
        quad(d1, acc[1], cc);
    }

    // ---- output: row r's columns 16h .. at r*k + 16h (nothing at or past B)
    u8 *out = const_cast<u8 *>(v.blk);
    const uintptr_t oa = reinterpret_cast<uintptr_t>(out);
    if (ngroups == 1 && (oa & 15) == 0 && (u32(k) & 3) == 0) {
        // k in {4, 8, 12, 16}, 16-aligned block: the quad's 4 rows are 4k
        // contiguous bytes = the first k/4 dwords of each row's accumulator;
        // written as k/4 16-byte stores (a wave's fill 256k contiguous bytes)
        const u32 kd = u32(k) >> 2;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const u32 r0 = r_begin + (u32(t) * u32(NT) + u32(tid)) * 4u;
            if (r0 >= v.ps)
                continue;
            const u64 base = u64(r0) * u64(k);
            const uint4 a0 = acc[t][0], a1 = acc[t][1], a2 = acc[t][2], a3 = acc[t][3];
            u8 *o = out + base;
            if (base + 4u * u64(k) <= u64(v.B)) {
                switch (kd) {  // row q's dwords are its accumulator's first kd
                case 1:
                    store16(o, a0.x, a1.x, a2.x, a3.x, false);
                    break;
                case 2:
                    store16(o, a0.x, a0.y, a1.x, a1.y, false);
                    store16(o + 16, a2.x, a2.y, a3.x, a3.y, false);
                    break;
                case 3:
                    store16(o, a0.x, a0.y, a0.z, a1.x, false);
                    store16(o + 16, a1.y, a1.z, a2.x, a2.y, false);
                    store16(o + 32, a2.z, a3.x, a3.y, a3.z, false);
                    break;
                default:
                    store16(o, a0.x, a0.y, a0.z, a0.w, false);
                    store16(o + 16, a1.x, a1.y, a1.z, a1.w, false);
                    store16(o + 32, a2.x, a2.y, a2.z, a2.w, false);
                    store16(o + 48, a3.x, a3.y, a3.z, a3.w, false);
                }
            } else {  // the block's last rows
                const uint4 aq[4] = {a0, a1, a2, a3};
                for (u32 c = 0; c < 4u * u32(k); ++c) {
                    const u32 q = c / u32(k), e = c % u32(k);
                    const uint4 x = aq[q];
                    const u32 wd = e < 4 ? x.x : e < 8 ? x.y : e < 12 ? x.z : x.w;
                    if (base + c < u64(v.B))
                        o[c] = u8(wd >> (8 * (e & 3)));
                }
            }
        }
    } else {
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32 r = r_begin + (u32(t) * u32(NT) + u32(tid)) * 4u + u32(q);
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
    if (!more)
        break;
    }
}

template <int MODE>
int launch_bign(const nkfs_geom *g, const uint8_t *work, const int32_t *status, bool pal, hipStream_t st)
{
    const int k = g->k;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    const u64 ngroups = (u64(k) + 15) / 16;
    const u64 nslices = (u64(ps_max) + BnShape<MODE>::ROWS - 1) / BnShape<MODE>::ROWS;
    const u32 ns = u32(nslices ? nslices : 1);
    // one chunk: workgroups per stripe enough for ~8 per CU in all, each
    // walking its share of the slices with the tables built once
    const bool one = k <= BnShape<MODE>::CW;
    u32 nwg = ns;
    if (one) {
        const u64 want = (u64(nkfs_cu_count()) * 8 + u64(g->nstripes) - 1) / u64(g->nstripes);
        nwg = u32(want < ns ? (want ? want : 1) : ns);
    }
    const u64 grid = (u64(g->nstripes) + 7) / 8 * 8 * ngroups * nwg;
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    const dim3 block(64 * BnShape<MODE>::WAVES);
    const u32 ng = u32(ngroups);
    if (one && pal)
        hipLaunchKernelGGL((k_decode_bign<MODE, true, true>), dim3(u32(grid)), block, 0, st, *g, work, status, ng, ns, nwg);
    else if (one)
        hipLaunchKernelGGL((k_decode_bign<MODE, false, true>), dim3(u32(grid)), block, 0, st, *g, work, status, ng, ns, nwg);
    else if (pal)
        hipLaunchKernelGGL((k_decode_bign<MODE, true, false>), dim3(u32(grid)), block, 0, st, *g, work, status, ng, ns, nwg);
    else
        hipLaunchKernelGGL((k_decode_bign<MODE, false, false>), dim3(u32(grid)), block, 0, st, *g, work, status, ng, ns, nwg);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// ---- decode, 8 < k <= 64: every output column of a slice in one workgroup
// (struct nkfs_tune.dec_bign 3).  k_decode_bign gives
// each 16-column output group its own workgroup, so a row's k bytes come
// from ceil(k/16) workgroups and rows that are not dword multiples (odd k)
// are written bytewise, 16-byte windows at a k-byte lane stride.  Here one
// workgroup owns all NG = ceil(k/16) groups of its rows:
//  - the stripe's K x K inverse (rows padded to 16 NG columns) and survivor
//    slots are copied to LDS once per workgroup;
//  - per slice of ROWS rows and per 16-survivor chunk, the chunk's survivor
//    dwords are loaded once (the next chunk's in flight) and feed all NG
//    groups: for each group the chunk's 16 byte tables U_c[x] = (W[c][16h]
//    x, ..., W[c][16h+15] x) are built (64 KiB) and every lane folds its 4
//    rows into the group's accumulators (acc[h], 16 bytes of 4 rows);
//  - output: a lane's 4 rows are 4k contiguous block bytes.  Row q is
//    shifted to its byte offset q k (a 64-bit funnel shift per dword, the
//    shift uniform) and written to an LDS stage as dwords -- the dword a row
//    shares with the next is OR-ed in (ds_or), the bytes past column k being
//    zero -- then the wave reads the stage back as 16-byte pieces in lane
//    order and stores them: every store instruction writes 1 KiB of
//    contiguous block bytes, whatever k.  The stage reuses the table LDS, in
//    two halves of the wave.
// Survivors past k sit in a chunk's tail and are skipped (uniform); output
// columns past k have zero W entries, so their accumulator bytes are zero.
#ifndef BR_PAIRS
#define BR_PAIRS 1  // survivor pairs whose lookups fly together in k_decode_bigr
#endif
template <int NG, int T>
struct BrShape {
    static constexpr int WAVES = 8, CW = 16, NT = 64 * WAVES;
    static constexpr u32 ROWS = u32(NT) * 4u * u32(T);
    static constexpr int KMAX = 16 * NG;
    static constexpr u32 WL = u32(KMAX) * u32(KMAX);  // inverse rows x padded columns, bytes
};

#ifndef BR_PREFETCH
// k_decode_bigr: 1 = the next chunk's survivor loads in flight under this
// chunk's groups; 0 (default) = each chunk's loads at its start, covered by
// the other workgroup on the CU (W3 875 vs 864, N40K17 1,700 vs 1,666 GB/s,
// profiles/r06/ab_bigr_variants.txt)
#define BR_PREFETCH 0
#endif
#ifndef BR_WPE
#define BR_WPE 4
#endif
// DIAG (dec_bign 5, NG <= 3): a (chunk, group)'s 16 tables in the diagonal
// layout of k_decode_bign MODE 4 (entry x of survivor j at x * 256 + j * 16),
// the survivor dwords rotated once per chunk by l & 15 and shared by the NG
// groups: every lookup of a b128 lane group in its own bank slot
template <int NG, int T, bool PAL, bool DIAG>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(BR_WPE, BR_WPE))) void k_decode_bigr(nkfs_geom g, const u8 *work, const int32_t *status,
                                                         u32 nslices, u32 nwg)
{
    static_assert(!DIAG || NG <= 3, "diagonal tables: branch-free survivor loads (NG <= 3)");
    using SH = BrShape<NG, T>;
    constexpr int CW = SH::CW, NT = SH::NT, KP = SH::KMAX;
    __shared__ __attribute__((aligned(16))) u8 tbl[CW * 4096];  // tables; the output stage after the lookups
    __shared__ __attribute__((aligned(16))) u8 wl[SH::WL];      // wl[c * KP + m] = W[c][m], 0 for m >= k
    __shared__ __attribute__((aligned(16))) u32 wsoff[KP];     // survivor c's part offset (slot * pitch), 0 past k

    const u32 b = blockIdx.x;
    const u32 s = b / nwg, wi = b % nwg;
    if (s >= g.nstripes || (status && status[s]))
        return;  // the whole workgroup
    const Stripe v = stripe_at(g, s);  // g.blocks = the output, g.n = slots per stripe
    if (wi * SH::ROWS >= v.ps)
        return;
    const int k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const u8 *wk = work + u64(s) * u64(k + k * k);
    for (int i = tid; i < KP * KP; i += NT) {
        const int c = i / KP, m = i % KP;
        wl[i] = c < k && m < k ? wk[k + c * k + m] : u8(0);
    }
    if (tid < KP)
        wsoff[tid] = tid < k ? u32(u64(wk[tid]) * v.pitch) : 0u;  // the launcher checks n * pitch < 2^32
    __syncthreads();

    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u8 *>(v.parts), (short)0, int(u64(g.n) * v.pitch), 0x00020000);
    // survivor loads: slot offsets from LDS at each chunk's load (PAL: one
    // buffer resource over the stripe's slots, the launcher checks n * pitch
    // < 2^31; otherwise clamped byte loads)
    // All CW loads are issued, branch-free (survivors past k read slot 0's
    // rows and are never looked up): a runtime break per survivor split the
    // loads into a chain of blocks, each load waited for (vmcnt(0)) and
    // spilled before the next one issued -- 14 VGPRs of scratch traffic per
    // slice, ~25 % of the W3 decode's HBM bytes (profiles/r06/pmc_w3_summary.txt)
    auto load = [&](u32 (&d)[CW], u32 r4, int cc) {
        if constexpr (NG >= 4) {  // (branch-free, NG = 4 spilled 1,292 VGPRs: the old form)
#pragma unroll
            for (int j = 0; j < CW; ++j) {
                if (CW * cc + j >= k)
                    break;  // uniform
                const u32 so = __builtin_amdgcn_readfirstlane(wsoff[CW * cc + j]);
                if constexpr (PAL)
                    d[j] = __builtin_amdgcn_raw_buffer_load_b32(prs, so + r4, 0, 0);
                else
                    d[j] = r4 < v.ps ? load4_any(v.parts + so + r4, v.ps - r4) : 0u;
            }
            return;
        }
        u32 so[CW];
#pragma unroll
        for (int i = 0; i < CW / 4; ++i) {
            const uint4 o4 = reinterpret_cast<const uint4 *>(wsoff + CW * cc)[i];
            so[4 * i] = __builtin_amdgcn_readfirstlane(o4.x);
            so[4 * i + 1] = __builtin_amdgcn_readfirstlane(o4.y);
            so[4 * i + 2] = __builtin_amdgcn_readfirstlane(o4.z);
            so[4 * i + 3] = __builtin_amdgcn_readfirstlane(o4.w);
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            if constexpr (PAL)
                d[j] = __builtin_amdgcn_raw_buffer_load_b32(prs, r4, so[j], 0);
            else
                d[j] = r4 < v.ps ? load4_any(v.parts + so[j] + r4, v.ps - r4) : 0u;
        }
    };
    // one row quad: the chunk's survivors' products for group h into a4
    auto quad = [&](const u32 (&d)[CW], uint4 (&a4)[4], int cc) {
        // tdep: 0 at run time, from an opaque move and then from the last
        // pair's accumulator; folded into every survivor dword before its
        // byte is extracted, so neither the extraction nor the address is
        // shared between the NG groups of a chunk (common-subexpression
        // elimination kept all 64 addresses of a chunk live across its groups:
        // 205 VGPRs, one workgroup per CU), and a pair's lookups wait for the
        // previous pair's (BR_PAIRS pairs in flight)
        u32 tdep;
        asm volatile("v_mov_b32 %0, 0" : "=v"(tdep));
#pragma unroll
        for (int j = 0; j < CW; j += 2) {
            if (CW * cc + j >= k)
                break;  // uniform: survivors past k
            // (odd k: the pair's second table is never built -- it may hold
            // the previous slice's stage -- so it is not read)
            const bool two = CW * cc + j + 1 < k;
            const u32 dj0 = d[j] ^ tdep, dj1 = d[j + 1] ^ tdep;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32 sel = 0x0C0C0C00u | u32(4 + q);
                const u32 P0 = __builtin_amdgcn_perm(dj0, 0u, sel) << 4;
                const u32 P1 = __builtin_amdgcn_perm(dj1, 0u, sel) << 4;
                const uint4 a = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + P0);
                const uint4 c2 = two ? *reinterpret_cast<const uint4 *>(tbl + u32(j + 1) * 4096u + P1)
                                     : make_uint4(0, 0, 0, 0);
                a4[q].x = xor3(a4[q].x, a.x, c2.x);
                a4[q].y = xor3(a4[q].y, a.y, c2.y);
                a4[q].z = xor3(a4[q].z, a.z, c2.z);
                a4[q].w = xor3(a4[q].w, a.w, c2.w);
            }
            // one pair's 8 lookups in flight at a time (two pairs, as in
            // k_decode_bign, cost this kernel 2 waves per SIMD: its NG
            // accumulators and the next chunk's survivors are live too)
            if ((j & (BR_PAIRS * 2 - 2)) == BR_PAIRS * 2 - 2)
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
        }
    };
    // the 16 byte tables of chunk cc, group h (survivor j: W[16cc + j][16h ..])
    auto build = [&](int cc, int h) {
#pragma unroll 1
        for (int j = wave; j < CW; j += SH::WAVES) {
            const int c = CW * cc + j;
            if (c >= k)
                break;  // uniform
            const uint4 r4 = *reinterpret_cast<const uint4 *>(wl + c * KP + 16 * h);
            const u32 row[4] = {r4.x, r4.y, r4.z, r4.w};
            u32 basis[8][4];
            make_basis<4>(basis, row);
            build_table16(tbl + u32(j) * 4096u, basis, lane);
        }
    };
    // DIAG: lane l builds table j = l & 15 of the (chunk, group), entries x =
    // (l >> 4) + 4 i + 32 wave (Gray-code walk over i < 8; the 8 lanes of a
    // ds_write_b128 group write 8 slots of one x row); rows past k are zero
    auto build_diag = [&](int cc, int h) {
        const int j = lane & 15, xl = lane >> 4;
        const uint4 r4 = *reinterpret_cast<const uint4 *>(wl + (CW * cc + j) * KP + 16 * h);
        const u32 row[4] = {r4.x, r4.y, r4.z, r4.w};
        u32 basis[8][4];
        make_basis<4>(basis, row);
        u32 hv[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            u32 e = 0;
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
                e ^= basis[bb][w] & (0u - ((u32(xl) >> bb) & 1u));
#pragma unroll
            for (int bb = 0; bb < 3; ++bb)
                e ^= basis[5 + bb][w] & (0u - ((u32(wave) >> bb) & 1u));
            hv[w] = e;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i) {
                const int bit = __builtin_ctz(i);
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    hv[w] ^= basis[2 + bit][w];
            }
            const u32 x = u32(xl) + 4u * u32(i ^ (i >> 1)) + 32u * u32(wave);
            *reinterpret_cast<uint4 *>(tbl + x * 256u + u32(j) * 16u) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
        }
    };
    // DIAG: byte i of dslot[gq] = the slot ((4 gq + i + (lane & 15)) & 15) * 16
    u32 dslot[4];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
        u32 x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            x |= (((u32(4 * gq + i) + u32(lane & 15)) & 15u) << 4) << (8 * i);
        dslot[gq] = x;
    }
    // DIAG: dd[t] = d[(t + (l & 15)) & 15], four mux stages
    auto rotate = [&](const u32 (&d)[CW], u32 (&dd)[CW]) {
#pragma unroll
        for (int t = 0; t < CW; ++t)
            dd[t] = d[t];
#pragma unroll
        for (int st2 = 3; st2 >= 0; --st2) {
            const u32 mk = (u32(lane) >> st2) & 1u ? ~0u : 0u;
            u32 nx[CW];
#pragma unroll
            for (int t = 0; t < CW; ++t)
                nx[t] = mux3(mk, dd[(t + (1 << st2)) & 15], dd[t]);
#pragma unroll
            for (int t = 0; t < CW; ++t)
                dd[t] = nx[t];
        }
    };
    auto quad_diag = [&](const u32 (&dd)[CW], uint4 (&a4)[4]) {
        u32 tdep;
        asm volatile("v_mov_b32 %0, 0" : "=v"(tdep));
#pragma unroll
        for (int j = 0; j < CW; j += 2) {
            const u32 dj0 = dd[j] ^ tdep, dj1 = dd[j + 1] ^ tdep;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // byte 0: the slot of survivor (j + r) & 15, byte 1: row q's byte
                const u32 s0 = 0x0C0C0004u | (u32(q) << 8) | u32(j & 3);
                const u32 s1 = 0x0C0C0004u | (u32(q) << 8) | u32((j + 1) & 3);
                const u32 P0 = __builtin_amdgcn_perm(dslot[j >> 2], dj0, s0);
                const u32 P1 = __builtin_amdgcn_perm(dslot[(j + 1) >> 2], dj1, s1);
                const uint4 a = *reinterpret_cast<const uint4 *>(tbl + P0);
                const uint4 c2 = *reinterpret_cast<const uint4 *>(tbl + P1);
                a4[q].x = xor3(a4[q].x, a.x, c2.x);
                a4[q].y = xor3(a4[q].y, a.y, c2.y);
                a4[q].z = xor3(a4[q].z, a.z, c2.z);
                a4[q].w = xor3(a4[q].w, a.w, c2.w);
            }
            if ((j & (BR_PAIRS * 2 - 2)) == BR_PAIRS * 2 - 2)
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(a4[3].x));
        }
    };

    u8 *out = const_cast<u8 *>(v.blk);
    const bool oal = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    // per row q of a lane's quad: the dword offset of its first byte in the
    // lane's 4k-byte region and its byte shift (uniform)
    u32 qd[4], qs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        qd[q] = (u32(q) * u32(k)) >> 2;
        qs[q] = (u32(q) * u32(k)) & 3u;
    }

    for (u32 slice = wi; slice < nslices; slice += nwg) {
        const u32 r_begin = slice * SH::ROWS;
        if (r_begin >= v.ps)
            break;
        uint4 acc[T][NG][4];
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int h = 0; h < NG; ++h)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[t][h][q] = make_uint4(0, 0, 0, 0);
        // survivor dwords, double-buffered over the chunks: chunk cc + 1's
        // loads fly under chunk cc's NG table builds and lookups
        u32 d[2][T][CW];
#pragma unroll
        for (int t = 0; t < T; ++t)
            load(d[0][t], r_begin + (u32(t) * u32(NT) + u32(tid)) * 4u, 0);
#pragma unroll
        for (int cc = 0; cc < NG; ++cc) {
            // the chunk's loads stay at the chunk: without this the
            // branch-free loads of all NG chunks were hoisted to the top of
            // the slice (NG = 4: 1,292 VGPRs spilled)
            asm volatile("" ::: "memory");
            if (!BR_PREFETCH && cc > 0)
#pragma unroll
                for (int t = 0; t < T; ++t)
                    load(d[cc & 1][t], r_begin + (u32(t) * u32(NT) + u32(tid)) * 4u, cc);
            if (BR_PREFETCH && cc + 1 < NG)
#pragma unroll
                for (int t = 0; t < T; ++t)
                    load(d[(cc + 1) & 1][t], r_begin + (u32(t) * u32(NT) + u32(tid)) * 4u, cc + 1);
            if constexpr (DIAG) {
                u32 dd[T][CW];
#pragma unroll
                for (int t = 0; t < T; ++t)
                    rotate(d[cc & 1][t], dd[t]);
#pragma unroll
                for (int h = 0; h < NG; ++h) {
                    lds_barrier();  // the previous tables' lookups (or stage reads) are done
                    build_diag(cc, h);
                    lds_barrier();
#pragma unroll
                    for (int t = 0; t < T; ++t)
                        quad_diag(dd[t], acc[t][h]);
                }
            } else {
#pragma unroll
            for (int h = 0; h < NG; ++h) {
                lds_barrier();  // the previous tables' lookups (or stage reads) are done
                build(cc, h);
                lds_barrier();
#pragma unroll
                for (int t = 0; t < T; ++t)
                    quad(d[cc & 1][t], acc[t][h], cc);
            }
            }
        }
        lds_barrier();  // every lookup is done: the table LDS becomes the stage

        // ---- output through the stage, half a wave's lanes at a time
        u8 *stage = tbl + u32(wave) * (32u * 4u * u32(KP));  // 32 lanes x 4 rows x KP bytes <= 8 KiB per wave
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const u32 wrow = r_begin + (u32(t) * u32(NT) + u32(wave) * 64u) * 4u;  // the wave's first row
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                if ((lane >> 5) == half) {
                    const u32 base = u32(lane & 31) * u32(k);  // the lane's region, in dwords
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        u32 R[4 * NG];
#pragma unroll
                        for (int h = 0; h < NG; ++h) {
                            R[4 * h] = acc[t][h][q].x;
                            R[4 * h + 1] = acc[t][h][q].y;
                            R[4 * h + 2] = acc[t][h][q].z;
                            R[4 * h + 3] = acc[t][h][q].w;
                        }
                        const u32 sh = 32u - 8u * qs[q];  // 32: no shift
                        const u32 nd = (qs[q] + u32(k) + 3u) >> 2;  // dwords the row touches
#pragma unroll
                        for (int w = 0; w <= 4 * NG; ++w) {
                            if (u32(w) >= nd)
                                break;  // uniform
                            const u64 pair = (u64(w < 4 * NG ? R[w] : 0u) << 32) | (w ? R[w - 1] : 0u);
                            const u32 dw = u32(pair >> sh);
                            u32 *dst = reinterpret_cast<u32 *>(stage) + base + qd[q] + u32(w);
                            if (w == 0 && qs[q])
                                __hip_atomic_fetch_or(dst, dw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            else
                                *dst = dw;
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // the half's 32 x 4k bytes back in lane order, 16 bytes per lane
                const u32 hbytes = 128u * u32(k);
                const u64 obase = (u64(wrow) + u64(half) * 128u) * u64(k);  // block offset of the half's region
#pragma unroll 1
                for (u32 o = u32(lane) * 16u; o < hbytes; o += 1024u) {
                    const u64 ob = obase + o;
                    if (ob >= u64(v.B))
                        break;
                    const uint4 x = *reinterpret_cast<const uint4 *>(stage + o);
                    if (oal && ob + 16u <= u64(v.B)) {
                        store16(out + ob, x.x, x.y, x.z, x.w, false);
                    } else {
                        const u32 tw[4] = {x.x, x.y, x.z, x.w};
                        for (u32 c = 0; c < 16u && ob + c < u64(v.B); ++c)
                            out[ob + c] = u8(tw[c >> 2] >> (8 * (c & 3)));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // the stage is read before the next half overwrites it
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
}

template <int NG, int T, bool DIAG>
int launch_bigr(const nkfs_geom *g, const uint8_t *work, const int32_t *status, bool pal, hipStream_t st)
{
    using SH = BrShape<NG, T>;
    const int k = g->k;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    const u64 nslices = (u64(ps_max) + SH::ROWS - 1) / SH::ROWS;
    const u32 ns = u32(nslices ? nslices : 1);
    // workgroups per stripe: enough for ~2 per CU in all, each walking its
    // share of the stripe's slices (the inverse copied to LDS once)
    const u64 want = (u64(nkfs_cu_count()) * 4 + u64(g->nstripes) - 1) / u64(g->nstripes);
    const u32 nwg = u32(want < ns ? (want ? want : 1) : ns);
    const u64 grid = u64(g->nstripes) * nwg;
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    // survivor offsets are 32-bit (a stripe's slots span < 4 GiB)
    const u64 pitch_max = g->block_sizes ? (u64(ps_max) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1) : g->part_pitch;
    if (u64(g->n) * pitch_max >= 0xFFFFFFFFull)
        return -ENOSYS;
    if (pal)
        hipLaunchKernelGGL((k_decode_bigr<NG, T, true, DIAG>), dim3(u32(grid)), dim3(SH::NT), 0, st, *g, work, status, ns, nwg);
    else
        hipLaunchKernelGGL((k_decode_bigr<NG, T, false, DIAG>), dim3(u32(grid)), dim3(SH::NT), 0, st, *g, work, status, ns, nwg);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// ---- encode, k <= 32 ------------------------------------------------------
// Reference arithmetic: crt/nk8.c:403-420 -- part_i[j] = XOR_m x_i^m
// d[j*k+m], d zero past block_size (:393-398); XXH64 of every part
// (crt/csum.c, crt/xxhash.c:791-916).
//
// Persistent: one workgroup of 16 waves per CU walks units = (stripe, group
// of 16 parts).  Per unit the k <= 32 columns' byte tables U_m[x] =
// (x_{p0}^m x, ..., x_{p0+15}^m x) are built once and stay resident (128
// KiB).  Waves 0..14 encode: a lane owns 4 consecutive rows per slice of
// 3,840 rows, loads each row's column bytes straight from the block
// (dword-aligned 16 + 4-byte buffer loads and v_alignbyte -- no LDS stage),
// looks up one 16-part product per (row, column), transposes its 4 rows x 16
// parts to one dword per part and stores it (64 lanes: 256 contiguous bytes
// of a part per instruction).  The next slice's loads are issued before the
// stores, so one wait covers both.  Wave 15 hashes: lane 4e + a is XXH64
// accumulator a of part p0 + e; once every encoder wave has stored slice i
// (its stores complete, then its LDS progress count), the hash wave folds
// slice i's 120 rounds from the L2.  The encoders never wait for it -- it
// may still be folding a unit while they encode the next -- and they
// synchronise among themselves through an LDS counter, so the tables of the
// next unit need no workgroup barrier.  The parts are read once from HBM
// (the hash re-read hits the L2).  Units u, u + 8, u + 16 are a stripe's
// part groups on one XCD (workgroup b runs on XCD b mod 8), side by side:
// they share the block's lines in its L2.
// NKFS_BE_SLC=1 (experiment builds): the block loads non-temporal (slc)
#ifndef NKFS_BE_SLC
#define NKFS_BE_SLC 0
#endif
// NKFS_BE_SLICE_BAR=1 (experiment builds): the encoder waves meet after every
// slice, bounding how long a slice's parts wait in the L2 for the hash wave
#ifndef NKFS_BE_SLICE_BAR
#define NKFS_BE_SLICE_BAR 0
#endif
// NKFS_BE_LATE_LOAD (default 1): the next slice's loads issue after this
// slice's stores, and the progress count waits for the stores only -- a
// vmcnt(0) after the loads made every slice's signal wait for the next
// slice's loads (W2 1,559 -> 1,690 GB/s, profiles/r05/ab_w2_late_load.txt)
#ifndef NKFS_BE_LATE_LOAD
#define NKFS_BE_LATE_LOAD 1
#endif
// NKFS_BE_DYN=1 (experiment builds): units from per-XCD counters (a
// workgroup takes the next unit of its own XCD -- a stripe's part groups stay
// on one XCD -- and steals from the other XCDs' counters once its own runs
// out, so every unit is taken even if an XCD holds no workgroup) instead of
// the static walk b, b + grid, ...
#ifndef NKFS_BE_DYN
#define NKFS_BE_DYN 0
#endif
// NKFS_BE_BATCH=1 (experiment builds): a column pair's lookups for all 4
// rows issued before any is folded -- lgkmcnt(6/4/2) waits instead of one
// per 2 lookups -- lost 4-8 % (W2 1,627 vs 1,776 GB/s,
// profiles/r06/ab_be_batch.txt): more lookups in flight per wave do not
// raise this kernel's LDS throughput
#ifndef NKFS_BE_BATCH
#define NKFS_BE_BATCH 0
#endif
// NKFS_BE_PROG=1 (experiment builds): the hash wave folds each encoder
// wave's 256-row segment of a slice as soon as that wave has stored it (its
// own progress count), in chain order, instead of waiting for all 15 waves
// (test whether the hash wave's lag is what makes its
// re-read of the parts miss the L2).  It is not: the PMC fetch stayed at 690
// vs 691 MB per W2 launch (the parts' 403 MB re-fetched either way) and the
// kernel ran 7-9 % slower (profiles/r06/ab_be_prog.txt, pmc_w2_prog*.txt)
#ifndef NKFS_BE_PROG
#define NKFS_BE_PROG 0
#endif
// NKFS_BE_HW: hash waves per workgroup, taking units in turn (default 4:
// the XXH64 chains, not the encoders, bounded the fused kernel --
// W2 1,703 -> 1,902, N24K20 1,665 -> 2,143, N20K17 1,382 -> 1,892 GB/s
// with NKFS_BE_HPRIO 3; 6 and 8 lose again: profiles/r06/ab_bign_hwn.txt)
#ifndef NKFS_BE_HW
#define NKFS_BE_HW 4
#endif
// NKFS_BE_RING: the hash waves' load ring, in batches of 8 rounds (RING - 1
// batches in flight while one is folded)
// NKFS_BE_LAG (experiment builds, 0 = off): encoder waves stay at most this
// many slices ahead of the unit's hash wave, so its re-read of the parts
// hits the XCD's L2 instead of HBM
#ifndef NKFS_BE_LAG
#define NKFS_BE_LAG 0
#endif
// NKFS_BE_DIAG8 (default 1): units of 8 parts (32 < k <= 64) take the
// diagonal tables whether or not enc_bign 3 pins them
#ifndef NKFS_BE_DIAG8
#define NKFS_BE_DIAG8 1
#endif
#ifndef NKFS_BE_RING
#define NKFS_BE_RING 4
#endif
// NKFS_BE_HPRIO: the hash waves' s_setprio level (default 3: an XXH64 chain
// is latency-bound and shares its SIMD with busy encoder waves; W2 1,704 ->
// 1,941 GB/s with one hash wave, profiles/r06/ab_bign_hprio.txt)
#ifndef NKFS_BE_HPRIO
#define NKFS_BE_HPRIO 3
#endif
constexpr u32 BE_END = 0xFFFFFFFFu;

// this wave's XCC (hardware register XCC_ID, bits 3:0)
__device__ inline u32 be_xcc() { return u32(__builtin_amdgcn_s_getreg(20 | (3 << 11))) & 7u; }
constexpr int BE_WAVES = 16, BE_EW = 15;
constexpr u32 BE_ROWS = 64u * BE_EW * 4u;  // 3,840 rows (120 XXH64 rounds) per slice
constexpr int BE_CMAX = 32;
// units of P = 8 parts (round 6, 32 < k <= 76): 8-byte table entries, k x 2
// KiB of tables, so every column's table of a unit still stays resident
constexpr int BE_CMAX8 = 76;
template <int P>
struct BeShape {
    static constexpr u32 TB = 256u * u32(P);              // bytes per column table
    static constexpr int CMAX = P == 16 ? BE_CMAX : BE_CMAX8;
};

// barrier of the encoder waves only (LDS counter; the hash wave runs on)
template <int EW>
__device__ __forceinline__ void enc_barrier(u32 *bar, u32 &gen, int lane)
{
    gen += EW;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if (lane == 0)
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// unit u -> stripe (nstripes or more: none) and part group
__device__ __forceinline__ u32 be_stripe(u32 u, u32 ngroups, u32 &grp)
{
    const u32 loc = u >> 3;
    grp = loc % ngroups;
    return (loc / ngroups) * 8 + (u & 7);
}

template <int P, bool HASH, int KC, bool DIAG, int HWV>
__global__ __launch_bounds__(64 * BE_WAVES, 1) void k_encode_bign(nkfs_geom g, const u8 *ids, u64 *digests,
                                                                   u32 ngroups, u32 nunits, u32 *uctr)
{
    static_assert(P == 16 || (P == 8 && KC == 0), "part groups of 16, or of 8 without contiguous-row loads");
    // DIAG with P = 8: 16-column chunks of 32 KiB (k <= 64, the launcher)
    // HWV hash waves (units go round them), EW encoders
    static_assert(HWV >= 1 && HWV <= 8, "one to eight hash waves");
    constexpr int EW = BE_WAVES - HWV;
    constexpr u32 ROWS = 64u * EW * 4u;  // rows per slice (3,840 with one hash wave: 120 XXH64 rounds)
    constexpr u32 TB = BeShape<P>::TB;
    constexpr int TPW = 64 / P;  // tables whose Vandermonde row one wave computes per pass
    // table passes per encoder wave: columns wave, wave + EW, ... must cover
    // every column (P = 16: 32; P = 8: 76), at most TPW per wave
    constexpr int TP = (BeShape<P>::CMAX + EW - 1) / EW;
    static_assert(TP <= TPW, "too few encoder waves to build every column's table");
    __shared__ __attribute__((aligned(16))) u8 tbl[BeShape<P>::CMAX * TB];
    __shared__ __attribute__((aligned(16))) u8 vrow[DIAG ? 2 * 16 * 16 : 16];  // DIAG: the Vandermonde rows
    __shared__ u32 done[BE_WAVES];  // slices stored so far, per encoder wave
    __shared__ u32 bar;
    __shared__ u32 uq[8];           // NKFS_BE_DYN: the workgroup's claimed units, in order
    __shared__ u32 uq_n, hdone;     // claims published / units the hash wave finished
    __shared__ u32 hseq[8];         // NKFS_BE_LAG: slices each hash wave has folded (or skipped)
    const bool dyn = NKFS_BE_DYN && uctr && HWV == 1;

    const int n = g.n, k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // KC != 0: k == KC, so the column loops' bounds are compile-time (the
    // runtime bound split every lookup pair into its own basic block, with a
    // wait for both lookups before the next pair issued)
    const int kk = KC ? KC : k;
    const int nch = (kk + 15) >> 4;
    if (tid < BE_WAVES)
        done[tid] = 0;
    if (tid < 8)
        hseq[tid] = 0;
    if (tid == 0) {
        bar = 0;
        uq_n = 0;
        hdone = 0;
    }
    __syncthreads();

    if (wave < EW) {
        u32 gen = 0, seq = 0;
#pragma unroll 1
        for (u32 ci = 0;; ++ci) {
            u32 u;
            if (dyn) {
                enc_barrier<EW>(&bar, gen, lane);  // the previous unit's lookups are done
                if (wave == 0) {
                    // at most 8 claims ahead of the hash wave (the uq ring)
                    while (ci >= __hip_atomic_load(&hdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + 8u)
                        __builtin_amdgcn_s_sleep(8);
                    u32 uu = BE_END;
                    if (lane == 0) {
                        const u32 x0 = be_xcc();
                        for (u32 t = 0; t < 8; ++t) {
                            const u32 xx = (x0 + t) & 7u;
                            const u32 cand = atomicAdd(uctr + xx, 1u) * 8u + xx;
                            if (cand < nunits) {
                                uu = cand;
                                break;
                            }
                        }
                        uq[ci % 8] = uu;
                        __hip_atomic_store(&uq_n, ci + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                enc_barrier<EW>(&bar, gen, lane);  // the claim is visible
                u = uq[ci % 8];
                if (u == BE_END)
                    break;
            } else {
                u = blockIdx.x + ci * gridDim.x;
                if (u >= nunits)
                    break;
            }
            u32 grp;
            const u32 s = be_stripe(u, ngroups, grp);
            if (s >= g.nstripes)
                continue;  // the whole workgroup
            const Stripe v = stripe_at(g, s);
            const int p0 = int(grp) * P, np = min(P, n - p0);

            // every encoder wave is done with the previous unit's tables
            enc_barrier<EW>(&bar, gen, lane);
            // Vandermonde rows of the group's parts, x^m by square and
            // multiply (crt/nk8.c:404-406 builds the same powers by repeated
            // multiplication): lane 16t + e computes byte e of the wave's
            // table t (columns wave, wave + 15, wave + 30), the rows are
            // gathered into scalars; parts past n and columns past k: 0
            // (P = 8: lane 8t + e, byte e of table t, t < 8: columns up to
            // wave + 105 >= 76)
            u32 xb;
            {
                const int t = lane / P, e = lane % P, m = wave + EW * t;
                u32 r = 0;
                if (e < np && m < k && t < TP) {
                    u32 x = ids[u64(s) * u64(n) + u64(p0 + e)];
                    r = 1;
#pragma unroll
                    for (int bit = 0; bit < 7; ++bit) {
                        if ((m >> bit) & 1)
                            r = gf_mul_packed(r, x);
                        x = gf_mul_packed(x, x);
                    }
                }
                xb = r;
            }
            if constexpr (DIAG) {
                // diagonal layout: entry x of column m at (m >> 4) * CB + x *
                // 16 P + (m & 15) * P (P = 16: 64 KiB chunks, 256-byte x rows;
                // P = 8: 32 KiB, 128-byte rows), so the 16 columns of a chunk
                // sit in 16 distinct bank slots of each x row.  The rows go
                // through the LDS; then job 4c + qt builds x = xl + 4 s + 64
                // qt of chunk c's 16 tables, lane 16 xl + j its table j: the
                // lanes of a ds_write group write distinct slots of one x row
                {
                    const int t = lane / P, e = lane % P, m = wave + EW * t;
                    if (t < TP && m < 16 * nch)
                        vrow[m * P + e] = u8(xb);
                }
                enc_barrier<EW>(&bar, gen, lane);
                constexpr int W4 = P / 4;
                constexpr u32 CB = P == 16 ? 65536u : 32768u, XB = 16u * u32(P);
#pragma unroll 1
                for (int job = wave; job < 4 * nch; job += EW) {
                    const int c = job >> 2, qt = job & 3, j = lane & 15, xl = lane >> 4;
                    u32 row[W4];
#pragma unroll
                    for (int w = 0; w < W4; ++w)
                        row[w] = reinterpret_cast<const u32 *>(vrow + (16 * c + j) * P)[w];
                    u32 basis[8][W4];
                    make_basis<W4>(basis, row);
                    u32 hv[W4];
#pragma unroll
                    for (int w = 0; w < W4; ++w)
                        hv[w] = (basis[0][w] & (0u - u32(xl & 1))) ^ (basis[1][w] & (0u - u32(xl >> 1))) ^
                                (basis[6][w] & (0u - u32(qt & 1))) ^ (basis[7][w] & (0u - u32(qt >> 1)));
                    u8 *tb = tbl + u32(c) * CB + u32(j) * u32(P);
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        if (i) {
                            const int bit = __builtin_ctz(i);
#pragma unroll
                            for (int w = 0; w < W4; ++w)
                                hv[w] ^= basis[2 + bit][w];
                        }
                        const u32 x = u32(xl) + 4u * u32(i ^ (i >> 1)) + 64u * u32(qt);
                        if constexpr (P == 16)
                            *reinterpret_cast<uint4 *>(tb + x * XB) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
                        else
                            *reinterpret_cast<uint2 *>(tb + x * XB) = make_uint2(hv[0], hv[1]);
                    }
                }
            }
#pragma unroll 1
            for (int t = 0; t < (DIAG ? 0 : TP); ++t) {
                const int m = wave + EW * t;
                // P = 16: columns k .. 16 nch - 1 get zero tables (lookups in
                // column pairs); P = 8: only columns < k exist -- 16 nch
                // tables would overrun the LDS at k = 76 -- and a pair's
                // second lookup past k is skipped instead
                if (m >= (P == 16 ? 16 * nch : k))
                    break;  // uniform
                if (m < k) {
                    u32 row[P / 4];
#pragma unroll
                    for (int w = 0; w < P / 4; ++w) {
                        u32 r = 0;
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            r |= u32(__builtin_amdgcn_readlane(int(xb), P * t + 4 * w + i)) << (8 * i);
                        row[w] = r;
                    }
                    u32 basis[8][P / 4];
                    make_basis<P / 4>(basis, row);
                    if constexpr (P == 16)
                        build_table16(tbl + m * TB, basis, lane);
                    else
                        build_table<2, 64>(tbl + m * TB, basis, lane);
                } else {  // columns k .. 16 nch - 1: zero (lookups go in column pairs)
#pragma unroll
                    for (int i = 0; i < int(TB / 1024u); ++i)
                        *reinterpret_cast<uint4 *>(tbl + m * TB + (lane + 64 * i) * 16) = make_uint4(0, 0, 0, 0);
                }
            }
            enc_barrier<EW>(&bar, gen, lane);

            if constexpr (P == 16) {
            // the block through a buffer resource based at the dword below
            // it: loads are dword aligned and anything past B reads 0 (the
            // bytes past B inside its last dword are masked in the last slice)
            const u32 mis = u32(reinterpret_cast<uintptr_t>(v.blk) & 3u);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<u8 *>(v.blk - mis), (short)0, int((v.B + mis + 3u) & ~3u), 0x00020000);
            const u32 nsl = (v.ps + ROWS - 1) / ROWS;
            const u32 rl = u32(wave * 64 + lane) * 4u;
            // DIAG: lane l walks a chunk's columns from (l & 15): its row
            // bytes rotated by r = l & 15 (dword rotation by two bit-field
            // selects, byte rotation by v_alignbyte), and step j's address
            // = x * 256 + slot((j + r) & 15), the slot bytes held in slot4[]:
            // the 16 lanes of every b128 lane group ({0-3,12-15,20-27}, ...:
            // distinct l & 15) read 16 distinct bank slots
            const u32 r16 = u32(lane & 15);
            const u32 mk2 = (r16 & 8u) ? ~0u : 0u, mk1 = (r16 & 4u) ? ~0u : 0u, rb = r16 & 3u;
            u32 slot4[4];
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                u32 x = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    x |= (((u32(4 * gq + i) + r16) & 15u) << 4) << (8 * i);
                slot4[gq] = x;
            }
            // every chunk's bytes of a slice's 4 rows, all loads in flight at
            // once: KC (k % 4 == 0, dword-aligned block) the 4k contiguous
            // bytes of the lane's rows in k/4 16-byte loads; otherwise per
            // row and chunk a 16 + 4-byte load, aligned by v_alignbyte
            constexpr int NR = KC ? 1 : 2;
            u32 raw[NR][4][5];
            u32 rw[KC ? KC : 1];
            auto load = [&](u32 r0) {
                if constexpr (KC) {
#pragma unroll
                    for (int i = 0; i < KC / 4; ++i) {
                        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, r0 * u32(KC) + 16u * u32(i), 0,
                                                                            NKFS_BE_SLC ? 2 : 0);
                        rw[4 * i] = x.x;
                        rw[4 * i + 1] = x.y;
                        rw[4 * i + 2] = x.z;
                        rw[4 * i + 3] = x.w;
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if (c >= nch)
                            break;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const u32 a = ((r0 + u32(q)) * u32(k) + 16u * u32(c) + mis) & ~3u;
                            const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, a, 0, 0);
                            raw[c][q][0] = x.x;
                            raw[c][q][1] = x.y;
                            raw[c][q][2] = x.z;
                            raw[c][q][3] = x.w;
                            raw[c][q][4] = __builtin_amdgcn_raw_buffer_load_b32(rs, a + 16u, 0, 0);
                        }
                    }
                }
            };
            load(rl);
#pragma unroll 1
            for (u32 sl = 0; sl < nsl; ++sl) {
                const u32 r0 = sl * ROWS + rl;
                if (HASH && NKFS_BE_LAG && !dyn) {
                    // at most NKFS_BE_LAG slices ahead of the unit's hash
                    // wave: its re-read of the parts stays in the XCD's L2
                    const u32 hw = ci % u32(HWV);
                    while (__hip_atomic_load(&hseq[hw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) +
                               u32(NKFS_BE_LAG) < seq + 1u)
                        __builtin_amdgcn_s_sleep(1);
                }
                const bool last = sl + 1 == nsl;
                uint4 acc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[q] = make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (c >= nch)
                        break;
                    u32 d[4][4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const u32 pos = (r0 + u32(q)) * u32(k) + 16u * u32(c);
                        if constexpr (KC) {
                            // dwords past the row's k bytes meet zero tables
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                d[q][w] = 4 * c + w < KC / 4 ? rw[q * (KC / 4) + 4 * c + w] : 0u;
                        } else {
                            const u32 sh = (pos + mis) & 3u;
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                d[q][w] = __builtin_amdgcn_alignbyte(raw[c % NR][q][w + 1], raw[c % NR][q][w], sh);
                        }
                        if (last) {
                            // bytes at or past B are zero (the reference
                            // zero-pads its tail row); columns past k meet
                            // zero tables
                            const u32 valid = v.B > pos ? min(v.B - pos, 16u) : 0u;
#pragma unroll
                            for (int w = 0; w < 4; ++w) {
                                const u32 keep = valid > u32(4 * w) ? min(valid - u32(4 * w), 4u) : 0u;
                                d[q][w] &= u32((u64(1) << (8 * keep)) - 1u);
                            }
                        }
                    }
                    if constexpr (DIAG) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            u32 a[4], b[4];
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                a[w] = mux3(mk2, d[q][(w + 2) & 3], d[q][w]);
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                b[w] = mux3(mk1, a[(w + 1) & 3], a[w]);
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                d[q][w] = __builtin_amdgcn_alignbyte(b[(w + 1) & 3], b[w], rb);
                        }
                    }
                    // columns in pairs (one three-input XOR per word folds
                    // both); tdep (0 at run time) keeps 16 lookups in flight
                    u32 tdep = u32(c) * 65536u;
#pragma unroll
                    for (int j = 0; j < 16; j += 2) {
                        if (!DIAG && 16 * c + j >= kk)
                            break;  // uniform (DIAG: every step, columns past k meet zero tables)
#if NKFS_BE_BATCH
                        // the pair's 8 lookups (4 rows x 2 columns) issued
                        // together, then folded: one LDS wait per 8 lookups
                        // (the per-row form waited for every 2)
                        uint4 la[4], lb[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if constexpr (DIAG) {
                                const u32 t0 = 0x0C0C0004u | (u32(j & 3) << 8) | u32(j & 3);
                                const u32 t1 = 0x0C0C0004u | (u32((j + 1) & 3) << 8) | u32((j + 1) & 3);
                                const u32 P0 = __builtin_amdgcn_perm(slot4[j >> 2], d[q][j >> 2], t0) + tdep;
                                const u32 P1 = __builtin_amdgcn_perm(slot4[(j + 1) >> 2], d[q][(j + 1) >> 2], t1) + tdep;
                                la[q] = *reinterpret_cast<const uint4 *>(tbl + P0);
                                lb[q] = *reinterpret_cast<const uint4 *>(tbl + P1);
                            } else {
                            const u32 s0 = 0x0C0C0C00u | u32(4 + (j & 3));
                            const u32 s1 = 0x0C0C0C00u | u32(4 + ((j + 1) & 3));
                            const u32 P0 = (__builtin_amdgcn_perm(d[q][j >> 2], 0u, s0) << 4) + tdep;
                            const u32 P1 = (__builtin_amdgcn_perm(d[q][(j + 1) >> 2], 0u, s1) << 4) + tdep;
                            la[q] = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + P0);
                            lb[q] = *reinterpret_cast<const uint4 *>(tbl + u32(j + 1) * 4096u + P1);
                            }
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            acc[q].x = xor3(acc[q].x, la[q].x, lb[q].x);
                            acc[q].y = xor3(acc[q].y, la[q].y, lb[q].y);
                            acc[q].z = xor3(acc[q].z, la[q].z, lb[q].z);
                            acc[q].w = xor3(acc[q].w, la[q].w, lb[q].w);
                        }
#else
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            uint4 a, c2;
                            if constexpr (DIAG) {
                                // byte 0: the slot of column (j + r) & 15, byte 1: x
                                const u32 t0 = 0x0C0C0004u | (u32(j & 3) << 8) | u32(j & 3);
                                const u32 t1 = 0x0C0C0004u | (u32((j + 1) & 3) << 8) | u32((j + 1) & 3);
                                const u32 P0 = __builtin_amdgcn_perm(slot4[j >> 2], d[q][j >> 2], t0) + tdep;
                                const u32 P1 = __builtin_amdgcn_perm(slot4[(j + 1) >> 2], d[q][(j + 1) >> 2], t1) + tdep;
                                a = *reinterpret_cast<const uint4 *>(tbl + P0);
                                c2 = *reinterpret_cast<const uint4 *>(tbl + P1);
                            } else {
                            const u32 s0 = 0x0C0C0C00u | u32(4 + (j & 3));
                            const u32 s1 = 0x0C0C0C00u | u32(4 + ((j + 1) & 3));
                            const u32 P0 = (__builtin_amdgcn_perm(d[q][j >> 2], 0u, s0) << 4) + tdep;
                            const u32 P1 = (__builtin_amdgcn_perm(d[q][(j + 1) >> 2], 0u, s1) << 4) + tdep;
                            a = *reinterpret_cast<const uint4 *>(tbl + u32(j) * 4096u + P0);
                            c2 = *reinterpret_cast<const uint4 *>(tbl + u32(j + 1) * 4096u + P1);
                            }
                            acc[q].x = xor3(acc[q].x, a.x, c2.x);
                            acc[q].y = xor3(acc[q].y, a.y, c2.y);
                            acc[q].z = xor3(acc[q].z, a.z, c2.z);
                            acc[q].w = xor3(acc[q].w, a.w, c2.w);
                        }
#endif
                        if (j & 2) {
                            u32 z;
                            asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(acc[3].x));
                            tdep = u32(c) * 65536u + z;
                        }
                    }
                }
                // (NKFS_BE_LATE_LOAD 0: the next slice's loads before the stores)
                if (!NKFS_BE_LATE_LOAD && !last)
                    load(r0 + ROWS);
                // row quad -> one dword of 4 rows per part
                if (r0 < v.ps) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const u32 *aw0 = &acc[0].x, *aw1 = &acc[1].x, *aw2 = &acc[2].x, *aw3 = &acc[3].x;
                        u32 o[4];
                        transpose4(aw0[w], aw1[w], aw2[w], aw3[w], o[0], o[1], o[2], o[3]);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int e = 4 * w + i;
                            if (e >= np)
                                break;
                            u8 *dst = v.parts + u64(p0 + e) * v.pitch + r0;
                            if (r0 + 4u <= v.ps) {
                                *reinterpret_cast<u32 *>(dst) = o[i];
                            } else {
                                for (u32 cb = 0; cb < 4 && r0 + cb < v.ps; ++cb)
                                    dst[cb] = u8(o[i] >> (8 * cb));
                            }
                        }
                    }
                }
                if constexpr (HASH) {
                    // this slice's stores are complete (in the L2) before
                    // the progress count the hash wave polls: a release
                    // fence orders them for the compiler (the s_waitcnt
                    // builtin alone does not: stores could sink below it),
                    // the asm wait for the hardware
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if constexpr (NKFS_BE_LATE_LOAD && KC != 0) {
                        // the KC/4 loads of the next slice may stay in flight
                        if (!last) {
                            load(r0 + ROWS);
                            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KC / 4) : "memory");
                        } else {
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        }
                    } else {
                        if (NKFS_BE_LATE_LOAD && !last)
                            load(r0 + ROWS);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    ++seq;
                    if (lane == 0)
                        __hip_atomic_store(&done[wave], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (NKFS_BE_SLICE_BAR)
                        enc_barrier<EW>(&bar, gen, lane);
                } else if (NKFS_BE_LATE_LOAD && !last) {
                    load(r0 + ROWS);
                }
            }
            } else {
            // P = 8 parts per unit, any k <= 76 (k > 32
            // without the column-chunked encoder's second XXH64 pass): per
            // slice, the lane's 4 rows in 16-column chunks -- a 16 + 4-byte
            // load per row and chunk, aligned by v_alignbyte (the byte shift
            // is uniform: a row starts at (4 l + q) k) -- chunk c + 1's loads
            // in flight under chunk c's lookups; one ds_read_b64 gives a
            // (row, column) term for the unit's 8 parts
            const u32 mis = u32(reinterpret_cast<uintptr_t>(v.blk) & 3u);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<u8 *>(v.blk - mis), (short)0, int((v.B + mis + 3u) & ~3u), 0x00020000);
            const u32 nsl = (v.ps + ROWS - 1) / ROWS;
            const u32 rl = u32(wave * 64 + lane) * 4u;
            constexpr int NCH = (BE_CMAX8 + 15) / 16;
            // DIAG: as the P = 16 path, with 8-byte entries at x * 128 + slot
            // * 8: the slot bytes hold slot * 16 and the address is halved
            const u32 r16 = u32(lane & 15);
            const u32 mk2 = (r16 & 8u) ? ~0u : 0u, mk1 = (r16 & 4u) ? ~0u : 0u, rb = r16 & 3u;
            u32 slot4[4];
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                u32 x = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    x |= (((u32(4 * gq + i) + r16) & 15u) << 4) << (8 * i);
                slot4[gq] = x;
            }
            u32 raw[2][4][5];
            auto load = [&](u32 (&x)[4][5], u32 r0, int c) {
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
            load(raw[0], rl, 0);
#pragma unroll 1
            for (u32 sl = 0; sl < nsl; ++sl) {
                const u32 r0 = sl * ROWS + rl;
                if (HASH && NKFS_BE_LAG && !dyn) {
                    // at most NKFS_BE_LAG slices ahead of the unit's hash
                    // wave: its re-read of the parts stays in the XCD's L2
                    const u32 hw = ci % u32(HWV);
                    while (__hip_atomic_load(&hseq[hw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) +
                               u32(NKFS_BE_LAG) < seq + 1u)
                        __builtin_amdgcn_s_sleep(1);
                }
                const bool last = sl + 1 == nsl;
                uint2 acc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[q] = make_uint2(0, 0);
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    if (c >= nch)
                        break;  // uniform
                    if (c + 1 < nch)
                        load(raw[(c + 1) & 1], r0, c + 1);
                    u32 d[4][4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const u32 pos = (r0 + u32(q)) * u32(k) + 16u * u32(c);
                        const u32 sh = (pos + mis) & 3u;
#pragma unroll
                        for (int w = 0; w < 4; ++w)
                            d[q][w] = __builtin_amdgcn_alignbyte(raw[c & 1][q][w + 1], raw[c & 1][q][w], sh);
                        if (last) {  // bytes at or past B are zero (crt/nk8.c:393-398)
                            const u32 valid = v.B > pos ? min(v.B - pos, 16u) : 0u;
#pragma unroll
                            for (int w = 0; w < 4; ++w) {
                                const u32 keep = valid > u32(4 * w) ? min(valid - u32(4 * w), 4u) : 0u;
                                d[q][w] &= u32((u64(1) << (8 * keep)) - 1u);
                            }
                        }
                    }
                    if constexpr (DIAG) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            u32 a[4], b[4];
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                a[w] = mux3(mk2, d[q][(w + 2) & 3], d[q][w]);
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                b[w] = mux3(mk1, a[(w + 1) & 3], a[w]);
#pragma unroll
                            for (int w = 0; w < 4; ++w)
                                d[q][w] = __builtin_amdgcn_alignbyte(b[(w + 1) & 3], b[w], rb);
                        }
                        // every step: columns past k meet zero tables
                        u32 tdep = u32(c) * 32768u;
#pragma unroll
                        for (int j = 0; j < 16; j += 2) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const u32 t0 = 0x0C0C0004u | (u32(j & 3) << 8) | u32(j & 3);
                                const u32 t1 = 0x0C0C0004u | (u32((j + 1) & 3) << 8) | u32((j + 1) & 3);
                                const u32 P0 = (__builtin_amdgcn_perm(slot4[j >> 2], d[q][j >> 2], t0) >> 1) + tdep;
                                const u32 P1 =
                                    (__builtin_amdgcn_perm(slot4[(j + 1) >> 2], d[q][(j + 1) >> 2], t1) >> 1) + tdep;
                                const uint2 a = *reinterpret_cast<const uint2 *>(tbl + P0);
                                const uint2 c2 = *reinterpret_cast<const uint2 *>(tbl + P1);
                                acc[q].x = xor3(acc[q].x, a.x, c2.x);
                                acc[q].y = xor3(acc[q].y, a.y, c2.y);
                            }
                            if (j & 2) {
                                u32 z;
                                asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(acc[3].x));
                                tdep = u32(c) * 32768u + z;
                            }
                        }
                        continue;
                    }
                    // columns in pairs, the bytes past k meet zero tables
                    u32 tdep = 0;
#pragma unroll
                    for (int j = 0; j < 16; j += 2) {
                        if (16 * c + j >= k)
                            break;  // uniform
                        const bool two = 16 * c + j + 1 < k;  // column j + 1 exists (no table past k)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const u32 s0 = 0x0C0C0C00u | u32(4 + (j & 3));
                            const u32 s1 = 0x0C0C0C00u | u32(4 + ((j + 1) & 3));
                            const u32 P0 = (__builtin_amdgcn_perm(d[q][j >> 2], 0u, s0) << 3) + tdep;
                            const u32 P1 = (__builtin_amdgcn_perm(d[q][(j + 1) >> 2], 0u, s1) << 3) + tdep;
                            const uint2 a = *reinterpret_cast<const uint2 *>(tbl + u32(16 * c + j) * TB + P0);
                            const uint2 c2 = two ? *reinterpret_cast<const uint2 *>(tbl + u32(16 * c + j + 1) * TB + P1)
                                                 : make_uint2(0, 0);
                            acc[q].x = xor3(acc[q].x, a.x, c2.x);
                            acc[q].y = xor3(acc[q].y, a.y, c2.y);
                        }
                        if (j & 2) {
                            u32 z;
                            asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(acc[3].x));
                            tdep = z;
                        }
                    }
                }
                // row quad -> one dword of 4 rows per part
                if (r0 < v.ps) {
#pragma unroll
                    for (int w = 0; w < 2; ++w) {
                        const u32 *aw0 = &acc[0].x, *aw1 = &acc[1].x, *aw2 = &acc[2].x, *aw3 = &acc[3].x;
                        u32 o[4];
                        transpose4(aw0[w], aw1[w], aw2[w], aw3[w], o[0], o[1], o[2], o[3]);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int e = 4 * w + i;
                            if (e >= np)
                                break;
                            u8 *dst = v.parts + u64(p0 + e) * v.pitch + r0;
                            if (r0 + 4u <= v.ps) {
                                *reinterpret_cast<u32 *>(dst) = o[i];
                            } else {
                                for (u32 cb = 0; cb < 4 && r0 + cb < v.ps; ++cb)
                                    dst[cb] = u8(o[i] >> (8 * cb));
                            }
                        }
                    }
                }
                // the next slice's first chunk after the stores; the progress
                // count waits for the stores only (the 8 loads stay in flight)
                if constexpr (HASH) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (!last) {
                        load(raw[0], r0 + ROWS, 0);
                        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    } else {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    ++seq;
                    if (lane == 0)
                        __hip_atomic_store(&done[wave], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else if (!last) {
                    load(raw[0], r0 + ROWS, 0);
                }
            }
            }
        }
    } else if constexpr (HASH) {
        if (NKFS_BE_HPRIO)
            __builtin_amdgcn_s_setprio(NKFS_BE_HPRIO);
        const int e = lane >> 2, a = lane & 3;
        u32 seq = 0;
#pragma unroll 1
        for (u32 ci = 0;; ++ci) {
            u32 u;
            if (dyn) {
                if (lane == 0)
                    __hip_atomic_store(&hdone, ci, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                while (__hip_atomic_load(&uq_n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= ci)
                    __builtin_amdgcn_s_sleep(8);
                u = uq[ci % 8];
                if (u == BE_END)
                    break;
            } else {
                u = blockIdx.x + ci * gridDim.x;
                if (u >= nunits)
                    break;
            }
            u32 grp;
            const u32 s = be_stripe(u, ngroups, grp);
            if (s >= g.nstripes)
                continue;
            const Stripe v = stripe_at(g, s);
            const int p0 = int(grp) * P, np = min(P, n - p0);  // P = 8: lanes 32.. idle (their e >= np)
            const u32 nsl = (v.ps + ROWS - 1) / ROWS;
            if (HWV > 1 && int(ci % u32(HWV)) != wave - EW) {
                seq += nsl;  // the other hash wave's unit
                if (NKFS_BE_LAG && lane == 0)
                    __hip_atomic_store(&hseq[wave - EW], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                continue;
            }
            const u32 nst = v.ps >> 5;  // whole 32-byte stripes of every part
            // the group's parts through one buffer resource (the launcher
            // checks n * pitch < 2^31); loads bypass the CU's L1 (sc0)
            const __amdgpu_buffer_rsrc_t pr =
                __builtin_amdgcn_make_buffer_rsrc(v.parts, (short)0, int(u64(n) * v.pitch), 0x00020000);
            const u32 pbase = u32(u64(p0 + min(e, np - 1)) * v.pitch);
            u64 hacc = xxh_acc_init(a, 0);
#pragma unroll 1
            for (u32 sl = 0; sl < nsl; ++sl) {
                if (NKFS_BE_LAG && lane == 0)  // the slices before this one are folded
                    __hip_atomic_store(&hseq[wave - EW], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                ++seq;
                if (!NKFS_BE_PROG) {
                    for (;;) {
                        const u32 dv = lane < EW ? __hip_atomic_load(&done[lane], __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP)
                                                    : 0xFFFFFFFFu;
                        if (!__ballot(dv < seq))
                            break;
                        __builtin_amdgcn_s_sleep(8);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
                const u32 rb = sl * (ROWS / 32u);
                const int re = int(min(rb + ROWS / 32u, nst));
                // a ring of 4 x 8 rounds: three batches' loads in flight
                // while one is folded (the chain is bound by its serial
                // rounds, ~35 ns each, not by the L2's latency).  Loads past
                // the slice's rounds are never folded and re-read its last
                // round: rows of the next slice are not stored yet, and a
                // line fetched early could still sit in the CU's L1 when
                // that slice is folded
                const u32 rlast = re > int(rb) ? u32(re) - 1u : rb;
                auto ld = [&](uint64_t (&w)[8], u32 r) {
                    if (NKFS_BE_PROG) {
                        // the 8 rounds from r (clamped like the loads) are
                        // encoder wave (r - rb) / 8's rows of this slice:
                        // wait for that wave's progress count only
                        const u32 sw = min((min(r, rlast) - rb) >> 3, u32(EW - 1));
                        while (__hip_atomic_load(&done[sw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < seq)
                            __builtin_amdgcn_s_sleep(2);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const u32 ri = min(r + u32(i), rlast);
                        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(pr, pbase + 32u * ri + 8u * u32(a), 0, 1);
                        w[i] = (u64(x.y) << 32) | x.x;
                    }
                };
                constexpr int RB = NKFS_BE_RING;  // batches of 8 rounds, RB - 1 in flight
                uint64_t w[RB][8];
#pragma unroll
                for (int i = 0; i < RB - 1; ++i)
                    ld(w[i], rb + 8u * u32(i));
#pragma unroll 1
                for (int r = int(rb); r < re; r += 8 * RB) {
#pragma unroll
                    for (int i = 0; i < RB; ++i) {
                        ld(w[(i + RB - 1) % RB], u32(r) + 8u * u32(i + RB - 1));
                        hacc = xxh_rounds<8>(hacc, w[i], re - r - 8 * i);
                    }
                }
            }
            if (NKFS_BE_LAG && lane == 0)
                __hip_atomic_store(&hseq[wave - EW], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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

// Decode a uniform or ragged batch with 2 <= k <= 254 from the plan
// k_decode_prep left in `work` (stripes with status != 0 are skipped), with
// table layout `mode` (0 byte tables, 1 nibble x 16 replicas in 16-survivor
// chunks, 2 nibble x 16 replicas in 8-survivor chunks, 3 every output column
// of a slice in one workgroup, 4 byte tables in the diagonal layout, 5 = 3
// with diagonal tables).
extern "C" int nkfs_bign_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, int mode,
                                hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > 254 || mode < 0 || mode > 5 || ((mode == 3 || mode == 5) && (k <= 8 || k > 64)))
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    if (u64(g->block_size) + 64u > 0x7FFFFFFFull)
        return -ENOSYS;
    // dword survivor loads through a buffer resource over a stripe's slots:
    // uniform batches with 4-byte aligned parts and pitch, slots < 2 GiB
    const bool pal = !g->block_sizes && ((reinterpret_cast<uintptr_t>(g->parts) | g->part_pitch) & 3) == 0 &&
                     u64(g->n) * g->part_pitch < 0x7FFFFFFFull;
    switch (mode) {
    case 0: return launch_bign<0>(g, work, status, pal, st);
    case 1: return launch_bign<1>(g, work, status, pal, st);
    case 2: return launch_bign<2>(g, work, status, pal, st);
    case 4: return launch_bign<4>(g, work, status, pal, st);
    case 5:  // layout 3 with diagonal tables (NG <= 3; beyond, layout 3)
        switch ((k + 15) / 16) {
        case 1: return launch_bigr<1, 1, true>(g, work, status, pal, st);
        case 2: return launch_bigr<2, 1, true>(g, work, status, pal, st);
        case 3: return launch_bigr<3, 1, true>(g, work, status, pal, st);
        default: return launch_bigr<4, 1, false>(g, work, status, pal, st);
        }
    default:
        switch ((k + 15) / 16) {
        case 1: return launch_bigr<1, 1, false>(g, work, status, pal, st);
        case 2: return launch_bigr<2, 1, false>(g, work, status, pal, st);
        case 3: return launch_bigr<3, 1, false>(g, work, status, pal, st);
        default: return launch_bigr<4, 1, false>(g, work, status, pal, st);
        }
    }
}

// Encode a uniform or ragged batch with k <= 32 on k_encode_bign (XXH64 of
// every part into digests when non-null), persistent or one workgroup per
// (stripe, part group).  -ENOSYS when the shape is outside
// what it handles (the caller takes the column-chunked encoder).
extern "C" int nkfs_bign_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, bool persist,
                                bool diag, hipStream_t st)
{
    const int k = g->k, n = g->n;
    if (k < 2 || k > BE_CMAX8 || n < k || g->part_min || g->part_max)
        return -ENOSYS;
    // k <= 32: units of 16 parts (16-byte table entries); 32 < k <= 76:
    // units of 8 parts, whose k tables of 8-byte entries still fit the LDS
    const int P = k <= BE_CMAX ? 16 : 8;
    if (!g->nstripes)
        return 0;
    // 4-byte aligned parts and pitch (dword stores); block offsets (rows +
    // one slice) and a stripe's part span inside 31 bits
    const u64 ps_max = (u64(g->block_size) + u64(k) - 1) / u64(k);  // ragged: block_size = the largest
    const u64 pitch_max = g->block_sizes ? (ps_max + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1) : g->part_pitch;
    if (((reinterpret_cast<uintptr_t>(g->parts) | (g->block_sizes ? 0 : g->part_pitch)) & 3) ||
        (ps_max + BE_ROWS) * u64(k) + 64 > 0x7FFFFFFFull || u64(n) * pitch_max > 0x7FFFFFFFull)
        return -ENOSYS;
    const u64 ngroups = (u64(n) + u64(P) - 1) / u64(P);
    const u64 nunits = (u64(g->nstripes) + 7) / 8 * 8 * ngroups;
    if (nunits > 0x7FFFFFFFull)
        return -EINVAL;
    // persist: one resident workgroup per CU (a multiple of 8: unit u stays
    // on XCD u mod 8); else one workgroup per unit
    const u64 cus = u64(nkfs_cu_count()) / 8 * 8;
    const u32 grid = u32(!persist || nunits < cus || !cus ? nunits : cus);
    // k % 4 == 0 with dword-aligned blocks (uniform batches): a lane's 4
    // rows in k/4 contiguous 16-byte loads (k-specialised kernels)
    const bool kc = !g->block_sizes && ((reinterpret_cast<uintptr_t>(g->blocks) | g->block_pitch) & 3) == 0;
    const int kk = P == 16 && kc && (k == 20 || k == 24 || k == 28 || k == 32) ? k : 0;
    // NKFS_BE_DYN: 8 zeroed per-XCD unit counters from the launch's scratch
    // (none to be had: the static walk)
    Scratch sc;
    u32 *uctr = nullptr;
    if (NKFS_BE_DYN && digests) {
        uctr = static_cast<u32 *>(sc.take(g, 256, st));
        if (uctr && hipMemsetAsync(uctr, 0, 32, st) != hipSuccess) {
            (void)hipGetLastError();
            uctr = nullptr;
        }
    }
    auto go = [&](auto hash, auto kcon) {
        if (diag || k == 32)
            hipLaunchKernelGGL((k_encode_bign<16, decltype(hash)::value, decltype(kcon)::value, true, NKFS_BE_HW>), dim3(grid),
                               dim3(64 * BE_WAVES), 0, st, *g, ids, digests, u32(ngroups), u32(nunits), uctr);
        else
            hipLaunchKernelGGL((k_encode_bign<16, decltype(hash)::value, decltype(kcon)::value, false, NKFS_BE_HW>), dim3(grid),
                               dim3(64 * BE_WAVES), 0, st, *g, ids, digests, u32(ngroups), u32(nunits), uctr);
    };
    auto pick = [&](auto hash) {
        if (P == 8) {
            if (k <= 64 && (diag || NKFS_BE_DIAG8))
                hipLaunchKernelGGL((k_encode_bign<8, decltype(hash)::value, 0, true, NKFS_BE_HW>), dim3(grid),
                                   dim3(64 * BE_WAVES), 0, st, *g, ids, digests, u32(ngroups), u32(nunits), uctr);
            else
            hipLaunchKernelGGL((k_encode_bign<8, decltype(hash)::value, 0, false, NKFS_BE_HW>), dim3(grid), dim3(64 * BE_WAVES), 0, st,
                               *g, ids, digests, u32(ngroups), u32(nunits), uctr);
            return;
        }
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
    const int rc = hipGetLastError() == hipSuccess ? 0 : -EIO;
    const int e = sc.finish();
    return rc ? rc : e;
}
