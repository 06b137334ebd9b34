// nk8_big.hip -- encode and decode for k > 16.  The reference accepts any
// 2 <= k <= n <= 255 with k <= 254 (crt/nk8.c:13-16, 356-360, 463-467), and
// its own load-time self test draws k uniform in [2, 254] (crt/nk8.c:735-744).
//
// Reference arithmetic: crt/nk8.c:403-420 -- part_i[j] = XOR_m x_i^m d[j*k+m]
// (d zero past block_size, :393-398); crt/nk8.c:552-582 -- block[j*k+m] =
// XOR_c part_c[j] W[c][m], W the inverse of the survivors' Vandermonde rows
// (k_decode_prep leaves the first k distinct survivors and W in `work`).
//
// Both directions are a per-stripe GF(2^8) matrix apply, k inputs -> n (or k)
// outputs per row.  With k > 16 the packed product tables of every input
// column no longer fit in LDS, so the inputs are taken 16 columns at a time:
// table j of a column chunk, U_j[x] = (M[j][o0] x, ..., M[j][o0+15] x),
// gives one row's term for 16 outputs per ds_read_b128, and a lane XORs the
// 16 terms of its row into a 16-byte accumulator that lives across chunks.
// Tables are rebuilt per chunk (64 KiB, four per wave by Gray-code walk) and
// amortised over a slice of thousands of rows.  Lane = row for the strided
// side (interleaved rows of k bytes: encode reads them, decode writes them),
// so one wave instruction covers 64 consecutive rows.
//
//  k_encode_big  workgroup = (stripe, group of 16 parts, slice of 4,096 rows);
//                a lane's row bytes come from dword-aligned 16+4-byte loads
//                and v_alignbyte (k is arbitrary); a slice's 16 x 256-row
//                outputs go through an LDS [part quad][row] stage and a 4x4
//                byte transpose, so each store instruction writes 256
//                contiguous bytes of one part.  The groups of a (stripe,
//                slice) are dispatched back to back on one XCD (workgroup b
//                runs on XCD b mod 8) and share the block's lines in its L2.
//  k_decode_big  workgroup = (stripe, group of 16 output columns, slice of
//                4,096 rows); a chunk's 16 survivor parts come through an
//                LDS [row][survivor] stage 512 rows at a time (coalesced
//                dword loads, 4x4 byte transposes); a lane writes its
//                rows' 16 columns, and the
//                groups of a (stripe, slice) run back to back on one XCD so
//                the rows' lines complete in its L2.
// XXH64 of the parts is fused into k_encode_big: a part's chain is serial over
// all of its rows and a stripe's rows are spread over slices, so slice i's
// workgroup continues the 64 chains of its part group from the accumulators
// slice i-1's workgroup published (BigChain, below).
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

constexpr int ENC_T = 16;                    // rows per lane per encode slice
constexpr u32 ENC_ROWS = 256u * ENC_T;       // rows per encode workgroup

__device__ inline __amdgpu_buffer_rsrc_t brsrc(const void *base, u32 bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}

// x^e over GF(2^8) by the log/antilog tables staged in LDS (x^0 = 1)
__device__ inline u32 gf_pow(const uint16_t *lg, const u8 *ex, u32 x, u32 e)
{
    if (!x)
        return e ? 0u : 1u;
    return ex[(u32(lg[x]) * e) % 255u];
}

// Chain hand-off of the fused XXH64 (HASH): one record per (stripe, group of
// 16 parts) -- the 64 accumulators (16 parts x 4) after the slices folded so
// far and a flag = the number of slices folded (agent-scope release/acquire).
struct BigChain {
    u64 *acc;       // [units][64]
    u32 *flag;      // [units], zeroed before the launch
    u32 *fail;      // set when a wait timed out: k_big_hash_fix recomputes the digests
    u64 *digests;   // [stripe][n]
};

// this wave's XCC (hardware register XCC_ID, bits 3:0)
__device__ inline u32 xcc_id() { return u32(__builtin_amdgcn_s_getreg(20 | (3 << 11))) & 15u; }

// NKFS_BIG_DIAG (default 1): k_encode_big's chunk tables in the diagonal
// layout -- entry x of column j at x * 256 + j * 16, the 16 tables in the 16
// bank slots of each x row -- and lane l walks a row's 16 columns from
// (l & 15) (its bytes rotated by l & 15): the 16 lanes of every b128 lane
// group read 16 distinct bank slots instead of random ones
#ifndef NKFS_BIG_DIAG
#define NKFS_BIG_DIAG 1
#endif

// a ^ b ^ c and mask ? a : b per bit, each one v_bitop3_b32 (operand truth
// tables S0 0xF0, S1 0xCC, S2 0xAA)
__device__ __forceinline__ u32 big_mux(u32 mask, u32 a, u32 b)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xE4" : "=v"(r) : "v"(a), "v"(b), "v"(mask));
    return r;
}

constexpr u64 CHAIN_TIMEOUT = 200000;  // s_memrealtime ticks (100 MHz): 2 ms (a slice takes ~35 us)

template <bool HASH>
__global__ __launch_bounds__(256, 2) void k_encode_big(nkfs_geom g, const u8 *ids, const GfTables *gft,
                                                       u32 ngroups, u32 nslices, BigChain ch)
{
    __shared__ __attribute__((aligned(16))) u8 tbl[16 * 256 * 16];   // 16 tables of 256 x 16 B
    __shared__ __attribute__((aligned(16))) u32 stage[4 * 256];      // [part quad][row]
    __shared__ __attribute__((aligned(16))) uint4 coef[256];         // coef[m] = (x_{p0+e}^m), e < 16
    // HASH: [part][row] copy of a 256-row unit for the XXH64 lanes, in
    // coef's 4 KiB (coef is dead once the last chunk's tables are built):
    // the LDS request stays at two workgroups per CU
    u8 *const hx = reinterpret_cast<u8 *>(coef);
    __shared__ uint16_t glog[256];
    __shared__ u8 gexp[256];

    // workgroup b runs on XCD b mod 8; slice-major over (slice, stripe octet,
    // group): the groups of a (stripe, slice) run back to back on one XCD
    // (they share the block's lines in its L2), and slice i of a (stripe,
    // group) is dispatched 8 * ngroups * octets workgroups after slice i-1,
    // on the same XCD (the XXH64 chain hand-off below waits on it)
    const u32 b = blockIdx.x;
    const u32 loc = b >> 3;
    const u32 noct = (g.nstripes + 7) / 8;
    const u32 grp = loc % ngroups;
    const u32 slice = loc / (ngroups * noct);
    const u32 s = ((loc / ngroups) % noct) * 8 + (b & 7);
    if (s >= g.nstripes || slice >= nslices)
        return;  // the whole workgroup: no barrier is skipped by part of it
    const Stripe v = stripe_at(g, s);
    const u32 r_begin = slice * ENC_ROWS;
    if (r_begin >= v.ps)
        return;
    const int n = g.n, k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int p0 = int(grp) * 16, np = min(16, n - p0);

    // Vandermonde rows of the group's parts: coef[m] byte e = x_{p0+e}^m
    // (crt/nk8.c:404-406 builds the same powers by repeated multiplication),
    // from log/antilog tables staged in LDS
    glog[tid] = gft->log[tid];
    gexp[tid] = gft->exp[tid];
    __syncthreads();
    {
        const u8 *sid = ids + u64(s) * u64(n) + p0;
        u32 xs[16];
#pragma unroll
        for (int e = 0; e < 16; ++e)
            xs[e] = e < np ? sid[e] : 0u;
        for (int m = tid; m < k; m += 256) {
            u32 w[4] = {0, 0, 0, 0};
#pragma unroll
            for (int e = 0; e < 16; ++e)
                if (e < np)
                    w[e >> 2] |= gf_pow(glog, gexp, xs[e], u32(m)) << (8 * (e & 3));
            coef[m] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }

    // the stripe's block through a buffer resource based at the dword below
    // it: loads are dword aligned and anything past B reads 0 (the tail
    // bytes inside the last dword are masked below)
    const u32 mis = u32(reinterpret_cast<uintptr_t>(v.blk) & 3u);
    const __amdgpu_buffer_rsrc_t rs = brsrc(v.blk - mis, (v.B + mis + 3u) & ~3u);

    uint4 acc[ENC_T];
#pragma unroll
    for (int t = 0; t < ENC_T; ++t)
        acc[t] = make_uint4(0, 0, 0, 0);
    // NKFS_BIG_DIAG: this lane's rotation r = l & 15 and the slot bytes
    // (byte i of dslot[gq] = ((4 gq + i + r) & 15) * 16)
    const u32 r16 = u32(lane & 15);
    const u32 mk8 = (r16 & 8u) ? ~0u : 0u, mk4 = (r16 & 4u) ? ~0u : 0u, rb3 = r16 & 3u;
    u32 dslot[4];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
        u32 x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            x |= (((u32(4 * gq + i) + r16) & 15u) << 4) << (8 * i);
        dslot[gq] = x;
    }

    const int nch = (k + 15) / 16;
    for (int cc = 0; cc < nch; ++cc) {
        __syncthreads();  // coef[] written / the previous chunk's lookups done
        if (NKFS_BIG_DIAG) {
            // lane l builds table j = l & 15, entries x = (l >> 4) + 4 i + 64
            // wave (Gray-code walk over i < 16): the 8 lanes of a
            // ds_write_b128 group write 8 slots of one x row (no conflict)
            const int j = lane & 15, xl = lane >> 4, m = 16 * cc + j;
            const uint4 c = m < k ? coef[m] : make_uint4(0, 0, 0, 0);  // columns past k: zero table
            const u32 row[4] = {c.x, c.y, c.z, c.w};
            u32 basis[8][4];
            make_basis<4>(basis, row);
            u32 hv[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                u32 e = 0;
#pragma unroll
                for (int bb = 0; bb < 2; ++bb) {
                    e ^= basis[bb][w] & (0u - ((u32(xl) >> bb) & 1u));
                    e ^= basis[6 + bb][w] & (0u - ((u32(wave) >> bb) & 1u));
                }
                hv[w] = e;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i) {
                    const int bit = __builtin_ctz(i);
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        hv[w] ^= basis[2 + bit][w];
                }
                const u32 x = u32(xl) + 4u * u32(i ^ (i >> 1)) + 64u * u32(wave);
                *reinterpret_cast<uint4 *>(tbl + x * 256u + u32(j) * 16u) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            }
        } else {
        // wave w builds tables j = w, w+4, w+8, w+12 of columns 16cc + j
#pragma unroll 1
        for (int q = 0; q < 4; ++q) {
            const int j = wave + 4 * q, m = 16 * cc + j;
            const uint4 c = m < k ? coef[m] : make_uint4(0, 0, 0, 0);  // columns past k: zero table
            const u32 row[4] = {c.x, c.y, c.z, c.w};
            u32 basis[8][4];
            make_basis<4>(basis, row);
            build_table16(tbl + j * 4096, basis, lane);
        }
        }
        __syncthreads();
        // tdep (0 at run time) chains each row's lookups and the next row's
        // loads behind the previous row's XORs: unchained, the compiler
        // hoists all 16 rows' loads and 256 lookups and spills
        // only the slice holding the stripe's last row reads bytes past B:
        // the masking is compiled into a second copy of the row loop
        const bool tail = (u64(r_begin) + ENC_ROWS) * u64(k) > u64(v.B);
        auto rows = [&](auto mask) {
            constexpr bool MASK = decltype(mask)::value;
            // tdep (0 at run time) chains each row's lookups and the next
            // row's loads behind the previous row's XORs: unchained, the
            // compiler hoists all 16 rows' loads and 256 lookups and spills
            u32 tdep = 0;
            auto load = [&](int t, v4u &x, u32 &x4, u32 &pos) {
                const u32 r = r_begin + u32(t) * 256u + u32(tid);
                pos = r * u32(k) + 16u * u32(cc);  // block byte of column 16cc of row r
                const u32 a = (pos + mis + tdep) & ~3u;
                x = __builtin_amdgcn_raw_buffer_load_b128(rs, a, 0, 0);
                x4 = __builtin_amdgcn_raw_buffer_load_b32(rs, a + 16u, 0, 0);
            };
            v4u xc, xn;
            u32 x4c, x4n, posc, posn;
            load(0, xc, x4c, posc);
#pragma unroll
            for (int t = 0; t < ENC_T; ++t) {
                if (t + 1 < ENC_T)
                    load(t + 1, xn, x4n, posn);
                const u32 sh = (posc + mis) & 3u;
                u32 d[4];
                d[0] = __builtin_amdgcn_alignbyte(xc.y, xc.x, sh);
                d[1] = __builtin_amdgcn_alignbyte(xc.z, xc.y, sh);
                d[2] = __builtin_amdgcn_alignbyte(xc.w, xc.z, sh);
                d[3] = __builtin_amdgcn_alignbyte(x4c, xc.w, sh);
                if constexpr (MASK) {
                    // bytes at or past B are zero (the reference zero-pads
                    // its tail row, crt/nk8.c:393-398); columns past k meet
                    // zero tables
                    const u32 valid = v.B > posc ? min(v.B - posc, 16u) : 0u;
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const u32 keep = valid > u32(4 * w) ? min(valid - u32(4 * w), 4u) : 0u;
                        d[w] &= u32((u64(1) << (8 * keep)) - 1u);
                    }
                }
                uint4 e = acc[t];
                if (NKFS_BIG_DIAG) {
                    // the row's 16 bytes rotated by r = l & 15 (dword
                    // rotation by two mux stages, byte rotation by
                    // v_alignbyte); step j: column (j + r) & 15, address
                    // x * 256 + its slot (dslot bytes)
                    u32 a[4], b2[4];
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        a[w] = big_mux(mk8, d[(w + 2) & 3], d[w]);
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        b2[w] = big_mux(mk4, a[(w + 1) & 3], a[w]);
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        d[w] = __builtin_amdgcn_alignbyte(b2[(w + 1) & 3], b2[w], rb3);
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const u32 sel = 0x0C0C0004u | (u32(j & 3) << 8) | u32(j & 3);
                        const u32 P = __builtin_amdgcn_perm(dslot[j >> 2], d[j >> 2], sel) + tdep;
                        const uint4 tv = *reinterpret_cast<const uint4 *>(tbl + P);
                        e.x ^= tv.x;
                        e.y ^= tv.y;
                        e.z ^= tv.z;
                        e.w ^= tv.w;
                    }
                } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const u32 byte = (d[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                    const uint4 tv = *reinterpret_cast<const uint4 *>(tbl + tdep + j * 4096 + byte * 16);
                    e.x ^= tv.x;
                    e.y ^= tv.y;
                    e.z ^= tv.z;
                    e.w ^= tv.w;
                }
                }
                acc[t] = e;
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(e.x), "v"(e.y), "v"(e.z), "v"(e.w));
                xc = xn;
                x4c = x4n;
                posc = posn;
            }
        };
        if (tail)
            rows(std::true_type{});
        else
            rows(std::false_type{});
    }

    // XXH64 of the group's parts, fused (HASH): lane 4j + a < 16 of wave w
    // is accumulator a of part p0 + 4w + j -- each wave hashes the four parts
    // it transposes and stores, so a unit's fold needs no workgroup barrier
    // and the four waves' serial rounds overlap.  The chain of a part is
    // serial over all its rows, so slice i continues from the accumulators
    // slice i-1's workgroup published (dispatched earlier on this XCD,
    // normally long done); each 256-row unit is folded from the wave's LDS
    // [part][row] copy of its outputs
    __shared__ int chain_bad;
    const int he = 4 * wave + (lane >> 2), ha = lane & 3;  // hash role of lanes < 16
    const bool hl = lane < 16;
    const u32 unit = s * ngroups + grp;
    const u32 nst = v.ps >> 5;  // whole 32-byte stripes of every part
    const u32 last = (v.ps - 1) / ENC_ROWS;
    u64 hacc = 0;
    bool hok = true;
    if (HASH) {
        hacc = xxh_acc_init(ha, 0);
        if (tid == 0)
            chain_bad = 0;
        if (slice > 0) {
            // the hand-off stays inside this XCD's L2: the producer (slice
            // i-1) ran on the same XCD, its stores reached the L2 before its
            // flag did, and these loads bypass the CU's L1 (sc0); an
            // agent-scope release would write the whole L2 back per slice
            const __amdgpu_buffer_rsrc_t fr = brsrc(ch.flag + unit, 4), xr = brsrc(ch.fail, 4);
            const u64 t0 = __builtin_amdgcn_s_memrealtime();
            u32 f;
            for (;;) {
                f = __builtin_amdgcn_raw_buffer_load_b32(fr, 0, 0, 1);
                if ((f & 0xFFFFFFu) >= slice || __builtin_amdgcn_raw_buffer_load_b32(xr, 0, 0, 1))
                    break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > CHAIN_TIMEOUT) {
                    if (lane == 0)
                        __hip_atomic_store(ch.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            // the hand-off is only coherent inside one XCD's L2: the flag
            // carries the producer's XCC id, and a chain whose
            // producer ran elsewhere is treated as lost -- recomputed by
            // k_big_hash_fix -- instead of trusting possibly stale lines
            hok = f != 0xFFFFFFFFu && (f & 0xFFFFFFu) >= slice && (f >> 24) == xcc_id();
            if (!hok && f != 0xFFFFFFFFu && (f & 0xFFFFFFu) >= slice && lane == 0)
                __hip_atomic_store(ch.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (hok) {
                const v2u w = __builtin_amdgcn_raw_buffer_load_b64(brsrc(ch.acc + u64(unit) * 64, 512),
                                                                   u32(16 * wave + (lane & 15)) * 8u, 0, 1);
                hacc = (u64(w.y) << 32) | w.x;
            }
        }
    }

    // 256 rows x 16 parts per t-unit: [part quad][row] in LDS (conflict-free
    // dword writes), read back as 4 rows x 4 parts (ds_read_b128), 4x4 byte
    // transpose, one dword of 4 rows per part: wave w stores parts
    // 4w..4w+3, 64 lanes x 4 B = 256 contiguous bytes per instruction
    const bool pal = ((reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 3) == 0;
    u64 tw[4] = {0, 0, 0, 0};  // a part's tail bytes (< 32), for its digest
#pragma unroll
    for (int t = 0; t < ENC_T; ++t) {
        const u32 rt = r_begin + u32(t) * 256u;
        if (rt >= v.ps)
            break;  // workgroup-uniform
        __syncthreads();
        stage[0 * 256 + tid] = acc[t].x;
        stage[1 * 256 + tid] = acc[t].y;
        stage[2 * 256 + tid] = acc[t].z;
        stage[3 * 256 + tid] = acc[t].w;
        __syncthreads();
        const uint4 q4 = *reinterpret_cast<const uint4 *>(stage + wave * 256 + 4 * lane);
        u32 o[4];
        transpose4(q4.x, q4.y, q4.z, q4.w, o[0], o[1], o[2], o[3]);
        const u32 rr = rt + 4u * u32(lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * wave + j;
            if constexpr (HASH)
                *reinterpret_cast<u32 *>(hx + e * 256 + 4 * lane) = o[j];  // this wave's own 1 KiB
            if (e < np && rr < v.ps) {
                u8 *dst = v.parts + u64(p0 + e) * v.pitch + rr;
                if (pal && rr + 4u <= v.ps) {
                    *reinterpret_cast<u32 *>(dst) = o[j];
                } else {
                    for (u32 c = 0; c < 4 && rr + c < v.ps; ++c)
                        dst[c] = u8(o[j] >> (8 * c));
                }
            }
        }
        if constexpr (HASH) {
            // this wave's parts only: its LDS writes above are ordered before
            // these reads (one wave), so no workgroup barrier is needed
            __builtin_amdgcn_wave_barrier();
            if (hl) {
                // rounds of the 32-byte stripes that lie wholly below ps
                const u8 *src = hx + he * 256 + 8 * ha;
                const u32 s0 = rt >> 5;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const u64 w = *reinterpret_cast<const u64 *>(src + 32 * r);
                    const u64 nx = xxh_round(hacc, w);
                    hacc = s0 + u32(r) < nst ? nx : hacc;
                }
                // the tail (ps & 31 bytes after the last whole stripe) lies
                // in this unit: keep its words for the digest
                if ((v.ps & 31) && nst * 32 >= rt && nst * 32 < rt + 256) {
                    const u64 *tp = reinterpret_cast<const u64 *>(hx + he * 256 + (nst * 32 - rt));
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        tw[w] = tp[w];
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if constexpr (HASH) {
        if (slice < last) {
            // publish: every wave's accumulators, then (after all of them
            // reached this XCD's L2) the flag; a chain that could not be
            // continued passes the failure on at once so no successor waits
            if (hl)
                ch.acc[u64(unit) * 64 + 16 * wave + lane] = hacc;
            if (!hok)
                chain_bad = 1;
            __builtin_amdgcn_s_waitcnt(0);  // the accumulators are in the L2 before the flag
            __syncthreads();
            if (tid == 0)
                __hip_atomic_store(ch.flag + unit, chain_bad ? 0xFFFFFFFFu : (xcc_id() << 24) | (slice + 1), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            const int base = lane & ~3;
            const u64 v1 = shfl64(hacc, base), v2 = shfl64(hacc, base + 1);
            const u64 v3 = shfl64(hacc, base + 2), v4 = shfl64(hacc, base + 3);
            if (hok && hl && ha == 0 && he < np) {
                u64 h = v.ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
                h += v.ps;
                ch.digests[u64(s) * u64(n) + u64(p0 + he)] = xxh_tail_regs(h, tw, v.ps & 31);
            }
        }
    }
}

// k_encode_big without the fused XXH64, in workgroups of 8 waves sharing one
// chunk table (NKFS_BIG_W8): k_encode_big's 72 KiB of LDS per 4-wave
// workgroup allow two per CU, 8 waves, and its SQ counters show half of
// their time waiting (W3: 7.7 waves per CU, 48 % wait,
// profiles/r06/sq_w3final_summary.txt); here two 8-wave workgroups share the
// CU's LDS the same way: 16 waves.  Same slice (4,096 rows = 512 lanes x 8),
// diagonal tables, output through a [part quad][512 rows] stage.  W3 1,001
// -> 1,135 GB/s, N40K33 1,074 -> 1,275, N80K70 850 -> 959 (with the XXH64
// pass; profiles/r06/ab_big8.txt)
#ifndef NKFS_BIG_W8
#define NKFS_BIG_W8 1
#endif
constexpr int ENC8_T = 8;  // rows per lane per slice (512 lanes: ENC_ROWS rows)
static_assert(512 * ENC8_T == int(ENC_ROWS), "same slice as k_encode_big");

__global__ __launch_bounds__(512, 4) void k_encode_big8(nkfs_geom g, const u8 *ids, const GfTables *gft,
                                                        u32 ngroups, u32 nslices)
{
    __shared__ __attribute__((aligned(16))) u8 tbl[16 * 256 * 16];   // 16 diagonal tables
    __shared__ __attribute__((aligned(16))) u32 stage[4 * 512];      // [part quad][row]
    __shared__ __attribute__((aligned(16))) uint4 coef[256];
    __shared__ uint16_t glog[256];
    __shared__ u8 gexp[256];

    const u32 b = blockIdx.x;
    const u32 loc = b >> 3;
    const u32 noct = (g.nstripes + 7) / 8;
    const u32 grp = loc % ngroups;
    const u32 slice = loc / (ngroups * noct);
    const u32 s = ((loc / ngroups) % noct) * 8 + (b & 7);
    if (s >= g.nstripes || slice >= nslices)
        return;  // the whole workgroup
    const Stripe v = stripe_at(g, s);
    const u32 r_begin = slice * ENC_ROWS;
    if (r_begin >= v.ps)
        return;
    const int n = g.n, k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int p0 = int(grp) * 16, np = min(16, n - p0);

    if (tid < 256) {
        glog[tid] = gft->log[tid];
        gexp[tid] = gft->exp[tid];
    }
    __syncthreads();
    {
        const u8 *sid = ids + u64(s) * u64(n) + p0;
        u32 xs[16];
#pragma unroll
        for (int e = 0; e < 16; ++e)
            xs[e] = e < np ? sid[e] : 0u;
        for (int m = tid; m < k; m += 512) {
            u32 w[4] = {0, 0, 0, 0};
#pragma unroll
            for (int e = 0; e < 16; ++e)
                if (e < np)
                    w[e >> 2] |= gf_pow(glog, gexp, xs[e], u32(m)) << (8 * (e & 3));
            coef[m] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    const u32 mis = u32(reinterpret_cast<uintptr_t>(v.blk) & 3u);
    const __amdgpu_buffer_rsrc_t rs = brsrc(v.blk - mis, (v.B + mis + 3u) & ~3u);
    uint4 acc[ENC8_T];
#pragma unroll
    for (int t = 0; t < ENC8_T; ++t)
        acc[t] = make_uint4(0, 0, 0, 0);
    const u32 r16 = u32(lane & 15);
    const u32 mk8 = (r16 & 8u) ? ~0u : 0u, mk4 = (r16 & 4u) ? ~0u : 0u, rb3 = r16 & 3u;
    u32 dslot[4];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
        u32 x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            x |= (((u32(4 * gq + i) + r16) & 15u) << 4) << (8 * i);
        dslot[gq] = x;
    }
    const int nch = (k + 15) / 16;
    for (int cc = 0; cc < nch; ++cc) {
        __syncthreads();  // coef[] written / the previous chunk's lookups done
        {
            // lane l of wave w builds table j = l & 15, entries x = (l >> 4)
            // + 4 i + 32 w (Gray-code walk over i < 8)
            const int j = lane & 15, xl = lane >> 4, m = 16 * cc + j;
            const uint4 c = m < k ? coef[m] : make_uint4(0, 0, 0, 0);
            const u32 row[4] = {c.x, c.y, c.z, c.w};
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
        }
        __syncthreads();
        const bool tail = (u64(r_begin) + ENC_ROWS) * u64(k) > u64(v.B);
        auto rows = [&](auto mask) {
            constexpr bool MASK = decltype(mask)::value;
            u32 tdep = 0;
            auto load = [&](int t, v4u &x, u32 &x4, u32 &pos) {
                const u32 r = r_begin + u32(t) * 512u + u32(tid);
                pos = r * u32(k) + 16u * u32(cc);
                const u32 a = (pos + mis + tdep) & ~3u;
                x = __builtin_amdgcn_raw_buffer_load_b128(rs, a, 0, 0);
                x4 = __builtin_amdgcn_raw_buffer_load_b32(rs, a + 16u, 0, 0);
            };
            v4u xc, xn;
            u32 x4c, x4n, posc, posn;
            load(0, xc, x4c, posc);
#pragma unroll
            for (int t = 0; t < ENC8_T; ++t) {
                if (t + 1 < ENC8_T)
                    load(t + 1, xn, x4n, posn);
                const u32 sh = (posc + mis) & 3u;
                u32 d[4];
                d[0] = __builtin_amdgcn_alignbyte(xc.y, xc.x, sh);
                d[1] = __builtin_amdgcn_alignbyte(xc.z, xc.y, sh);
                d[2] = __builtin_amdgcn_alignbyte(xc.w, xc.z, sh);
                d[3] = __builtin_amdgcn_alignbyte(x4c, xc.w, sh);
                if constexpr (MASK) {
                    const u32 valid = v.B > posc ? min(v.B - posc, 16u) : 0u;
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const u32 keep = valid > u32(4 * w) ? min(valid - u32(4 * w), 4u) : 0u;
                        d[w] &= u32((u64(1) << (8 * keep)) - 1u);
                    }
                }
                u32 a[4], b2[4];
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    a[w] = big_mux(mk8, d[(w + 2) & 3], d[w]);
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    b2[w] = big_mux(mk4, a[(w + 1) & 3], a[w]);
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    d[w] = __builtin_amdgcn_alignbyte(b2[(w + 1) & 3], b2[w], rb3);
                uint4 e = acc[t];
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    if (j == 8) {  // eight lookups in flight at most (128 VGPRs)
                        u32 z;
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(e.x));
                        tdep += z;
                    }
                    const u32 sel = 0x0C0C0004u | (u32(j & 3) << 8) | u32(j & 3);
                    const u32 P = __builtin_amdgcn_perm(dslot[j >> 2], d[j >> 2], sel) + tdep;
                    const uint4 tv = *reinterpret_cast<const uint4 *>(tbl + P);
                    e.x ^= tv.x;
                    e.y ^= tv.y;
                    e.z ^= tv.z;
                    e.w ^= tv.w;
                }
                acc[t] = e;
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(e.x), "v"(e.y), "v"(e.z), "v"(e.w));
                xc = xn;
                x4c = x4n;
                posc = posn;
            }
        };
        if (tail)
            rows(std::true_type{});
        else
            rows(std::false_type{});
    }

    // 512 rows x 16 parts per t-unit: [part quad][row] in LDS, read back as 4
    // rows x 4 parts, 4x4 byte transpose: wave w stores part quad w & 3 of
    // rows (w >> 2) * 256 .., 256 contiguous bytes of a part per instruction
    const bool pal = ((reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 3) == 0;
    const int pq = wave & 3, half = wave >> 2;
#pragma unroll
    for (int t = 0; t < ENC8_T; ++t) {
        const u32 rt = r_begin + u32(t) * 512u;
        if (rt >= v.ps)
            break;  // workgroup-uniform
        __syncthreads();
        stage[0 * 512 + tid] = acc[t].x;
        stage[1 * 512 + tid] = acc[t].y;
        stage[2 * 512 + tid] = acc[t].z;
        stage[3 * 512 + tid] = acc[t].w;
        __syncthreads();
        const uint4 q4 = *reinterpret_cast<const uint4 *>(stage + pq * 512 + half * 256 + 4 * lane);
        u32 o[4];
        transpose4(q4.x, q4.y, q4.z, q4.w, o[0], o[1], o[2], o[3]);
        const u32 rr = rt + u32(half) * 256u + 4u * u32(lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * pq + j;
            if (e < np && rr < v.ps) {
                u8 *dst = v.parts + u64(p0 + e) * v.pitch + rr;
                if (pal && rr + 4u <= v.ps) {
                    *reinterpret_cast<u32 *>(dst) = o[j];
                } else {
                    for (u32 c = 0; c < 4 && rr + c < v.ps; ++c)
                        dst[c] = u8(o[j] >> (8 * c));
                }
            }
        }
    }
}

// The fused hash's safety net: when a chain wait timed out (ch.fail; not
// expected -- slice i-1 is dispatched long before slice i on the same XCD),
// every part's digest is recomputed here, four lanes per part; otherwise
// every workgroup returns at once.
__global__ __launch_bounds__(256) void k_big_hash_fix(nkfs_geom g, const u32 *fail, u64 *digests)
{
    if (!__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return;
    const u64 t = u64(blockIdx.x) * blockDim.x + threadIdx.x;
    const u64 msg = t >> 2;
    const int a = int(t & 3);
    const bool live = msg < u64(g.nstripes) * u64(g.n);
    const u8 *p = nullptr;
    u32 len = 0;
    if (live) {
        const u32 s = u32(msg / u32(g.n)), i = u32(msg % u32(g.n));
        const Stripe v = stripe_at(g, s);
        p = v.parts + u64(i) * v.pitch;
        len = v.ps;
    }
    u64 acc = xxh_acc_init(a, 0);
    const u32 nst = len >> 5;
    for (u32 r = 0; r < nst; ++r) {
        u64 w = 0;
        for (int c = 0; c < 8; ++c)  // ragged part bases: byte loads
            w |= u64(p[u64(r) * 32 + 8 * a + c]) << (8 * c);
        acc = xxh_round(acc, w);
    }
    const int base = int(threadIdx.x & 63) & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    if (!live || a != 0)
        return;
    u64 h = len >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
    h += len;
    u64 tw[4] = {0, 0, 0, 0};
    for (u32 c = 0; c < (len & 31); ++c)
        tw[c >> 3] |= u64(p[u64(nst) * 32 + c]) << (8 * (c & 7));
    digests[msg] = xxh_tail_regs(h, tw, len & 31);
}

// Up to 4 bytes (left >= 1; fewer when left < 4) from an unaligned address,
// byte by byte: ragged batches with unaligned part offsets only.
// Branch-free (clamped addresses, then a select): conditional loads would
// cost the common path its registers in exec-mask juggling.
__device__ __forceinline__ u32 load4_bytes(const u8 *p, u32 left)
{
    u32 w = 0;
#pragma unroll
    for (u32 e = 0; e < 4; ++e) {
        const u32 b = p[e < left ? e : left - 1];
        w |= (e < left ? b : 0u) << (8 * e);
    }
    return w;
}

// Decode: one workgroup per (stripe, group of 16 output columns, slice of
// 256*DEC_T rows); the survivors come through the LDS stage SUB rows at a
// time, so a chunk's tables serve the whole slice.
constexpr int DEC_T = 16;                 // rows per lane per slice
constexpr u32 DEC_ROWS = 256u * DEC_T;    // 4,096
constexpr u32 SUB = 512;                  // rows per survivor stage: 64 KiB tables + 10 KiB, two workgroups per CU

// PAL: every stripe's parts 16-byte aligned (the launcher knows it for
// uniform batches; ragged ones take the byte-wise form)
template <bool PAL>
__global__ __launch_bounds__(256, 2) void k_decode_big(nkfs_geom g, const u8 *work, const int32_t *status,
                                                       u32 ngroups, u32 nslices)
{
    __shared__ __attribute__((aligned(16))) u8 tbl[16 * 256 * 16];
    // survivor bytes of a sub-block, [row][survivor] at a 20-byte row pitch
    // (odd in dwords: the transposing byte writes spread over the banks)
    __shared__ __attribute__((aligned(16))) u8 ins[20 * SUB];
    // W[16cc+j][16h..16h+15] for a chunk's table build, in the stage (whose
    // rows are written only after the tables are built)
    uint4 *const wq = reinterpret_cast<uint4 *>(ins);
    const u32 b = blockIdx.x;
    const u32 loc = b >> 3;
    const u32 h = loc % ngroups;
    const u32 slice = (loc / ngroups) % nslices;
    const u32 s = (loc / ngroups / nslices) * 8 + (b & 7);
    if (s >= g.nstripes || (status && status[s]))
        return;
    const Stripe v = stripe_at(g, s);  // g.blocks = the output, g.n = slots per stripe
    const u32 r_begin = slice * DEC_ROWS;
    if (r_begin >= v.ps)
        return;
    const int k = g.k;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const u8 *wk = work + u64(s) * u64(k + k * k);

    uint4 acc[DEC_T];
#pragma unroll
    for (int t = 0; t < DEC_T; ++t)
        acc[t] = make_uint4(0, 0, 0, 0);

    const int nch = (k + 15) / 16;
    for (int cc = 0; cc < nch; ++cc) {
        __syncthreads();  // the previous chunk's tables are consumed
        {
            // byte e of row j: thread 16j + e (zero past k; clamped loads,
            // no branch)
            const int j = tid >> 4, e = tid & 15, c = 16 * cc + j, m = 16 * int(h) + e;
            const bool live = c < k && m < k;
            const u8 wv = wk[k + (live ? c * k + m : 0)];
            reinterpret_cast<u8 *>(wq)[tid] = live ? wv : u8(0);
        }
        __syncthreads();
        // table j: survivor 16cc+j, U_j[x] = (W[c][16h] x, ..., W[c][16h+15] x)
#pragma unroll 1
        for (int q = 0; q < 4; ++q) {
            const int j = wave + 4 * q;
            const uint4 wv = wq[j];
            const u32 row[4] = {wv.x, wv.y, wv.z, wv.w};
            u32 basis[8][4];
            make_basis<4>(basis, row);
            build_table16(tbl + j * 4096, basis, lane);
        }
        // Survivor stage: thread t takes row group rg = t & 127 (rows
        // 4rg..4rg+3 of the sub-block) of survivor quads t >> 7 and
        // (t >> 7) + 2: one dword of each of the quad's four parts (a wave
        // reads 256 contiguous bytes of one part per instruction), a 4x4
        // byte transpose, and four dword writes into [row][20-byte pitch]
        // (at most 2-way bank conflicts; the lanes' reads below, at a
        // 5-dword stride, none).
        const int rg = tid & 127, sq0 = tid >> 7;
        const u8 *qsrc[2][4];
        bool qlive[2][4];
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int c = 16 * cc + 4 * (sq0 + 2 * b2) + jj;
                qlive[b2][jj] = c < k;
                qsrc[b2][jj] = v.parts + (c < k ? u64(wk[c]) * v.pitch : 0);
            }
        u32 tdep = 0;  // 0 at run time: chains each row's lookups behind the previous row's
        // Not unrolled (unrolled, the compiler's schedule spills): the rows
        // of sub-block `sub` are acc[0..SUB/256-1], and the accumulators
        // rotate by SUB/256 after each sub-block, back in order after all
#pragma unroll 1
        for (int sub = 0; sub < int(DEC_ROWS / SUB); ++sub) {
            const u32 r4 = r_begin + u32(sub) * SUB + 4u * u32(rg);  // first of the thread's 4 rows
            u32 dq[2][4];
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    // below ps the dword lies inside the part's pitch; bytes
                    // past ps feed rows that are never stored
                    const bool ok = qlive[b2][jj] && r4 < v.ps;
                    if constexpr (PAL)
                        dq[b2][jj] = ok ? *reinterpret_cast<const u32 *>(qsrc[b2][jj] + r4) : 0u;
                    else
                        dq[b2][jj] = ok ? load4_bytes(qsrc[b2][jj] + r4, v.ps - r4) : 0u;
                }
            __syncthreads();  // tables built / the previous sub-block's rows consumed
            u32 *iw = reinterpret_cast<u32 *>(ins);
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2) {
                u32 o[4];
                transpose4(dq[b2][0], dq[b2][1], dq[b2][2], dq[b2][3], o[0], o[1], o[2], o[3]);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    iw[(4 * rg + i) * 5 + sq0 + 2 * b2] = o[i];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < int(SUB / 256); ++i) {
                const int t = i;
                const u32 rl = u32(i) * 256u + u32(tid);  // row within the sub-block
                const u32 *ip = reinterpret_cast<const u32 *>(ins) + rl * 5;
                const u32 in[4] = {ip[0], ip[1], ip[2], ip[3]};
                uint4 e = acc[t];
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const u32 byte = (in[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                    const uint4 tv = *reinterpret_cast<const uint4 *>(tbl + tdep + j * 4096 + byte * 16);
                    e.x ^= tv.x;
                    e.y ^= tv.y;
                    e.z ^= tv.z;
                    e.w ^= tv.w;
                }
                acc[t] = e;
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(e.x), "v"(e.y), "v"(e.z), "v"(e.w));
            }
            constexpr int R = int(SUB / 256);
            uint4 keep[R];
#pragma unroll
            for (int i = 0; i < R; ++i)
                keep[i] = acc[i];
#pragma unroll
            for (int i = 0; i + R < DEC_T; ++i)
                acc[i] = acc[i + R];
#pragma unroll
            for (int i = 0; i < R; ++i)
                acc[DEC_T - R + i] = keep[i];
        }
    }

    // row r's bytes 16h..16h+15 at r*k + 16h (fewer in the last group;
    // nothing at or past B); the other groups' workgroups of this slice run
    // on the same XCD, so the lines complete in its L2
    u8 *out = const_cast<u8 *>(v.blk);
    const uintptr_t oa = reinterpret_cast<uintptr_t>(out);
#pragma unroll
    for (int t = 0; t < DEC_T; ++t) {
        const u32 r = r_begin + u32(t) * 256u + u32(tid);
        if (r >= v.ps)
            continue;
        const u64 rb = u64(r) * u64(k);
        const u64 off = rb + 16u * h;
        const u32 tw[4] = {acc[t].x, acc[t].y, acc[t].z, acc[t].w};
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

}  // namespace

// Encode a uniform or ragged batch with any 2 <= k <= 254, n <= 255 through
// 16-column chunks, with the XXH64 of every part fused when `digests` is
// given (the chain hand-off records live in the launch's scratch,
// scratch.h).  -ENOSYS where a stripe's buffer offsets would not fit 31 bits
// (or no scratch could be had for the hand-off: the caller hashes after).
extern "C" int nkfs_big_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, const void *gf,
                               hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > 254 || g->n < k || g->n > 255)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    if (u64(g->block_size) + 64u > 0x7FFFFFFFull)
        return -ENOSYS;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    const u64 ngroups = (u64(g->n) + 15) / 16;
    const u64 nslices = (u64(ps_max) + ENC_ROWS - 1) / ENC_ROWS;
    const u64 grid = (u64(g->nstripes) + 7) / 8 * 8 * ngroups * (nslices ? nslices : 1);
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    if (!digests) {
        constexpr bool w8 = NKFS_BIG_W8 != 0 && NKFS_BIG_DIAG != 0;
        if (w8)
            hipLaunchKernelGGL(k_encode_big8, dim3(u32(grid)), dim3(512), 0, st, *g, ids, (const GfTables *)gf,
                               u32(ngroups), u32(nslices ? nslices : 1));
        else
            hipLaunchKernelGGL(k_encode_big<false>, dim3(u32(grid)), dim3(256), 0, st, *g, ids, (const GfTables *)gf,
                               u32(ngroups), u32(nslices ? nslices : 1), BigChain{});
        return hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    // hand-off records: per (stripe, group) 64 accumulators + a flag, and the failure word
    const u64 units = u64(g->nstripes) * ngroups;
    const u64 acc_b = (units * 64 * 8 + 255) & ~u64(255), flag_b = (units * 4 + 4 + 255) & ~u64(255);
    Scratch sc;
    u8 *rec = static_cast<u8 *>(sc.take(g, acc_b + flag_b, st));
    if (!rec)
        return -ENOSYS;
    BigChain ch{reinterpret_cast<u64 *>(rec), reinterpret_cast<u32 *>(rec + acc_b),
                reinterpret_cast<u32 *>(rec + acc_b) + units, digests};
    int rc = hipMemsetAsync(ch.flag, 0, units * 4 + 4, st) == hipSuccess ? 0 : -EIO;
    if (!rc) {
        hipLaunchKernelGGL(k_encode_big<true>, dim3(u32(grid)), dim3(256), 0, st, *g, ids, (const GfTables *)gf,
                           u32(ngroups), u32(nslices ? nslices : 1), ch);
        const u64 threads = u64(g->nstripes) * u64(g->n) * 4;
        hipLaunchKernelGGL(k_big_hash_fix, dim3(u32((threads + 255) / 256)), dim3(256), 0, st, *g,
                           (const u32 *)ch.fail, digests);
        rc = hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    const int e = sc.finish();
    return rc ? rc : e;
}

// Decode a uniform or ragged batch with 2 <= k <= 254 from the plan
// k_decode_prep left in `work` (stripes with status != 0 are skipped).
extern "C" int nkfs_big_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, hipStream_t st)
{
    const int k = g->k;
    if (k < 2 || k > 254)
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    if (u64(g->block_size) + 64u > 0x7FFFFFFFull)
        return -ENOSYS;
    const u32 ps_max = g->block_size / u32(k) + ((g->block_size % u32(k)) ? 1u : 0u);
    const u64 ngroups = (u64(k) + 15) / 16;
    const u64 nslices = (u64(ps_max) + DEC_ROWS - 1) / DEC_ROWS;
    const u64 grid = (u64(g->nstripes) + 7) / 8 * 8 * ngroups * (nslices ? nslices : 1);
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    const bool pal = !g->block_sizes && ((reinterpret_cast<uintptr_t>(g->parts) | g->part_pitch) & 15) == 0;
    if (pal)
        hipLaunchKernelGGL(k_decode_big<true>, dim3(u32(grid)), dim3(256), 0, st, *g, work, status, u32(ngroups),
                           u32(nslices ? nslices : 1));
    else
        hipLaunchKernelGGL(k_decode_big<false>, dim3(u32(grid)), dim3(256), 0, st, *g, work, status, u32(ngroups),
                           u32(nslices ? nslices : 1));
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
