// nk8_pair.hip -- decode for k = 2 (the C2 shape, N4K2 4 KiB stripes):
// one wave per stripe (or per row slice of a long one), the 2 x 2 inverse
// in closed form.
//
// Reference: crt/nk8.c:446-599 (nk8_assemble_block): the first k offered
// parts with distinct ids (:512-537) and block[j*k + m] = XOR_c part_c[j]
// W[c][m] with W the inverse of the survivors' Vandermonde rows.  For k = 2
// the encode is part_i[j] = d0 ^ x_i d1 (crt/nk8.c:403-420, d0 = block[2j],
// d1 = block[2j+1]), so from parts a, b (ids x_a != x_b):
//     d1 = (p_a ^ p_b) / (x_a ^ x_b),   d0 = p_a ^ x_a d1
// -- the same bytes the inverse gives (it is unique).  One product table
// T[y] = (x_a c y) | (c y) << 8 with c = 1 / (x_a ^ x_b) yields both terms
// of a row from one lookup: (T[p_a ^ p_b] ^ p_a) & 0xFFFF = (d0, d1).  That
// is one LDS lookup per row instead of the general decoder's k, and the
// selection + inverse collapse to a scalar id compare and one inverse.
//
// The wave's first part loads are issued as soon as its offered slots are
// known (speculatively: the first two offers are the selection unless their
// ids repeat), beside the loads of the two ids; the table is built while
// they are in flight.  XP: each unit's 2 KiB of output goes through a
// per-wave LDS stage so every store instruction writes one contiguous
// 1 KiB run (a lane's rows are 32 contiguous bytes).
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nk8_dev.h"
#include "nkfs_internal.h"
#include "runtime.h"
#include "scratch.h"

using namespace nkfs;
using namespace nkfs::dev;

namespace {

// bit-serial GF(2^8)/0x11B product (crt/nk8.c:54-74) in registers
__device__ inline u32 gfm_bits(u32 a, u32 b)
{
    u32 r = 0;
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        r ^= a & (0u - ((b >> bit) & 1u));
        a = ((a << 1) ^ (0x11Bu & (0u - ((a >> 7) & 1u)))) & 0xFFu;
    }
    return r;
}

constexpr int R = 1024;  // rows per unit: 16 per lane

// WPB waves per workgroup, each an independent (stripe, slice) with its own
// LDS: only wave-level ordering inside (no workgroup barrier), so a wave
// that finds its stripe out of range or undecodable simply leaves.  WPB = 4
// quarters the workgroups the dispatcher launches for 4 KiB stripes.
template <int U, bool XP, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_decode_pair(nkfs_geom g, int n_slots, const u8 *ids,
                                                          const u8 *avail, int navail, int32_t *status,
                                                          const GfTables *gft, u32 slices)
{
    constexpr int RS = R * U;  // rows per step
    __shared__ __attribute__((aligned(16))) u32 tbl_all[WPB][256];
    __shared__ __attribute__((aligned(16))) u8 stage_all[WPB][XP ? 2 * R : 16];
    __shared__ __attribute__((aligned(4))) u8 inv_all[WPB][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 *const tbl = tbl_all[wave];
    u8 *const stage = stage_all[wave];
    u8 *const inv_s = inv_all[wave];
    const u32 vw = blockIdx.x * WPB + wave;  // this wave's (stripe, slice)
    const u32 s = vw / slices, slice = vw % slices;
    if (s >= g.nstripes)
        return;
    const u32 sl = g.order ? g.order[s] : s;
    // the field's inverses into LDS, first: used once the ids are known
    reinterpret_cast<u32 *>(inv_s)[lane] = reinterpret_cast<const u32 *>(gft->inv)[lane];

    // geometry: uniform, or ragged as nkfs_nk8_encode_ragged lays it out
    u32 B = g.block_size;
    u64 ppitch = g.part_pitch;
    const u8 *pbase;
    u8 *out;
    if (g.block_sizes) {
        B = g.block_sizes[sl];
        ppitch = (u64(part_size_of(B, 2)) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
        pbase = g.parts + g.part_off[sl];
        out = const_cast<u8 *>(g.blocks) + g.block_off[sl];
    } else {
        pbase = g.parts + u64(sl) * u64(n_slots) * g.part_pitch;
        out = const_cast<u8 *>(g.blocks) + u64(sl) * g.block_pitch;
    }
    const u32 ps = part_size_of(B, 2);
    const u32 steps = (ps + RS - 1) / RS, per = (steps + slices - 1) / slices;
    const u32 rend = min(ps, (slice + 1) * per * RS);
    const u32 rfirst = slice * per * RS + 16 * lane;
    // ragged part offsets are caller data: byte loads where not 16-byte aligned
    const bool pal = (reinterpret_cast<uintptr_t>(pbase) & 15) == 0;

    // offered slots (wave-uniform) and the speculative part loads
    const u8 *sav = avail + u64(sl) * u64(navail);
    const u8 *sid = ids + u64(sl) * u64(n_slots);
    const u32 a0 = sav[0];
    u32 a1 = sav[1];
    u32 pa[U][4], pb[U][4];
    auto load_part = [&](u32 (&x)[U][4], u32 slot, u32 r0) {
        const u8 *src = pbase + u64(slot) * ppitch + r0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u && r0 + u * R >= rend)
                continue;
            if (pal) {
                const uint4 t = *reinterpret_cast<const uint4 *>(src + u * R);  // pitch >= round16(ps)
                x[u][0] = t.x;
                x[u][1] = t.y;
                x[u][2] = t.z;
                x[u][3] = t.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    u32 w = 0;
                    for (int e = 0; e < 4; ++e)
                        w |= u32(src[u * R + 4 * q + e]) << (8 * e);  // within the pitch
                    x[u][q] = w;
                }
            }
        }
    };
    if (rfirst < rend) {
        load_part(pa, a0, rfirst);
        load_part(pb, a1, rfirst);
    }
    const u32 x0 = sid[a0];
    u32 x1 = sid[a1];
    if (x1 == x0) {
        // the second offer repeats the first's id: the first later offer
        // with another id (crt/nk8.c:512-537), or -EINVAL (block untouched)
        u32 pick = 256;
        for (int c = 2; c < navail; ++c) {
            const u32 sc = sav[c], xc = sid[sc];
            if (xc != x0) {
                pick = sc;
                x1 = xc;
                break;
            }
        }
        if (pick == 256) {
            if (lane == 0 && status && slice == 0)
                status[sl] = -EINVAL;
            return;
        }
        a1 = pick;
        if (rfirst < rend)
            load_part(pb, a1, rfirst);
    }
    if (lane == 0 && status && slice == 0)
        status[sl] = 0;
    __builtin_amdgcn_wave_barrier();  // inv_s (this wave's LDS: in order within the wave)
    // T[y] = (x_a c y) | (c y) << 8, c = 1 / (x_a ^ x_b): linear in y, so
    // eight basis products and a Gray-code walk fill it (build_table)
    const u32 c = inv_s[x0 ^ x1];
    const u32 row[1] = {gfm_bits(x0, c) | (c << 8)};
    u32 basis[8][1];
    make_basis<1>(basis, row);
    build_table<1, 64>(reinterpret_cast<u8 *>(tbl), basis, lane);
    __builtin_amdgcn_wave_barrier();

    const bool oal = ((reinterpret_cast<uintptr_t>(out) | (g.block_sizes ? 0 : g.block_pitch)) & 15) == 0;
    // the step loop runs on a wave-uniform row (the output stage needs every
    // lane at its barrier and read-back, also lanes past the stripe's last row)
    for (u32 rb = rfirst - 16 * lane; rb < rend; rb += RS) {
        const u32 r0 = rb + 16 * lane;
        u32 o[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r0 + u * R >= rend)
                continue;  // this lane's rows of the unit lie past the stripe (or its slice)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32 y = pa[u][q] ^ pb[u][q];
                const u32 e0 = tbl[y & 0xFFu], e1 = tbl[(y >> 8) & 0xFFu];
                const u32 e2 = tbl[(y >> 16) & 0xFFu], e3 = tbl[y >> 24];
                // rows 4q..4q+3 -> (d0 d1) pairs: low halves of the entries,
                // XOR the part-a bytes spread to bytes 0 and 2
                o[u][2 * q] = __builtin_amdgcn_perm(e1, e0, 0x05040100u) ^
                              __builtin_amdgcn_perm(0u, pa[u][q], 0x04010400u);
                o[u][2 * q + 1] = __builtin_amdgcn_perm(e3, e2, 0x05040100u) ^
                                  __builtin_amdgcn_perm(0u, pa[u][q], 0x04030402u);
            }
        }
        if (r0 + RS < rend) {  // the next step's rows, in flight under this step's stores
            load_part(pa, a0, r0 + RS);
            load_part(pb, a1, r0 + RS);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 ru = rb + u * R;  // first row of the unit (wave-uniform)
            if (ru >= rend)
                continue;  // wave-uniform
            if constexpr (XP) {
                // lane l's 32 bytes at 32l; lane l then stores bytes 16l and
                // 1024 + 16l of the unit: one contiguous 1 KiB per instruction
                *reinterpret_cast<uint4 *>(stage + 32 * lane) = make_uint4(o[u][0], o[u][1], o[u][2], o[u][3]);
                *reinterpret_cast<uint4 *>(stage + 32 * lane + 16) = make_uint4(o[u][4], o[u][5], o[u][6], o[u][7]);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint4 t = *reinterpret_cast<const uint4 *>(stage + 1024 * h + 16 * lane);
                    const u64 off = u64(ru) * 2 + 1024u * h + 16u * lane;  // output byte
                    const u32 rlim = min(rend, ru + u32(R));
                    const u64 lim = min(u64(B), u64(rlim) * 2);  // this unit's bytes (within the slice)
                    if (oal && off + 16 <= lim) {
                        store16(out + off, t.x, t.y, t.z, t.w, false);
                    } else if (off < lim) {
                        const u32 tw[4] = {t.x, t.y, t.z, t.w};
                        for (u32 b = 0; b < 16 && off + b < lim; ++b)
                            out[off + b] = u8(tw[b >> 2] >> (8 * (b & 3)));
                    }
                }
                __builtin_amdgcn_wave_barrier();
            } else {
                const u32 rl = ru + 16 * lane;
                if (rl >= rend)
                    continue;
                const u64 off = u64(rl) * 2;
                const u64 lim = min(u64(B), u64(rend) * 2);
                if (oal && off + 32 <= lim) {
                    store16(out + off, o[u][0], o[u][1], o[u][2], o[u][3], false);
                    store16(out + off + 16, o[u][4], o[u][5], o[u][6], o[u][7], false);
                } else {
                    for (u32 b = 0; b < 32 && off + b < lim; ++b)
                        out[off + b] = u8(o[u][b >> 2] >> (8 * (b & 3)));
                }
            }
        }
    }
}

// Persistent, pipelined form for uniform batches of one-step stripes (ps <=
// 2,048 rows: C2's 4 KiB blocks).  A 4 KiB stripe is one load round trip
// and one store per wave, and each needs its offered slots first: the
// one-shot grid leaves every wave behind two dependent round trips (slots,
// then parts and ids).  Here a wave walks stripes s, s + G, s + 2G, ...
// with the round trips of the next two stripes in flight under the current
// one: at step j the slots of stripe j + 2 and the parts and ids of stripe
// j + 1 (whose slots came with step j - 1) are loaded before stripe j is
// decoded.  All loads are buffer loads with clamped, branch-free
// addresses, so the waits stay counted (vmcnt(n), not vmcnt(0)).
template <bool XP, bool FULL>
__global__ __launch_bounds__(64) void k_decode_pair_pipe(nkfs_geom g, int n_slots, const u8 *ids, const u8 *avail,
                                                         int navail, int32_t *status, const GfTables *gft)
{
    constexpr int U = 2;
    __shared__ __attribute__((aligned(16))) u32 tbl[256];
    __shared__ __attribute__((aligned(16))) u8 stage[XP ? 2 * R : 16];
    __shared__ __attribute__((aligned(4))) u8 inv_s[256];
    const int lane = threadIdx.x;
    const u32 G = gridDim.x;
    u32 s = blockIdx.x;
    if (s >= g.nstripes)
        return;
    reinterpret_cast<u32 *>(inv_s)[lane] = reinterpret_cast<const u32 *>(gft->inv)[lane];

    const u32 B = g.block_size, ps = part_size_of(B, 2);
    const u64 ppitch = g.part_pitch;
    // byte loads of the offered slots and ids (wave-uniform values through
    // vector loads: scalar loads would share lgkmcnt with the LDS traffic)
    const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<u8 *>(avail), (short)0,
                                                                         0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(const_cast<u8 *>(ids), (short)0,
                                                                         0x7FFFFFFF, 0x00020000);
    auto ldb = [&](__amdgpu_buffer_rsrc_t r, u64 off) -> u32 {
        return u32(__builtin_amdgcn_raw_buffer_load_b8(r, u32(off), 0, 0));
    };
    const u32 r0 = 16u * u32(lane);
    // a stripe's two offered parts, rows r0 .. r0 + 15 of each unit (rows
    // past ps read the part's padding or its neighbour: never stored)
    auto ldp = [&](u32 (&x)[U][4], u32 st, u32 slot) {
        const u8 *pb = g.parts + u64(st) * u64(n_slots) * ppitch + u64(slot) * ppitch;
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(const_cast<u8 *>(pb), (short)0,
                                                                             int(ppitch), 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const v4u t = __builtin_amdgcn_raw_buffer_load_b128(pr, r0 + u32(u * R), 0, 0);
            x[u][0] = t.x;
            x[u][1] = t.y;
            x[u][2] = t.z;
            x[u][3] = t.w;
        }
    };
    auto clampst = [&](u32 t) { return t < g.nstripes ? t : s; };

    // prologue: stripe s's slots (waited), its parts and ids; stripe s + G's slots
    u32 sn = clampst(s + G);
    u32 pa[U][4], pb[U][4], qa[U][4], qb[U][4];
    u32 x0, x1, y0 = 0, y1 = 0;
    {
        const u32 a0 = __builtin_amdgcn_readfirstlane(ldb(ar, u64(s) * u64(navail)));
        const u32 a1 = __builtin_amdgcn_readfirstlane(ldb(ar, u64(s) * u64(navail) + 1));
        ldp(pa, s, a0);
        ldp(pb, s, a1);
        x0 = ldb(ir, u64(s) * u64(n_slots) + a0);
        x1 = ldb(ir, u64(s) * u64(n_slots) + a1);
    }
    u32 na0 = ldb(ar, u64(sn) * u64(navail)), na1 = ldb(ar, u64(sn) * u64(navail) + 1);
    __builtin_amdgcn_wave_barrier();  // inv_s

    const bool oal = ((reinterpret_cast<uintptr_t>(g.blocks) | g.block_pitch) & 15) == 0;
    // the table of (x_a, x_b) and stripe t's rows from parts da, db
    auto emit = [&](u32 t, const u32 (&da)[U][4], const u32 (&db)[U][4], u32 c0, u32 c1) {
        // T[y] = (x_a c y) | (c y) << 8, c = 1 / (x_a ^ x_b)
        const u32 c = inv_s[c0 ^ c1];
        const u32 row[1] = {gfm_bits(c0, c) | (c << 8)};
        u32 basis[8][1];
        make_basis<1>(basis, row);
        __builtin_amdgcn_wave_barrier();  // the previous stripe's lookups are done
        build_table<1, 64>(reinterpret_cast<u8 *>(tbl), basis, lane);
        __builtin_amdgcn_wave_barrier();
        u8 *out = const_cast<u8 *>(g.blocks) + u64(t) * g.block_pitch;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 ru = u32(u * R);  // first row of the unit
            if (!FULL && ru >= ps)
                break;  // wave-uniform
            u32 o[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32 y = da[u][q] ^ db[u][q];
                const u32 e0 = tbl[y & 0xFFu], e1 = tbl[(y >> 8) & 0xFFu];
                const u32 e2 = tbl[(y >> 16) & 0xFFu], e3 = tbl[y >> 24];
                o[2 * q] = __builtin_amdgcn_perm(e1, e0, 0x05040100u) ^
                           __builtin_amdgcn_perm(0u, da[u][q], 0x04010400u);
                o[2 * q + 1] = __builtin_amdgcn_perm(e3, e2, 0x05040100u) ^
                               __builtin_amdgcn_perm(0u, da[u][q], 0x04030402u);
            }
            const u64 lim = min(u64(B), u64(min(ps, ru + u32(R))) * 2);  // this unit's bytes
            if constexpr (XP) {
                // lane l's 32 bytes at 32l; lane l then stores bytes 16l and
                // 1024 + 16l of the unit: 1 KiB contiguous per instruction
                *reinterpret_cast<uint4 *>(stage + 32 * lane) = make_uint4(o[0], o[1], o[2], o[3]);
                *reinterpret_cast<uint4 *>(stage + 32 * lane + 16) = make_uint4(o[4], o[5], o[6], o[7]);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint4 tt = *reinterpret_cast<const uint4 *>(stage + 1024 * h + 16 * lane);
                    const u64 off = u64(ru) * 2 + 1024u * h + 16u * lane;
                    if (FULL || (oal && off + 16 <= lim)) {
                        store16(out + off, tt.x, tt.y, tt.z, tt.w, false);
                    } else if (off < lim) {
                        const u32 tw[4] = {tt.x, tt.y, tt.z, tt.w};
                        for (u32 bb = 0; bb < 16 && off + bb < lim; ++bb)
                            out[off + bb] = u8(tw[bb >> 2] >> (8 * (bb & 3)));
                    }
                }
                __builtin_amdgcn_wave_barrier();
            } else {
                const u64 off = (u64(ru) + r0) * 2;
                if (FULL || (oal && off + 32 <= lim)) {
                    store16(out + off, o[0], o[1], o[2], o[3], false);
                    store16(out + off + 16, o[4], o[5], o[6], o[7], false);
                } else {
                    for (u32 bb = 0; bb < 32 && off + bb < lim; ++bb)
                        out[off + bb] = u8(o[bb >> 2] >> (8 * (bb & 3)));
                }
            }
        }
    };
    // decode stripe t from its parts and ids.  A repeated id is handled out
    // of line with its own part loads, so the common path's waits for da / db
    // stay counted (a reload of db on one path would make them vmcnt(0))
    auto decode = [&](u32 t, const u32 (&da)[U][4], const u32 (&db)[U][4], u32 i0, u32 i1) {
        const u32 c0 = __builtin_amdgcn_readfirstlane(i0), c1 = __builtin_amdgcn_readfirstlane(i1);
        if (c1 != c0) {
            if (lane == 0 && status)
                status[t] = 0;
            emit(t, da, db, c0, c1);
            return;
        }
        // the second offer repeats the first's id: the first later offer
        // with another id (crt/nk8.c:512-537), or -EINVAL (block untouched)
        const u8 *sav = avail + u64(t) * u64(navail);
        const u8 *sid = ids + u64(t) * u64(n_slots);
        u32 pick = 256, cx = c1;
        for (int c = 2; c < navail; ++c) {
            const u32 sc = sav[c], xc = sid[sc];
            if (xc != c0) {
                pick = sc;
                cx = xc;
                break;
            }
        }
        if (lane == 0 && status)
            status[t] = pick == 256 ? -EINVAL : 0;
        if (pick == 256)
            return;
        u32 tb[U][4];
        ldp(tb, t, pick);
        emit(t, da, tb, c0, cx);
    };
    // one step: the slots of the stripe two ahead, then the parts and ids of
    // the next stripe (slots from the last step), then the current stripe;
    // the two buffer sets alternate between steps (no register copies of
    // loads in flight), and the slots -- the step's first loads -- are the
    // only values carried over
    auto step = [&](u32 (&ca)[U][4], u32 (&cb)[U][4], u32 ci0, u32 ci1, u32 (&fa)[U][4], u32 (&fb)[U][4],
                    u32 &fi0, u32 &fi1) -> bool {
        const bool more = s + G < g.nstripes;
        const u32 s2 = clampst(sn + G);
        const u32 nb0 = ldb(ar, u64(s2) * u64(navail)), nb1 = ldb(ar, u64(s2) * u64(navail) + 1);
        const u32 b0 = __builtin_amdgcn_readfirstlane(na0), b1 = __builtin_amdgcn_readfirstlane(na1);
        ldp(fa, sn, b0);
        ldp(fb, sn, b1);
        fi0 = ldb(ir, u64(sn) * u64(n_slots) + b0);
        fi1 = ldb(ir, u64(sn) * u64(n_slots) + b1);
        decode(s, ca, cb, ci0, ci1);
        s = sn;
        sn = s2;
        na0 = nb0;
        na1 = nb1;
        return more;
    };
#pragma unroll 1
    for (;;) {
        if (!step(pa, pb, x0, x1, qa, qb, y0, y1))
            break;
        if (!step(qa, qb, y0, y1, pa, pb, x0, x1))
            break;
    }
}

}  // namespace

// k = 2 decode of a uniform or ragged batch (g->order honoured), no
// integrity check (the verifying form stays on the wave decoder).  xp: stage
// the output through LDS; waves: waves per workgroup (1 or 4); pipe: waves
// per CU of the persistent pipelined form (uniform 4 KiB-or-smaller blocks;
// 0 = the one-shot grid).  -ENOSYS outside k = 2.
extern "C" int nkfs_pair_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                                int navail, int32_t *status, const void *gf, int xp, int waves, int pipe,
                                hipStream_t st)
{
    if (g->k != 2 || navail < 2 || (!g->block_sizes && (g->part_pitch & 15)))
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    // pipe > 0: uniform batches of one-step stripes on the persistent
    // pipelined form, `pipe` waves per CU
    if (pipe > 0 && !g->block_sizes && !g->order && g->block_size <= 2u * R * 2u &&
        (reinterpret_cast<uintptr_t>(g->parts) & 15) == 0 && g->part_pitch < 0x7FFFFFFFull &&
        u64(g->nstripes) * u64(n_slots) < 0x7FFFFFFFull && u64(g->nstripes) * u64(navail) < 0x7FFFFFFFull) {
        const u64 want = u64(nkfs_cu_count()) * u64(pipe);
        const u32 grid = u32(want < g->nstripes ? want : g->nstripes);
        const GfTables *t = static_cast<const GfTables *>(gf);
        // FULL: 4 KiB blocks at 16-byte aligned addresses, every store whole
        const bool full = g->block_size == 2u * R * 2u &&
                          ((reinterpret_cast<uintptr_t>(g->blocks) | g->block_pitch) & 15) == 0;
#define NKFS_PIPE(XX, FF)                                                                                 \
    hipLaunchKernelGGL((k_decode_pair_pipe<XX, FF>), dim3(grid), dim3(64), 0, st, *g, n_slots, ids, avail, \
                       navail, status, t)
        if (xp && full)
            NKFS_PIPE(true, true);
        else if (xp)
            NKFS_PIPE(true, false);
        else if (full)
            NKFS_PIPE(false, true);
        else
            NKFS_PIPE(false, false);
#undef NKFS_PIPE
        return hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    // slices: enough waves to fill the chip (4,096), never a slice under 4 steps
    constexpr u32 U = 2;
    const u32 ps = g->block_size / 2u + (g->block_size & 1u);  // ragged: the bound on block sizes
    const u32 steps = (ps + R * U - 1) / (R * U);
    u32 slices = 1;
    while (u64(g->nstripes) * slices < 4096 && steps / (slices * 2) >= 4)
        slices *= 2;
    const u64 grid = u64(g->nstripes) * slices;
    if (grid > 0x7FFFFFFFull)
        return -EINVAL;
    const GfTables *t = static_cast<const GfTables *>(gf);
    // one wave per workgroup, or four (waves 1..3 of the last workgroup may
    // find no stripe and leave)
    const u32 wpb = waves >= 4 ? 4 : 1;
    const dim3 gd(u32((grid + wpb - 1) / wpb)), bd(64 * wpb);
#define NKFS_PAIR(XX, WW) \
    hipLaunchKernelGGL((k_decode_pair<U, XX, WW>), gd, bd, 0, st, *g, n_slots, ids, avail, navail, status, t, slices)
    if (wpb == 4) {
        if (xp)
            NKFS_PAIR(true, 4);
        else
            NKFS_PAIR(false, 4);
    } else if (xp) {
        NKFS_PAIR(true, 1);
    } else {
        NKFS_PAIR(false, 1);
    }
#undef NKFS_PAIR
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
