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

}  // namespace

// k = 2 decode of a uniform or ragged batch (g->order honoured), no
// integrity check (the verifying form stays on the wave decoder).  xp: stage
// the output through LDS; waves: waves per workgroup (1 or 4).  -ENOSYS
// outside k = 2.
extern "C" int nkfs_pair_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                                int navail, int32_t *status, const void *gf, int xp, int waves, hipStream_t st)
{
    if (g->k != 2 || navail < 2 || (!g->block_sizes && (g->part_pitch & 15)))
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
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
