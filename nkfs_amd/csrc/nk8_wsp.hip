// nk8_wsp.hip -- persistent warp-specialised fused encode + XXH64 for
// n <= 8, k <= 8, uniform and ragged batches.
//
// Reference: crt/nk8.c:344-444 (nk8_split_block: part_i[j] = XOR_m
// ids[i]^m * d[j*k+m], crt/nk8.c:403-420) and crt/xxhash.c:358-496 (XXH64,
// seed 0 as crt/csum.c:5), per part.  Stripes are independent.
//
// k_encode_ws (nk8_ws.hip) runs one workgroup per group of S stripes: S
// encoder waves (one stripe each) feed HW hash waves through an LDS exchange,
// one barrier per 1,024-row chunk.  A CU holds one such workgroup (~100 KiB of
// LDS), so every workgroup change drains the CU: the last chunk's fold, the
// next workgroup's launch, its ids, its table build and its first loads run
// with no HBM traffic on that CU -- about three chunk-times per group, i.e.
// ~1.4 % of C3 (205 chunks per stripe) and ~5 % of C4 (52), and on a ragged
// batch the groups of 4 KiB / 64 KiB stripes are mostly transition.
//
// Here one workgroup per CU stays resident and walks a stream of groups:
//   * encoder wave e streams stripe slot e of the current group and keeps
//     PF chunks of loads in flight ACROSS group boundaries (the next group's
//     first chunks are loaded under the current group's last ones); its
//     packed tables (wave-private, one stripe) are rebuilt in its own step
//     when a group starts, hidden behind those loads;
//   * the hash waves fold chunk t-1 from the double-buffered exchange while
//     the encoders produce chunk t, and emit a stripe's digests right after
//     its own last chunk;
//   * a scheduler wave keeps a ring of group descriptors in LDS (stripe
//     index, block size, block / part offsets, ids of every stripe) far
//     enough ahead that no wave ever waits for metadata: uniform batches walk
//     the groups statically (workgroup b: groups b, b + grid, ...); ragged
//     batches run in size order (largest first, k_order_by_size) and take
//     groups from a device-wide counter (g.queue), one big group at a time
//     near the end of the current one, many small ones at once -- greedy
//     longest-first, so the grid ends together.
// All waves advance through the same task sequence (task = one chunk of one
// group) and meet at one barrier per task, so every wave executes the same
// number of barriers; the scheduler's loads are pipelined over steps (claim,
// stripe order, geometry, publish), and a descriptor becomes visible HZ
// steps before any wave needs it (the bound is derived at HZ below).
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nk8_dev.h"
#include "nkfs_internal.h"
#include "scratch.h"
#include "xxh64_dev.h"

using namespace nkfs;
using namespace nkfs::dev;

namespace {

constexpr u32 WSP_END = 0xFFFFFFFFu;  // ring_nch of the entry after the last group
constexpr u32 WSP_DEAD = 0xFFFFFFFFu; // stripe slot past the batch
constexpr int RD = 32;                // ring entries (groups)

struct RingStripe {
    u32 s;      // stripe index, WSP_DEAD past the batch
    u32 B;      // block bytes
    u64 boff;   // block offset from g.blocks
    u64 poff;   // parts offset from g.parts
    u64 idw;    // ids, byte i = id of part i (n <= 8)
};

// K: data parts; E: packed table bytes (4: n <= 4, 8: n <= 8); HW: hash waves;
// PF: chunks of block loads in flight per encoder wave; RAGGED / DYN: ragged
// geometry / device-wide group counter.
// NKFS_WS_HPRIO (experiment builds): the hash waves' s_setprio level
#ifndef NKFS_WS_HPRIO
#define NKFS_WS_HPRIO 0
#endif
template <int K, int E, int HW, int PF, bool RAGGED, bool DYN>
__global__ __launch_bounds__(64 * (HW * 16 / E + HW + 1)) void k_encode_wsp(nkfs_geom g, const u8 *ids,
                                                                            u64 *digests, u32 ngroups, bool nt)
{
    constexpr int SPH = 16 / E;     // stripes per hash wave: 4 accumulators x E parts x SPH = 64 chains
    constexpr int S = HW * SPH;     // stripes per group = encoder waves
    constexpr int CR = 1024;        // rows per stripe per chunk (64 lanes x 16 rows)
    constexpr int SP = CR + 32;     // exchange bytes per part (+32: bank spread, tail room)
    constexpr int TB = 256 * E;     // bytes per packed table
    constexpr int W = E / 4;        // dwords per packed entry
    constexpr int RPC = CR / 32;    // XXH64 rounds per chain per chunk
    constexpr int GPJ = 64 / S;     // groups one scheduler job can fetch (one lane per stripe)
    // Descriptor lead.  The scheduler publishes a job's groups 3 steps after
    // claiming them (claim; stripe order; geometry + ids; publish: each stage
    // consumes the previous step's loads), visible one step later; with one
    // job in flight it claims whenever the published chunks fall short of
    // t + HZ.  Encoders at step t need tasks t .. t+PF known, i.e. at the
    // claim step t the published chunks must cover t+3 .. t+3+PF: HZ >= PF+5;
    // a job that brings a single chunk shrinks the lead by 2, and the next
    // job claims ceil(HZ / last group's chunks) groups, so +3 keeps one such
    // job safe.
    constexpr u32 HZ = PF + 8;

    __shared__ __attribute__((aligned(16))) u8 tbl[S * (K - 1) * TB];
    __shared__ __attribute__((aligned(16))) u8 xbuf[2][S * E * SP];
    __shared__ __attribute__((aligned(16))) RingStripe ring[RD][S];
    __shared__ u32 ring_nch[RD];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = g.n;
    const u32 grid = gridDim.x, b = blockIdx.x;

    // geometry of ring stripe (j, e)
    auto ring_at = [&](u32 j, int e) -> RingStripe { return ring[j % RD][e]; };

    // ------------------------------------------------------ scheduler wave
    // lane l of a job: group i = l / S of the job, stripe slot e = l % S
    const int sj_i = lane / S, sj_e = lane % S;
    auto sched_order = [&](u32 gid, u32 &s) {
        const u64 p = u64(gid) * S + u32(sj_e);
        if (gid >= ngroups || p >= g.nstripes) {
            s = WSP_DEAD;
            return;
        }
        s = g.order ? g.order[p] : u32(p);
        if (s >= g.nstripes)  // never an index past the batch (a torn order entry)
            s = WSP_DEAD;
    };
    auto sched_geom = [&](u32 s, RingStripe &r) {
        r.s = s;
        r.B = 0;
        r.boff = r.poff = 0;
        r.idw = 0;
        if (s == WSP_DEAD)
            return;
        if constexpr (RAGGED) {
            r.B = g.block_sizes[s];
            r.boff = g.block_off[s];
            r.poff = g.part_off[s];
#ifdef NKFS_DEBUG_BOUNDS
            // debug-bounds build: report and skip a stripe whose block reads
            // (bytes [boff, boff + B): 16-byte loads only when the whole
            // 16 K-byte run lies inside B) or part stores would leave the
            // caller's buffers
            {
                const u64 pp = (u64(part_size_of(r.B, K)) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
                if ((g.blocks_bytes && r.boff + u64(r.B) > g.blocks_bytes) ||
                    (g.parts_bytes && r.poff + u64(n) * pp > g.parts_bytes) || (r.poff & 15) ||
                    (g.block_size && r.B > g.block_size) || r.B == 0) {
                    printf("nkfs bounds: k_encode_wsp stripe %u: B %u block [%llu,+%u) of %llu, parts [%llu,+%llu) "
                           "of %llu\n",
                           s, r.B, (unsigned long long)r.boff, r.B, (unsigned long long)g.blocks_bytes,
                           (unsigned long long)r.poff, (unsigned long long)(u64(n) * pp),
                           (unsigned long long)g.parts_bytes);
                    r.s = WSP_DEAD;
                    r.B = 0;
                    r.boff = r.poff = 0;
                    return;
                }
            }
#endif
        } else {
            r.B = g.block_size;
            r.boff = u64(s) * g.block_pitch;
            r.poff = u64(s) * u64(n) * g.part_pitch;
        }
        const u8 *sid = ids + u64(s) * u64(n);
        u64 w = 0;
        for (int i = 0; i < n; ++i)
            w |= u64(sid[i]) << (8 * i);
        r.idw = w;
    };
    // publish a job of m groups (gids in gid_of(i)): every lane of the job
    // writes its stripe; returns the chunks published, sets end / last_nch
    auto sched_publish = [&](u32 &written, u32 m, u32 first_gid_valid, const RingStripe &r, bool &ended,
                             u32 &last_nch) -> u32 {
        // this lane's stripe chunks; the group's = the max over its S lanes
        u32 cc = 0;
        if (r.s != WSP_DEAD)
            cc = (part_size_of(r.B, K) + CR - 1) / CR;
#pragma unroll
        for (int d = 1; d < S; d <<= 1)
            cc = max(cc, u32(__shfl_xor(int(cc), d, 64)));
        cc = max(cc, 1u);  // an all-empty group still takes one step (its digests)
        const bool valid = u32(sj_i) < first_gid_valid;
        if (u32(sj_i) < m && valid) {
            ring[(written + sj_i) % RD][sj_e] = r;
            if (sj_e == 0)
                ring_nch[(written + sj_i) % RD] = cc;
        }
        u32 total = 0, last = last_nch;
        for (u32 i = 0; i < first_gid_valid && i < m; ++i) {
            const u32 ci = u32(__shfl(int(cc), int(i) * S, 64));
            total += ci;
            last = ci;
        }
        last_nch = last;
        const u32 nv = min(first_gid_valid, m);
        if (nv < m) {  // the counter ran past the last group: end marker
            if (lane == 0)
                ring_nch[(written + nv) % RD] = WSP_END;
            ended = true;
        }
        written += nv;
        return total;
    };

    if (wave == S + HW) {
        // prologue: group b (static first for both modes), then synchronous
        // jobs until HZ chunks are published
        u32 written = 0, avail = 0, last_nch = 1, next_static = 1;
        bool ended = false;
        {
            u32 s;
            RingStripe r;
            sched_order(sj_i == 0 ? b : ngroups, s);
            sched_geom(s, r);
            avail += sched_publish(written, 1, b < ngroups ? 1u : 0u, r, ended, last_nch);
        }
        auto claim = [&](u32 m, u32 &base) {
            if constexpr (DYN) {
                u32 r0 = 0;
                if (lane == 0)
                    r0 = atomicAdd(g.queue, m);
                base = grid + u32(__shfl(int(r0), 0, 64));
            } else {
                base = next_static;  // sequence index: gid = b + (base + i) * grid
                next_static += m;
            }
        };
        auto gid_of = [&](u32 base, u32 i) -> u32 {
            if constexpr (DYN)
                return base + i;
            const u64 gg = u64(b) + u64(base + i) * grid;
            return gg < ngroups ? u32(gg) : ngroups;
        };
        auto valid_count = [&](u32 base, u32 m) -> u32 {
            u32 v = 0;
            for (u32 i = 0; i < m; ++i)
                v += gid_of(base, i) < ngroups ? 1u : 0u;
            return v;  // gids rise with i, so the valid ones come first
        };
        while (!ended && avail < HZ) {
            const u32 m = min(u32(GPJ), max(1u, (HZ + last_nch - 1) / last_nch));
            u32 base;
            claim(m, base);
            u32 s;
            RingStripe r;
            sched_order(u32(sj_i) < m ? gid_of(base, u32(sj_i)) : ngroups, s);
            sched_geom(s, r);
            avail += sched_publish(written, m, valid_count(base, m), r, ended, last_nch);
        }
        __syncthreads();  // prologue: ring published

        // steady state: one job in flight, one stage per step
        int jstate = 0;  // 0 idle, 1 claimed, 2 order known, 3 geometry known
        u32 jbase = 0, jm = 0, js = WSP_DEAD;
        u32 jr0 = 0;     // DYN: the counter's old value (lane 0), read a step later
        RingStripe jr{};
        u32 j = 0, c = 0, nchj = ring_nch[0];
        for (u32 t = 0;; ++t) {
            if (jstate == 3) {
                avail += sched_publish(written, jm, valid_count(jbase, jm), jr, ended, last_nch);
                jstate = 0;
            } else if (jstate == 2) {
                sched_geom(js, jr);
                jstate = 3;
            } else if (jstate == 1) {
                if constexpr (DYN)
                    jbase = grid + u32(__shfl(int(jr0), 0, 64));
                sched_order(u32(sj_i) < jm ? gid_of(jbase, u32(sj_i)) : ngroups, js);
                jstate = 2;
            }
            if (jstate == 0 && !ended && avail < t + HZ) {
                jm = min(u32(GPJ), max(1u, (HZ + last_nch - 1) / last_nch));
                if constexpr (DYN) {
                    if (lane == 0)
                        jr0 = atomicAdd(g.queue, jm);  // consumed next step
                } else {
                    jbase = next_static;
                    next_static += jm;
                }
                jstate = 1;
            }
            __syncthreads();
            if (++c >= nchj) {
                ++j;
                c = 0;
                nchj = ring_nch[j % RD];
                if (nchj == WSP_END)
                    break;
            }
        }
        return;
    }

    if (wave < S) {
        // ------------------------------------------------------ encoder wave
        const int e = wave;
        __syncthreads();  // prologue: ring published

        struct Geo {
            const u8 *blk;
            u8 *parts;
            u64 pitch;
            u32 B, ps;
            bool live, aligned;
            u64 idw;
        };
        auto geo = [&](u32 jj) -> Geo {
            const RingStripe r = ring_at(jj, e);
            Geo v;
            v.live = r.s != WSP_DEAD;
            v.B = r.B;
            v.ps = part_size_of(r.B, K);
            v.blk = g.blocks + r.boff;
            v.parts = g.parts + r.poff;
            if constexpr (RAGGED)
                v.pitch = (u64(v.ps) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
            else
                v.pitch = g.part_pitch;
            v.aligned = ((reinterpret_cast<uintptr_t>(v.blk) | reinterpret_cast<uintptr_t>(v.parts) | v.pitch) & 15) == 0;
            v.idw = r.idw;
            if (!v.live)
                v.ps = 0;
            return v;
        };
        const u32 rbase = 16 * lane;  // this lane's first row in every chunk

        // load pointer: task t+PF
        u32 jl = 0, cl = 0, nchl = ring_nch[0];
        Geo gl = geo(0);
        // issue the loads of the task at the load pointer (no LDS access:
        // the pointer is advanced at the top of the next step, so the ring
        // reads never sit between the table lookups and their uses)
        auto load_issue = [&](u32 (&x)[4 * K]) {
            if (nchl == WSP_END)
                return;
            const u32 r0 = cl * CR + rbase;
            const u64 off = u64(r0) * K;
            if (gl.live && r0 < gl.ps) {
                if (gl.aligned && off + 16 * K <= gl.B) {
                    const uint4 *src = reinterpret_cast<const uint4 *>(gl.blk + off);
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        const uint4 tq = src[q];
                        x[4 * q] = tq.x;
                        x[4 * q + 1] = tq.y;
                        x[4 * q + 2] = tq.z;
                        x[4 * q + 3] = tq.w;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4 * K; ++q) {
                        u32 y = 0;
                        for (int bb = 0; bb < 4; ++bb) {
                            const u64 p = off + 4 * q + bb;
                            if (p < gl.B)
                                y |= u32(gl.blk[p]) << (8 * bb);
                        }
                        x[q] = y;
                    }
                }
            }
        };
        auto load_advance = [&]() {
            if (nchl == WSP_END)
                return;
            if (++cl >= nchl) {
                ++jl;
                cl = 0;
                nchl = ring_nch[jl % RD];
                if (nchl != WSP_END)
                    gl = geo(jl);
            }
        };

        u32 d[PF][4 * K];
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            load_issue(d[p]);
            load_advance();
        }

        u8 *mytbl = tbl + e * (K - 1) * TB;
        u32 j = 0, c = 0, nchj = ring_nch[0];
        Geo ge = geo(0);

        auto chunk = [&](u32 (&x)[4 * K], u32 t) {
            if (t > 0)
                load_advance();  // to task t + PF (issued at the end of this step's lookups)
            if (c == 0 && ge.live) {
                // a new group: this wave's stripe's tables (the previous
                // group's last lookups are behind us in program order)
                u32 coef[W], idw[W];
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const u32 x4 = u32(ge.idw >> (32 * w));
                    idw[w] = x4;
                    coef[w] = x4;
                }
#pragma unroll
                for (int m = 1; m < K; ++m) {
                    u32 basis[8][W];
                    make_basis<W>(basis, coef);
                    build_table<W, 64>(mytbl + (m - 1) * TB, basis, lane);
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        coef[w] = gf_mul_packed(coef[w], idw[w]);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            const u32 r0 = c * CR + rbase;
            if (ge.live && r0 < ge.ps) {
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
                            const u8 *te = mytbl + tdep + (m - 1) * TB + byte * E;
                            if constexpr (E == 8) {
                                const uint2 tv = *reinterpret_cast<const uint2 *>(te);
                                row[rr][0] ^= tv.x;
                                row[rr][1] ^= tv.y;
                            } else {
                                row[rr][0] ^= *reinterpret_cast<const u32 *>(te);
                            }
                        }
                    }
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        transpose4(row[0][w], row[1][w], row[2][w], row[3][w], out[4 * w][q], out[4 * w + 1][q],
                                   out[4 * w + 2][q], out[4 * w + 3][q]);
                    if constexpr (K * W > 8)
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(tdep) : "v"(out[0][q]));
                }
                load_issue(x);  // task t + PF, in flight under what follows
                u8 *xb = xbuf[t & 1] + e * E * SP + 16 * lane;
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    if (i < n) {
                        u8 *dst = ge.parts + u64(i) * ge.pitch + r0;
                        if (ge.aligned) {
                            store16(dst, out[i][0], out[i][1], out[i][2], out[i][3], nt);
                        } else {
                            for (int bb = 0; bb < 16 && r0 + bb < ge.ps; ++bb)
                                dst[bb] = u8(out[i][bb >> 2] >> (8 * (bb & 3)));
                        }
                        *reinterpret_cast<uint4 *>(xb + i * SP) = make_uint4(out[i][0], out[i][1], out[i][2], out[i][3]);
                    }
                }
            } else {
                load_issue(x);
            }
            __syncthreads();
        };
        for (u32 t = 0;; t += PF) {
            chunk(d[0], t);
            if (++c >= nchj) {
                ++j;
                c = 0;
                nchj = ring_nch[j % RD];
                if (nchj == WSP_END)
                    break;
                ge = geo(j);
            }
            if constexpr (PF == 2) {
                chunk(d[1], t + 1);
                if (++c >= nchj) {
                    ++j;
                    c = 0;
                    nchj = ring_nch[j % RD];
                    if (nchj == WSP_END)
                        break;
                    ge = geo(j);
                }
            }
        }
        return;
    }

    // ------------------------------------------------------------ hash wave
    if (NKFS_WS_HPRIO)
        __builtin_amdgcn_s_setprio(NKFS_WS_HPRIO);
    constexpr int LPS = 64 / SPH;  // hash lanes per stripe (4 x E)
    const int hs = (wave - S) * SPH + lane / LPS, hli = lane % LPS;
    const int hi = hli >> 2, ha = hli & 3;
    __syncthreads();  // prologue: ring published

    u32 s_h = WSP_DEAD, ps = 0, nst = 0, own = 0, tstart = 0;
    bool hlane = false;
    u64 acc = 0;
    // fold task tp = chunk cp of group jp (exchange buffer tp & 1)
    auto fold = [&](u32 jp, u32 cp, u32 tp) {
        if (cp == 0) {
            const RingStripe r = ring_at(jp, hs);
            s_h = r.s;
            ps = r.s != WSP_DEAD ? part_size_of(r.B, K) : 0u;
            nst = ps >> 5;
            own = (ps + CR - 1) / CR;
            hlane = r.s != WSP_DEAD && hi < n;
            acc = xxh_acc_init(ha, 0);
            tstart = tp;
        }
        const u8 *src = xbuf[tp & 1] + (hs * E + hi) * SP + 8 * ha;
        if (hlane && cp < own) {
            const int left = int(nst) - int(cp * RPC);
            if (left >= RPC) {
#pragma unroll 8
                for (int r = 0; r < RPC; ++r)
                    acc = xxh_round(acc, *reinterpret_cast<const u64 *>(src + 32 * r));
            } else {
                for (int r = 0; r < left; ++r)
                    acc = xxh_round(acc, *reinterpret_cast<const u64 *>(src + 32 * r));
            }
        }
        // a stripe's digests right after its own last chunk (max(own, 1) - 1:
        // an empty part is digested at the group's first step), while that
        // chunk's exchange buffer still holds its tail
        const bool fin = hlane && cp + 1 == max(own, 1u);
        if (__ballot(fin)) {
            const int base = lane & ~3;
            const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
            const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
            if (fin && ha == 0) {
                u64 h = ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
                h += ps;
                u64 tw[4] = {0, 0, 0, 0};
                const u32 lft = ps & 31;
                if (lft) {
                    const u32 toff = nst * 32 - (own - 1) * CR;
                    const u64 *tp64 = reinterpret_cast<const u64 *>(xbuf[(tstart + own - 1) & 1] + (hs * E + hi) * SP + toff);
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        tw[w] = tp64[w];
                }
                digests[u64(s_h) * n + hi] = xxh_tail_regs(h, tw, lft);
            }
        }
    };
    u32 j = 0, c = 0, nchj = ring_nch[0];
    u32 jp = 0, cp = 0;
    for (u32 t = 0;; ++t) {
        if (t > 0)
            fold(jp, cp, t - 1);
        __syncthreads();
        jp = j;
        cp = c;
        if (++c >= nchj) {
            ++j;
            c = 0;
            nchj = ring_nch[j % RD];
            if (nchj == WSP_END) {
                fold(jp, cp, t);
                break;
            }
        }
    }
}

template <int E, int HW, int PF, bool RAGGED, bool DYN>
int launch_wsp(int k, hipStream_t st, const nkfs_geom &g, const u8 *ids, u64 *dig, u32 ngroups, u32 grid, bool nt)
{
    constexpr int S = HW * 16 / E;
    const dim3 block(64 * (S + HW + 1));
    switch (k) {
#define NKFS_K(KK)                                                                                              \
    case KK:                                                                                                    \
        hipLaunchKernelGGL((k_encode_wsp<KK, E, HW, PF, RAGGED, DYN>), dim3(grid), block, 0, st, g, ids, dig, \
                           ngroups, nt);                                                                        \
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

template <int E, int HW, int PF>
int launch_wsp_mode(int k, hipStream_t st, const nkfs_geom &g, const u8 *ids, u64 *dig, u32 ngroups, u32 grid,
                    bool nt, bool dyn)
{
    if (g.block_sizes)
        return launch_wsp<E, HW, PF, true, true>(k, st, g, ids, dig, ngroups, grid, nt);
    if (dyn)
        return launch_wsp<E, HW, PF, false, true>(k, st, g, ids, dig, ngroups, grid, nt);
    return launch_wsp<E, HW, PF, false, false>(k, st, g, ids, dig, ngroups, grid, nt);
}

}  // namespace

// Persistent fused encode + XXH64 (n <= 8, k <= 8, digests required).
// Ragged batches need the size order and its zeroed group counter
// (g->order, g->queue: with_size_order); -ENOSYS otherwise.  One workgroup
// per CU (its LDS request: tables, the exchange, the descriptor ring).
extern "C" int nkfs_wsp_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, bool nt, hipStream_t st)
{
    if (g->n > 8 || g->k > 8 || g->k < 2 || !digests || g->part_min || g->part_max)
        return -ENOSYS;
    if (g->block_sizes && (!g->order || !g->queue))
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    const nkfs_tune t = nkfs_tune_now();
    const bool e4 = g->n <= 4;
    const u32 S = 4;  // stripes per group: E = 4 with one hash wave, E = 8 with two
    const u64 ngroups = (u64(g->nstripes) + S - 1) / S;
    const u32 cus = u32(nkfs_cu_count());
    const u32 grid = u32(ngroups < cus ? ngroups : cus);
    // uniform batches: groups from a device-wide counter as well (a CU whose
    // HBM share runs slower takes fewer groups; the static walk -- workgroup
    // b: groups b, b + grid, ... -- measured 0.4 % slower on C3), the
    // counter a zeroed word of the launch's scratch; static when every
    // workgroup has one group
    const bool dyn = !g->block_sizes && ngroups > grid;
    nkfs_geom g2 = *g;
    Scratch sc;
    if (dyn && !g2.queue) {
        g2.queue = static_cast<u32 *>(sc.take(g, 256, st));
        if (!g2.queue || hipMemsetAsync(g2.queue, 0, 4, st) != hipSuccess) {
            (void)hipGetLastError();
            sc.finish();
            return -ENOSYS;
        }
    }
    int rc;
    if (e4)
        rc = t.enc_ws_prefetch >= 2 ? launch_wsp_mode<4, 1, 2>(g2.k, st, g2, ids, digests, u32(ngroups), grid, nt, dyn)
                                    : launch_wsp_mode<4, 1, 1>(g2.k, st, g2, ids, digests, u32(ngroups), grid, nt, dyn);
    else
        rc = t.enc_ws_prefetch >= 2 ? launch_wsp_mode<8, 2, 2>(g2.k, st, g2, ids, digests, u32(ngroups), grid, nt, dyn)
                                    : launch_wsp_mode<8, 2, 1>(g2.k, st, g2, ids, digests, u32(ngroups), grid, nt, dyn);
    if (!rc && hipGetLastError() != hipSuccess)
        rc = -EIO;
    const int e = sc.finish();
    return rc ? rc : e;
}
