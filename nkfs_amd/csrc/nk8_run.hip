// nk8_run.hip -- the run decoder for k <= 8 (crt/nk8.c:446-599 per stripe):
// a persistent grid of the resident waves over the batch's chunks of
// 1,024-row units, uniform or ragged, with each chunk's stripe lookup and
// descriptor prefetched under the previous chunk (details below).
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

#include "../../include/nkfs_gpu.h"
#include "gf256.h"
#include "nk8_dev.h"
#include "nkfs_internal.h"

using namespace nkfs;
using namespace nkfs::dev;

namespace {

constexpr size_t LDS_PER_CU = 160 * 1024;

// Launch shape that caps residency at `target` one-wave workgroups per CU:
// the dynamic LDS request that makes only `target` fit beside the kernel's
// static LDS, and the number of workgroups per CU that are then really
// resident (a persistent grid must not exceed it).  Cached per kernel.
struct Shape {
    size_t pad;
    int per_cu;
};

Shape occupancy_shape(const void *kern, int target)
{
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, Shape> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({kern, target});
    if (it != cache.end())
        return it->second;
    hipFuncAttributes a{};
    size_t stat = 0;
    if (hipFuncGetAttributes(&a, kern) == hipSuccess)
        stat = a.sharedSizeBytes;
    if (target < 4)
        target = 4;  // keeps the request under the 64 KiB dynamic default
    const size_t per = LDS_PER_CU / size_t(target);
    Shape sh{per > stat ? per - stat : 0, target};
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64, sh.pad) == hipSuccess && occ > 0)
        sh.per_cu = occ < target ? occ : target;
    cache[{kern, target}] = sh;
    return sh;
}

u32 part_size_of_host(u32 B, int k) { return B / u32(k) + ((B % u32(k)) ? 1u : 0u); }

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

}  // namespace

// ------------------------------------------------------------ run decoder
//
// k_run_plan<K> + k_decode_run<K,E,U,RAGGED>: a persistent grid of the
// resident waves over the batch's chunks of U 1,024-row units (stripe by
// stripe, batch order), interleaved: wave w takes chunks w, w + G, w + 2G,
// ... so the waves in flight work on neighbouring chunks (a contiguous run
// per wave measured 6-9 % slower on uniform batches: every wave then
// streams its own region).  A chunk's stripe is found from a two-level
// prefix of the chunk counts (per 256-stripe group in LDS, within the group
// by one ballot over 256 loaded prefixes), and the lookup of chunk c + G
// and its stripe's descriptor (size, offsets, selection and inverse) are
// loaded while chunk c is rebuilt, so no chunk waits on a metadata chain.
// The plan kernel leaves the selection, the inverse, every stripe's chunk
// prefix within its group and each group's total in the caller's
// workspace: no scratch allocation and no single-workgroup setup launch.
//
// Workspace (nkfs_decode_work_bytes): plan[s] at s * run_plan_stride(k)
// (k slots, then W row-major; slot byte 0xFF: fewer than k distinct ids),
// then u32 loc[nstripes] (exclusive prefix of the chunks of the stripes
// before s in its group), then u32 gsum[ceil(nstripes / 256)].
constexpr u32 RUN_MAX_GROUPS = 256;  // prefix of the group totals in LDS (1 KiB): 65,536 stripes

template <int K>
__global__ __launch_bounds__(256) void k_run_plan(const nkfs_geom g, const u8 *ids, const u8 *avail, int n_slots,
                                                  int navail, u8 *work, int32_t *status, const GfTables *gft,
                                                  u32 chunk_rows)
{
    constexpr u32 PS = (K + K * K + 3) & ~3;
    __shared__ u32 wtot[4];
    const u32 s = blockIdx.x * 256u + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32 chunks = 0;
    if (s < g.nstripes) {
        const u8 *sid = ids + u64(s) * n_slots;
        const u8 *sav = avail + u64(s) * navail;
        u8 *pl = work + u64(s) * PS;
        u32 x[K], sl[K];
        int h = 0;
        for (int c = 0; c < navail && h < K; ++c) {  // crt/nk8.c:512-537
            const u32 slot = sav[c];
            const u32 id = sid[slot];
            bool dup = false;
#pragma unroll
            for (int j = 0; j < K; ++j)
                dup |= j < h && x[j] == id;
            if (dup)
                continue;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (j == h) {
                    x[j] = id;
                    sl[j] = slot;
                }
            ++h;
        }
        if (status)
            status[s] = h < K ? -EINVAL : 0;
        if (h < K) {
            pl[0] = 0xFF;
        } else {
            const u32 ps = part_size_of(g.block_sizes ? g.block_sizes[s] : g.block_size, K);
            chunks = (ps + chunk_rows - 1) / chunk_rows;
            // W = V^-1 in closed form, as k_decode_plan (crt/nk8.c:199-266)
            u32 M[K + 1];
            M[0] = 1;
#pragma unroll
            for (int c = 0; c < K; ++c) {
                M[c + 1] = M[c];
#pragma unroll
                for (int i = c; i >= 1; --i)
                    M[i] = M[i - 1] ^ gfm_bits(x[c], M[i]);
                M[0] = gfm_bits(x[c], M[0]);
            }
            u32 words[PS / 4];
#pragma unroll
            for (int i = 0; i < int(PS / 4); ++i)
                words[i] = 0;
            auto put = [&](int at, u32 v) {
#pragma unroll
                for (int i = 0; i < int(PS / 4); ++i)
                    if (i == at / 4)
                        words[i] |= (v & 0xFFu) << (8 * (at % 4));
            };
#pragma unroll
            for (int c = 0; c < K; ++c) {
                put(c, sl[c]);
                u32 q[K];
                u32 a = M[K];
                q[K - 1] = a;
#pragma unroll
                for (int i = K - 1; i >= 1; --i) {
                    a = M[i] ^ gfm_bits(x[c], a);
                    q[i - 1] = a;
                }
                u32 dd = 0;
#pragma unroll
                for (int i = K - 1; i >= 0; --i)
                    dd = gfm_bits(dd, x[c]) ^ q[i];
                const u32 dinv = gft->inv[dd];
#pragma unroll
                for (int i = 0; i < K; ++i)
                    put(K + c * K + i, gfm_bits(q[i], dinv));
            }
#pragma unroll
            for (int i = 0; i < int(PS / 4); ++i)
                reinterpret_cast<u32 *>(pl)[i] = words[i];
        }
    }
    // exclusive prefix of the chunks within the 256-stripe group
    u32 inc = chunks;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(inc, d, 64);
        if (lane >= d)
            inc += y;
    }
    if (lane == 63)
        wtot[wv] = inc;
    __syncthreads();
    u32 before = 0;
    for (int i = 0; i < wv; ++i)
        before += wtot[i];
    u32 *loc = reinterpret_cast<u32 *>(work + run_loc_off(g.nstripes, K));
    if (s < g.nstripes)
        loc[s] = before + inc - chunks;
    if (threadIdx.x == 255)
        reinterpret_cast<u32 *>(work + run_gsum_off(g.nstripes, K))[blockIdx.x] = before + inc;
}

// A chunk's stripe, its chunk index within the stripe and the stripe's
// descriptor: plan words, size, part base and block base (wave-uniform,
// held in VGPRs and loaded by vector loads: a scalar load shares lgkmcnt
// with the LDS traffic, so waiting on any LDS access would wait on the
// prefetch too).
template <int K>
struct RunDesc {
    static constexpr int PW = (K + K * K + 3) / 4;
    u32 pw[PW];
    u32 B;
    u32 ci;
    u64 poff;
    u64 boff;
};

template <int K, bool RAGGED>
__device__ inline void run_desc_load(const nkfs_geom &g, int n_slots, const u8 *work, u32 s, u32 ci, u32 vz,
                                     RunDesc<K> &d)
{
    // vz: 0 at run time, but a VGPR -- keeps these loads on the vector path
    const u32 *pw = reinterpret_cast<const u32 *>(work + u64(s) * run_plan_stride(K)) + vz;
#pragma unroll
    for (int i = 0; i < RunDesc<K>::PW; ++i)
        d.pw[i] = pw[i];
    d.ci = ci;
    if constexpr (RAGGED) {
        d.B = g.block_sizes[s + vz];
        d.poff = g.part_off[s + vz];
        d.boff = g.block_off[s + vz];
#ifdef NKFS_DEBUG_BOUNDS
        // debug-bounds build: a stripe whose block stores or survivor loads
        // would leave the caller's buffers (or whose plan names a slot past
        // n_slots) is reported and skipped like a stripe with fewer than K
        // distinct ids
        {
            const u64 pp = (u64(part_size_of(d.B, K)) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
            bool bad = (g.blocks_bytes && d.boff + d.B > g.blocks_bytes) ||
                       (g.parts_bytes && d.poff + u64(n_slots) * pp > g.parts_bytes) || (d.poff & 15) ||
                       (g.block_size && d.B > g.block_size) || s >= g.nstripes;
            if ((d.pw[0] & 0xFFu) != 0xFFu)
                for (int cc = 0; cc < K; ++cc)
                    bad |= ((d.pw[cc / 4] >> (8 * (cc % 4))) & 0xFFu) >= u32(n_slots);
            if (bad) {
                if ((threadIdx.x & 63) == 0)
                    printf("nkfs bounds: k_decode_run stripe %u chunk %u: B %u block [%llu,+%u) of %llu, parts "
                           "[%llu,+%llu) of %llu\n",
                           s, ci, d.B, (unsigned long long)d.boff, d.B, (unsigned long long)g.blocks_bytes,
                           (unsigned long long)d.poff, (unsigned long long)(u64(n_slots) * pp),
                           (unsigned long long)g.parts_bytes);
                d.pw[0] |= 0xFFu;
            }
        }
#endif
    } else {
        d.B = g.block_size;
        d.poff = u64(s) * u64(n_slots) * g.part_pitch;
        d.boff = u64(s) * g.block_pitch;
    }
}

template <int K, int E, int U, bool RAGGED>
__global__ __launch_bounds__(64) void k_decode_run(nkfs_geom g, int n_slots, const u8 *work, u32 subs)
{
    constexpr int W = E / 4;
    constexpr int TB = 256 * E;
    constexpr int LS = 16 * K + (K % 2 == 0 ? 16 : 0);  // transpose bytes per lane (even K padded)
    constexpr bool XPOSE = K >= 3;
    constexpr u32 SR = 1024u * U;  // rows per sub-chunk (one set of loads)
    const u32 CR = SR * subs;      // rows per chunk (one table build)
    __shared__ __attribute__((aligned(16))) u8 tbl[K * TB];
    __shared__ __attribute__((aligned(16))) u8 obuf[XPOSE ? 64 * LS : 16];
    __shared__ u32 gpre[RAGGED ? RUN_MAX_GROUPS + 1 : 1];  // exclusive prefix of the group totals
    const int li = threadIdx.x;
    u32 vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));

    const u32 ngroups = (g.nstripes + 255u) / 256u;
    const u32 *loc = reinterpret_cast<const u32 *>(work + run_loc_off(g.nstripes, K));
    u32 total;  // chunks in the batch
    u32 cps = 0;  // uniform: chunks per stripe
    if constexpr (RAGGED) {
        const u32 *gsum = reinterpret_cast<const u32 *>(work + run_gsum_off(g.nstripes, K));
        u32 carry = 0;
        for (u32 c = 0; c < ngroups; c += 64) {
            const u32 i = c + u32(li);
            const u32 v = i < ngroups ? gsum[i] : 0u;
            u32 inc = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const u32 y = __shfl_up(inc, d, 64);
                if (li >= d)
                    inc += y;
            }
            if (i < ngroups)
                gpre[i] = carry + inc - v;
            carry += __shfl(inc, 63, 64);
        }
        total = carry;
        if (li == 0)
            gpre[ngroups] = total;
        __syncthreads();
    } else {
        cps = (part_size_of(g.block_size, K) + CR - 1) / CR;
        total = cps * g.nstripes;  // the launcher checks it fits 32 bits
    }

    // stripe s and chunk ci of chunk c
    auto locate = [&](u32 c, u32 &s, u32 &ci) {
        if constexpr (RAGGED) {
            // last group whose prefix is <= c (gpre is nondecreasing)
            u32 lo = 0, hi = ngroups;  // gpre[lo] <= c < gpre[hi]
            while (hi - lo > 1) {
                const u32 mid = (lo + hi) >> 1;
                if (gpre[mid] <= c)
                    lo = mid;
                else
                    hi = mid;
            }
            const u32 rel = c - gpre[lo];
            int cnt = 0;
            u32 lq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32 i = lo * 256u + u32(64 * q + li);
                lq[q] = i < g.nstripes ? loc[i] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                cnt += __popcll(__ballot(lq[q] <= rel));
            const int sl = cnt - 1;  // >= 0: the group's first prefix is 0
            u32 ls = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32 y = __shfl(lq[q], sl & 63, 64);
                if (q == (sl >> 6))
                    ls = y;
            }
            s = lo * 256u + u32(sl);
            ci = rel - ls;
        } else {
            s = c / cps;
            ci = c % cps;
        }
    };

    u32 c = blockIdx.x;
    if (c >= total)
        return;
    RunDesc<K> cur;
    {
        u32 s0, ci0;
        locate(c, s0, ci0);
        run_desc_load<K, RAGGED>(g, n_slots, work, s0, ci0, vz, cur);
    }
    for (;;) {
        const u32 cn = c + gridDim.x;  // this wave's next chunk
        const bool more = cn < total;
        if ((cur.pw[0] & 0xFFu) == 0xFFu) {
            // fewer than K distinct ids: status says -EINVAL, block untouched
            // (uniform batches only; a ragged batch gives such a stripe no chunks)
            if (!more)
                return;
            u32 s1, ci1;
            locate(cn, s1, ci1);
            run_desc_load<K, RAGGED>(g, n_slots, work, s1, ci1, vz, cur);
            c = cn;
            continue;
        }
        const u32 ps = part_size_of(cur.B, K);
        const u64 ppitch = RAGGED ? (u64(ps) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1) : g.part_pitch;
        const u8 *pbase = g.parts + cur.poff;
        u8 *out = const_cast<u8 *>(g.blocks) + cur.boff;
        const u32 B = cur.B;
        const bool pal = !RAGGED || (reinterpret_cast<uintptr_t>(pbase) & 15) == 0;
        RunDesc<K> nxt;
        for (u32 sb = 0; sb < subs; ++sb) {
            const u32 rbase = (cur.ci * subs + sb) * SR;
            if (rbase >= ps)
                break;  // wave-uniform

            // this chunk's loads first (their latency hides under the next
            // chunk's lookup and the table build)
            const u8 *src[K];
#pragma unroll
            for (int cc = 0; cc < K; ++cc)
                src[cc] = pbase + u64((cur.pw[cc / 4] >> (8 * (cc % 4))) & 0xFFu) * ppitch;
            u32 pv[U][K][4];
#pragma unroll
            for (int uu = 0; uu < U; ++uu) {
                const u32 r0 = rbase + uu * 1024 + 16 * li;
                if (r0 < ps)
#pragma unroll
                    for (int cc = 0; cc < K; ++cc) {
                        if (pal) {
                            const uint4 t = *reinterpret_cast<const uint4 *>(src[cc] + r0);  // pitch >= round16(ps)
                            pv[uu][cc][0] = t.x;
                            pv[uu][cc][1] = t.y;
                            pv[uu][cc][2] = t.z;
                            pv[uu][cc][3] = t.w;
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                u32 x = 0;
                                for (int e = 0; e < 4; ++e)
                                    x |= u32(src[cc][r0 + 4 * q + e]) << (8 * e);  // within the pitch
                                pv[uu][cc][q] = x;
                            }
                        }
                    }
            }
            // the next chunk's stripe and descriptor, in flight under this chunk
            if (sb == 0 && more) {
                u32 s1, ci1;
                locate(cn, s1, ci1);
                run_desc_load<K, RAGGED>(g, n_slots, work, s1, ci1, vz, nxt);
            }
            // U_c[x] = (W[c][0] x, ..., W[c][K-1] x), packed: once per chunk
            if (sb == 0) {
#pragma unroll
            for (int cc = 0; cc < K; ++cc) {
                u32 rw[W];
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    u32 x = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if (4 * w + b < K) {
                            const int at = K + cc * K + 4 * w + b;
                            x |= ((cur.pw[at / 4] >> (8 * (at % 4))) & 0xFFu) << (8 * b);
                        }
                    rw[w] = x;
                }
                u32 basis[8][W];
                make_basis<W>(basis, rw);
                build_table<W, 64>(tbl + cc * TB, basis, li);
            }
            __syncthreads();
            }

            const bool aligned = ((reinterpret_cast<uintptr_t>(out) | (RAGGED ? 0 : g.block_pitch)) & 15) == 0;
#pragma unroll
            for (int uu = 0; uu < U; ++uu) {
                const u32 ru = rbase + uu * 1024;
                if (ru >= ps)
                    break;
                const u32 r0 = ru + 16 * li;
                u32 o[4 * K];
                if (r0 < ps) {
                    u32 ent[2][4][K][W];
                    auto look = [&](int gq, u32 (&e)[4][K][W]) {
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int r = 4 * gq + rr;
#pragma unroll
                            for (int cc = 0; cc < K; ++cc) {
                                const u32 byte = (pv[uu][cc][r >> 2] >> (8 * (r & 3))) & 0xFFu;
                                const u8 *ep = tbl + cc * TB + byte * E;
                                if constexpr (E == 8) {
                                    const uint2 t = *reinterpret_cast<const uint2 *>(ep);
                                    e[rr][cc][0] = t.x;
                                    e[rr][cc][W - 1] = t.y;
                                } else {
                                    e[rr][cc][0] = *reinterpret_cast<const u32 *>(ep);
                                }
                            }
                        }
                    };
                    look(0, ent[0]);
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        if (gq < 3)
                            look(gq + 1, ent[(gq + 1) & 1]);
                        u32 row[4 * W];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                            for (int w = 0; w < W; ++w) {
                                u32 x = ent[gq & 1][rr][0][w];
#pragma unroll
                                for (int cc = 1; cc < K; ++cc)
                                    x ^= ent[gq & 1][rr][cc][w];
                                row[rr * W + w] = x;
                            }
#pragma unroll
                        for (int q = 0; q < K; ++q)
                            o[gq * K + q] = pack_dword<K, W>(row, q);
                    }
                }
                const u64 ubyte = u64(ru) * K;  // first output byte of the unit
                if constexpr (XPOSE) {
                    if (r0 < ps)
#pragma unroll
                        for (int q = 0; q < K; ++q)
                            *reinterpret_cast<uint4 *>(obuf + li * LS + 16 * q) =
                                make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                    __syncthreads();
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        const int j = q * 64 + li;  // 16-byte piece of the unit's output
                        const uint4 t = *reinterpret_cast<const uint4 *>(obuf + (j / K) * LS + (j % K) * 16);
                        const u64 off = ubyte + u64(j) * 16;
                        if (aligned && off + 16 <= B) {
                            store16(out + off, t.x, t.y, t.z, t.w, false);
                        } else if (off < B) {
                            const u32 tw[4] = {t.x, t.y, t.z, t.w};
                            for (int b = 0; b < 16 && off + b < B; ++b)
                                out[off + b] = u8(tw[b >> 2] >> (8 * (b & 3)));
                        }
                    }
                    __syncthreads();
                } else if (r0 < ps) {
                    const u64 off = u64(r0) * K;
                    if (aligned && off + 16 * K <= B) {
                        uint4 *dst = reinterpret_cast<uint4 *>(out + off);
#pragma unroll
                        for (int q = 0; q < K; ++q)
                            store16(dst + q, o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3], false);
                    } else {
#pragma unroll
                        for (int q = 0; q < 4 * K; ++q)
                            for (int b = 0; b < 4; ++b)
                                if (off + 4 * q + b < B)
                                    out[off + 4 * q + b] = u8(o[q] >> (8 * b));
                    }
                }
            }
        }
        if (!more)
            return;
        __syncthreads();  // this chunk's lookups are done before the next build
        c = cn;
        cur = nxt;
    }
}

// ------------------------------------------------------- run decoder launch

// chunk = `units` 1,024-row units: U = 2 units per set of loads (1 for
// single-unit chunks), subs = units / U sets per chunk sharing one table build
template <int K, int E, int U>
static void launch_run(hipStream_t st, const nkfs_geom &g, int n_slots, const u8 *work, int waves, int cus,
                       u32 subs)
{
    if (g.block_sizes) {
        const Shape sh = occupancy_shape(reinterpret_cast<const void *>(&k_decode_run<K, E, U, true>), waves);
        hipLaunchKernelGGL((k_decode_run<K, E, U, true>), dim3(u32(cus) * u32(sh.per_cu)), dim3(64), sh.pad, st, g,
                           n_slots, work, subs);
    } else {
        const Shape sh = occupancy_shape(reinterpret_cast<const void *>(&k_decode_run<K, E, U, false>), waves);
        hipLaunchKernelGGL((k_decode_run<K, E, U, false>), dim3(u32(cus) * u32(sh.per_cu)), dim3(64), sh.pad, st, g,
                           n_slots, work, subs);
    }
}

template <int K, int E>
static void launch_run_u(int units, hipStream_t st, const nkfs_geom &g, int n_slots, const u8 *work, int waves,
                         int cus)
{
    if (units >= 2)
        launch_run<K, E, 2>(st, g, n_slots, work, waves, cus, u32(units / 2));
    else
        launch_run<K, E, 1>(st, g, n_slots, work, waves, cus, 1u);
}

extern "C" uint64_t nkfs_run_work_bytes(uint32_t nstripes, int k)
{
    return run_gsum_off(nstripes, k) + u64((nstripes + 255u) / 256u) * 4u;
}

// Run decoder, k <= 8, uniform or ragged (g->order ignored: batch order):
// k_run_plan (selection, inverse, unit prefix per 256 stripes, in `work`)
// then one persistent wave per resident slot walking its run of units.
// -ENOSYS outside its shapes.
extern "C" int nkfs_run_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                               int navail, void *work, int32_t *status, const void *gf, int units, int waves,
                               int cus, hipStream_t st)
{
    if (g->k > 8 || g->k < 2 || (reinterpret_cast<uintptr_t>(g->parts) & 15) ||
        (!g->block_sizes && (g->part_pitch & 15)) || (reinterpret_cast<uintptr_t>(work) & 15))
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    u8 *w = static_cast<u8 *>(work);
    const GfTables *gft = static_cast<const GfTables *>(gf);
    const dim3 pgrid((g->nstripes + 255) / 256);
    units = units >= 16 ? 16 : units >= 8 ? 8 : units >= 4 ? 4 : units >= 2 ? 2 : 1;
    // ragged: the group prefix lives in LDS; uniform: chunk indices fit 32 bits
    const u64 cps = (u64(part_size_of_host(g->block_size, g->k)) + 1024u * units - 1) / (1024u * units);
    if (g->block_sizes ? (g->nstripes + 255u) / 256u > RUN_MAX_GROUPS : cps * g->nstripes > 0xFFFFFFFFull)
        return -ENOSYS;
    switch (g->k) {
#define NKFS_RK(KK, EE)                                                                                          \
    case KK:                                                                                                     \
        hipLaunchKernelGGL((k_run_plan<KK>), pgrid, dim3(256), 0, st, *g, ids, avail, n_slots, navail, w, status, \
                           gft, 1024u * u32(units));                                                             \
        launch_run_u<KK, EE>(units, st, *g, n_slots, w, waves, cus);                                             \
        break;
        NKFS_RK(2, 4)
        NKFS_RK(3, 4)
        NKFS_RK(4, 4)
        NKFS_RK(5, 8)
        NKFS_RK(6, 8)
        NKFS_RK(7, 8)
        NKFS_RK(8, 8)
#undef NKFS_RK
    default:
        return -ENOSYS;
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
