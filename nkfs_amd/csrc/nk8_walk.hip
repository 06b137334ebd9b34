// nk8_walk.hip -- streaming N-K kernels shaped by what MI355X's HBM rewards
// (profiles/r02/sol_shapes.txt, tools/sol.hip):
//
//  * every wave owns ONE stripe, and every global load / store instruction
//    moves one contiguous 1 KiB run of one block or part;
//  * about 8 resident waves per CU (capped through the LDS request): the
//    same data movement runs 6.2-6.3 TB/s at 8 waves/CU and 5.8 TB/s
//    uncapped (C2 shape), 5.8 TB/s for whole-stripe walks at 8/CU vs
//    5.4-5.6 at 4/CU;
//  * no lane stores with a lane stride of more than 16 B: the decode's
//    row-major output goes through an LDS transpose (stride-80 stores cost
//    30 % at K = 5).
//
// k_encode_walk -- fused encode + XXH64 of every part (crt/nk8.c:403-420,
//   crt/xxhash.c:358-496 with seed 0 as crt/csum.c:5).  The wave walks its
//   stripe in chunks of R = 1024*U rows: lane l encodes rows 16l..16l+15 of
//   each 1024-row unit (k 16-byte loads), XORs k-1 lookups of packed product
//   tables T_m[x] = (ids_0^m x, ..., ids_{n-1}^m x) per row, transposes 16
//   rows into 16 bytes of every part (v_perm), stores them (1 KiB per
//   instruction) and drops them into an LDS exchange.  Lane 4i+a (i < n) is
//   accumulator a of part i's XXH64: it folds chunk c-1 from the exchange
//   while the wave encodes chunk c, so the hash rides along the stream.
//   XXH64 is serial per accumulator, so a stripe has exactly 4n chains; a
//   wave hashes one stripe with 4n active lanes (one round costs ~45 SIMD
//   cycles whatever the active lane count, tools/sol.hip).
//
// k_decode_slice -- decode (crt/nk8.c:446-599) as one-shot waves: wave =
//   one slice of 1024*U rows of one stripe; the stripe's selection and
//   K x K inverse come precomputed from k_decode_plan (one lane per stripe).
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
#include "scratch.h"
#include "xxh64_dev.h"

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

[[maybe_unused]] Shape occupancy_shape(const void *kern, int target)
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

[[maybe_unused]] u32 part_size_of_host(u32 B, int k) { return B / u32(k) + ((B % u32(k)) ? 1u : 0u); }

typedef unsigned int v2u __attribute__((ext_vector_type(2)));

// bit-serial GF(2^8)/0x11B product (crt/nk8.c:54-74) in registers
[[maybe_unused]] __device__ inline u32 gfm_bits(u32 a, u32 b)
{
    u32 r = 0;
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        r ^= a & (0u - ((b >> bit) & 1u));
        a = ((a << 1) ^ (0x11Bu & (0u - ((a >> 7) & 1u)))) & 0xFFu;
    }
    return r;
}

// 16 rows starting at byte `off` of the stripe's block into d[4K] (zero
// beyond B: the reference zero-pads the tail row, crt/nk8.c:393-398)
template <int K>
__device__ inline void load_rows(u32 (&d)[4 * K], const Stripe &v, u64 off, bool aligned)
{
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
}

}  // namespace

// The walk encoder's buffer offsets (block bytes plus a chunk's reach, a
// stripe's part span, the digest array) all below 2^31 (host-side check;
// tests/test_abi.py exercises the bound through nkfs_walk_offsets_fit)
__host__ __device__ inline bool walk_offsets_fit(u64 block_size, u64 part_span, u64 nstripes, u64 n)
{
    return block_size + 2048u * 8u <= 0x7FFFFFFFull && part_span <= 0x7FFFFFFFull && nstripes * n * 8u <= 0x7FFFFFFFull;
}

#ifndef NKFS_WALK_K
extern "C" int nkfs_walk_offsets_fit(uint64_t block_size, uint64_t part_span, uint64_t nstripes, uint64_t n)
{
    return walk_offsets_fit(block_size, part_span, nstripes, n);
}
#endif

// Buffer offset `off` (< 2^31) when `live`, else past every num_records
// (the load reads 0 / the store is dropped), as plain
// arithmetic: a select here tempts the compiler to branch around each
// load/store, which splits the step's straight-line block
__device__ inline u32 live_off(bool live, u32 off) { return off | (u32(!live) << 31); }

__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void *base, u32 bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}

// Persistent walk.  Wave w walks stripes w, w + grid, w + 2*grid, ...
// (per_wave of them; ragged batches: exactly one, g.order applied), each in
// chunks of R = 1024*U rows; every (stripe, chunk) is one task and step t
//   1. loads task t+P (P = 1 or 2 tasks of loads in flight ahead),
//   2. folds task t-1's parts into the XXH64 chains (finishing a stripe's
//      digests after its last chunk),
//   3. encodes task t (tables rebuilt when it starts a stripe), stores it and
//      drops it into the exchange.
// Every global access is a buffer load/store issued on every step
// unconditionally (out-of-range offsets read 0 / drop the write), so the
// compiler's s_waitcnt accounting is exact and the loads of task t+1 stay
// in flight under steps 2-3 (the wait before task t's data covers only what
// was issued before it).  Two register sets alternate; step 0 is peeled so
// the loop is entered in the same state it loops back in.
template <int K, int E, int U, int P, bool HASH, bool NIB, bool RAGGED>
__global__ __launch_bounds__(64, 2) void k_encode_walk(nkfs_geom g, const u8 *ids, u64 *digests, u32 per_wave)
{
    constexpr int R = 1024 * U;                // rows per chunk
    constexpr int SP = R + 32;                 // exchange bytes per part: 32-B skew -> conflict-free hash reads
    constexpr int TB = (NIB ? 32 : 256) * E;   // bytes per packed table
    constexpr int W = E / 4;                   // dwords per packed entry
    constexpr int RPC = R / 32;                // XXH64 rounds per chain per chunk
    __shared__ __attribute__((aligned(16))) u8 tbl[(K - 1) * TB];
    __shared__ __attribute__((aligned(16))) u8 xbuf[HASH ? E * SP : 16];

    const int li = threadIdx.x;
    const int n = g.n;
    const u32 grid = gridDim.x;

    // ---- geometry (uniform batches: one shape; ragged: this wave's stripe)
    u32 B, s0;
    u64 ppitch;
    const u8 *blk0;
    u8 *par0;
    if constexpr (RAGGED) {
        s0 = g.order ? g.order[blockIdx.x] : blockIdx.x;
#ifdef NKFS_DEBUG_BOUNDS
        // debug-bounds build (make DEBUG_BOUNDS=1): report and skip a stripe
        // whose accesses would leave the caller's buffers
        if (s0 >= g.nstripes) {
            if (li == 0)
                printf("nkfs bounds: k_encode_walk wave %u: order gives stripe %u of %u\n", blockIdx.x, s0,
                       g.nstripes);
            return;
        }
#endif
        B = g.block_sizes[s0];
        ppitch = (u64(part_size_of(B, K)) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
        blk0 = g.blocks + g.block_off[s0];
        par0 = g.parts + g.part_off[s0];
#ifdef NKFS_DEBUG_BOUNDS
        {
            const u64 bo = g.block_off[s0], po = g.part_off[s0];
            const bool bad = (g.blocks_bytes && bo + ((u64(B) + 3) & ~u64(3)) > g.blocks_bytes) ||
                             (g.parts_bytes && po + u64(g.n) * ppitch > g.parts_bytes) || (po & 15) ||
                             (g.block_size && B > g.block_size);
            if (bad) {
                if (li == 0)
                    printf("nkfs bounds: k_encode_walk stripe %u: B %u block [%llu,+%u) of %llu, parts [%llu,+%llu) "
                           "of %llu\n",
                           s0, B, (unsigned long long)bo, B, (unsigned long long)g.blocks_bytes,
                           (unsigned long long)po, (unsigned long long)(u64(g.n) * ppitch),
                           (unsigned long long)g.parts_bytes);
                return;
            }
        }
#endif
    } else {
        s0 = blockIdx.x;
        B = g.block_size;
        ppitch = g.part_pitch;
        blk0 = g.blocks;
        par0 = g.parts;
    }
    const u32 ps = part_size_of(B, K);
    if constexpr (RAGGED)  // part-size window of this launch (whole wave)
        if ((g.part_min && ps < g.part_min) || (g.part_max && ps >= g.part_max))
            return;
    const u32 nch = (ps + R - 1) / R;
    const u32 ntask = per_wave * nch;
    auto stripe_of = [&](u32 j) { return RAGGED ? s0 : s0 + j * grid; };
    auto blk_of = [&](u32 s) { return RAGGED ? blk0 : blk0 + u64(s) * g.block_pitch; };
    auto par_of = [&](u32 s) { return RAGGED ? par0 : par0 + u64(s) * u64(n) * ppitch; };
    auto task_ok = [&](u32 t, u32 j) { return t < ntask && stripe_of(j) < g.nstripes; };

    // ids of this wave's stripes, staged in LDS once (per_wave <= 64)
    __shared__ u64 idl[64];
    {
        u64 x = 0;
        if (u32(li) < per_wave && stripe_of(li) < g.nstripes)
            for (int b = 0; b < n; ++b)
                x |= u64(ids[u64(stripe_of(li)) * n + b]) << (8 * b);
        idl[li] = x;
    }

    const __amdgpu_buffer_rsrc_t drs = rsrc(digests, g.nstripes * u32(n) * 8u);
    const u32 pbytes = u32(n) * u32(ppitch);

    using Buf = u32[U][4 * K];
    auto load_task = [&](Buf &x, u32 t, u32 j, u32 c) {
        const bool ok = task_ok(t, j);
        // The resource starts at the chunk and spans the stripe's remaining
        // bytes (scalar work per task); the lane offsets are loop-invariant,
        // so no per-task VALU address temps exist for the compiler to fence
        // with a wait before the loads issue.  num_records is rounded up to a
        // dword: the buffer unit range-checks whole dwords (a dword
        // straddling num_records reads 0); bytes past B in it are masked
        // below (a dword never crosses a page, so it is mapped).  A task
        // past the end gets num_records 0: nothing is read.
        const u32 cb = c * u32(R * K);
        const u32 left = ok && B > cb ? ((B - cb + 3u) & ~3u) : 0u;
        const __amdgpu_buffer_rsrc_t r = rsrc(blk_of(stripe_of(j)) + cb, left);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const u32 off = u32((u * 1024 + 16 * li) * K + 16 * q);
                const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
                x[u][4 * q] = v.x;
                x[u][4 * q + 1] = v.y;
                x[u][4 * q + 2] = v.z;
                x[u][4 * q + 3] = v.w;
            }
    };

    // XXH64 lane: part hi, accumulator ha (lanes 4n.. idle)
    const int hi = li >> 2, ha = li & 3;
    const u8 *hsrc = xbuf + (hi < E ? hi : 0) * SP + 8 * ha;
    const u32 nst = ps >> 5;  // whole 32-byte stripes of every part
    const u32 left = ps & 31;
    const u32 toff = nst * 32 - (nch - 1) * R;  // tail offset inside the last chunk
    u64 acc = xxh_acc_init(ha, 0);

    auto step = [&](Buf &cur, Buf &nxt, u32 t) {
        // task cursors: t-1 (fold), t (encode), t+P (load); uniform shapes
        const u32 je = t / nch, ce = t - je * nch;
        const u32 jl = (t + P) / nch, cl = (t + P) - jl * nch;
        load_task(nxt, t + P, jl, cl);
        const u32 jf = t >= 1 ? (t - 1) / nch : 0, cf = t >= 1 ? (t - 1) - jf * nch : 0;
        const bool fok = HASH && t >= 1 && task_ok(t - 1, jf);
        const bool fin = fok && cf == nch - 1;
        const bool eok = task_ok(t, je);

        // wave-uniform, rare: the tables of a stripe that starts here, and
        // the zero padding of a stripe's last 16-byte piece
        if (eok) {
            if (ce == 0) {
                // packed product tables T_m, m = 1..K-1, of the stripe starting here
                const u64 idv = idl[je];
                u32 coef[W], idw[W];
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    idw[w] = u32(idv >> (32 * w));
                    coef[w] = idw[w];
                }
#pragma unroll
                for (int m = 1; m < K; ++m) {
                    u32 basis[8][W];
                    make_basis<W>(basis, coef);
                    u8 *tm = tbl + (m - 1) * TB;
                    if constexpr (NIB) {
                        if (li < 32) {
                            const int val = li & 15, h = li >> 4;
                            u32 e[W];
#pragma unroll
                            for (int w = 0; w < W; ++w) {
                                u32 x = 0;
#pragma unroll
                                for (int b = 0; b < 4; ++b)
                                    x ^= basis[4 * h + b][w] & (0u - u32((val >> b) & 1));
                                e[w] = x;
                            }
                            if constexpr (W == 2)
                                *reinterpret_cast<uint2 *>(tm + li * E) = make_uint2(e[0], e[1]);
                            else
                                *reinterpret_cast<u32 *>(tm + li * E) = e[0];
                        }
                    } else {
                        build_table<W, 64>(tm, basis, li);
                    }
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        coef[w] = gf_mul_packed(coef[w], idw[w]);
                }
            }
            if (ce == nch - 1 && (B & 15)) {
                // zero the bytes of the stripe's last 16-byte piece that lie past B
                // (the reference zero-pads its tail row, crt/nk8.c:393-398)
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int q = 0; q < 4 * K; ++q) {
                        const u32 off = ce * u32(R * K) + u32((u * 1024 + 16 * li) * K + 4 * q);
                        const u32 keep = off >= B ? 0u : B - off >= 4 ? 4u : B - off;
                        cur[u][q] &= keep >= 4 ? 0xFFFFFFFFu : (1u << (8 * keep)) - 1u;
                    }
            }
        }

        // ---- one straight-line block: fold task t-1 (serial XXH64 rounds
        // from words read out of the exchange up front), encode task t
        // (table lookups in flight a row group ahead), the exchange write,
        // the stores.  Work past the end (!eok) computes on zeros and its
        // stores are dropped, so no branch splits the block.
        u64 wv[HASH ? RPC : 1];
        u64 tw[4] = {0, 0, 0, 0};
        if constexpr (HASH) {
#pragma unroll
            for (int r = 0; r < RPC; ++r)
                wv[r] = *reinterpret_cast<const u64 *>(hsrc + 32 * r);
            // the tail words of a part whose last chunk this is (read
            // before the exchange is overwritten; used only when fin)
            const u64 *tsrc = reinterpret_cast<const u64 *>(xbuf + (hi < E ? hi : 0) * SP + toff);
#pragma unroll
            for (int w = 0; w < 4; ++w)
                tw[w] = tsrc[w];
        }
        u32 out[U][E][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (!NIB) {
                // byte tables: the 4(K-1) lookups of a group of 4 rows are
                // issued together, one group ahead of the XORs that use
                // them, so a wave keeps up to 8(K-1) LDS reads in flight
                // instead of waiting on every row's K-1
                u32 ent[2][4][K - 1][W];
                auto look = [&](int q, u32 (&e)[4][K - 1][W]) {
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                        for (int m = 1; m < K; ++m) {
                            const int p = (4 * q + rr) * K + m;
                            const u32 byte = (cur[u][p >> 2] >> (8 * (p & 3))) & 0xFFu;
                            const u8 *ep = tbl + (m - 1) * TB + byte * E;
                            if constexpr (E == 8) {
                                const uint2 tt = *reinterpret_cast<const uint2 *>(ep);
                                e[rr][m - 1][0] = tt.x;
                                e[rr][m - 1][W - 1] = tt.y;
                            } else {
                                e[rr][m - 1][0] = *reinterpret_cast<const u32 *>(ep);
                            }
                        }
                };
                look(0, ent[0]);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q < 3)
                        look(q + 1, ent[(q + 1) & 1]);
                    u32 row[4][W];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int p0 = (4 * q + rr) * K;
                        const u32 rep = __builtin_amdgcn_perm(0u, cur[u][p0 >> 2], 0x01010101u * u32(p0 & 3));
#pragma unroll
                        for (int w = 0; w < W; ++w) {
                            u32 x = rep;
#pragma unroll
                            for (int m = 1; m < K; ++m)
                                x ^= ent[q & 1][rr][m - 1][w];
                            row[rr][w] = x;
                        }
                    }
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        transpose4(row[0][w], row[1][w], row[2][w], row[3][w], out[u][4 * w][q],
                                   out[u][4 * w + 1][q], out[u][4 * w + 2][q], out[u][4 * w + 3][q]);
                }
            } else {
                // nibble tables: T_m[x] = L_m[x & 15] ^ H_m[x >> 4], two
                // conflict-free lookups per byte; a row group's lookups are
                // issued before its XORs
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    u32 e[4][K - 1][2][W];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                        for (int m = 1; m < K; ++m) {
                            const int p = (4 * q + rr) * K + m;
                            const u32 byte = (cur[u][p >> 2] >> (8 * (p & 3))) & 0xFFu;
                            const u8 *tb = tbl + (m - 1) * TB;
                            const u8 *e0 = tb + (byte & 15u) * E;
                            const u8 *e1 = tb + (16u + (byte >> 4)) * E;
                            if constexpr (E == 8) {
                                const uint2 t0 = *reinterpret_cast<const uint2 *>(e0);
                                const uint2 t1 = *reinterpret_cast<const uint2 *>(e1);
                                e[rr][m - 1][0][0] = t0.x;
                                e[rr][m - 1][0][W - 1] = t0.y;
                                e[rr][m - 1][1][0] = t1.x;
                                e[rr][m - 1][1][W - 1] = t1.y;
                            } else {
                                e[rr][m - 1][0][0] = *reinterpret_cast<const u32 *>(e0);
                                e[rr][m - 1][1][0] = *reinterpret_cast<const u32 *>(e1);
                            }
                        }
                    u32 row[4][W];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int p0 = (4 * q + rr) * K;
                        const u32 rep = __builtin_amdgcn_perm(0u, cur[u][p0 >> 2], 0x01010101u * u32(p0 & 3));
#pragma unroll
                        for (int w = 0; w < W; ++w) {
                            u32 x = rep;
#pragma unroll
                            for (int m = 1; m < K; ++m)
                                x ^= e[rr][m - 1][0][w] ^ e[rr][m - 1][1][w];
                            row[rr][w] = x;
                        }
                    }
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        transpose4(row[0][w], row[1][w], row[2][w], row[3][w], out[u][4 * w][q],
                                   out[u][4 * w + 1][q], out[u][4 * w + 2][q], out[u][4 * w + 3][q]);
                }
            }
        }

        if constexpr (HASH) {
            const u32 rbase = fok ? cf * RPC : nst;
#pragma unroll
            for (int r = 0; r < RPC; ++r) {
                const u64 nx = xxh_round(acc, wv[r]);
                acc = rbase + r < nst ? nx : acc;
            }
            // this task's parts into the exchange, after the reads above
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int i = 0; i < E; ++i)
                    *reinterpret_cast<uint4 *>(xbuf + i * SP + u * 1024 + 16 * li) =
                        make_uint4(out[u][i][0], out[u][i][1], out[u][i][2], out[u][i][3]);
        }
        // stores: n parts x U units of 1 KiB runs; dropped where not live
        const __amdgpu_buffer_rsrc_t prs = rsrc(par_of(stripe_of(je)), pbytes);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 r0 = ce * u32(R) + u32(u * 1024 + 16 * li);
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const u32 off = live_off(eok & (i < n) & (r0 < ps), u32(i) * u32(ppitch) + r0);
                const v4u v = {out[u][i][0], out[u][i][1], out[u][i][2], out[u][i][3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, prs, off, 0, 0);
            }
        }
        if constexpr (HASH) {
            // a stripe's last chunk was folded: its digests (merge, length,
            // tail, avalanche); one digest store per step, dropped unless a
            // stripe finished here
            u64 dval = 0;
            if (fin) {
                const int base = li & ~3;
                const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
                const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
                u64 h = ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
                h += ps;
                dval = xxh_tail_regs(h, tw, left);
                acc = xxh_acc_init(ha, 0);
            }
            const u32 doff = live_off(fin & (hi < n) & (ha == 0), (stripe_of(jf) * u32(n) + u32(hi)) * 8u);
            const v2u dv = {u32(dval), u32(dval >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(dv, drs, doff, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();
    };

    // P + 1 register sets in rotation: step t encodes set t % (P+1) and
    // loads task t + P into set (t + P) % (P+1)
    u32 xb[P + 1][U][4 * K];
#pragma unroll
    for (int p = 0; p < P; ++p)
        load_task(xb[p], u32(p), u32(p) / nch, u32(p) % nch);
    const u32 last = HASH ? ntask : ntask - 1;  // step ntask only folds
    step(xb[0], xb[P], 0);
    for (u32 t = 1; t <= last;) {
#pragma unroll
        for (int q = 1; q <= P + 1; ++q) {
            if (t > last)
                break;
            step(xb[q % (P + 1)], xb[(q + P) % (P + 1)], t++);
        }
    }
}

// ------------------------------------------------------------------ decode
//
// k_decode_plan: K lanes per stripe, lane c of a stripe computes row c of
// W.  First K offered slots with distinct ids (crt/nk8.c:512-537) and
// W = V^-1 for V[m][c] = x_c^m in closed form (Lagrange basis: W[c][m] =
// [t^m] M(t)/(t + x_c) / M'(x_c) with M(t) = prod_c (t + x_c)): the unique
// inverse, so identical to the reference's Gauss-Jordan
// (crt/nk8.c:199-266).  plan[s] = K slots then W row-major; slot byte 0xFF
// marks a stripe with fewer than K distinct ids.  The plan is a serial chain
// of bit-serial GF products on one lane, so spreading the K rows over K
// lanes (and loading the first 16 offers before walking them) cuts the
// kernel -- a fixed cost of every uniform k >= 3 decode -- from ~9 us.
template <int K>
__global__ __launch_bounds__(256) void k_decode_plan(const u8 *ids, const u8 *avail, int n_slots, int navail,
                                                     u32 nstripes, u8 *plan, int32_t *status, const GfTables *gft)
{
    const u64 t = u64(blockIdx.x) * blockDim.x + threadIdx.x;
    const u32 s = u32(t / K);
    const int col = int(t % K);
    if (s >= nstripes)
        return;
    const u8 *sid = ids + u64(s) * n_slots;
    const u8 *sav = avail + u64(s) * navail;
    u8 *pl = plan + u64(s) * (K + K * K);
    u32 x[K], sl[K];
    int h = 0;
    auto offer = [&](u32 slot, u32 id) {
        bool dup = false;
#pragma unroll
        for (int j = 0; j < K; ++j)
            dup |= j < h && x[j] == id;
        if (dup || h >= K)
            return;
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j == h) {
                x[j] = id;
                sl[j] = slot;
            }
        ++h;
    };
    // the first 16 offers: all loads issued before any is used
    constexpr int PRE = 16;
    u32 pslot[PRE], pid[PRE];
#pragma unroll
    for (int c = 0; c < PRE; ++c)
        pslot[c] = c < navail ? sav[c] : 0u;
#pragma unroll
    for (int c = 0; c < PRE; ++c)
        pid[c] = c < navail ? sid[pslot[c]] : 0u;
#pragma unroll
    for (int c = 0; c < PRE; ++c)
        if (c < navail)
            offer(pslot[c], pid[c]);
    for (int c = PRE; c < navail && h < K; ++c) {
        const u32 slot = sav[c];
        offer(slot, sid[slot]);
    }
    if (col == 0 && status)
        status[s] = h < K ? -EINVAL : 0;
    if (h < K) {
        if (col == 0)
            pl[0] = 0xFF;
        return;
    }
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
    // this lane's row: x_c, slot of column col
    u32 xc = 0, sc = 0;
#pragma unroll
    for (int c = 0; c < K; ++c)
        if (c == col) {
            xc = x[c];
            sc = sl[c];
        }
    pl[col] = u8(sc);
    u32 q[K];
    u32 a = M[K];
    q[K - 1] = a;
#pragma unroll
    for (int i = K - 1; i >= 1; --i) {
        a = M[i] ^ gfm_bits(xc, a);
        q[i - 1] = a;
    }
    u32 dd = 0;
#pragma unroll
    for (int i = K - 1; i >= 0; --i)
        dd = gfm_bits(dd, xc) ^ q[i];
    const u32 dinv = gft->inv[dd];
#pragma unroll
    for (int i = 0; i < K; ++i)
        pl[K + col * K + i] = u8(gfm_bits(q[i], dinv));
}

// One-shot slice: rows [slice*R, slice*R + R) of one stripe, R = 1024*U.
// XPOSE: output rows go through LDS so every store instruction writes one
// contiguous 1 KiB run (lane l owns 16 rows = 16K contiguous bytes; stored
// directly that is a 16K-byte lane stride).
// RAGGED: a persistent grid walks the (stripe, slice) list of a ragged
// batch -- smap[w] = (processing position << 32) | slice of slice w (g.order
// applied; k_slice_scan + k_slice_map), *stotal = all slices -- and each
// slice is one pass of the same one-shot body.
template <int K, int E, int U, bool XPOSE, bool RAGGED>
__global__ __launch_bounds__(64) void k_decode_slice(nkfs_geom g, int n_slots, const u8 *plan, u32 slices,
                                                     const u64 *smap, const u32 *stotal)
{
    constexpr int W = E / 4;
    constexpr int TB = 256 * E;
    constexpr int R = 1024 * U;
    constexpr int LS = 16 * K + (K % 2 == 0 ? 16 : 0);  // transpose bytes per lane (even K padded: bank spread)
    __shared__ __attribute__((aligned(16))) u8 tbl[K * TB];
    __shared__ __attribute__((aligned(16))) u8 obuf[XPOSE ? 64 * LS : 16];

    const int li = threadIdx.x;
    const u32 total = RAGGED ? *stotal : 0u;
    for (u32 w = blockIdx.x;; w += gridDim.x) {
    u32 s, slice;
    if constexpr (RAGGED) {
        if (w >= total)
            return;
        const u64 e = smap[w];
        slice = u32(e);
        s = g.order ? g.order[u32(e >> 32)] : u32(e >> 32);
#ifdef NKFS_DEBUG_BOUNDS
        if (s >= g.nstripes || u32(e >> 32) >= g.nstripes ||
            (g.blocks_bytes && g.block_off[s] + g.block_sizes[s] > g.blocks_bytes) ||
            (g.parts_bytes && g.part_off[s] + u64(n_slots) * ((u64(part_size_of(g.block_sizes[s], K)) + 255) & ~u64(255)) >
                                  g.parts_bytes)) {
            if (li == 0)
                printf("nkfs bounds: k_decode_slice map entry %u -> stripe %u slice %u out of range\n", w, s, slice);
            continue;
        }
#endif
    } else {
        s = w / slices;
        slice = w % slices;
        if (s >= g.nstripes)
            return;
    }
    const u8 *pl = plan + u64(s) * (K + K * K);
    const u32 sl0 = pl[0];
    if (sl0 == 0xFF) {  // fewer than K distinct ids: status says -EINVAL, block untouched
        if constexpr (RAGGED)
            continue;
        return;
    }
    const u32 B = RAGGED ? g.block_sizes[s] : g.block_size;
    const u32 ps = part_size_of(B, K);
    const u64 ppitch = RAGGED ? (u64(ps) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1) : g.part_pitch;
    const u32 rbase = slice * R;
    const u8 *pbase = RAGGED ? g.parts + g.part_off[s] : g.parts + u64(s) * n_slots * g.part_pitch;
    u8 *out = const_cast<u8 *>(g.blocks) + (RAGGED ? g.block_off[s] : u64(s) * g.block_pitch);
    // ragged part offsets are caller data: byte loads where a stripe's parts
    // are not 16-byte aligned (uniform batches are checked by the launcher)
    const bool pal = !RAGGED || (reinterpret_cast<uintptr_t>(pbase) & 15) == 0;

    // loads first (their latency hides under the table build)
    const u8 *src[K];
#pragma unroll
    for (int c = 0; c < K; ++c)
        src[c] = pbase + u64(c ? pl[c] : sl0) * ppitch;
    u32 pv[U][K][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32 r0 = rbase + u * 1024 + 16 * li;
        if (r0 < ps)
#pragma unroll
            for (int c = 0; c < K; ++c) {
                if (pal) {
                    const uint4 t = *reinterpret_cast<const uint4 *>(src[c] + r0);  // pitch >= round16(ps)
                    pv[u][c][0] = t.x;
                    pv[u][c][1] = t.y;
                    pv[u][c][2] = t.z;
                    pv[u][c][3] = t.w;
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        u32 x = 0;
                        for (int e = 0; e < 4; ++e)
                            x |= u32(src[c][r0 + 4 * q + e]) << (8 * e);  // within the pitch
                        pv[u][c][q] = x;
                    }
                }
            }
    }
    // U_c[x] = (W[c][0] x, ..., W[c][K-1] x), packed
#pragma unroll
    for (int c = 0; c < K; ++c) {
        u32 rw[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            u32 x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (4 * w + b < K)
                    x |= u32(pl[K + c * K + 4 * w + b]) << (8 * b);
            rw[w] = x;
        }
        u32 basis[8][W];
        make_basis<W>(basis, rw);
        build_table<W, 64>(tbl + c * TB, basis, li);
    }
    __syncthreads();

    const bool aligned = ((reinterpret_cast<uintptr_t>(out) | (RAGGED ? 0 : g.block_pitch)) & 15) == 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32 ru = rbase + u * 1024;  // first row of this unit
        if (ru >= ps)
            break;
        const u32 r0 = ru + 16 * li;
        u32 o[4 * K];
        if (r0 < ps) {
            // the K lookups of each of a 4-row group's rows issued together,
            // one group ahead of the XORs that consume them (up to 8K LDS
            // reads in flight per lane instead of waiting on each group)
            u32 ent[2][4][K][W];
            auto look = [&](int gq, u32 (&e)[4][K][W]) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int r = 4 * gq + rr;
#pragma unroll
                    for (int c = 0; c < K; ++c) {
                        const u32 byte = (pv[u][c][r >> 2] >> (8 * (r & 3))) & 0xFFu;
                        const u8 *ep = tbl + c * TB + byte * E;
                        if constexpr (E == 8) {
                            const uint2 t = *reinterpret_cast<const uint2 *>(ep);
                            e[rr][c][0] = t.x;
                            e[rr][c][W - 1] = t.y;
                        } else {
                            e[rr][c][0] = *reinterpret_cast<const u32 *>(ep);
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
                        for (int c = 1; c < K; ++c)
                            x ^= ent[gq & 1][rr][c][w];
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
    if constexpr (!RAGGED)
        return;
    __syncthreads();  // the next slice rebuilds the tables
    }
}

#ifndef NKFS_WALK_K
// Exclusive prefix of the slices per stripe of a ragged batch in processing
// order (g.order applied): sfirst[0..nstripes], *stotal = sfirst[nstripes].
// One workgroup; every thread sums a contiguous run of stripes.
__global__ __launch_bounds__(1024) void k_slice_scan(const u32 *sizes, const u32 *order, u32 nstripes, int k,
                                                     u32 rows, u32 *sfirst, u32 *stotal)
{
    // thread t owns the contiguous positions [t*per, t*per + per); the
    // per-stripe slice counts are loaded once, all independently (clamped
    // indices, no branch), and kept in registers for the prefix pass
    constexpr int MAXP = 64;  // the launcher keeps nstripes <= 64 * 1024
    __shared__ u32 part[1024];
    const u32 t = threadIdx.x;
    const u32 per = (nstripes + 1023) / 1024;
    const u32 a = t * per;
    u32 cnt[MAXP];
    u32 sum = 0;
#pragma unroll
    for (int j = 0; j < MAXP; ++j) {
        const u32 p = a + u32(j);
        const bool live = u32(j) < per && p < nstripes;
        const u32 pc = live ? p : 0u;
        const u32 sz = sizes[order ? order[pc] : pc];
        const u32 ps = part_size_of(sz, k);
        const u32 c = ps ? (ps + rows - 1) / rows : 1u;  // an empty stripe is one (empty) pass
        cnt[j] = live ? c : 0u;
        sum += cnt[j];
    }
    part[t] = sum;
    __syncthreads();
    for (u32 d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
        const u32 v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    u32 run = t ? part[t - 1] : 0u;
#pragma unroll
    for (int j = 0; j < MAXP; ++j) {
        const u32 p = a + u32(j);
        if (u32(j) < per && p < nstripes)
            sfirst[p] = run;
        run += cnt[j];
    }
    if (t == 1023) {
        sfirst[nstripes] = part[1023];
        *stotal = part[1023];
    }
}

// smap[sfirst[p] + j] = (p << 32) | j for the slices j of the stripe at
// processing position p: one wave per stripe, lanes over its slices.
__global__ __launch_bounds__(256) void k_slice_map(const u32 *sfirst, u32 nstripes, u64 *smap)
{
    const u32 p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= nstripes)
        return;
    const u32 a = sfirst[p], n = sfirst[p + 1] - a;
    for (u32 j = threadIdx.x & 63; j < n; j += 64)
        smap[a + j] = (u64(p) << 32) | j;
}

#endif  // !NKFS_WALK_K

// ----------------------------------------------------------------- launchers

template <int K, int E, int U, int P, bool HASH, bool NIB>
static void launch_walk_kk(hipStream_t st, const nkfs_geom &g, const u8 *ids, u64 *dig, int waves, int cus)
{
    // uniform batches: persistent grid of the resident waves, walking stripes
    // grid-stride (at most 64 stripes per wave: their ids are staged in LDS);
    // ragged: one wave per stripe
    if (g.block_sizes) {
        const Shape sh = occupancy_shape(reinterpret_cast<const void *>(&k_encode_walk<K, E, U, P, HASH, NIB, true>),
                                         waves);
        hipLaunchKernelGGL((k_encode_walk<K, E, U, P, HASH, NIB, true>), dim3(g.nstripes), dim3(64), sh.pad, st, g,
                           ids, dig, 1u);
        return;
    }
    const Shape sh =
        occupancy_shape(reinterpret_cast<const void *>(&k_encode_walk<K, E, U, P, HASH, NIB, false>), waves);
    const u32 cap = u32(cus) * u32(sh.per_cu);
    u32 grid = g.nstripes < cap ? g.nstripes : cap;
    u32 per_wave = (g.nstripes + grid - 1) / grid;
    if (per_wave > 64) {
        per_wave = 64;
        grid = (g.nstripes + 63) / 64;
    }
    hipLaunchKernelGGL((k_encode_walk<K, E, U, P, HASH, NIB, false>), dim3(grid), dim3(64), sh.pad, st, g, ids, dig,
                       per_wave);
}

// prefetch depth 2 only for the byte-table forms (nibble tables keep P = 1)
template <int K, int E, int U, bool HASH, bool NIB>
static void launch_walk_k(hipStream_t st, const nkfs_geom &g, const u8 *ids, u64 *dig, int waves, int cus)
{
    if constexpr (!NIB)
        if (nkfs_tune_now().enc_prefetch >= 2)
            return launch_walk_kk<K, E, U, 2, HASH, NIB>(st, g, ids, dig, waves, cus);
    launch_walk_kk<K, E, U, 1, HASH, NIB>(st, g, ids, dig, waves, cus);
}

// Per-k entry points.  The Makefile compiles this file once per k
// (-DNKFS_WALK_K=2..8: that k's kernels and these two functions) and once
// without (the dispatchers below): the kernels of all seven k in one
// translation unit took ~400 s to compile, one k takes a seventh of it.
namespace nkfs {
template <int K>
void walk_encode_k(const nkfs_geom &g, const u8 *ids, u64 *dig, int units, int nib, int waves, int cus,
                   hipStream_t st)
{
    const bool h = dig != nullptr;
    if (g.n <= 4) {
        if (units == 2)
            h ? launch_walk_k<K, 4, 2, true, false>(st, g, ids, dig, waves, cus)
              : launch_walk_k<K, 4, 2, false, false>(st, g, ids, dig, waves, cus);
        else
            h ? launch_walk_k<K, 4, 1, true, false>(st, g, ids, dig, waves, cus)
              : launch_walk_k<K, 4, 1, false, false>(st, g, ids, dig, waves, cus);
    } else if (nib) {
        h ? launch_walk_k<K, 8, 1, true, true>(st, g, ids, dig, waves, cus)
          : launch_walk_k<K, 8, 1, false, true>(st, g, ids, dig, waves, cus);
    } else {
        h ? launch_walk_k<K, 8, 1, true, false>(st, g, ids, dig, waves, cus)
          : launch_walk_k<K, 8, 1, false, false>(st, g, ids, dig, waves, cus);
    }
}

#ifdef NKFS_WALK_K
template void walk_encode_k<NKFS_WALK_K>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
#else
extern template void walk_encode_k<2>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
extern template void walk_encode_k<3>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
extern template void walk_encode_k<4>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
extern template void walk_encode_k<5>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
extern template void walk_encode_k<6>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
extern template void walk_encode_k<7>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
extern template void walk_encode_k<8>(const nkfs_geom &, const u8 *, u64 *, int, int, int, int, hipStream_t);
#endif
}  // namespace nkfs

#ifndef NKFS_WALK_K
// Walk encoder for n <= 8, k <= 8 (uniform or ragged; g->order honoured).
// units: 1,024-row units per chunk.  -ENOSYS where the buffer offsets of a
// stripe would not fit 31 bits (the generic kernels take those).
extern "C" int nkfs_walk_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, int units, int nib,
                                int waves, int cus, hipStream_t st)
{
    if (g->n > 8 || g->k > 8 || (!g->block_sizes && (g->part_min || g->part_max)))
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    const u64 ps = part_size_of_host(g->block_size, g->k);
    const u64 pitch = g->block_sizes ? ((ps + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1)) : g->part_pitch;
    // every buffer offset must fit 31 bits: live_off() drops a store by
    // setting bit 31, which lands past num_records only for offsets below 2^31
    if (!walk_offsets_fit(g->block_size, u64(g->n) * pitch, g->nstripes, g->n))
        return -ENOSYS;
    switch (g->k) {
    case 2: walk_encode_k<2>(*g, ids, digests, units, nib, waves, cus, st); break;
    case 3: walk_encode_k<3>(*g, ids, digests, units, nib, waves, cus, st); break;
    case 4: walk_encode_k<4>(*g, ids, digests, units, nib, waves, cus, st); break;
    case 5: walk_encode_k<5>(*g, ids, digests, units, nib, waves, cus, st); break;
    case 6: walk_encode_k<6>(*g, ids, digests, units, nib, waves, cus, st); break;
    case 7: walk_encode_k<7>(*g, ids, digests, units, nib, waves, cus, st); break;
    case 8: walk_encode_k<8>(*g, ids, digests, units, nib, waves, cus, st); break;
    default: return -ENOSYS;
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
#endif  // !NKFS_WALK_K

// uniform: one wave per (stripe, slice); ragged: a persistent grid of the
// resident waves over the scanned slice list
template <int K, int E, int U, bool XP>
static void launch_slice(hipStream_t st, const nkfs_geom &g, int n_slots, const u8 *plan, u32 slices, int waves,
                         const u64 *smap, const u32 *stotal, int cus)
{
    if (smap) {
        const Shape sh = occupancy_shape(reinterpret_cast<const void *>(&k_decode_slice<K, E, U, XP, true>), waves);
        hipLaunchKernelGGL((k_decode_slice<K, E, U, XP, true>), dim3(u32(cus) * u32(sh.per_cu)), dim3(64), sh.pad,
                           st, g, n_slots, plan, 0u, smap, stotal);
        return;
    }
    const Shape sh = occupancy_shape(reinterpret_cast<const void *>(&k_decode_slice<K, E, U, XP, false>), waves);
    hipLaunchKernelGGL((k_decode_slice<K, E, U, XP, false>), dim3(g.nstripes * slices), dim3(64), sh.pad, st, g,
                       n_slots, plan, slices, (const u64 *)nullptr, (const u32 *)nullptr);
}

template <int K, int E>
static void launch_slice_u(int units, hipStream_t st, const nkfs_geom &g, int n_slots, const u8 *plan, u32 slices,
                           int waves, const u64 *smap, const u32 *stotal, int cus)
{
    constexpr bool XP = K >= 3;
    if (units >= 4)
        launch_slice<K, E, 4, XP>(st, g, n_slots, plan, slices, waves, smap, stotal, cus);
    else if (units == 2)
        launch_slice<K, E, 2, XP>(st, g, n_slots, plan, slices, waves, smap, stotal, cus);
    else
        launch_slice<K, E, 1, XP>(st, g, n_slots, plan, slices, waves, smap, stotal, cus);
}

namespace nkfs {
template <int K>
void slice_decode_k(const nkfs_geom &g, int n_slots, const u8 *ids, const u8 *avail, int navail, u8 *plan,
                    int32_t *status, const GfTables *gft, int units, u32 slices, int waves, const u64 *smap,
                    const u32 *stotal, int cus, hipStream_t st)
{
    const dim3 pgrid(u32((u64(g.nstripes) * u64(K) + 255) / 256));  // k_decode_plan: k lanes per stripe
    hipLaunchKernelGGL((k_decode_plan<K>), pgrid, dim3(256), 0, st, ids, avail, n_slots, navail, g.nstripes, plan,
                       status, gft);
    launch_slice_u<K, (K <= 4 ? 4 : 8)>(units, st, g, n_slots, plan, slices, waves, smap, stotal, cus);
}

#ifdef NKFS_WALK_K
template void slice_decode_k<NKFS_WALK_K>(const nkfs_geom &, int, const u8 *, const u8 *, int, u8 *, int32_t *,
                                          const GfTables *, int, u32, int, const u64 *, const u32 *, int,
                                          hipStream_t);
#else
#define NKFS_EXT(KK)                                                                                            \
    extern template void slice_decode_k<KK>(const nkfs_geom &, int, const u8 *, const u8 *, int, u8 *, int32_t *, \
                                            const GfTables *, int, u32, int, const u64 *, const u32 *, int,     \
                                            hipStream_t);
NKFS_EXT(2)
NKFS_EXT(3)
NKFS_EXT(4)
NKFS_EXT(5)
NKFS_EXT(6)
NKFS_EXT(7)
NKFS_EXT(8)
#undef NKFS_EXT
#endif
}  // namespace nkfs

#ifndef NKFS_WALK_K
// Slice decoder, k <= 8: plan kernel (selection + inverse per stripe into
// `work`, nkfs_decode_work_bytes layout) then one-shot slice waves; a ragged
// batch (g->order honoured) first scans its slice counts into stream-ordered
// scratch.  -ENOSYS outside its shapes.
extern "C" int nkfs_slice_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                                 int navail, void *work, int32_t *status, const void *gf, int units, int waves,
                                 int cus, hipStream_t st)
{
    if (g->k > 8 || (reinterpret_cast<uintptr_t>(g->parts) & 15) || (!g->block_sizes && (g->part_pitch & 15)) ||
        (g->block_sizes && g->nstripes > 64u * 1024u))  // k_slice_scan: 64 stripes per thread
        return -ENOSYS;
    if (!g->nstripes)
        return 0;
    u8 *plan = static_cast<u8 *>(work);
    const GfTables *gft = static_cast<const GfTables *>(gf);
    const u32 ps = part_size_of_host(g->block_size, g->k);  // ragged: the bound on block sizes
    units = units >= 4 ? 4 : units >= 2 ? 2 : 1;
    // a stripe that fits in fewer units takes one wave of just those
    while (!g->block_sizes && units > 1 && u32(units / 2) * 1024u >= ps)
        units /= 2;
    const u32 slices = (ps + 1024u * units - 1) / (1024u * units);
    // ragged: slice list in the launch's scratch (scratch.h) -- nstripes + 2
    // u32 of prefix and total, then at most nstripes * slices(max) u64 map
    // entries
    u32 *scan = nullptr;
    u64 *smap = nullptr;
    Scratch sc;
    if (g->block_sizes) {
        const size_t head = ((size_t(g->nstripes) + 2) * sizeof(u32) + 15) & ~size_t(15);
        // the caller's scratch is sized for 1,024-row units: any units fit
        scan = static_cast<u32 *>(sc.take(g, head + size_t(g->nstripes) * slices * sizeof(u64), st, true));
        if (!scan)
            return -ENOSYS;
        smap = reinterpret_cast<u64 *>(reinterpret_cast<u8 *>(scan) + head);
        hipLaunchKernelGGL(k_slice_scan, dim3(1), dim3(1024), 0, st, g->block_sizes, g->order, g->nstripes, g->k,
                           1024u * u32(units), scan, scan + g->nstripes + 1);
        hipLaunchKernelGGL(k_slice_map, dim3((g->nstripes + 3) / 4), dim3(256), 0, st, scan, g->nstripes, smap);
    }
    const u32 *stotal = scan ? scan + g->nstripes + 1 : nullptr;
    int rc = 0;
    switch (g->k) {
    case 2: slice_decode_k<2>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    case 3: slice_decode_k<3>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    case 4: slice_decode_k<4>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    case 5: slice_decode_k<5>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    case 6: slice_decode_k<6>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    case 7: slice_decode_k<7>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    case 8: slice_decode_k<8>(*g, n_slots, ids, avail, navail, plan, status, gft, units, slices, waves, smap, stotal, cus, st); break;
    default:
        rc = -ENOSYS;
    }
    const int e = sc.finish();
    if (!rc)
        rc = e;
    if (rc)
        return rc;
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
#endif  // !NKFS_WALK_K
