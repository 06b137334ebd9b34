// nk8_kernels.hip -- gfx950 kernels for the nkfs N-K erasure code and its
// per-part XXH64 (reference: irqlevel/nkfs crt/nk8.c, crt/xxhash.c).
//
// Kernels in this file are the general path: any (n, k) the reference
// accepts (2<=k<=n<=255, k<=254), any block size, uniform or ragged
// batches.  The streaming fast path for n <= 8 (fused encode + XXH64 with
// per-stripe packed product tables in LDS) lives in nk8_fast.hip and is
// preferred by the dispatch in nkfs_launch_encode when it applies.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "../../include/nkfs_gpu.h"
#include "gf256.h"
#include "nkfs_internal.h"
#include "runtime.h"
#include "scratch.h"
#include "xxh64_dev.h"

using namespace nkfs;
typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

namespace {

__host__ __device__ inline u32 part_size_of(u32 block_size, int k)
{
    return block_size / u32(k) + ((block_size % u32(k)) ? 1u : 0u);
}

__host__ __device__ inline u64 pitch_of(u32 block_size, int k)
{
    return (u64(part_size_of(block_size, k)) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
}

struct StripeView {
    const u8 *blk;
    u8 *parts;
    u64 pitch;
    u32 B;
    u32 ps;
};

__device__ inline StripeView stripe_view(const nkfs_geom &g, u32 s)
{
    StripeView v;
    if (g.block_sizes) {
        v.B = g.block_sizes[s];
        v.blk = g.blocks + g.block_off[s];
        v.parts = g.parts + g.part_off[s];
        v.pitch = pitch_of(v.B, g.k);
    } else {
        v.B = g.block_size;
        v.blk = g.blocks + u64(s) * g.block_pitch;
        v.parts = g.parts + u64(s) * u64(g.n) * g.part_pitch;
        v.pitch = g.part_pitch;
    }
    v.ps = part_size_of(v.B, g.k);
    return v;
}

// GF(2^8) log/antilog in LDS.
struct GfLds {
    uint16_t log[256];
    u8 exp[768];
};

__device__ inline void gf_stage(GfLds &L, const GfTables *g)
{
    for (int i = threadIdx.x; i < 256; i += blockDim.x)
        L.log[i] = g->log[i];
    for (int i = threadIdx.x; i < 768; i += blockDim.x)
        L.exp[i] = g->exp[i];
    __syncthreads();
}

__device__ inline u8 gf_mul(const GfLds &L, u8 a, u8 b)
{
    return (a && b) ? L.exp[L.log[a] + L.log[b]] : u8(0);
}

__device__ inline u64 shfl64(u64 v, int src)
{
    u32 lo = __shfl(u32(v), src, 64);
    u32 hi = __shfl(u32(v >> 32), src, 64);
    return (u64(hi) << 32) | lo;
}

}  // namespace

// ----------------------------------------------------------- GF tables

__global__ void k_gf_init(GfTables *t)
{
    if (threadIdx.x != 0 || blockIdx.x != 0)
        return;
    u8 x = 1;
    for (int i = 0; i < 255; ++i) {
        t->exp[i] = x;
        t->exp[i + 255] = x;
        t->log[x] = uint16_t(i);
        x = gf_mul_slow(x, 3);
    }
    for (int i = 510; i < 768; ++i)
        t->exp[i] = 0;
    t->log[0] = LOG_ZERO;
    t->inv[0] = 0;
    for (int a = 1; a < 256; ++a)
        t->inv[a] = t->exp[255 - t->log[a]];
}

// ------------------------------------------------------ generic encode
//
// grid (nstripes, ceil(max_ps / 256)); one thread per row j of stripe
// blockIdx.x, computing byte j of every part:
//   part_i[j] = XOR_m ids[i]^m * d[j*k + m]     (crt/nk8.c:403-420)
// with d zero beyond block_size (the reference's padded tail row).
__global__ __launch_bounds__(256) void k_encode_generic(nkfs_geom g, const u8 *ids, const GfTables *gft)
{
    __shared__ GfLds L;
    __shared__ uint16_t lid[256];
    gf_stage(L, gft);
    const u32 s = blockIdx.x;
    const StripeView v = stripe_view(g, s);
    for (int i = threadIdx.x; i < g.n; i += blockDim.x)
        lid[i] = L.log[ids[u64(s) * g.n + i]];
    __syncthreads();
    const int kk = g.k;
    // rows grid-stride over grid.y (capped at 65,535 by the launcher)
    for (u32 j = blockIdx.y * blockDim.x + threadIdx.x; j < v.ps; j += gridDim.y * blockDim.x) {
        const u64 row = u64(j) * kk;
        for (int i = 0; i < g.n; ++i) {
            const int li = lid[i];
            int la = 0;  // log of ids[i]^m
            u8 acc = 0;
            for (int m = 0; m < kk; ++m) {
                const u64 pos = row + m;
                const u8 x = pos < v.B ? v.blk[pos] : u8(0);
                if (x)
                    acc ^= L.exp[la + L.log[x]];
                la += li;
                if (la >= 255)
                    la -= 255;
            }
            v.parts[u64(i) * v.pitch + j] = acc;
        }
    }
}

// ---------------------------------------------------- XXH64 over parts
//
// Four lanes per part (accumulator a = lane & 3 consumes words a, a+4, ...),
// converge + tail + avalanche in lane a == 0.  Part bases are 16-byte
// aligned (pitch is a multiple of 16).
__global__ __launch_bounds__(256) void k_hash_parts(nkfs_geom g, u64 *digests)
{
    const u64 t = u64(blockIdx.x) * blockDim.x + threadIdx.x;
    const u64 msg = t >> 2;
    const int a = int(t & 3);
    const u64 total = u64(g.nstripes) * u64(g.n);
    const bool live = msg < total;
    const u8 *p = nullptr;
    u32 len = 0;
    if (live) {
        const u32 s = u32(msg / u32(g.n));
        const u32 i = u32(msg % u32(g.n));
        const StripeView v = stripe_view(g, s);
        p = v.parts + u64(i) * v.pitch;
        len = v.ps;
    }
    u64 acc = xxh_acc_init(a, 0);
    const u32 nst = len >> 5;
    const u64 *w = reinterpret_cast<const u64 *>(p) + a;
    for (u32 r = 0; r < nst; ++r)
        acc = xxh_round(acc, w[4 * r]);
    const int base = int(threadIdx.x & 63) & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    if (!live || a != 0)
        return;
    u64 h = len >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
    h += len;
    digests[msg] = xxh_tail(h, p + (u64(nst) << 5), len & 31);
}

// Same, for an arbitrary message list (offsets multiple of 8).
__global__ __launch_bounds__(256) void k_xxh64_batch(const u8 *base, const u64 *off, const u64 *lenv,
                                                     u32 count, u64 seed, u64 *out)
{
    const u64 t = u64(blockIdx.x) * blockDim.x + threadIdx.x;
    const u64 msg = t >> 2;
    const int a = int(t & 3);
    const bool live = msg < count;
    const u8 *p = live ? base + off[msg] : nullptr;
    const u64 len = live ? lenv[msg] : 0;
    u64 acc = xxh_acc_init(a, seed);
    const u64 nst = len >> 5;
    const u64 *w = reinterpret_cast<const u64 *>(p) + a;
    for (u64 r = 0; r < nst; ++r)
        acc = xxh_round(acc, w[4 * r]);
    const int b = int(threadIdx.x & 63) & ~3;
    const u64 v1 = shfl64(acc, b), v2 = shfl64(acc, b + 1);
    const u64 v3 = shfl64(acc, b + 2), v4 = shfl64(acc, b + 3);
    if (!live || a != 0)
        return;
    u64 h = len >= 32 ? xxh_converge(v1, v2, v3, v4) : seed + XP5;
    h += len;
    out[msg] = xxh_tail(h, p + (nst << 5), u32(len & 31));
}

// ------------------------------------------------------------- decode
//
// Per stripe: pick the first k offered parts with distinct ids
// (crt/nk8.c:512-537), then W = V^-1 for V[m][c] = x_c^m (crt/nk8.c:509-546).
// W is computed in closed form: column c of the decode is the Lagrange basis
// polynomial L_c(t) = prod_{c' != c} (t + x_c') / (x_c + x_c'), so
// W[c][m] = [t^m] L_c(t).  The inverse of a matrix is unique, so this is
// bit-identical to the reference's Gauss-Jordan (checked against the oracle
// and the golden fixtures); it costs O(k^2) per stripe instead of O(k^3)
// and spreads over one thread per column.
// work per stripe: k bytes of slot index, then W row-major (k*k bytes).
__global__ __launch_bounds__(64) void k_decode_prep(const u8 *ids, const u8 *avail, int n_slots, int navail,
                                                    int k, u8 *work, int32_t *status, const GfTables *gft)
{
    __shared__ GfLds L;
    __shared__ u8 sid[256], sav[256], x[256], slot[256], M[2][260];
    __shared__ u8 q[64][256];  // one column's quotient per thread
    __shared__ int firstoff[256];  // first offer of each id
    gf_stage(L, gft);
    const u32 s = blockIdx.x;
    const int tid = threadIdx.x;
    u8 *wk = work + u64(s) * u64(k + k * k);
    for (int i = tid; i < n_slots; i += 64)
        sid[i] = ids[u64(s) * n_slots + i];
    for (int i = tid; i < navail; i += 64)
        sav[i] = avail[u64(s) * navail + i];
    for (int i = tid; i < 256; i += 64)
        firstoff[i] = 0x7FFFFFFF;
    __syncthreads();
    for (int c = tid; c < navail; c += 64)
        atomicMin(&firstoff[sid[sav[c]]], c);
    __syncthreads();
    // first k offered slots with distinct ids, in offer order
    // (crt/nk8.c:512-537): offer c is kept iff it is its id's first offer;
    // a ballot prefix places the kept ones
    int h = 0;
    for (int base = 0; base < navail && h < k; base += 64) {
        const int c = base + tid;
        bool keep = false;
        u8 id = 0, sl = 0;
        if (c < navail) {
            sl = sav[c];
            id = sid[sl];
            keep = firstoff[id] == c;
        }
        const u64 bal = __ballot(keep);
        const int pos = h + __popcll(bal & ((1ull << tid) - 1ull));
        if (keep && pos < k) {
            x[pos] = id;
            slot[pos] = sl;
        }
        h += __popcll(bal);
    }
    if (tid == 0 && status)
        status[s] = h < k ? -EINVAL : 0;
    if (h < k)
        return;  // wave-uniform
    // M(t) = prod_c (t + x_c), coefficients M[0..k]: k steps, lanes over
    // the coefficients (double-buffered)
    for (int i = tid; i <= k; i += 64) {
        M[0][i] = i == 0 ? 1 : 0;
        M[1][i] = 0;
    }
    __syncthreads();
    for (int c = 0; c < k; ++c) {
        const int cur = c & 1;
        for (int i = tid; i <= c + 1; i += 64)
            M[cur ^ 1][i] = (i ? M[cur][i - 1] : u8(0)) ^ gf_mul(L, x[c], M[cur][i]);
        __syncthreads();
    }
    const u8 *Mk = M[k & 1];
    for (int c = tid; c < k; c += 64) {
        wk[c] = slot[c];
        u8 *qc = q[tid];
        const u8 xc = x[c];
        // Q(t) = M(t) / (t + x_c), synthetic division from the top
        u8 qq = Mk[k];
        qc[k - 1] = qq;
        for (int i = k - 1; i >= 1; --i) {
            qq = Mk[i] ^ gf_mul(L, xc, qq);
            qc[i - 1] = qq;
        }
        // D = Q(x_c) = prod_{c' != c} (x_c + x_c'): a sum of k - 1
        // independent logs (the ids are distinct, so no factor is 0)
        u32 lsum = 0;
        for (int j = 0; j < k; ++j)
            lsum += j == c ? 0u : u32(L.log[xc ^ x[j]]);
        const u32 ld = lsum % 255u;
        // W[c][i] = q_i / D, eight at a time: loads before stores
        u8 *row = wk + k + c * k;
        for (int i0 = 0; i0 < k; i0 += 8) {
            u8 qv[8], ov[8];
#pragma unroll
            for (int t = 0; t < 8; ++t)
                qv[t] = i0 + t < k ? qc[i0 + t] : u8(0);
#pragma unroll
            for (int t = 0; t < 8; ++t)
                ov[t] = qv[t] ? L.exp[L.log[qv[t]] + 255u - ld] : u8(0);
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (i0 + t < k)
                    row[i0 + t] = ov[t];
        }
    }
}

// grid (nstripes, ceil(ps/256)); thread = row j:
//   block[j*k + m] = XOR_c part_c[j] * W[c][m]        (crt/nk8.c:552-582)
// only bytes below block_size are written (the tail row's padding is not).
__global__ __launch_bounds__(256) void k_decode_generic(nkfs_geom g, int n_slots, const u8 *work,
                                                        const int32_t *status, const GfTables *gft)
{
    __shared__ GfLds L;
    gf_stage(L, gft);
    const u32 s = blockIdx.x;
    if (status && status[s])
        return;
    const int k = g.k;
    const StripeView v = stripe_view(g, s);  // g.n = n_slots; blocks = the output
    const u8 *wk = work + u64(s) * u64(k + k * k);
    u8 *out = const_cast<u8 *>(v.blk);
    for (u32 j = blockIdx.y * blockDim.x + threadIdx.x; j < v.ps; j += gridDim.y * blockDim.x) {
        const u64 row = u64(j) * k;
        for (int m = 0; m < k; ++m) {
            if (row + m >= v.B)
                break;
            u8 acc = 0;
            for (int c = 0; c < k; ++c) {
                const u8 pv = v.parts[u64(wk[c]) * v.pitch + j];
                acc ^= gf_mul(L, pv, wk[k + c * k + m]);
            }
            out[row + m] = acc;
        }
    }
}

// Integrity check for the general decode path: XXH64 of the k parts the
// prep kernel selected, compared with their stored digests; a mismatch sets
// status -EIO and the slot's bit in badmask (bit 63 for slots >= 63).
__global__ __launch_bounds__(64) void k_verify_generic(nkfs_geom g, int n_slots, const u8 *work, int32_t *status,
                                                       const u64 *expect, u64 *badmask)
{
    const u32 s = blockIdx.x;
    const int k = g.k;
    if (status && status[s] == -EINVAL)
        return;
    const u8 *wk = work + u64(s) * u64(k + k * k);
    const StripeView v = stripe_view(g, s);
    const u32 ps = v.ps;
    const u32 nst = ps >> 5;
    if (threadIdx.x == 0 && badmask)
        badmask[s] = 0;
    __syncthreads();
    for (int c0 = 0; c0 < k; c0 += 16) {
        const int c = c0 + int(threadIdx.x >> 2), a = int(threadIdx.x & 3);
        const bool live = c < k;
        const u8 sl = live ? wk[c] : 0;
        const u8 *p = v.parts + u64(sl) * v.pitch;
        u64 acc = xxh_acc_init(a, 0);
        const u64 *w = reinterpret_cast<const u64 *>(p) + a;
        for (u32 r = 0; live && r < nst; ++r)
            acc = xxh_round(acc, w[4 * r]);
        const int b = int(threadIdx.x & 63) & ~3;
        const u64 v1 = shfl64(acc, b), v2 = shfl64(acc, b + 1);
        const u64 v3 = shfl64(acc, b + 2), v4 = shfl64(acc, b + 3);
        if (live && a == 0) {
            u64 h = ps >= 32 ? xxh_converge(v1, v2, v3, v4) : XP5;
            h += ps;
            if (xxh_tail(h, p + (u64(nst) << 5), ps & 31) != expect[u64(s) * n_slots + sl]) {
                if (badmask)
                    atomicOr(reinterpret_cast<unsigned long long *>(badmask + s), 1ull << (sl < 63 ? sl : 63));
                if (status)
                    status[s] = -EIO;
            }
        }
    }
}

// ------------------------------------------------- ragged batch order
//
// Ragged batches (mixed stripe sizes) are processed largest-first, with
// stripes of similar size side by side: the fused kernels run G stripes of a
// wave in lock step (a 1 MiB stripe next to a 4 KiB one idles half the wave
// for the whole stripe) and the longest stripes must not start last (the
// grid's tail).  One workgroup bucket-sorts the stripes by part size into
// perm (256 buckets: 8 per octave, largest first).  The order inside a
// bucket depends on atomics; it changes timing only, never an output.
constexpr u32 ORDER_MAXP = 60;  // stripes per thread of k_order_by_size (LDS bytes)

__device__ inline u32 size_bucket(u32 B, int k)
{
    const u32 ps = part_size_of(B, k);
    if (!ps)
        return 255;
    const u32 lz = 31u - u32(__builtin_clz(ps));
    const u32 top = lz >= 3 ? (ps >> (lz - 3)) & 7u : (ps << (3 - lz)) & 7u;
    return 255u - (lz * 8u + top);  // lz <= 28 for 32-bit sizes: no wrap
}

__global__ __launch_bounds__(1024) void k_order_by_size(const u32 *sizes, u32 count, int k, u32 *perm)
{
    // thread t takes positions t, t + 1024, ... (at most ORDER_MAXP: the
    // launcher caps count); the buckets are computed once, all loads
    // independent, into LDS bytes, then counted and placed with
    // wave-aggregated LDS atomics (one per distinct bucket in a wave: a few
    // size classes would otherwise serialise thousands of adds on one word)
    __shared__ u32 cnt[256];
    __shared__ u8 bks[ORDER_MAXP * 1024];
    const u32 t = threadIdx.x;
    if (t < 256)
        cnt[t] = 0;
    const u32 rounds = (count + 1023) / 1024;
#pragma unroll 4
    for (u32 j = 0; j < rounds; ++j) {
        const u32 i = t + 1024u * j;
        bks[i] = u8(i < count ? size_bucket(sizes[i < count ? i : 0], k) : 0u);
    }
    __syncthreads();
    const u64 lt = (1ull << (t & 63)) - 1ull;
    auto rank = [&](u32 bk, bool live) -> u32 {
        u64 todo = __ballot(live);
        u32 pos = 0;
        while (todo) {
            const int leader = __builtin_ctzll(todo);
            const u32 lb = __shfl(bk, leader, 64);
            const u64 same = __ballot(live && bk == lb);
            u32 base = 0;
            if (int(t & 63) == leader)
                base = atomicAdd(&cnt[lb], u32(__popcll(same)));
            base = __shfl(base, leader, 64);
            if (live && bk == lb)
                pos = base + u32(__popcll(same & lt));
            todo &= ~same;
        }
        return pos;
    };
#pragma unroll 1
    for (u32 j = 0; j < rounds; ++j) {
        const u32 i = t + 1024u * j;
        (void)rank(bks[i], i < count);
    }
    __syncthreads();
    if (t < 64) {  // exclusive prefix over the 256 counters: 4 per lane
        const u32 c0 = cnt[4 * t], c1 = cnt[4 * t + 1], c2 = cnt[4 * t + 2], c3 = cnt[4 * t + 3];
        u32 s = c0 + c1 + c2 + c3, x = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(x, d, 64);
            if (int(t) >= d)
                x += y;
        }
        x -= s;
        cnt[4 * t] = x;
        cnt[4 * t + 1] = x + c0;
        cnt[4 * t + 2] = x + c0 + c1;
        cnt[4 * t + 3] = x + c0 + c1 + c2;
    }
    __syncthreads();
#pragma unroll 1
    for (u32 j = 0; j < rounds; ++j) {
        const u32 i = t + 1024u * j;
        const u32 pos = rank(bks[i], i < count);
        if (i < count)
            perm[pos] = i;
    }
    if (t == 0)
        perm[count] = 0;  // the launcher's group counter for a persistent grid over the order
}

// ---------------------------------------------------------- synthetic
// word(seed, s, w) = mix64(seed + GAMMA*((s << 32) + w + 1)) -- synth.py.
__device__ inline u64 mix64(u64 z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_synth(u8 *blocks, u64 pitch, u32 B, u32 nstripes, u64 seed, u64 first)
{
    const u32 nw = (B + 7) / 8;
    const u64 total = u64(nw) * nstripes;
    for (u64 t = u64(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += u64(gridDim.x) * blockDim.x) {
        const u64 s = t / nw, w = t % nw;
        const u64 val = mix64(seed + 0x9E3779B97F4A7C15ull * (((first + s) << 32) + w + 1));
        u8 *dst = blocks + s * pitch + w * 8;
        if (w * 8 + 8 <= B) {
            if ((reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
                *reinterpret_cast<u64 *>(dst) = val;
                continue;
            }
        }
        for (u32 b = 0; b < 8 && w * 8 + b < B; ++b)
            dst[b] = u8(val >> (8 * b));
    }
}

// Ragged form: one workgroup per stripe s, d_block_size[s] bytes at
// d_block_off[s], stripe index first + s (the same bytes k_synth gives that
// stripe).
__global__ __launch_bounds__(256) void k_synth_ragged(u8 *blocks, const u64 *boff, const u32 *bsize, u64 seed,
                                                      u64 first)
{
    const u64 s = blockIdx.x;
    const u32 B = bsize[s];
    u8 *dst0 = blocks + boff[s];
    const u32 nw = (B + 7) / 8;
    for (u32 w = threadIdx.x; w < nw; w += blockDim.x) {
        const u64 val = mix64(seed + 0x9E3779B97F4A7C15ull * (((first + s) << 32) + w + 1));
        u8 *dst = dst0 + u64(w) * 8;
        if (w * 8 + 8 <= B && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
            *reinterpret_cast<u64 *>(dst) = val;
            continue;
        }
        for (u32 b = 0; b < 8 && w * 8 + b < B; ++b)
            dst[b] = u8(val >> (8 * b));
    }
}

// ----------------------------------------------------------- launchers

extern "C" int nkfs_fast_encode(const nkfs_geom *g, const u8 *ids, u64 *digests, int rules, int nib, hipStream_t st);
extern "C" int nkfs_ws_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, int ne, bool nt,
                              hipStream_t st);
extern "C" int nkfs_fast_xxh64_list(const u8 *base, const u64 *off, const u64 *len, u32 count, u64 seed, u64 *out,
                                    hipStream_t st);
extern "C" int nkfs_fast_xxh64_parts(const nkfs_geom *g, u64 *out, hipStream_t st);
extern "C" int nkfs_fast_decode(const nkfs_geom *g, int n_slots, const u8 *ids, const u8 *avail, int navail,
                                int32_t *status, const void *gf, hipStream_t st, const u64 *expect, u64 *badmask);

static int launch_ok(void)
{
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -EIO;
}

// grid.y of the general kernels: 256 rows per block, at most 65,535 blocks
// (the kernels grid-stride over the rest: parts beyond ~16 MiB)
static u32 row_blocks(u32 ps)
{
    const u32 b = (ps + 255) / 256;
    return b < 1 ? 1 : b > 65535 ? 65535 : b;
}

static u32 max_part_size(const nkfs_geom *g, u32 max_block)
{
    return part_size_of(g->block_sizes ? max_block : g->block_size, g->k);
}

extern "C" size_t nkfs_gf_tables_bytes(void) { return sizeof(GfTables); }

extern "C" uint64_t nkfs_run_work_bytes(uint32_t nstripes, int k);

// the larger of the plan layouts: k + k*k bytes per stripe (k_decode_plan,
// k_decode_prep) and the run decoder's padded plans + unit prefixes
extern "C" uint64_t nkfs_decode_work_bytes(uint32_t nstripes, int k)
{
    const u64 a = u64(nstripes) * u64(k + k * k), b = nkfs_run_work_bytes(nstripes, k);
    return a > b ? a : b;
}

extern "C" int nkfs_launch_gf_init(void *gf, void *stream)
{
    hipLaunchKernelGGL(k_gf_init, dim3(1), dim3(64), 0, (hipStream_t)stream, (GfTables *)gf);
    return launch_ok();
}

// ---------------------------------------------------------------- scratch
//
// A launch's own metadata (the ragged size order, the ragged slice map)
// lives in the caller's scratch when nkfs_geom.scratch provides it (the host
// pipeline carves it from its context buffer), else in stream-ordered
// allocations from a private per-device pool.  The private pool allows
// reuse only along stream-ordered dependencies: opportunistic and
// driver-inserted cross-stream reuse are off, so a block freed on one stream
// never goes to another stream's allocation before the freeing work is
// ordered before it (the default pool allows both; round-3 fault audit,
// DESIGN.md §5.6).  Allocation stays stream-ordered, so calls remain
// graph-capturable.
static std::mutex g_pool_mu;
static hipMemPool_t g_pool[NKFS_MAX_DEVICES];

extern "C" hipMemPool_t nkfs_private_pool(hipStream_t st)
{
    int dev = -1;
    if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= NKFS_MAX_DEVICES)
        return nullptr;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (g_pool[dev])
        return g_pool[dev];
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t p = nullptr;
    if (hipMemPoolCreate(&p, &props) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    int off = 0, on = 1;
    uint64_t keep = 64ull << 20;  // keep up to 64 MiB cached across syncs
    if (hipMemPoolSetAttribute(p, hipMemPoolReuseAllowOpportunistic, &off) != hipSuccess ||
        hipMemPoolSetAttribute(p, hipMemPoolReuseAllowInternalDependencies, &off) != hipSuccess ||
        hipMemPoolSetAttribute(p, hipMemPoolReuseFollowEventDependencies, &on) != hipSuccess ||
        hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipMemPoolDestroy(p);
        return nullptr;
    }
    g_pool[dev] = p;
    return p;
}

extern "C" uint64_t nkfs_ragged_scratch_bytes(uint32_t nstripes, uint64_t sum_units)
{
    const u64 perm = ((u64(nstripes) + 1) * 4 + 255) & ~u64(255);  // + the persistent launches' group counter
    const u64 head = ((u64(nstripes) + 2) * 4 + 15) & ~u64(15);
    return perm + ((head + sum_units * 8 + 255) & ~u64(255));
}

// ragged batches pass the bound on block sizes in g->block_size
// Fast-path launch of a ragged batch in size order (k_order_by_size); the
// permutation lives in the launch's scratch (above), so the call stays
// capturable.  Returns -ENOSYS when the batch is uniform or ordering is
// switched off.
template <class F>
static int with_size_order(const nkfs_geom *g, hipStream_t st, F launch)
{
    if (!g->block_sizes || g->order || !nkfs_tune_now().size_order || g->nstripes > ORDER_MAXP * 1024u)
        return -ENOSYS;  // (k_order_by_size: ORDER_MAXP stripes per thread)
    Scratch sc;
    // the permutation, then one zeroed word: the group counter of a
    // persistent launch over the order (nk8_wsp.hip)
    u32 *perm = static_cast<u32 *>(sc.take(g, (u64(g->nstripes) + 1) * sizeof(u32), st));
    if (!perm)
        return -ENOSYS;
    hipLaunchKernelGGL(k_order_by_size, dim3(1), dim3(1024), 0, st, g->block_sizes, g->nstripes, g->k, perm);
    int rc = launch_ok();
    nkfs_geom g2 = *g;
    g2.order = perm;
    g2.queue = perm + g->nstripes;
    sc.rest(&g2);
    if (!rc)
        rc = launch(&g2);
    const int e = sc.finish();
    return rc ? rc : e;
}

extern "C" int nkfs_walk_encode(const nkfs_geom *g, const u8 *ids, u64 *digests, int units, int nib, int waves,
                                int cus, hipStream_t st);
extern "C" int nkfs_wsp_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, bool nt, hipStream_t st);
extern "C" int nkfs_wide_encode(const nkfs_geom *g, const uint8_t *ids, int cus, hipStream_t st);
extern "C" int nkfs_wide_ws_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, hipStream_t st);
extern "C" int nkfs_big_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, const void *gf,
                               hipStream_t st);
extern "C" int nkfs_big_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, hipStream_t st);
extern "C" int nkfs_bign_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, int mode,
                                hipStream_t st);
extern "C" int nkfs_bign_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, bool persist,
                                bool diag, hipStream_t st);
extern "C" int nkfs_wide_decode(const nkfs_geom *g, const uint8_t *work, const int32_t *status, int cus,
                                hipStream_t st);
extern "C" int nkfs_slice_decode(const nkfs_geom *g, int n_slots, const u8 *ids, const u8 *avail, int navail,
                                 void *work, int32_t *status, const void *gf, int units, int waves, int cus,
                                 hipStream_t st);
extern "C" int nkfs_pair_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                                int navail, int32_t *status, const void *gf, int xp, int waves, int pipe,
                                hipStream_t st);
extern "C" int nkfs_run_decode(const nkfs_geom *g, int n_slots, const u8 *ids, const u8 *avail, int navail,
                               void *work, int32_t *status, const void *gf, int units, int waves, int cus,
                               hipStream_t st);

// Fast-path encoder choice (n <= 8, k <= 8), struct nkfs_tune.enc_kernel:
// AUTO = the walk encoder for ragged batches (one wave per stripe in size
// order; the fused kernel would pair unequal stripes in one wave) and for
// mid-size uniform N8 shapes (walk_by_rule), else the fused /
// warp-specialised shape rules (the walk encoder is slower on N4K2 4 KiB,
// where one stripe is one chunk).
static int walk_by_rule(const nkfs_geom *g, const u64 *digests)
{
    // uniform n > 4 batches: the walk encoder, except parts of 64 KiB and up,
    // parts of 32 KiB and up on at most 1,024 stripes and parts of 8 KiB and
    // up on at most 256 stripes, which take the warp-specialised kernel
    // (nkfs_fast_encode).  Round-3 seam sweep, N8K5 (profiles/r03/
    // seam_sweep_box{1,2}.txt): 1,024 x 64 KiB walk 3,502 / fused 2,211 / ws
    // 3,045 GB/s; 65,536 x 4 KiB walk 3,027 / fused 2,669; 2,048 x 256 KiB
    // walk 4,373 / ws 4,263; 256 x 64 KiB ws 1,552 / walk 1,111; 16,384 x
    // 512 KiB ws 4,964 / walk 4,881.
    // Round 4: with two hash waves per workgroup (>= 1,024 stripes) the
    // warp-specialised kernel also wins from 48 KiB parts: 16,384 x 256 KiB
    // ws2 4,960 / walk 4,901, 2,048 x 256 KiB 4,650 / 4,549; 131,072-byte
    // blocks (26 KiB parts) stay on the walk encoder, 4,764 / 4,875
    // (profiles/r04/seam_ws2.txt).
    // Round 4 (seam_mid.txt, seam_sweep_r04_boxA.txt): up to 1,024 stripes
    // the warp-specialised grid fits one round of workgroups and wins from
    // 4 KiB parts (N8K5 512 x 128 KiB 3,713 / walk 2,388, 1,024 x 64 KiB
    // 4,329 / 3,781, 256 x 20 KiB 1,028 / 763; 1 KiB parts stay on the walk,
    // 767 / 921).
    if (g->block_sizes || !digests || g->n <= 4)
        return 0;
    const u32 ps = (g->block_size + u32(g->k) - 1) / u32(g->k);
    const int hwt = nkfs_tune_now().enc_ws_hash_waves;
    const bool ws2 = hwt == 2 || (!hwt && nkfs_ws_auto_hash_waves(g->nstripes) == 2);
    const bool ws = ps >= 65536 || (ps >= 4096 && g->nstripes <= 1024) || (ws2 && ps >= 49152);
    return !ws;
}

static int fast_encode(const nkfs_geom *g, const u8 *ids, u64 *digests, hipStream_t st)
{
    const nkfs_tune t = nkfs_tune_now();
    int kern = t.enc_kernel != NKFS_ENC_AUTO ? t.enc_kernel
               : g->block_sizes || walk_by_rule(g, digests) ? NKFS_ENC_WALK
                                                            : NKFS_ENC_AUTO;
    // enc_persist: n > 4 batches with digests take the persistent
    // warp-specialised encoder where the choice above is the walk encoder on
    // a ragged batch (1, the default: C5 4,839 -> 5,051 GB/s) or also the
    // warp-specialised grid on a uniform one (2: C3 5,109 -> 5,064, C4 5,148
    // -> 5,144; profiles/r05/ab_wsp.txt)
    if (t.enc_kernel == NKFS_ENC_AUTO && t.enc_persist && digests && g->n > 4 &&
        (g->block_sizes ? kern == NKFS_ENC_WALK : t.enc_persist == 2 && kern == NKFS_ENC_AUTO))
        kern = NKFS_ENC_WSP;
    if (kern == NKFS_ENC_WSP) {
        const int rc = nkfs_wsp_encode(g, ids, digests, false, st);
        if (rc != -ENOSYS)
            return rc;
        kern = g->block_sizes ? NKFS_ENC_WALK : NKFS_ENC_AUTO;
    }
    if (kern == NKFS_ENC_WALK && g->block_sizes && digests && g->n > 4 && t.enc_ragged_split &&
        !g->part_min && !g->part_max) {
        // ragged n > 4: stripes with parts of at least enc_ragged_split bytes
        // on the warp-specialised kernel (C3's), the rest on the walk
        // encoder; two launches over the same size order with complementary
        // part-size windows (nkfs_geom.part_min / part_max)
        nkfs_geom big = *g, small = *g;
        big.part_min = u32(t.enc_ragged_split);
        small.part_max = u32(t.enc_ragged_split);
        int rc = nkfs_ws_encode(&big, ids, digests, 4, false, st);
        if (!rc)
            rc = nkfs_walk_encode(&small, ids, digests, 1, t.enc_nib < 0 ? 0 : t.enc_nib, t.enc_waves_per_cu,
                                  nkfs_cu_count(), st);
        if (rc != -ENOSYS)
            return rc;
    }
    if (kern == NKFS_ENC_WALK) {
        // two 1,024-row units per chunk for n <= 4 (a 4 KiB N4K2 stripe is one chunk)
        const int units = g->n <= 4 ? (t.enc_units ? t.enc_units : 2) : 1;
        const int nib = t.enc_nib < 0 ? 0 : t.enc_nib;
        const int rc = nkfs_walk_encode(g, ids, digests, units, nib, t.enc_waves_per_cu, nkfs_cu_count(), st);
        if (rc != -ENOSYS)
            return rc;
    }
    if (kern == NKFS_ENC_WS && digests)
        return nkfs_ws_encode(g, ids, digests, 4, false, st);
    return nkfs_fast_encode(g, ids, digests, kern == NKFS_ENC_AUTO, t.enc_nib, st);
}

// A handful of big stripes (the drop-in nk8_split_block: one block per
// call) would leave the fast kernels' one wave per stripe alone on the chip;
// the general kernel spreads every stripe's rows over the whole GPU (1 MiB
// N8K5 split: 855 -> see DESIGN.md §5, per-call table).
static bool few_big_stripes(const nkfs_geom *g)
{
    const u32 ps = max_part_size(g, g->block_size);
    const nkfs_tune t = nkfs_tune_now();
    return !g->block_sizes && t.enc_kernel == NKFS_ENC_AUTO && u64(g->nstripes) * ps < (u64(16) << 20) &&
           g->nstripes <= u32(t.enc_few_max) && ps >= 1024;
}

extern "C" int nkfs_launch_encode(const nkfs_geom *g, const uint8_t *ids, uint64_t *digests, const void *gf,
                                  void *stream)
{
    if (!g->nstripes)
        return 0;
    hipStream_t st = (hipStream_t)stream;
    int rc = -ENOSYS;
    const int kern = nkfs_tune_now().enc_kernel;
    if (g->n <= 8 && g->k <= 8 && kern != NKFS_ENC_GENERIC && kern != NKFS_ENC_WIDE && kern != NKFS_ENC_BIG &&
        kern != NKFS_ENC_WIDE_WS && !few_big_stripes(g)) {
        rc = with_size_order(g, st, [&](const nkfs_geom *go) { return fast_encode(go, ids, digests, st); });
        if (rc == -ENOSYS)
            rc = fast_encode(g, ids, digests, st);
    }
    if (rc != -ENOSYS)
        return rc;
    // 16 < k <= 32 with digests: the stage-free encoder with a hash wave
    // (nk8_bign.hip; tune enc_bign).  Its units of 8 parts (32 < k <= 76,
    // pinned with enc_bign 1) lose to the column-chunked encoder + hash
    // pass: W3 723 / 887, N40K33 762 / 977 GB/s (profiles/r06/ab_bign8_enc.txt)
    const int eb = nkfs_tune_now().enc_bign;
    if (kern != NKFS_ENC_GENERIC &&
        (eb > 0 || (eb == -1 && digests && g->k > 16 && g->k <= 32 && kern == NKFS_ENC_AUTO))) {
        // diagonal tables for k = 32, or every k with enc_bign 3
        rc = nkfs_bign_encode(g, ids, digests, eb != 2, eb == 3, st);
        if (rc != -ENOSYS)
            return rc;
    }
    // n > 8 (or a few big stripes), k <= 16: with digests and a batch that
    // fills the chip (two workgroups of 16 parts per CU), the part-group
    // encoder with XXH64 fused (nk8_wide.hip, k_encode_wide_ws)
    if (digests && g->k <= 16 &&
        (kern == NKFS_ENC_WIDE_WS ||
         (kern == NKFS_ENC_AUTO && u64(g->nstripes) * u64((g->n + 15) / 16) >= 2u * u64(nkfs_cu_count())))) {
        rc = nkfs_wide_ws_encode(g, ids, digests, st);
        if (rc != -ENOSYS)
            return rc;
    }
    // else part groups of 8 for k <= 16 (then the batched XXH64 of the
    // parts), 16-column chunks beyond (nk8_big.hip): XXH64 fused with
    // nkfs_tune.enc_big_fused (HBM traffic 1.0x instead of 1.6x, but the
    // chains' serial rounds in the store phase cost W2 ~6 %,
    // profiles/r04/ab_w2_fused_*.txt), else a second pass (default)
    if (kern != NKFS_ENC_GENERIC) {
        rc = kern == NKFS_ENC_BIG ? -ENOSYS : nkfs_wide_encode(g, ids, nkfs_cu_count(), st);
        if (rc != -ENOSYS)
            return rc || !digests ? rc : nkfs_launch_hash_parts(g, digests, stream);
        // -1 auto: the XXH64 pass (round 6, with the diagonal tables the
        // slices' serial chain hand-off became the fused form's bound: W3
        // 941 -> 1,039, N40K33 968 -> 1,078, N80K70 796 -> 866 GB/s,
        // profiles/r06/ab_w3_enc.txt; it had won 880 -> 914 on W3 before)
        const int fz = nkfs_tune_now().enc_big_fused;
        rc = digests && fz > 0 ? nkfs_big_encode(g, ids, digests, gf, st) : -ENOSYS;
        if (rc != -ENOSYS)
            return rc;
        rc = nkfs_big_encode(g, ids, nullptr, gf, st);
        if (rc != -ENOSYS)
            return rc || !digests ? rc : nkfs_launch_hash_parts(g, digests, stream);
    }
    const u32 ps = max_part_size(g, g->block_size);
    dim3 grid(g->nstripes, row_blocks(ps));
    hipLaunchKernelGGL(k_encode_generic, grid, dim3(256), 0, st, *g, ids, (const GfTables *)gf);
    if ((rc = launch_ok()))
        return rc;
    if (digests)
        return nkfs_launch_hash_parts(g, digests, stream);
    return 0;
}

extern "C" int nkfs_launch_hash_parts(const nkfs_geom *g, uint64_t *digests, void *stream)
{
    if (nkfs_tune_now().enc_kernel != NKFS_ENC_GENERIC)
        return nkfs_fast_xxh64_parts(g, digests, (hipStream_t)stream);
    const u64 threads = u64(g->nstripes) * u64(g->n) * 4;
    if (!threads)
        return 0;
    hipLaunchKernelGGL(k_hash_parts, dim3(u32((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *g,
                       digests);
    return launch_ok();
}

extern "C" int nkfs_launch_decode(const nkfs_geom *g, int n_slots, const uint8_t *ids, const uint8_t *avail,
                                  int navail, void *work, int32_t *status, const void *gf, void *stream,
                                  const uint64_t *expect, uint64_t *badmask)
{
    if (!g->nstripes)
        return 0;
    hipStream_t st = (hipStream_t)stream;
    const nkfs_tune t = nkfs_tune_now();
    int rc = -ENOSYS;
    if (g->k <= 8 && t.dec_kernel != NKFS_DEC_GENERIC && t.dec_kernel != NKFS_DEC_WIDE && t.dec_kernel != NKFS_DEC_BIG) {
        // uniform batches without the integrity check: one-shot slice waves;
        // ragged batches and the verifying form: the wave-per-stripe decoder
        // default: one-shot slices for k >= 3 (C3/C4 decode +10-15 %); for
        // k = 2 a 4 KiB stripe is one wave either way and the wave decoder's
        // in-wave inverse saves the plan launch
        // ragged batches with k >= 3: the run decoder (no per-slice metadata
        // chain, no setup scan; C5 decode +6 % over the ragged slice grid)
        // k = 2: the wave decoder's in-wave inverse saves the plan launch on
        // small stripes; from 64 KiB parts the slice grid wins (N4K2 65,536 x
        // 256 KiB slice 5,636 / wave 5,314 GB/s, 1,024 x 256 KiB 4,962 /
        // 4,551; 1,024 x 64 KiB wave 5,412 / slice 4,584; C2's 4 KiB: 5,236
        // / 4,796; profiles/r03/seam_sweep_box{2,3}.txt)
        const bool small_k2 = g->k < 3 && (g->block_sizes || part_size_of(g->block_size, g->k) < 65536);
        // ragged: the run decoder on batches that give its persistent grid
        // several chunks per wave; the host pipeline's sub-batches (tens of
        // stripes) keep the slice grid (C5 GET from host memory: run 20.7,
        // slice 31.6 GiB/s; profiles/r03/pcie.txt)
        // dec_pair_pipe > 0: uniform k = 2 batches of blocks up to 4 KiB on
        // the persistent pipelined pair decoder
        const bool pipe2 = g->k == 2 && !g->block_sizes && g->block_size <= 4096 && t.dec_pair_pipe > 0;
        const int kern = t.dec_kernel != NKFS_DEC_AUTO         ? t.dec_kernel
                         : pipe2 && !expect                    ? NKFS_DEC_PAIR
                         : small_k2                            ? NKFS_DEC_WAVE
                         : g->block_sizes && g->nstripes >= 2048 ? NKFS_DEC_RUN
                                                                 : NKFS_DEC_SLICE;
        if (kern == NKFS_DEC_PAIR && !expect) {
            auto pair = [&](const nkfs_geom *go) {
                return nkfs_pair_decode(go, n_slots, ids, avail, navail, status, gf, t.dec_pair_stage,
                                        t.dec_pair_waves, t.dec_pair_pipe, st);
            };
            rc = with_size_order(g, st, pair);
            if (rc == -ENOSYS)
                rc = pair(g);
        }
        if (kern == NKFS_DEC_RUN && !expect)
            rc = nkfs_run_decode(g, n_slots, ids, avail, navail, work, status, gf, t.dec_run_units, t.dec_waves_per_cu,
                                 nkfs_cu_count(), st);
        if (kern == NKFS_DEC_SLICE && !expect) {
            // ragged: in size order (largest first), so the grid's tail is short slices
            auto slice = [&](const nkfs_geom *go) {
                return nkfs_slice_decode(go, n_slots, ids, avail, navail, work, status, gf, t.dec_units,
                                         t.dec_waves_per_cu, nkfs_cu_count(), st);
            };
            rc = with_size_order(g, st, slice);
            if (rc == -ENOSYS)
                rc = slice(g);
        }
        if (rc == -ENOSYS)
            rc = with_size_order(g, st, [&](const nkfs_geom *go) {
                return nkfs_fast_decode(go, n_slots, ids, avail, navail, status, gf, st, expect, badmask);
            });
        if (rc == -ENOSYS)
            rc = nkfs_fast_decode(g, n_slots, ids, avail, navail, status, gf, st, expect, badmask);
    }
    if (rc != -ENOSYS)
        return rc;
    hipLaunchKernelGGL(k_decode_prep, dim3(g->nstripes), dim3(64), 0, st, ids, avail, n_slots, navail, g->k,
                       (u8 *)work, status, (const GfTables *)gf);
    rc = launch_ok();
    if (rc)
        return rc;
    // k <= 16: survivor tables of 16-byte products (nk8_wide.hip); beyond:
    // 16-column chunks (nk8_big.hip); pinned GENERIC: thread per row
    // the stage-free decoder (nk8_bign.hip): dec_bign >= 0 pins a table
    // layout for every k > 8; -2 (auto, the default) takes byte tables where
    // they win: k % 4 == 0 except 16 -- W2 N48K32 1,315 -> 2,082 GB/s,
    // N24K20 926 -> 1,211, W1 N16K12 3,330 -> 4,296; k = 16 (4,087 / 3,952)
    // keeps the survivor-table decoder (profiles/r05/ab_bign.txt), and k with
    // rows not a dword multiple keep the column-chunked one, whose output goes
    // through an LDS stage (the stage-free one writes such rows bytewise:
    // N40K17 696 / 413, N40K18 736 / 598, N40K33 524 / 523;
    // profiles/r05/ab_oddk.txt)
    // round 6: rows that are not a dword multiple (16 < k <= 64) take the
    // all-groups stage-free decoder, whose output goes through an LDS stage
    // (dec_bign 3, k_decode_bigr): N40K17 696 -> 1,700, N40K33 524 -> 1,095,
    // W3 N64K41 491 -> 875 GB/s (profiles/r06/ab_bigr_*.txt); k % 4 == 0 keeps
    // the byte-table form (W2 2,064 vs 1,341).  The automatic choice applies
    // to NKFS_DEC_AUTO only: a pinned NKFS_DEC_BIG runs the column-chunked
    // decoder unless dec_bign pins a stage-free layout.
    // Round 6 (later): the byte tables in the diagonal layout (dec_bign 4:
    // conflict-free lookups) replace layout 0 in the automatic choice -- W2
    // 2,068 -> 2,680 GB/s, N24K20 1,116 -> 1,180, N32K28 608 -> 639, W1
    // 4,292 -> 4,301 (profiles/r06/ab_diag_dec.txt); the all-groups decoder
    // with diagonal tables (dec_bign 5) replaces layout 3 -- W3 985 -> 1,489,
    // N40K33 1,242 -> 1,636, N24K18 1,688 -> 1,895, N40K17 1,637 -> 1,784
    // (profiles/r06/ab_bigr_diag.txt)
    rc = -ENOSYS;
    if (t.dec_kernel == NKFS_DEC_AUTO || t.dec_kernel == NKFS_DEC_BIG) {
        int mode = t.dec_bign;
        if (mode == -2 && t.dec_kernel == NKFS_DEC_AUTO)
            mode = g->k % 4 == 0 && g->k != 16 ? 4 : g->k > 16 && g->k <= 64 ? 5 : -1;
        if (mode >= 0)
            rc = nkfs_bign_decode(g, (const u8 *)work, status, mode, st);
    }
    if (rc == -ENOSYS)
        rc = t.dec_kernel == NKFS_DEC_GENERIC || t.dec_kernel == NKFS_DEC_BIG
                 ? -ENOSYS
                 : nkfs_wide_decode(g, (const u8 *)work, status, nkfs_cu_count(), st);
    if (rc == -ENOSYS && t.dec_kernel != NKFS_DEC_GENERIC)
        rc = nkfs_big_decode(g, (const u8 *)work, status, st);
    if (rc == -ENOSYS) {
        const u32 ps = part_size_of(g->block_size, g->k);
        dim3 grid(g->nstripes, row_blocks(ps));
        hipLaunchKernelGGL(k_decode_generic, grid, dim3(256), 0, st, *g, n_slots, (const u8 *)work,
                           (const int32_t *)status, (const GfTables *)gf);
        rc = launch_ok();
    }
    if (rc || !expect)
        return rc;
    hipLaunchKernelGGL(k_verify_generic, dim3(g->nstripes), dim3(64), 0, st, *g, n_slots, (const u8 *)work, status,
                       expect, badmask);
    return launch_ok();
}

extern "C" int nkfs_launch_xxh64_batch(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                                       uint32_t count, uint64_t seed, uint64_t *out, void *stream)
{
    if (!count)
        return 0;
    if (nkfs_tune_now().enc_kernel != NKFS_ENC_GENERIC)
        return nkfs_fast_xxh64_list(base, off, len, count, seed, out, (hipStream_t)stream);
    const u64 threads = u64(count) * 4;
    hipLaunchKernelGGL(k_xxh64_batch, dim3(u32((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, base,
                       off, len, count, seed, out);
    return launch_ok();
}

extern "C" int nkfs_launch_synth(uint8_t *blocks, uint64_t pitch, uint32_t B, uint32_t nstripes, uint64_t seed,
                                 uint64_t first, void *stream)
{
    if (!nstripes || !B)
        return 0;
    const u64 total = u64((B + 7) / 8) * nstripes;
    const u32 grid = u32(total / 256 + 1 < 8192 ? total / 256 + 1 : 8192);
    hipLaunchKernelGGL(k_synth, dim3(grid), dim3(256), 0, (hipStream_t)stream, blocks, pitch, B, nstripes, seed,
                       first);
    return launch_ok();
}

extern "C" int nkfs_launch_synth_ragged(uint8_t *blocks, const uint64_t *boff, const uint32_t *bsize,
                                        uint32_t nstripes, uint64_t seed, uint64_t first, void *stream)
{
    if (!nstripes)
        return 0;
    hipLaunchKernelGGL(k_synth_ragged, dim3(nstripes), dim3(256), 0, (hipStream_t)stream, blocks, boff, bsize, seed,
                       first);
    return launch_ok();
}
