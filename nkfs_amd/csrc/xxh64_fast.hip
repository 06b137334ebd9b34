// xxh64_fast.hip -- batched XXH64 (seeded, crt/xxhash.c:358-496) over many
// independent messages at HBM speed: the csum of every part of a batch, or
// of every 64 KiB block of the core's integrity path (core/dio.c:26-37,
// core/inode.c:147-155), in one launch.
//
// One wave = 16 messages.  XXH64 of one message is serial with exactly four
// independent accumulators, so lane 4m+a owns accumulator a of message m
// for the whole message.  The wave streams CH = 512 bytes of each message
// per iteration: all 64 lanes load cooperatively (8 x 16 B per lane, two
// messages per wave-instruction, fully coalesced), the chunk goes through
// LDS, and each hash lane then runs its 4 rounds per 128 bytes from
// registers.  Two chunks of loads stay in flight behind the rounds.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nkfs_internal.h"
#include "xxh64_dev.h"

using namespace nkfs;
typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

namespace {

constexpr int MSGS = 16;               // messages per wave
constexpr int CH = 512;                // bytes per message per iteration
constexpr int PIECES = MSGS * CH / 16; // 16-byte pieces per iteration
constexpr int PPL = PIECES / 64;       // pieces per lane (8)
constexpr int SPAD = CH + 32;          // LDS bytes per message (bank spread)

// A message source maps message m to (descriptor, length) and a byte
// offset inside the message to its address.  Every source guarantees that
// an aligned 16-byte piece never straddles a discontinuity.
struct MsgList {  // explicit (offset, length) list
    typedef const u8 *Desc;
    const u8 *base;
    const u64 *off;
    const u64 *len;
    u32 count;
    __device__ bool get(u32 m, Desc &d, u64 &n) const
    {
        if (m >= count)
            return false;
        d = base + off[m];
        n = len[m];
        return true;
    }
    __device__ static const u8 *at(Desc d, u64 pos) { return d + pos; }
};

struct Strided {  // count messages of len bytes, pitch apart (clusters)
    typedef const u8 *Desc;
    const u8 *base;
    u64 pitch;
    u64 len;
    u32 count;
    __device__ bool get(u32 m, Desc &d, u64 &n) const
    {
        if (m >= count)
            return false;
        d = base + u64(m) * pitch;
        n = len;
        return true;
    }
    __device__ static const u8 *at(Desc d, u64 pos) { return d + pos; }
};

struct PageList {  // message m = first len[m] bytes of pages[first[m]..]
    struct Desc {
        const u8 *const *pg;
        u32 shift;
    };
    const u8 *const *pages;
    const u64 *first;
    const u64 *len;
    u32 count;
    u32 shift;  // log2(page size), >= log2(CH)
    __device__ bool get(u32 m, Desc &d, u64 &n) const
    {
        d.shift = shift;
        if (m >= count) {
            d.pg = nullptr;
            return false;
        }
        d.pg = pages + first[m];
        n = len[m];
        return true;
    }
    __device__ static const u8 *at(Desc d, u64 pos)
    {
        return d.pg[pos >> d.shift] + (pos & ((u64(1) << d.shift) - 1));
    }
};

struct PartsOf {  // every part of a batch laid out by nkfs_geom
    typedef const u8 *Desc;
    nkfs_geom g;
    __device__ bool get(u32 m, Desc &p, u64 &n) const
    {
        const u64 total = u64(g.nstripes) * u64(g.n);
        if (m >= total)
            return false;
        const u32 s = u32(m / u32(g.n)), i = u32(m % u32(g.n));
        const u32 B = g.block_sizes ? g.block_sizes[s] : g.block_size;
        const u32 ps = B / u32(g.k) + ((B % u32(g.k)) ? 1u : 0u);
        u64 pitch;
        const u8 *base;
        if (g.block_sizes) {
            pitch = (u64(ps) + NKFS_PART_ALIGN - 1) & ~u64(NKFS_PART_ALIGN - 1);
            base = g.parts + g.part_off[s];
        } else {
            pitch = g.part_pitch;
            base = g.parts + u64(s) * u64(g.n) * g.part_pitch;
        }
        p = base + u64(i) * pitch;
        n = ps;
        return true;
    }
    __device__ static const u8 *at(Desc d, u64 pos) { return d + pos; }
};

__device__ inline u64 shfl64(u64 v, int src)
{
    u32 lo = __shfl(u32(v), src, 64);
    u32 hi = __shfl(u32(v >> 32), src, 64);
    return (u64(hi) << 32) | lo;
}

}  // namespace

// expect != NULL: status[m] = 0 when out[m] == expect[m], else -EINVAL
// (the compare of nkfs_inode_block_check_sum, core/inode.c:561-575).
template <class Src>
__global__ __launch_bounds__(64) void k_xxh64_fast(Src src, u64 seed, u64 *out, const u64 *expect,
                                                   int32_t *status)
{
    __shared__ __attribute__((aligned(16))) u8 buf[MSGS * SPAD];
    const int lane = threadIdx.x;
    const u32 m0 = blockIdx.x * MSGS;

    // loader role: piece q of lane = message (lane + 64q) / 32, 16-B piece
    // (lane + 64q) % 32 of that message's chunk
    typename Src::Desc lp[PPL];
    u64 llen[PPL];
    int lmsg[PPL], lpos[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
        const int pc = lane + 64 * q;
        lmsg[q] = pc / (CH / 16);
        lpos[q] = (pc % (CH / 16)) * 16;
        u64 n = 0;
        src.get(m0 + lmsg[q], lp[q], n);
        llen[q] = n;
    }
    // hash role: message hm, accumulator ha
    const int hm = lane >> 2, ha = lane & 3;
    typename Src::Desc hp;
    u64 hlen = 0;
    const bool hlive = src.get(m0 + hm, hp, hlen);
    const u64 nst = hlen >> 5;
    const u32 nchunks = u32((hlen + CH - 1) / CH);
    u64 acc = xxh_acc_init(ha, seed);

    auto load = [&](uint4 (&d)[PPL], u32 c) {
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const u64 pos = u64(c) * CH + lpos[q];
            // at() may read a page table: only for bytes inside the message
            if (pos + 16 <= llen[q]) {
                const u8 *a = Src::at(lp[q], pos);
                if ((reinterpret_cast<uintptr_t>(a) & 15) == 0) {
                    d[q] = *reinterpret_cast<const uint4 *>(a);
                } else {  // 8-byte aligned (API contract)
                    const u64 *w = reinterpret_cast<const u64 *>(a);
                    const u64 lo = w[0], hi = w[1];
                    d[q] = make_uint4(u32(lo), u32(lo >> 32), u32(hi), u32(hi >> 32));
                }
            } else if (pos < llen[q]) {
                const u8 *a = Src::at(lp[q], pos);
                u32 x[4] = {0, 0, 0, 0};
                for (u32 b = 0; b < 16 && pos + b < llen[q]; ++b)
                    x[b >> 2] |= u32(a[b]) << (8 * (b & 3));
                d[q] = make_uint4(x[0], x[1], x[2], x[3]);
            }
        }
    };
    auto stage = [&](const uint4 (&d)[PPL], u32 c) {
#pragma unroll
        for (int q = 0; q < PPL; ++q)
            if (u64(c) * CH + lpos[q] < llen[q])
                *reinterpret_cast<uint4 *>(buf + lmsg[q] * SPAD + lpos[q]) = d[q];
    };

    // any message left in this wave?
    u32 wchunks = nchunks;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        wchunks = max(wchunks, u32(__shfl_xor(int(wchunks), o, 64)));

    uint4 d0[PPL], d1[PPL];
    if (wchunks > 0)
        load(d0, 0);
    if (wchunks > 1)
        load(d1, 1);
    auto step = [&](uint4 (&d)[PPL], u32 c) {
        stage(d, c);
        __syncthreads();
        u64 hw[CH / 32];
#pragma unroll
        for (int r = 0; r < CH / 32; ++r)
            hw[r] = *reinterpret_cast<const u64 *>(buf + hm * SPAD + 32 * r + 8 * ha);
        __syncthreads();
        if (c + 2 < wchunks)
            load(d, c + 2);  // refill this ring slot behind the rounds
        if (hlive && c < nchunks) {
            const u64 first = u64(c) * (CH / 32);
#pragma unroll
            for (int r = 0; r < CH / 32; ++r) {
                const u64 nxt = xxh_round(acc, hw[r]);
                acc = first + r < nst ? nxt : acc;
            }
        }
    };
    for (u32 c = 0; c < wchunks; c += 2) {
        step(d0, c);
        if (c + 1 < wchunks)
            step(d1, c + 1);
    }

    const int base = lane & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    if (hlive && ha == 0) {
        u64 h = hlen >= 32 ? xxh_converge(v1, v2, v3, v4) : seed + XP5;
        h += hlen;
        u64 tw[4] = {0, 0, 0, 0};
        const u32 left = u32(hlen & 31);
        if (left) {
            // the tail is in this message's LDS slot from its last chunk
            const u32 toff = u32(nst * 32 - u64(nchunks - 1) * CH);
            const u64 *t = reinterpret_cast<const u64 *>(buf + hm * SPAD + toff);
#pragma unroll
            for (int w = 0; w < 4; ++w)
                tw[w] = t[w];
        }
        const u64 dig = xxh_tail_regs(h, tw, left);
        out[m0 + hm] = dig;
        if (expect)
            status[m0 + hm] = dig == expect[m0 + hm] ? 0 : -EINVAL;
    }
}

extern "C" int nkfs_fast_xxh64_list(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint32_t count,
                                    uint64_t seed, uint64_t *out, hipStream_t st)
{
    if (!count)
        return 0;
    MsgList src{base, off, len, count};
    hipLaunchKernelGGL(k_xxh64_fast<MsgList>, dim3((count + MSGS - 1) / MSGS), dim3(64), 0, st, src, seed, out,
                       (const u64 *)nullptr, (int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_fast_xxh64_parts(const nkfs_geom *g, uint64_t *out, hipStream_t st)
{
    const u64 total = u64(g->nstripes) * u64(g->n);
    if (!total)
        return 0;
    PartsOf src{*g};
    hipLaunchKernelGGL(k_xxh64_fast<PartsOf>, dim3(u32((total + MSGS - 1) / MSGS)), dim3(64), 0, st, src,
                       u64(0), out, (const u64 *)nullptr, (int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_fast_xxh64_strided(const uint8_t *base, uint64_t pitch, uint64_t len, uint32_t count,
                                       uint64_t *out, const uint64_t *expect, int32_t *status, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (!count)
        return 0;
    Strided src{base, pitch, len, count};
    hipLaunchKernelGGL(k_xxh64_fast<Strided>, dim3((count + MSGS - 1) / MSGS), dim3(64), 0, st, src, u64(0), out,
                       expect, status);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_fast_xxh64_pages(const uint8_t *const *pages, const uint64_t *first, const uint64_t *len,
                                     uint32_t count, uint32_t page_shift, uint64_t *out, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (!count)
        return 0;
    PageList src{pages, first, len, count, page_shift};
    hipLaunchKernelGGL(k_xxh64_fast<PageList>, dim3((count + MSGS - 1) / MSGS), dim3(64), 0, st, src, u64(0), out,
                       (const u64 *)nullptr, (int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
