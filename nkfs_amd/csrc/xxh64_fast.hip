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
#include <stdlib.h>

#include "nkfs_internal.h"
#include "xxh64_dev.h"

using namespace nkfs;
typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

namespace {

constexpr int MSGS = 16;               // messages per wave
constexpr int CH = 512;                // bytes per message per iteration
constexpr int PIECES = MSGS * CH / 16; // 16-byte pieces per iteration
constexpr int PPL = PIECES / 64;       // pieces per lane (8)
constexpr int SPAD = CH + 32;          // LDS bytes per message (bank spread)

// Pieces outside a message load from here instead (branch-free loads keep
// the ring slots in flight); g_zero_page is a one-entry page table for it.
__device__ __attribute__((aligned(16))) u8 g_zero16[16];
__device__ const u8 *g_zero_page[1];

// A message source maps message m to (descriptor, length).  base(d, c)
// is the address that byte offset off(c*CH + x) of chunk c is relative to,
// for 0 <= x < CH: the message start for contiguous sources, the page
// holding the chunk for page lists (pages are >= CH and powers of two, so
// a chunk never straddles two pages).  base() may read memory; the kernel
// calls it one ring slot ahead so no load waits on a fresh pointer.
struct MsgList {  // explicit (offset, length) list
    typedef const u8 *Desc;
    static constexpr bool kPaged = false;
    const u8 *base_;
    const u64 *off;
    const u64 *len;
    u32 count;
    __device__ u64 total() const { return count; }
    __device__ bool get(u32 m, Desc &d, u64 &n) const
    {
        if (m >= count)
            return false;
        d = base_ + off[m];
        n = len[m];
        return true;
    }
    __device__ const u8 *base(Desc d, u32, u64) const { return d; }
    __device__ static Desc dummy() { return g_zero16; }
    __device__ u64 off_in(u64 pos) const { return pos; }
    __device__ u32 page_shift() const { return 0; }
    __device__ const u8 *addr(Desc d, u64 pos) const { return d + pos; }
};

struct Strided {  // count messages of len bytes, pitch apart (clusters)
    typedef const u8 *Desc;
    static constexpr bool kPaged = false;
    const u8 *base_;
    u64 pitch;
    u64 len;
    u32 count;
    __device__ u64 total() const { return count; }
    __device__ bool get(u32 m, Desc &d, u64 &n) const
    {
        if (m >= count)
            return false;
        d = base_ + u64(m) * pitch;
        n = len;
        return true;
    }
    __device__ const u8 *base(Desc d, u32, u64) const { return d; }
    __device__ static Desc dummy() { return g_zero16; }
    __device__ u64 off_in(u64 pos) const { return pos; }
    __device__ u32 page_shift() const { return 0; }
    __device__ const u8 *addr(Desc d, u64 pos) const { return d + pos; }
};

struct PageList {  // message m = first len[m] bytes of pages[first[m]..]
    typedef const u8 *const *Desc;
    static constexpr bool kPaged = true;
    const u8 *const *pages;
    const u64 *first;
    const u64 *len;
    u32 count;
    u32 shift;  // log2(page size), >= log2(CH)
    __device__ bool get(u32 m, Desc &d, u64 &n) const
    {
        if (m >= count)
            return false;
        d = pages + first[m];
        n = len[m];
        return true;
    }
    __device__ const u8 *base(Desc d, u32 c, u64 lastpg) const
    {
        const u64 pg = (u64(c) * CH) >> shift;
        return d[pg < lastpg ? pg : lastpg];
    }
    __device__ static Desc dummy() { return g_zero_page; }
    __device__ u64 off_in(u64 pos) const { return pos & ((u64(1) << shift) - 1); }
    __device__ u32 page_shift() const { return shift; }
    __device__ const u8 *addr(Desc d, u64 pos) const { return d[pos >> shift] + off_in(pos); }
};

struct PartsOf {  // every part of a batch laid out by nkfs_geom
    typedef const u8 *Desc;
    static constexpr bool kPaged = false;
    nkfs_geom g;
    __device__ u64 total() const { return u64(g.nstripes) * u64(g.n); }
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
    __device__ const u8 *base(Desc d, u32, u64) const { return d; }
    __device__ static Desc dummy() { return g_zero16; }
    __device__ u64 off_in(u64 pos) const { return pos; }
    __device__ u32 page_shift() const { return 0; }
    __device__ const u8 *addr(Desc d, u64 pos) const { return d + pos; }
};

__device__ inline u64 shfl64(u64 v, int src)
{
    u32 lo = __shfl(u32(v), src, 64);
    u32 hi = __shfl(u32(v >> 32), src, 64);
    return (u64(hi) << 32) | lo;
}

}  // namespace

// One wave, 16 messages.  The hot loop moves whole 16-byte pieces only
// (pieces past a message's last full piece are skipped): the chunk loop has
// no data-dependent control flow inside the loads, so the compiler keeps
// both ring slots in flight.  The < 32-byte tail the accumulators do not
// consume is read by the finishing lane straight from memory.
//
// A16: every piece address is 16-byte aligned (one dwordx4 load), else two
// dwordx2 loads (8-byte aligned data, the API contract).
// expect != NULL: status[m] = 0 when out[m] == expect[m], else -EINVAL
// (the compare of nkfs_inode_block_check_sum, core/inode.c:561-575).
template <class Src, bool A16>
__global__ __launch_bounds__(64) void k_xxh64_fast(Src src, u64 seed, u64 *out, const u64 *expect,
                                                   int32_t *status)
{
    __shared__ __attribute__((aligned(16))) u8 buf[MSGS * SPAD];
    const int lane = threadIdx.x;
    const u32 m0 = blockIdx.x * MSGS;

    // loader role: piece q of lane = message (lane + 64q) / 32, 16-B piece
    // (lane + 64q) % 32 of that message's chunk
    typename Src::Desc ld[PPL];
    u64 llen[PPL], lastpg[PPL];
    int lmsg[PPL], lpos[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
        const int pc = lane + 64 * q;
        lmsg[q] = pc / (CH / 16);
        lpos[q] = (pc % (CH / 16)) * 16;
        u64 n = 0;
        if (!src.get(m0 + lmsg[q], ld[q], n))
            n = 0;
        llen[q] = n & ~u64(15);  // whole pieces only
        if (!llen[q])
            ld[q] = Src::dummy();
        lastpg[q] = Src::kPaged && llen[q] ? (llen[q] - 1) >> src.page_shift() : 0;
    }
    const u8 *const zero = g_zero16;
    // hash role: message hm, accumulator ha
    const int hm = lane >> 2, ha = lane & 3;
    typename Src::Desc hd = typename Src::Desc();
    u64 hlen = 0;
    const bool hlive = src.get(m0 + hm, hd, hlen);
    const u64 nst = hlen >> 5;
    const u32 nchunks = u32((nst * 32 + CH - 1) / CH);  // chunks holding whole stripes
    u64 acc = xxh_acc_init(ha, seed);

    // any stripe left in this wave?
    u32 wchunks = nchunks;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        wchunks = max(wchunks, u32(__shfl_xor(int(wchunks), o, 64)));

    // chunk bases one ring slot ahead (page lists: the page of each chunk)
    auto bases = [&](const u8 *(&b)[PPL], u32 c) {
#pragma unroll
        for (int q = 0; q < PPL; ++q)
            b[q] = src.base(ld[q], c, lastpg[q]);
    };
    auto load = [&](uint4 (&d)[PPL], const u8 *const (&b)[PPL], u32 c) {
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const u64 pos = u64(c) * CH + lpos[q];
            const u8 *a = pos < llen[q] ? b[q] + src.off_in(pos) : zero;
            if (A16) {
                const v4u t = *reinterpret_cast<const v4u *>(a);
                d[q] = make_uint4(t.x, t.y, t.z, t.w);
            } else {
                const u64 *w = reinterpret_cast<const u64 *>(a);
                const u64 lo = w[0], hi = w[1];
                d[q] = make_uint4(u32(lo), u32(lo >> 32), u32(hi), u32(hi >> 32));
            }
        }
    };

    // The ring is always refilled and both steps always run (wchunks is
    // even; chunks past a message load the zero block and are not hashed):
    // one straight-line loop body, so the compiler's wait counts keep the
    // other slot in flight.
    wchunks = (wchunks + 1) & ~1u;
    uint4 d0[PPL], d1[PPL];
    const u8 *b0[PPL], *b1[PPL];
    bases(b0, 0);
    load(d0, b0, 0);
    bases(b1, 1);
    load(d1, b1, 1);
    if (Src::kPaged) {  // pointers for chunks 2 and 3 ride with slots 0 and 1
        bases(b0, 2);
        bases(b1, 3);
    }
    auto step = [&](uint4 (&d)[PPL], const u8 *(&b)[PPL], u32 c) {
#pragma unroll
        for (int q = 0; q < PPL; ++q)  // pieces past a message are zeros, never hashed
            *reinterpret_cast<uint4 *>(buf + lmsg[q] * SPAD + lpos[q]) = d[q];
        __syncthreads();
        u64 hw[CH / 32];
#pragma unroll
        for (int r = 0; r < CH / 32; ++r)
            hw[r] = *reinterpret_cast<const u64 *>(buf + hm * SPAD + 32 * r + 8 * ha);
        __syncthreads();
        // refill this ring slot behind the rounds
        if (!Src::kPaged)
            bases(b, c + 2);
        load(d, b, c + 2);
        if (Src::kPaged)
            bases(b, c + 4);
        const u64 first = u64(c) * (CH / 32);
        acc = xxh_rounds<CH / 32>(acc, hw, first >= nst ? 0 : int(min(nst - first, u64(CH / 32))));
    };
    for (u32 c = 0; c < wchunks; c += 2) {
        step(d0, b0, c);
        step(d1, b1, c + 1);
    }

    const int base = lane & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    if (hlive && ha == 0) {
        u64 h = hlen >= 32 ? xxh_converge(v1, v2, v3, v4) : seed + XP5;
        h += hlen;
        u64 tw[4] = {0, 0, 0, 0};
        const u32 left = u32(hlen & 31);
        if (left) {  // < 32 bytes, never across a page (pages are >= 512 B)
            const u8 *t = src.addr(hd, nst * 32);
            for (u32 b = 0; b < left; ++b)
                tw[b >> 3] |= u64(t[b]) << (8 * (b & 7));
        }
        const u64 dig = xxh_tail_regs(h, tw, left);
        out[m0 + hm] = dig;
        if (expect)
            status[m0 + hm] = dig == expect[m0 + hm] ? 0 : -EINVAL;
    }
}

// LDS-DMA ring form (contiguous sources, 16-byte aligned pieces): the 64 lanes copy each chunk
// global -> LDS with global_load_lds_dwordx4 (no VGPR staging), NS chunks
// deep, so a wave keeps (NS-1) x 8 KB in flight whatever the compiler's
// scheduling; the wait for chunk c is an explicit counted vmcnt.  Used when
// the batch has few messages per SIMD (long messages, e.g. whole 64 KiB
// clusters), where latency rather than VALU bounds the register form.
//
// LDS image of a slot: message m's 512-byte chunk at m*512, 16-byte unit j
// holding the message's piece j ^ swz(m) (swizzled through the SOURCE
// address, as glds writes lane-linear), so the hash lanes' 8-byte reads of
// one round fall in distinct banks.
__device__ inline u32 ring_swz(u32 m) { return 2u * (m & 7u); }

template <class Src, int NS>
__global__ __launch_bounds__(64) void k_xxh64_ring(Src src, u64 seed, u64 *out, const u64 *expect,
                                                   int32_t *status)
{
    __shared__ __attribute__((aligned(16))) u8 ring[NS * MSGS * CH];
    const int lane = threadIdx.x;
    const u32 m0 = blockIdx.x * MSGS;

    // lane m < 16 looks message m up; everyone else reads it by shuffle
    typename Src::Desc md = Src::dummy();
    u64 mlen = 0;
    if (lane < MSGS && !src.get(m0 + lane, md, mlen)) {
        md = Src::dummy();
        mlen = 0;
    }
    const u8 *mbase = src.base(md, 0, 0);
    // loader: instruction q moves messages 2q (lanes 0-31) and 2q+1
    const u32 lj = lane & 31;
    const u8 *lb[PPL];
    u64 lfull[PPL];
    u32 lsw[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
        const int mq = 2 * q + (lane >> 5);
        lb[q] = reinterpret_cast<const u8 *>(shfl64(reinterpret_cast<uintptr_t>(mbase), mq));
        lfull[q] = shfl64(mlen, mq) & ~u64(15);
        lsw[q] = 16u * (lj ^ ring_swz(u32(mq)));
    }
    // hash role: message hm, accumulator ha
    const int hm = lane >> 2, ha = lane & 3;
    const u64 hlen = shfl64(mlen, hm);
    const bool hlive = m0 + u32(hm) < src.total();
    const u64 nst = hlen >> 5;
    const u32 nchunks = u32((nst * 32 + CH - 1) / CH);
    u64 acc = xxh_acc_init(ha, seed);
    u32 wchunks = nchunks;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        wchunks = max(wchunks, u32(__shfl_xor(int(wchunks), o, 64)));

    const u8 *const zero = g_zero16;
    auto issue = [&](u32 c) {  // always PPL instructions (the wait counts rely on it)
        u8 *dst = ring + (c % NS) * (MSGS * CH);
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const u64 pos = u64(c) * CH + lsw[q];
            const u8 *a = pos < lfull[q] ? lb[q] + pos : zero;
            __builtin_amdgcn_global_load_lds((const void *)a, (__attribute__((address_space(3))) void *)(dst + q * 1024),
                                             16, 0, 0);
        }
    };
#pragma unroll
    for (int c = 0; c < NS - 1; ++c)
        issue(u32(c));
    // hash lane's read offsets inside a slot (round r: piece 2r + ha/2)
    u32 hoff[CH / 32];
#pragma unroll
    for (int r = 0; r < CH / 32; ++r)
        hoff[r] = u32(hm) * CH + 16u * ((2u * r + (u32(ha) >> 1)) ^ ring_swz(u32(hm))) + 8u * (u32(ha) & 1u);
    for (u32 c = 0; c < wchunks; ++c) {
        issue(c + NS - 1);  // into the slot chunk c-1 was read from
        if constexpr (NS == 4)
            asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        const u8 *slot = ring + (c % NS) * (MSGS * CH);
        u64 hw[CH / 32];
#pragma unroll
        for (int r = 0; r < CH / 32; ++r)
            hw[r] = *reinterpret_cast<const u64 *>(slot + hoff[r]);
        const u64 first = u64(c) * (CH / 32);
        acc = xxh_rounds<CH / 32>(acc, hw, first >= nst ? 0 : int(min(nst - first, u64(CH / 32))));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave

    const int base = lane & ~3;
    const u64 v1 = shfl64(acc, base), v2 = shfl64(acc, base + 1);
    const u64 v3 = shfl64(acc, base + 2), v4 = shfl64(acc, base + 3);
    // shuffles need every lane active: fetch the tail's message base here
    const u8 *hbase = reinterpret_cast<const u8 *>(shfl64(reinterpret_cast<uintptr_t>(mbase), hm));
    if (hlive && ha == 0) {
        u64 h = hlen >= 32 ? xxh_converge(v1, v2, v3, v4) : seed + XP5;
        h += hlen;
        u64 tw[4] = {0, 0, 0, 0};
        const u32 left = u32(hlen & 31);
        if (left) {
            const u8 *t = hbase + nst * 32;
            for (u32 b = 0; b < left; ++b)
                tw[b >> 3] |= u64(t[b]) << (8 * (b & 7));
        }
        const u64 dig = xxh_tail_regs(h, tw, left);
        out[m0 + hm] = dig;
        if (expect)
            status[m0 + hm] = dig == expect[m0 + hm] ? 0 : -EINVAL;
    }
}

// Register form below ~this many waves per SIMD, ring form under it.
static bool use_ring(u64 messages)
{
    return (messages + MSGS - 1) / MSGS <= 2048;  // <= 2 waves per SIMD
}

#define NKFS_XXH_LAUNCH(SRC, A16, grid, st, src, seed, out, expect, status)                                    \
    do {                                                                                                       \
        if (A16)                                                                                               \
            hipLaunchKernelGGL((k_xxh64_fast<SRC, true>), grid, dim3(64), 0, st, src, seed, out, expect, status); \
        else                                                                                                   \
            hipLaunchKernelGGL((k_xxh64_fast<SRC, false>), grid, dim3(64), 0, st, src, seed, out, expect,       \
                               status);                                                                        \
    } while (0)

extern "C" int nkfs_fast_xxh64_list(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint32_t count,
                                    uint64_t seed, uint64_t *out, hipStream_t st)
{
    if (!count)
        return 0;
    MsgList src{base, off, len, count};
    // offsets live on the device: only 8-byte alignment is known
    hipLaunchKernelGGL((k_xxh64_fast<MsgList, false>), dim3((count + MSGS - 1) / MSGS), dim3(64), 0, st, src, seed,
                       out, (const u64 *)nullptr, (int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_fast_xxh64_parts(const nkfs_geom *g, uint64_t *out, hipStream_t st)
{
    const u64 total = u64(g->nstripes) * u64(g->n);
    if (!total)
        return 0;
    PartsOf src{*g};
    // ragged part offsets are caller data: assume only 8-byte alignment there
    const bool a16 = !g->block_sizes && ((reinterpret_cast<uintptr_t>(g->parts) | g->part_pitch) & 15) == 0;
    if (a16 && use_ring(total)) {  // the DMA form needs 16-byte aligned pieces
        hipLaunchKernelGGL((k_xxh64_ring<PartsOf, 4>), dim3(u32((total + MSGS - 1) / MSGS)), dim3(64), 0, st, src,
                           u64(0), out, (const u64 *)nullptr, (int32_t *)nullptr);
        return hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    NKFS_XXH_LAUNCH(PartsOf, a16, dim3(u32((total + MSGS - 1) / MSGS)), st, src, u64(0), out, (const u64 *)nullptr,
                    (int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_fast_xxh64_strided(const uint8_t *base, uint64_t pitch, uint64_t len, uint32_t count,
                                       uint64_t *out, const uint64_t *expect, int32_t *status, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (!count)
        return 0;
    Strided src{base, pitch, len, count};
    const bool a16 = ((reinterpret_cast<uintptr_t>(base) | (count > 1 ? pitch : 0)) & 15) == 0;
    if (a16 && use_ring(count)) {  // the DMA form needs 16-byte aligned pieces
        hipLaunchKernelGGL((k_xxh64_ring<Strided, 4>), dim3((count + MSGS - 1) / MSGS), dim3(64), 0, st, src, u64(0),
                           out, expect, status);
        return hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    NKFS_XXH_LAUNCH(Strided, a16, dim3((count + MSGS - 1) / MSGS), st, src, u64(0), out, expect, status);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_fast_xxh64_pages(const uint8_t *const *pages, const uint64_t *first, const uint64_t *len,
                                     uint32_t count, uint32_t page_shift, uint64_t *out, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (!count)
        return 0;
    PageList src{pages, first, len, count, page_shift};
    // page pointers are device data: only 8-byte alignment is known
    hipLaunchKernelGGL((k_xxh64_fast<PageList, false>), dim3((count + MSGS - 1) / MSGS), dim3(64), 0, st, src,
                       u64(0), out, (const u64 *)nullptr, (int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
