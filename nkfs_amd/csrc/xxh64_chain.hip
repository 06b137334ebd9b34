// xxh64_chain.hip -- one message's XXH64 at the latency of its four serial
// chains, for the per-call drop-in entry points (XXH64, XXH64_update /
// _digest, csum_*; crt/xxhash.c:358-496, 736-930; crt/csum.c:3-27).
//
// One message has exactly four dependent chains of rounds (the accumulators,
// crt/xxhash.c:791-810), so one wave folds it: lane a runs accumulator a
// (lanes 4.. mirror lane a & 3 and are ignored), reading the message
// straight from the caller-staged pinned host buffer over PCIe (no copy
// engine, no host-side wait) or from device memory, far enough ahead that
// a round waits only on the previous round (~80-100 SIMD cycles,
// tools/sol.hip): 32 bytes per round per chain, so a 64 KiB message is
// 2,048 dependent rounds and 1 MiB 32,768.  No barrier.  The same launch can start from accumulators passed
// by value or kept on the device, leave them on the device (a long stream
// folded chunk by chunk), and finish: merge, length, the <32-byte tail
// passed by value, avalanche, then the digest and a completion word stored
// to host memory with a system-scope release, so the host spins on one word
// instead of synchronising the stream.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nkfs_internal.h"
#include "xxh64_dev.h"

using namespace nkfs;

namespace {

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// The message streams through an LDS ring of NS slots of 1 KiB (32
// stripes): each slot is one global_load_lds_dwordx4 of the whole wave (no
// VGPR staging), issued NS-1 slots ahead -- 31 KiB in flight, so the PCIe
// latency of pinned host memory (several us) hides under ~500 rounds -- and
// waited for with a counted vmcnt (the loop issues no other vector memory
// instruction).  Lane a then reads its 32 words of the slot (ds_read_b64)
// and runs its 32 rounds.
constexpr int NS = 32;

// pre: slot 0 (a message of at most 32 stripes) is already in flight into
// ring slot 0 (the service wave's inline read)
__device__ __forceinline__ void chain_run(const nkfs_xxh_args &a, u8 *ring, bool pre = false)
{
    const int li = threadIdx.x, lane = li & 3;
    // (selects, not a.v[lane]: a dynamically indexed argument goes through
    // scratch -- a memory round trip before the first round.  The compiler
    // folds a select chain over a.v back into that index, so the four
    // values are made opaque first)
    u64 w0 = a.v[0], w1 = a.v[1], w2 = a.v[2], w3 = a.v[3];
    asm volatile("" : "+s"(w0), "+s"(w1), "+s"(w2), "+s"(w3));
    u64 acc = lane == 0 ? w0 : lane == 1 ? w1 : lane == 2 ? w2 : w3;
    if (a.flags & NKFS_XXH_FROM_DEV)
        acc = a.v_dev[lane];
    const u64 nst = a.nst;
    const u64 nslots = (nst + 31) / 32;
    // slot c = stripes 32c..32c+31; lane li moves bytes 16li..16li+15 of it
    // (slots past the message read its first KiB again: unused)
    auto issue = [&](u64 c) {
        const u64 off = c < nslots ? c * 1024 + 16 * li : 16 * li;
        const u8 *src = a.src + (off + 16 <= nst * 32 ? off : 0);
        __builtin_amdgcn_global_load_lds((const void *)src,
                                         (__attribute__((address_space(3))) void *)(ring + (c % NS) * 1024), 16,
                                         0, 0);
    };
    if (nst) {
        // only the message's own slots are fetched (a short message is one
        // PCIe round trip, not NS KiB of ring fill); the last NS - 1 slots
        // are waited for together
#pragma unroll
        for (int c = 0; c < NS - 1; ++c)
            if (u64(c) < nslots && !(pre && c == 0))
                issue(u64(c));
        // full slots: no per-round select on the chain's critical path
        const u64 nfull = nst / 32;
        for (u64 c = 0; c < nslots; ++c) {
            if (c + NS - 1 < nslots) {
                issue(c + NS - 1);  // into the slot slot c-1 was read from
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // The multiplies by P2 do not depend on the chain: all 64 lanes
            // take them for the whole slot (two words each, in place), so
            // the four chain lanes' rounds are add, rotate, multiply by P1.
            // A wave issues its 64-bit multiplies for all 64 lanes whatever
            // the exec mask: this cuts the chain's multiply issue by half.
            u8 *sb = ring + (c % NS) * 1024;
            {
                // read and written back by asm: compiler-visible LDS accesses
                // here make it wait for every DMA still landing in the ring
                // (vmcnt(0)); the wave's own LDS operations stay in order, so
                // the chain lanes' reads below see the products
                const u32 la = u32(reinterpret_cast<uintptr_t>(
                    (__attribute__((address_space(3))) u8 *)(sb + 16 * li)));
                v4u q;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(q) : "v"(la) : "memory");
                const u64 m0 = ((u64(q.y) << 32) | q.x) * XP2, m1 = ((u64(q.w) << 32) | q.z) * XP2;
                const v4u mv = {u32(m0), u32(m0 >> 32), u32(m1), u32(m1 >> 32)};
                asm volatile("ds_write_b128 %0, %1" ::"v"(la), "v"(mv) : "memory");
            }
            const u8 *slot = sb + 8 * lane;
            u64 w[32];
#pragma unroll
            for (int r = 0; r < 32; ++r)
                w[r] = *reinterpret_cast<const u64 *>(slot + 32 * r);
            if (c < nfull) {
#pragma unroll
                for (int r = 0; r < 32; ++r)
                    acc = rotl64_31(acc + w[r]) * XP1;
            } else {
                const u32 left = u32(nst - c * 32);
#pragma unroll
                for (int r = 0; r < 32; ++r) {
                    const u64 nx = rotl64_31(acc + w[r]) * XP1;
                    acc = u32(r) < left ? nx : acc;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave
    }
    if (a.flags & NKFS_XXH_TO_DEV)
        if (threadIdx.x < 4)
            a.v_dev[lane] = acc;
    if (!(a.flags & (NKFS_XXH_FINISH | NKFS_XXH_EMIT)))
        return;
    const u64 v1 = __shfl(acc, 0, 64), v2 = __shfl(acc, 1, 64);
    const u64 v3 = __shfl(acc, 2, 64), v4 = __shfl(acc, 3, 64);
    if (threadIdx.x != 0)
        return;
    // The answer words are written through to memory (system-scope stores)
    // and the completion word follows once they are acknowledged: the
    // ordering a release would give, without its write-back of the whole L2
    // before the completion word (these kernels leave nothing else in it)
    auto put = [](u64 *p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    auto complete = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        put(a.out + 1, a.flag);
    };
    if (a.flags & NKFS_XXH_EMIT) {  // the accumulators back to the host state
        put(a.out + 2, v1);
        put(a.out + 3, v2);
        put(a.out + 4, v3);
        put(a.out + 5, v4);
    }
    if (!(a.flags & NKFS_XXH_FINISH)) {
        complete();
        return;
    }
    // merge (crt/xxhash.c:849-877), length (:884), tail (:886-910),
    // avalanche (:912-916)
    u64 h = a.total_len >= 32 ? xxh_converge(v1, v2, v3, v4) : a.seed + XP5;
    h += a.total_len;
    u64 tw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        u64 x = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            x |= u64(a.tail[8 * w + b]) << (8 * b);
        tw[w] = x;
    }
    const u64 dig = xxh_tail_regs(h, tw, a.tail_len);
    if (!(a.flags & NKFS_XXH_EMIT) && (reinterpret_cast<uintptr_t>(a.out) & 15) == 0) {
        // digest and completion word in one 16-byte system-scope store:
        // one posted write over the link, so the host that sees the word
        // sees the digest (the NVMe completion-entry pattern) -- the
        // two-store form waited for the digest's acknowledgement (a link
        // round trip) before the word could leave
        const v4u pk = {u32(dig), u32(dig >> 32), u32(a.flag), u32(a.flag >> 32)};
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(a.out), "v"(pk) : "memory");
        return;
    }
    put(a.out, dig);
    complete();  // the completion word after the digest, visible in order
}

__global__ __launch_bounds__(64) void k_xxh64_chain(nkfs_xxh_args a)
{
    __shared__ __attribute__((aligned(16))) u8 ring[NS * 1024];
    chain_run(a, ring);
}

// The opt-in resident service (nkfs_percall_service): one wave polls a
// mailbox in fine-grained (coherent) host memory and runs each posted
// message exactly as k_xxh64_chain would, so a per-call digest needs no
// kernel launch -- the host writes the arguments, then the request number,
// and spins on the message's own completion word as before.  The wave leaves
// after `idle` ticks (s_memrealtime, 100 MHz) without a request, after
// `life` ticks in all, or on a stop request, and clears `alive` as it goes:
// no schedule can leave it running, and the host relaunches it when a
// request finds it gone.
// The request half (seq, op, args, inline bytes) is read from `mb` -- host
// memory, or (mode 2) fine-grained device memory the host writes over the
// BAR -- and the answer half (taken, alive) written to `ob` in host memory.
#ifndef NKFS_SVC_RELAXED_POLL
#define NKFS_SVC_RELAXED_POLL 0
#endif
__global__ __launch_bounds__(64) void k_xxh64_service(nkfs_svc_box *mb, nkfs_svc_box *ob, u64 idle, u64 life)
{
    __shared__ __attribute__((aligned(16))) u8 ring[NS * 1024];
    u64 last = __hip_atomic_load(&ob->taken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    u64 tl = t0;
    for (;;) {
        // NKFS_SVC_RELAXED_POLL (experiment builds): poll relaxed and acquire
        // only once a request is seen
        const u64 sq = NKFS_SVC_RELAXED_POLL
                           ? __hip_atomic_load(&mb->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                           : __hip_atomic_load(&mb->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (sq != last) {
            if (NKFS_SVC_RELAXED_POLL)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            last = sq;
            // the inline message bytes (up to 1 KiB) into ring slot 0 in the
            // same round trip as the arguments
            __builtin_amdgcn_global_load_lds((const void *)(mb->inl + 16 * threadIdx.x),
                                             (__attribute__((address_space(3))) void *)ring, 16, 0, 0);
            // op and the arguments in the same round trip as the inline bytes
            // (all three are complete before seq is published); the branch on
            // op waits for all of them at once.  (The clobber keeps the
            // argument loads behind the inline read: scheduled first, the
            // read waited for one of them before it was issued.)
            asm volatile("" ::: "memory");
            const u64 op = mb->op;
            nkfs_xxh_args a = mb->args;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (op != NKFS_SVC_XXH && op != NKFS_SVC_XXH_INL) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // a stop uses a request number too: mark it taken, so the next
                // wave (which starts from `taken`) sees no request pending
                // (off -> on left taken one behind seq)
                if (threadIdx.x == 0)
                    __hip_atomic_store(&ob->taken, sq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                break;  // stop
            }
            const bool inl = op == NKFS_SVC_XXH_INL;
            if (!inl)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the unused inline read lands first
            // the arguments are in registers (lgkmcnt(0) above): the box may be
            // reused.  A relaxed store -- a release here would write back the
            // L2 and wait for it before the chain starts; the host reads
            // `taken` only to tell a lost wave from a slow one
            if (threadIdx.x == 0)
                __hip_atomic_store(&ob->taken, sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            chain_run(a, ring, inl);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (a message under 32 B left the inline read unused)
            tl = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        const u64 now = __builtin_amdgcn_s_memrealtime();
        if (now - tl > idle || now - t0 > life)
            break;
        __builtin_amdgcn_s_sleep(2);
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(&ob->alive, u64(0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

extern "C" int nkfs_launch_xxh64_chain(const nkfs_xxh_args *a, void *stream)
{
    if (!a || (a->nst && !a->src) || ((a->flags & (NKFS_XXH_FROM_DEV | NKFS_XXH_TO_DEV)) && !a->v_dev) ||
        ((a->flags & (NKFS_XXH_FINISH | NKFS_XXH_EMIT)) && !a->out) || a->tail_len > 31)
        return -EINVAL;
    hipLaunchKernelGGL(k_xxh64_chain, dim3(1), dim3(64), 0, (hipStream_t)stream, *a);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int nkfs_launch_xxh64_service(nkfs_svc_box *mb, nkfs_svc_box *ob, uint64_t idle_ticks, uint64_t life_ticks,
                                         void *stream)
{
    if (!mb || !ob)
        return -EINVAL;
    hipLaunchKernelGGL(k_xxh64_service, dim3(1), dim3(64), 0, (hipStream_t)stream, mb, ob, idle_ticks, life_ticks);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
