// xxh64_chain.hip -- one message's XXH64 at the latency of its four serial
// chains, for the per-call drop-in entry points (XXH64, XXH64_update /
// _digest, csum_*; crt/xxhash.c:358-496, 736-930; crt/csum.c:3-27).
//
// One message has exactly four dependent chains of rounds (the accumulators,
// crt/xxhash.c:791-810), so one wave folds it: lane a runs accumulator a
// (lanes 4.. mirror lane a & 3 and are ignored).  Each lane keeps the words
// of the next D stripes in flight in a register ring -- loads are issued D
// rounds ahead, straight from the caller-staged pinned host buffer over
// PCIe (no copy engine, no host-side wait) or from device memory -- so a
// round waits only on the previous round (~96 SIMD cycles, tools/sol.hip).
// No LDS, no barrier.  The same launch can start from accumulators passed
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

constexpr int D = 48;  // rounds of loads in flight per lane (vmcnt holds 63)

__global__ __launch_bounds__(64) void k_xxh64_chain(nkfs_xxh_args a)
{
    const int lane = threadIdx.x & 3;
    u64 acc = (a.flags & NKFS_XXH_FROM_DEV) ? a.v_dev[lane] : a.v[lane];
    const u64 nst = a.nst;
    const u8 *src = a.src + 8 * lane;
    // word of stripe i; stripes past the end read stripe 0 (unused): every
    // slot is loaded unconditionally, so the in-order vmcnt waits are exact
    auto ld = [&](u64 i) { return *reinterpret_cast<const u64 *>(src + 32 * (i < nst ? i : 0)); };
    if (nst) {
        u64 ring[D];
#pragma unroll
        for (int j = 0; j < D; ++j)
            ring[j] = ld(u64(j));
        for (u64 base = 0; base < nst; base += D) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const u64 w = ring[j];
                ring[j] = ld(base + D + j);
                const u64 nx = xxh_round(acc, w);
                acc = base + j < nst ? nx : acc;
            }
        }
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
    if (a.flags & NKFS_XXH_EMIT) {  // the accumulators back to the host state
        a.out[2] = v1;
        a.out[3] = v2;
        a.out[4] = v3;
        a.out[5] = v4;
    }
    if (!(a.flags & NKFS_XXH_FINISH)) {
        __hip_atomic_store(a.out + 1, a.flag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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
    a.out[0] = dig;
    // the completion word after the digest, visible to the host in order
    __hip_atomic_store(a.out + 1, a.flag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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
