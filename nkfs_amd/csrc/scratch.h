// scratch.h -- per-launch device scratch of the launchers (C++ only): bump
// allocation from nkfs_geom.scratch when the caller provides it, else one
// stream-ordered block of the library's private pool (nk8_kernels.hip,
// nkfs_private_pool: cross-stream reuse only along stream order).
#ifndef NKFS_SCRATCH_H
#define NKFS_SCRATCH_H
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "nkfs_internal.h"

extern "C" hipMemPool_t nkfs_private_pool(hipStream_t st);

namespace nkfs {

// One launch's scratch: bump allocation from the geometry's scratch, else
// one stream-ordered block of the private pool (released by finish()).
struct Scratch {
    uint8_t *base = nullptr;
    uint64_t left = 0;
    void *pooled = nullptr;
    hipStream_t st = nullptr;

    // take `bytes` (256-B aligned) from g's scratch, or the pool when g has
    // none; with `all`, everything g's scratch has left (the caller sized it
    // for the exact need, which only the device knows; `bytes` is then the
    // host-side upper bound the pool would be asked for)
    void *take(const nkfs_geom *g, uint64_t bytes, hipStream_t s, bool all = false)
    {
        bytes = (bytes + 255) & ~uint64_t(255);
        if (g->scratch) {
            if (all)
                bytes = g->scratch_bytes & ~uint64_t(255);
            if (g->scratch_bytes < bytes || !bytes)
                return nullptr;  // the caller sized its scratch: too small is a bug, not a reason to allocate
            base = g->scratch;
            left = g->scratch_bytes;
        } else {
            hipMemPool_t p = nkfs_private_pool(s);
            if (!p || hipMallocFromPoolAsync(&pooled, bytes, p, s) != hipSuccess) {
                (void)hipGetLastError();
                pooled = nullptr;
                return nullptr;
            }
            st = s;
            base = static_cast<uint8_t *>(pooled);
            left = bytes;
        }
        uint8_t *r = base;
        base += bytes;
        left -= bytes;
        return r;
    }
    // the rest of the caller's scratch, for a nested launch (NULL: pool)
    void rest(nkfs_geom *g2) const
    {
        g2->scratch = pooled ? nullptr : base;
        g2->scratch_bytes = pooled ? 0 : left;
    }
    int finish()
    {
        if (!pooled)
            return 0;
        const hipError_t e = hipFreeAsync(pooled, st);
        pooled = nullptr;
        return e == hipSuccess ? 0 : -EIO;
    }
};

}  // namespace nkfs

#endif
