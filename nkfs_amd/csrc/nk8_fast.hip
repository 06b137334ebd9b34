// nk8_fast.hip -- streaming fast path (placeholder until the fused kernel lands)
#include <hip/hip_runtime.h>
#include <errno.h>
#include "nkfs_internal.h"

extern "C" int nkfs_fast_encode(const nkfs_geom *, const uint8_t *, uint64_t *, const void *, hipStream_t)
{
    return -ENOSYS;
}
