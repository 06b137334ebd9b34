// boxprobe.hip -- measurement helper for bench.py (not part of the product
// library): the HBM rate THIS box sustains for a given read:write mix with
// the arithmetic stripped, so every bench line can state its kernel's
// fraction of the box's own ceiling next to the fraction of the 8 TB/s spec.
//
// Why: the encode/decode kernels are HBM-mix-bound.  Measured across boxes
// (profiles/r03/sol3_*.txt) a pure read stream runs 6.0-6.3 TB/s and a pure
// write stream 5.0-6.3, but a 5:8 read:write mix (the N8K5 encode's) only
// 5.1-5.7 TB/s depending on the box; the spread between boxes is larger
// than any kernel change measured this round.
//
// k_mix<L,S>: persistent grid, one wave per workgroup; step t of wave w
// loads L KiB (one contiguous 1 KiB run per instruction) from chunk t*G + w
// of the input and stores S KiB to the same chunk of the output (compact
// chip-wide front: the fastest arrangement measured); the next step's loads
// issue before this step's stores.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stddef.h>
#include <stdint.h>

typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

namespace {

template <int L, int S>
__global__ __launch_bounds__(64) void k_mix(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, u32 nsteps)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t pad[];
    const int li = threadIdx.x;
    const u32 G = gridDim.x;
    v4u d[2][L];
    auto load = [&](v4u (&x)[L], u32 t) {
        const u64 base = t < nsteps ? (u64(t) * G + blockIdx.x) * (L * 1024u) : 0;
#pragma unroll
        for (int q = 0; q < L; ++q)
            x[q] = *reinterpret_cast<const v4u *>(in + base + q * 1024 + li * 16);
    };
    auto store = [&](v4u (&x)[L], u32 t) {
        uint8_t *p = out + (u64(t) * G + blockIdx.x) * (S * 1024u);
#pragma unroll
        for (int q = 0; q < S; ++q) {
            v4u v = x[q % L];
            v.x ^= u32(q);
            *reinterpret_cast<v4u *>(p + q * 1024 + li * 16) = v;
        }
    };
    load(d[0], 0);
    for (u32 t = 0; t < nsteps; t += 2) {
        load(d[1], t + 1);
        store(d[0], t);
        if (t + 1 >= nsteps)
            break;
        load(d[0], t + 2);
        store(d[1], t + 1);
    }
}

// The microarch guide's anchor (MI355X_MICROARCH.md, "HBM3E peak BW: 6.29
// TB/s measured (float4 copy)"): plain grid-stride float4 kernels with no
// shaping at all -- copy (1:1), pure read (xor-reduced, one store per
// thread), pure write.  256-thread workgroups, grid = `blocks`.
__global__ __launch_bounds__(256) void k_copy4(const float4 *__restrict__ in, float4 *__restrict__ out, u64 n)
{
    for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += u64(gridDim.x) * blockDim.x)
        out[i] = in[i];
}

__global__ __launch_bounds__(256) void k_read4(const v4u *__restrict__ in, v4u *__restrict__ sink, u64 n)
{
    v4u acc = {0, 0, 0, 0};
    for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += u64(gridDim.x) * blockDim.x)
        acc ^= in[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u)  // practically never: keeps the loads alive
        sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_write4(v4u *__restrict__ out, u64 n)
{
    const v4u v = {blockIdx.x, threadIdx.x, 0x6E6B3846u, 0u};
    for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += u64(gridDim.x) * blockDim.x)
        out[i] = v;
}

// median of `reps` timed launches of `launch` (one untimed first)
template <class F>
int time_median(F launch, int reps, hipStream_t st, float *ms)
{
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess)
        return -EIO;
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return -EIO;
    }
    float t[33];
    if (reps > 33)
        reps = 33;
    if (reps < 1)
        reps = 1;
    int rc = 0;
    launch();
    for (int r = 0; r < reps && !rc; ++r) {
        (void)hipEventRecord(e0, st);
        launch();
        (void)hipEventRecord(e1, st);
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t[r], e0, e1) != hipSuccess)
            rc = -EIO;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc)
        return rc;
    for (int a = 0; a < reps; ++a)
        for (int b = a + 1; b < reps; ++b)
            if (t[b] < t[a]) {
                const float x = t[a];
                t[a] = t[b];
                t[b] = x;
            }
    *ms = t[reps / 2];
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

template <int L, int S>
int run(const void *in, size_t in_bytes, void *out, size_t out_bytes, int waves_per_cu, int reps, hipStream_t st,
        float *ms, double *bytes)
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return -ENODEV;
    const u32 G = u32(cus) * u32(waves_per_cu);
    const u64 steps = in_bytes / (u64(L) * 1024u * G) < out_bytes / (u64(S) * 1024u * G)
                          ? in_bytes / (u64(L) * 1024u * G)
                          : out_bytes / (u64(S) * 1024u * G);
    if (steps < 2 || steps > 0xFFFFFFFFull)
        return -EINVAL;
    // dynamic LDS that caps residency at waves_per_cu one-wave workgroups
    size_t lds = 160u * 1024u / size_t(waves_per_cu);
    if (lds > 65536)
        lds = 65536;
    auto kern = k_mix<L, S>;
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            65536) != hipSuccess)
        return -EIO;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess)
        return -EIO;
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return -EIO;
    }
    float t[33];
    if (reps > 33)
        reps = 33;
    if (reps < 1)
        reps = 1;
    int rc = 0;
    hipLaunchKernelGGL(kern, dim3(G), dim3(64), lds, st, (const uint8_t *)in, (uint8_t *)out, u32(steps));
    for (int r = 0; r < reps && !rc; ++r) {
        (void)hipEventRecord(e0, st);
        hipLaunchKernelGGL(kern, dim3(G), dim3(64), lds, st, (const uint8_t *)in, (uint8_t *)out, u32(steps));
        (void)hipEventRecord(e1, st);
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t[r], e0, e1) != hipSuccess)
            rc = -EIO;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc)
        return rc;
    for (int a = 0; a < reps; ++a)
        for (int b = a + 1; b < reps; ++b)
            if (t[b] < t[a]) {
                const float x = t[a];
                t[a] = t[b];
                t[b] = x;
            }
    *ms = t[reps / 2];
    *bytes = double(steps) * G * 1024.0 * (L + S);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Shader clock under load: every wave spins a dependent integer chain and
// reads the shader cycle counter (s_memtime) and the 100 MHz real-time
// counter (s_memrealtime) around it (record the box's
// clock in the line, to attribute box-to-box swings).
__global__ __launch_bounds__(64) void k_clock(u64 *out, u32 iters)
{
    const u64 t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    u32 x = threadIdx.x + blockIdx.x;
    for (u32 i = 0; i < iters; ++i)
        x = x * 1664525u + 1013904223u;
    const u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
    }
    if (x == 0x12345678u)
        out[2] = x;  // keeps the chain
}

}  // namespace

// Loaded shader clock (MHz) from k_clock over 4 waves per CU, and the CU
// count and peak clock the runtime reports.
extern "C" int nkfs_probe_clock(hipStream_t st, double *mhz_loaded, int *cus, int *mhz_peak)
{
    if (!mhz_loaded || !cus || !mhz_peak)
        return -EINVAL;
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev) ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev))
        return -ENODEV;
    *mhz_peak = khz / 1000;
    u64 *d = nullptr, h[3] = {0, 0, 0};
    if (hipMalloc(reinterpret_cast<void **>(&d), 3 * sizeof(u64)) != hipSuccess)
        return -ENOMEM;
    hipLaunchKernelGGL(k_clock, dim3(4 * *cus), dim3(64), 0, st, d, 1u << 20);  // warm-up: clocks ramp
    hipLaunchKernelGGL(k_clock, dim3(4 * *cus), dim3(64), 0, st, d, 1u << 22);
    const bool ok = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess;
    (void)hipFree(d);
    if (!ok || !h[1])
        return -EIO;
    *mhz_loaded = double(h[0]) / (double(h[1]) / 100.0);  // s_memrealtime ticks at 100 MHz
    return 0;
}

// Median time (ms) of `reps` launches streaming the read:write mix
// read_kib:write_kib (one of 4:8, 5:8, 6:8, 8:8, 8:4) from `in` to `out` at
// waves_per_cu resident waves per CU, and the bytes one launch moves.
extern "C" int nkfs_probe_stream(const void *in, size_t in_bytes, void *out, size_t out_bytes, int read_kib,
                                 int write_kib, int waves_per_cu, int reps, hipStream_t st, float *ms, double *bytes)
{
    if (!in || !out || !ms || !bytes || waves_per_cu < 1 || waves_per_cu > 32)
        return -EINVAL;
#define NKFS_MIX(LL, SS)                                                                              \
    if (read_kib == LL && write_kib == SS)                                                            \
        return run<LL, SS>(in, in_bytes, out, out_bytes, waves_per_cu, reps, st, ms, bytes);
    NKFS_MIX(4, 8)
    NKFS_MIX(5, 8)
    NKFS_MIX(6, 8)
    NKFS_MIX(8, 8)
    NKFS_MIX(8, 4)
#undef NKFS_MIX
    return -EINVAL;
}

// The guide's plain float4 anchor: kind 0 = copy (in -> out, `bytes` read
// and `bytes` written), 1 = pure read of `in`, 2 = pure write of `out`;
// `bytes` (a multiple of 16) per buffer, grid of `blocks` 256-thread
// workgroups (0: 8 per CU).  *moved = HBM bytes one launch moves.
extern "C" int nkfs_probe_plain(const void *in, void *out, size_t bytes, int kind, int blocks, int reps,
                                hipStream_t st, float *ms, double *moved)
{
    if (!ms || !moved || bytes < 16 || (bytes & 15) || kind < 0 || kind > 2 || (kind != 2 && !in) ||
        (kind != 1 && !out) || blocks < 0)
        return -EINVAL;
    if (!blocks) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return -ENODEV;
        blocks = 8 * cus;
    }
    const u64 n = bytes / 16;
    static v4u *sink = nullptr;  // k_read4's never-taken store target
    if (!sink && hipMalloc(reinterpret_cast<void **>(&sink), 256 * sizeof(v4u)) != hipSuccess)
        return -ENOMEM;
    int rc;
    if (kind == 0) {
        rc = time_median([&] { hipLaunchKernelGGL(k_copy4, dim3(blocks), dim3(256), 0, st, (const float4 *)in,
                                                  (float4 *)out, n); },
                         reps, st, ms);
        *moved = 2.0 * double(bytes);
    } else if (kind == 1) {
        rc = time_median([&] { hipLaunchKernelGGL(k_read4, dim3(blocks), dim3(256), 0, st, (const v4u *)in, sink,
                                                  n); },
                         reps, st, ms);
        *moved = double(bytes);
    } else {
        rc = time_median([&] { hipLaunchKernelGGL(k_write4, dim3(blocks), dim3(256), 0, st, (v4u *)out, n); },
                         reps, st, ms);
        *moved = double(bytes);
    }
    return rc;
}
