// tools/membench2.hip -- tighter HBM speed-of-light probes for the encode
// (read 1 : write 2) and decode (read 1 : write 1) traffic mixes: U 16-byte
// accesses in flight per lane, one-shot grids (every lane touches U pieces
// once) and persistent grid-stride grids, 256- or 64-thread workgroups.
// Bytes counted = bytes read + bytes written, like bench.py's roofline.
//   hipcc --offload-arch=gfx950 -O3 tools/membench2.hip -o tools/membench2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// one-shot: block b, lane t handles pieces base + t + j*BS, j < U (coalesced per j)
template <int U, int BS, int NOUT>
__global__ __launch_bounds__(BS) void k_oneshot(const uint4 *__restrict__ a, uint4 *__restrict__ b,
                                                uint4 *__restrict__ c, size_t n)
{
    const size_t base = size_t(blockIdx.x) * BS * U + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
        if (base + size_t(j) * BS < n)
            v[j] = a[base + size_t(j) * BS];
#pragma unroll
    for (int j = 0; j < U; ++j)
        if (base + size_t(j) * BS < n) {
            b[base + size_t(j) * BS] = v[j];
            if (NOUT == 2)
                c[base + size_t(j) * BS] = make_uint4(v[j].y, v[j].z, v[j].w, v[j].x);
        }
}

// persistent grid-stride with U pieces per lane per iteration
template <int U, int BS, int NOUT>
__global__ __launch_bounds__(BS) void k_stride(const uint4 *__restrict__ a, uint4 *__restrict__ b,
                                               uint4 *__restrict__ c, size_t n)
{
    const size_t step = size_t(gridDim.x) * BS * U;
    for (size_t base = size_t(blockIdx.x) * BS * U + threadIdx.x; base < n; base += step) {
        uint4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (base + size_t(j) * BS < n)
                v[j] = a[base + size_t(j) * BS];
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (base + size_t(j) * BS < n) {
                b[base + size_t(j) * BS] = v[j];
                if (NOUT == 2)
                    c[base + size_t(j) * BS] = make_uint4(v[j].y, v[j].z, v[j].w, v[j].x);
            }
    }
}

// pure read (sink) for reference
template <int U, int BS>
__global__ __launch_bounds__(BS) void k_read(const uint4 *__restrict__ a, uint4 *sink, size_t n)
{
    const size_t base = size_t(blockIdx.x) * BS * U + threadIdx.x;
    uint4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < U; ++j)
        if (base + size_t(j) * BS < n) {
            const uint4 v = a[base + size_t(j) * BS];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u)
        sink[0] = acc;
}

template <class F>
static float timeit(F f)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        f();
    float best = 1e30f;
    for (int r = 0; r < 10; ++r) {
        hipEventRecord(e0, 0);
        f();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    return best;
}

int main()
{
    const size_t bytes = size_t(1) << 30;  // 1 GiB input
    const size_t n = bytes / 16;
    uint4 *a, *b, *c, *sink;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&c, bytes));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(a, 1, bytes));
    CHK(hipMemset(b, 0, bytes));
    CHK(hipMemset(c, 0, bytes));

#define ONESHOT(U, BS, NO)                                                                                   \
    do {                                                                                                     \
        const unsigned grid = unsigned((n + size_t(BS) * U - 1) / (size_t(BS) * U));                         \
        float ms = timeit([&] { hipLaunchKernelGGL((k_oneshot<U, BS, NO>), grid, BS, 0, 0, a, b, c, n); }); \
        printf("oneshot r1w%d U=%2d BS=%3d grid=%7u  %7.1f GB/s\n", NO, U, BS, grid,                          \
               double(bytes) * (1 + NO) / (ms * 1e-3) / 1e9);                                                \
    } while (0)
#define STRIDE(U, BS, NO, G)                                                                               \
    do {                                                                                                   \
        float ms = timeit([&] { hipLaunchKernelGGL((k_stride<U, BS, NO>), G, BS, 0, 0, a, b, c, n); });   \
        printf("stride  r1w%d U=%2d BS=%3d grid=%7u  %7.1f GB/s\n", NO, U, BS, unsigned(G),               \
               double(bytes) * (1 + NO) / (ms * 1e-3) / 1e9);                                              \
    } while (0)
#define READ(U, BS)                                                                                          \
    do {                                                                                                     \
        const unsigned grid = unsigned((n + size_t(BS) * U - 1) / (size_t(BS) * U));                         \
        float ms = timeit([&] { hipLaunchKernelGGL((k_read<U, BS>), grid, BS, 0, 0, a, sink, n); });        \
        printf("read         U=%2d BS=%3d grid=%7u  %7.1f GB/s\n", U, BS, grid,                               \
               double(bytes) / (ms * 1e-3) / 1e9);                                                           \
    } while (0)

    READ(1, 256); READ(4, 256); READ(8, 256); READ(4, 64); READ(8, 64);
    ONESHOT(1, 256, 1); ONESHOT(2, 256, 1); ONESHOT(4, 256, 1); ONESHOT(8, 256, 1);
    ONESHOT(4, 64, 1); ONESHOT(8, 64, 1); ONESHOT(16, 64, 1);
    ONESHOT(1, 256, 2); ONESHOT(2, 256, 2); ONESHOT(4, 256, 2); ONESHOT(8, 256, 2);
    ONESHOT(2, 64, 2); ONESHOT(4, 64, 2); ONESHOT(8, 64, 2); ONESHOT(16, 64, 2);
    for (unsigned G : {1024u, 2048u, 4096u, 8192u}) {
        STRIDE(4, 256, 1, G);
        STRIDE(4, 256, 2, G);
        STRIDE(8, 64, 2, G);
    }
    return 0;
}
