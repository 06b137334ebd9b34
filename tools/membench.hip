// tools/membench.hip -- HBM speed-of-light probes for the traffic mixes of
// the nkfs kernels (read:write = 1:2 for N4K2 encode, 1:1 copy, read-only,
// write-only).  Standalone: hipcc --offload-arch=gfx950 -O3 tools/membench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_read(const uint4 *__restrict__ a, size_t n, uint4 *sink)
{
    uint4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = a[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = acc;
}

__global__ void k_write(uint4 *__restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4(i, i + 1, i + 2, i + 3);
}

__global__ void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

// read n, write 2n (two output planes), like an N=4,K=2 encode
__global__ void k_r1w2(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint4 *__restrict__ c, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = a[i];
        b[i] = v;
        c[i] = make_uint4(v.y, v.z, v.w, v.x);
    }
}

// each lane reads K consecutive 16-byte pieces (K*16 B per lane, stride K*16
// across lanes) -- the encode's per-lane row-block load for k = K
template <int K>
__global__ void k_read_lane_contig(const uint4 *__restrict__ a, size_t n, uint4 *sink)
{
    uint4 acc = {0, 0, 0, 0};
    const size_t tasks = n / K;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tasks; t += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int q = 0; q < K; ++q) {
            uint4 v = a[t * K + q];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = acc;
}

int main()
{
    const size_t bytes = (size_t)1 << 30;
    const size_t n = bytes / 16;
    uint4 *a, *b, *c;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&c, bytes));
    CHK(hipMemset(a, 1, bytes));
    CHK(hipMemset(b, 2, bytes));
    CHK(hipMemset(c, 3, bytes));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int grids[] = {1024, 2048, 4096, 8192, 16384};
    for (int gi = 0; gi < 5; ++gi) {
        int grid = grids[gi];
        for (int kind = 0; kind < 4; ++kind) {
            float best = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL(k_read, grid, 256, 0, 0, a, n, c);
                if (kind == 1) hipLaunchKernelGGL(k_write, grid, 256, 0, 0, b, n);
                if (kind == 2) hipLaunchKernelGGL(k_copy, grid, 256, 0, 0, a, b, n);
                if (kind == 3) hipLaunchKernelGGL(k_r1w2, grid, 256, 0, 0, a, b, c, n / 2);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            double moved = kind == 0 ? bytes : kind == 1 ? bytes : kind == 2 ? 2.0 * bytes : 1.5 * bytes;
            const char *nm[] = {"read", "write", "copy 1:1", "read1:write2"};
            printf("grid %5d  %-13s %7.1f GB/s\n", grid, nm[kind], moved / best / 1e6);
        }
    }
    for (int gi = 0; gi < 5; ++gi) {
        int grid = grids[gi];
        for (int kind = 0; kind < 3; ++kind) {
            float best = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL(k_read_lane_contig<2>, grid, 64, 0, 0, a, n, c);
                if (kind == 1) hipLaunchKernelGGL(k_read_lane_contig<5>, grid, 64, 0, 0, a, n, c);
                if (kind == 2) hipLaunchKernelGGL(k_read_lane_contig<1>, grid, 64, 0, 0, a, n, c);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            const char *nm[] = {"read 32B/lane", "read 80B/lane", "read 16B/lane"};
            printf("grid %5d x64  %-13s %7.1f GB/s\n", grid, nm[kind], bytes / best / 1e6);
        }
    }
    return 0;
}
