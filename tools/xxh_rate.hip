// XXH64 round rate on one CU's SIMDs: is a serial chain latency- or
// issue-bound?  Each lane runs C independent chains of R rounds; the grid
// is 256 workgroups (one per CU) of W waves.
//   hipcc --offload-arch=gfx950 -O3 -o tools/xxh_rate tools/xxh_rate.hip && tools/xxh_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../nkfs_amd/csrc/xxh64_dev.h"
using namespace nkfs;

template <int C>
__global__ void k_rounds(const uint64_t *in, uint64_t *out, int R)
{
    uint64_t acc[C], w[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        acc[c] = in[(blockIdx.x * blockDim.x + threadIdx.x) * C + c];
        w[c] = acc[c] ^ 0x1234567ull;
    }
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            acc[c] = xxh_round(acc[c], w[c]);
            w[c] += 0x9E37ull;
        }
    }
    uint64_t x = 0;
#pragma unroll
    for (int c = 0; c < C; ++c)
        x ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int C>
static void run(int waves, int R, uint64_t *in, uint64_t *out)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256;
    hipLaunchKernelGGL(k_rounds<C>, dim3(blocks), dim3(64 * waves), 0, 0, in, out, R);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL(k_rounds<C>, dim3(blocks), dim3(64 * waves), 0, 0, in, out, R);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double ns = ms * 1e6 / 5;
    // per CU: waves * 64 lanes * C chains * R rounds
    const double rounds_cu = double(waves) * 64 * C * R;
    printf("waves/CU %2d chains/lane %d: %8.1f us  %6.2f ns per wave-round-step  %7.2f Ground/s per CU (%.1f GB/s hashed per CU, %.2f TB/s chip)\n",
           waves, C, ns / 1e3, ns / (double(R) * C), rounds_cu / ns, rounds_cu * 8 / ns, rounds_cu * 8 / ns * 256 / 1e3);
}

int main()
{
    uint64_t *in, *out;
    hipMalloc(&in, 256 * 1024 * 8 * 8);
    hipMalloc(&out, 256 * 1024 * 8);
    hipMemset(in, 7, 256 * 1024 * 8 * 8);
    const int R = 1 << 16;
    for (int w : {1, 2, 4, 8}) {
        run<1>(w, R, in, out);
        run<2>(w, R / 2, in, out);
        run<4>(w, R / 4, in, out);
    }
    hipDeviceSynchronize();
    return 0;
}
