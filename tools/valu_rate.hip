// VALU issue cost per wave64 instruction on gfx950 for the byte-product
// instructions (nk8_vp.hip): v_perm_b32 with SGPR table operands, the
// three-input XOR v_bitop3_b32, and v_xor_b32 / v_fma_f32 for reference.
// 256 workgroups (one per CU) of W waves; each lane runs 8 independent
// chains of R x 8 instructions; cycles per instruction per SIMD =
// time x clock x 4 SIMDs / (waves x R x 64).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip && tools/valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int OP>
__global__ void k_ops(const uint32_t *in, uint32_t *out, int R, uint32_t t0, uint32_t t1)
{
    uint32_t a[8];
    const uint32_t s = in[blockIdx.x * blockDim.x + threadIdx.x];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        a[c] = s + c;
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        f[c] = float(s + c);
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (OP == 0)
                    asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(a[c]) : "s"(t0));
                else if (OP == 1)
                    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[c]) : "v"(a[(c + 1) & 7]), "v"(a[(c + 2) & 7]));
                else if (OP == 2)
                    asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[c]) : "s"(t1));
                else if (OP == 3)
                    asm volatile("v_fma_f32 %0, %0, %0, %1" : "+v"(f[c]) : "s"(t1));
                else if (OP == 4)
                    asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[c]) : "s"(t1));
                else if (OP == 5)
                    asm volatile("v_lshrrev_b32 %0, 2, %0" : "+v"(a[c]));
                else
                    asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(a[c]) : "v"(a[(c + 3) & 7]));
            }
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c)
        x ^= a[c] ^ __float_as_uint(f[c]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

static const char *NAMES[] = {"v_perm_b32 s,s,v", "v_bitop3_b32 v,v,v", "v_xor_b32 s,v", "v_fma_f32 v,v,s",
                              "v_and_b32 s,v", "v_lshrrev_b32", "v_perm_b32 v,v,v"};

template <int OP>
static void run(int waves, int R, uint32_t *in, uint32_t *out, double ghz)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int it = 0; it < 2; ++it)
        hipLaunchKernelGGL(k_ops<OP>, dim3(256), dim3(64 * waves), 0, 0, in, out, R, 0x0C0B0A09u, 0x12345u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_ops<OP>, dim3(256), dim3(64 * waves), 0, 0, in, out, R, 0x0C0B0A09u, 0x12345u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double insts = double(waves) * R * 64.0;  // per CU (one workgroup each)
    printf("%-22s waves/CU %2d  %8.3f ms  %5.2f cycles per wave64 instruction per SIMD\n", NAMES[OP], waves, ms,
           ms * 1e-3 * ghz * 1e9 * 4.0 / insts);
}

int main()
{
    uint32_t *in, *out;
    hipMalloc(&in, 256 * 1024 * 4);
    hipMalloc(&out, 256 * 1024 * 4);
    hipMemset(in, 1, 256 * 1024 * 4);
    const double ghz = 2.4;
    const int R = 20000;
    for (int w : {4, 8, 16}) {
        run<0>(w, R, in, out, ghz);
        run<6>(w, R, in, out, ghz);
        run<1>(w, R, in, out, ghz);
        run<2>(w, R, in, out, ghz);
        run<4>(w, R, in, out, ghz);
        run<5>(w, R, in, out, ghz);
        run<3>(w, R, in, out, ghz);
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
