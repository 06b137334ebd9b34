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

// store flavours: 0 plain, 1 nontemporal (nt), 2 write-through (sc1 via
// __hip_atomic store relaxed agent would be scalar; use inline asm)
template <int FL>
__device__ inline void st16(uint4 *p, uint4 v)
{
    if constexpr (FL == 0) {
        *p = v;
    } else if constexpr (FL == 1) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        v4u x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(x) : "memory");
    }
}

template <int FL>
__global__ void k_r1w2_fl(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint4 *__restrict__ c, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = a[i];
        st16<FL>(b + i, v);
        st16<FL>(c + i, make_uint4(v.y, v.z, v.w, v.x));
    }
}

template <int FL>
__global__ void k_write_fl(uint4 *__restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        st16<FL>(a + i, make_uint4(i, i + 1, i + 2, i + 3));
}

// the encode's write pattern: one 64-lane wave owns a REGION-byte output
// region of STREAMS planar streams (stride REGION/STREAMS) and writes SEG
// bytes to each stream per iteration (lanes spread evenly over streams).
template <int STREAMS, int SEG>
__global__ void k_wave_streams(uint4 *__restrict__ out, size_t region, size_t n_waves)
{
    const size_t w = blockIdx.x;
    if (w >= n_waves) return;
    const int lane = threadIdx.x;
    constexpr int LPS = 64 / STREAMS;          // lanes per stream
    constexpr int PER = SEG / 16 / LPS;        // 16-B stores per lane per stream per iteration
    const int st = lane / LPS, li = lane % LPS;
    const size_t stride = region / STREAMS;
    char *base = reinterpret_cast<char *>(out) + w * region + st * stride;
    for (size_t off = 0; off < stride; off += SEG)
#pragma unroll
        for (int q = 0; q < PER; ++q)
            *reinterpret_cast<uint4 *>(base + off + (size_t)(q * LPS + li) * 16) = make_uint4(off, q, li, st);
}

// encode-shaped copy: wave w reads its IN-byte input region (32 B per lane
// per iteration, like N4K2's 16 rows x 2 B) and writes 4 parts x 4 stripes
// (16 streams x 256 B per iteration) of its 2*IN-byte output region.
__global__ void k_wave_r1w2(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n_waves)
{
    const size_t w = blockIdx.x;
    const int lane = threadIdx.x;
    constexpr size_t IN = 16384;
    const char *src = reinterpret_cast<const char *>(in) + w * IN;
    char *dst = reinterpret_cast<char *>(out) + w * 2 * IN;
    const int st = lane / 16, li = lane % 16;  // stripe of 4, lane in stripe
    for (int c = 0; c < 8; ++c) {               // 8 chunks of 256 rows
        const uint4 *p = reinterpret_cast<const uint4 *>(src + st * 4096 + c * 512 + li * 32);
        uint4 a = p[0], b = p[1];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint4 v = make_uint4(a.x ^ i, a.y ^ b.x, a.z ^ b.y, a.w ^ b.z + i);
            *reinterpret_cast<uint4 *>(dst + (st * 4 + i) * 2048 + c * 256 + li * 16) = v;
        }
    }
}

// encode-shaped copy variants.  SPW stripes per wave (4 KiB in, 4 x 2 KiB
// out each), ROWS16 16-row tasks per lane per chunk.
template <int SPW, int T16>
__global__ void k_enc_shape(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n_waves)
{
    const size_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (w >= n_waves) return;
    const int lane = threadIdx.x & 63;
    constexpr int LPS = 64 / SPW;                  // lanes per stripe
    constexpr int R = 16 * T16 * LPS;              // rows per chunk per stripe
    const int st = lane / LPS, li = lane % LPS;
    const char *src = reinterpret_cast<const char *>(in) + (w * SPW + st) * 4096;
    char *dst = reinterpret_cast<char *>(out) + (w * SPW + st) * 8192;
    for (int c = 0; c < 2048 / R; ++c) {
        uint4 a[2 * T16];
#pragma unroll
        for (int t = 0; t < T16; ++t) {
            const uint4 *p = reinterpret_cast<const uint4 *>(src + (c * R + (t * LPS + li) * 16) * 2);
            a[2 * t] = p[0];
            a[2 * t + 1] = p[1];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int t = 0; t < T16; ++t)
                *reinterpret_cast<uint4 *>(dst + i * 2048 + c * R + (t * LPS + li) * 16) =
                    make_uint4(a[2 * t].x ^ i, a[2 * t].y, a[2 * t + 1].z, a[2 * t + 1].w + i);
    }
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
        for (int kind = 0; kind < 6; ++kind) {
            float best = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL(k_write_fl<0>, grid, 256, 0, 0, b, n);
                if (kind == 1) hipLaunchKernelGGL(k_write_fl<1>, grid, 256, 0, 0, b, n);
                if (kind == 2) hipLaunchKernelGGL(k_write_fl<2>, grid, 256, 0, 0, b, n);
                if (kind == 3) hipLaunchKernelGGL(k_r1w2_fl<0>, grid, 256, 0, 0, a, b, c, n / 2);
                if (kind == 4) hipLaunchKernelGGL(k_r1w2_fl<1>, grid, 256, 0, 0, a, b, c, n / 2);
                if (kind == 5) hipLaunchKernelGGL(k_r1w2_fl<2>, grid, 256, 0, 0, a, b, c, n / 2);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            const char *nm[] = {"write plain", "write nt", "write sc1", "r1w2 plain", "r1w2 nt", "r1w2 sc1"};
            double moved = kind < 3 ? bytes : 1.5 * bytes;
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
    {
        const size_t region = 32768, waves = bytes / region;
        for (int kind = 0; kind < 5; ++kind) {
            float best = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL((k_wave_streams<16, 256>), waves, 64, 0, 0, b, region, waves);
                if (kind == 1) hipLaunchKernelGGL((k_wave_streams<16, 512>), waves, 64, 0, 0, b, region, waves);
                if (kind == 2) hipLaunchKernelGGL((k_wave_streams<16, 1024>), waves, 64, 0, 0, b, region, waves);
                if (kind == 3) hipLaunchKernelGGL((k_wave_streams<4, 1024>), waves, 64, 0, 0, b, region, waves);
                if (kind == 4) hipLaunchKernelGGL((k_wave_streams<1, 1024>), waves, 64, 0, 0, b, region, waves);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            const char *nm[] = {"16 streams x 256B", "16 streams x 512B", "16 streams x 1KB", "4 streams x 1KB", "1 stream x 1KB"};
            printf("wave-region write  %-18s %7.1f GB/s\n", nm[kind], bytes / best / 1e6);
        }
        const size_t w2 = (bytes / 2) / 16384;
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_wave_r1w2, w2, 64, 0, 0, a, b, w2);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        printf("wave-region r1w2 (encode-shaped, 16 KB in / 32 KB out per wave) %7.1f GB/s\n", 1.5 * bytes / best / 1e6);
        const size_t stripes = (bytes / 2) / 4096;
        for (int kind = 0; kind < 6; ++kind) {
            float bb = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL((k_enc_shape<4, 1>), stripes / 4, 64, 0, 0, a, b, stripes / 4);
                if (kind == 1) hipLaunchKernelGGL((k_enc_shape<1, 1>), stripes, 64, 0, 0, a, b, stripes);
                if (kind == 2) hipLaunchKernelGGL((k_enc_shape<1, 1>), stripes / 4, 256, 0, 0, a, b, stripes);
                if (kind == 3) hipLaunchKernelGGL((k_enc_shape<1, 2>), stripes, 64, 0, 0, a, b, stripes);
                if (kind == 4) hipLaunchKernelGGL((k_enc_shape<4, 2>), stripes / 4, 64, 0, 0, a, b, stripes / 4);
                if (kind == 5) hipLaunchKernelGGL((k_enc_shape<4, 1>), stripes / 16, 256, 0, 0, a, b, stripes / 4);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < bb) bb = ms;
            }
            const char *nm[] = {"4 stripes/wave, 256 rows", "1 stripe/wave, 1024 rows", "1 stripe/wave, WG 4 waves",
                                "1 stripe/wave, 2048 rows", "4 stripes/wave, 512 rows", "4 stripes/wave, WG 4 waves"};
            printf("enc-shape r1w2 %-28s %7.1f GB/s\n", nm[kind], 1.5 * bytes / bb / 1e6);
        }
    }
    return 0;
}
