// tools/sol3.hip -- round-3 access-shape probe for the C3 encode (N8K5,
// 8,192 x 1 MiB -> 8 x 209,716 at a 209,920 pitch), arithmetic stripped (a
// XOR per 16 B).  Bytes counted = algorithmic bytes (B + n*ps per stripe),
// as bench.py's roofline.  Question answered: which data-movement shape can
// carry the fused encode above 5.6 TB/s (0.70 of 8 TB/s)?
//   hipcc --offload-arch=gfx950 -O3 tools/sol3.hip -o tools/sol3 && tools/sol3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr u32 CB = 1048576, CPS = 209716, CPP = 209920, CN = 8, CK = 5;
constexpr u32 NU = (CPS + 1023) / 1024;  // 1,024-row units per stripe (205)
constexpr u32 NS = 8192;

__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void *base, u32 bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}
__device__ inline u32 live_off(bool live, u32 off) { return off | (u32(!live) << 31); }

// aux cache-policy bits (gfx940+): sc0 = 1, nt = 2, sc1 = 16
template <int POL>
__device__ inline v4u bload(__amdgpu_buffer_rsrc_t r, u32 off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, POL);
}
template <int POL>
__device__ inline void bstore(v4u v, __amdgpu_buffer_rsrc_t r, u32 off)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, POL);
}

// ------------------------------------------------------------------ walk
// A wave's task list: (stripe, chunk of U units).  MAP 0: stripes
// grid-stride (s = w + j*G); MAP 1: contiguous stripes per wave; WPS > 1:
// WPS consecutive waves share a stripe, each a contiguous range of its
// chunks.  OUT 0: planar parts (the product layout); OUT 1: the wave's
// 8 x U KiB of a step written as one contiguous run (layout-free ideal).
// LDMA: loads land in LDS by global_load_lds (then read back lane-linear).
template <int U, int SPOL, int LPOL, int MAP, int WPS, int OUT, bool LDMA>
__global__ __launch_bounds__(64) void k_walk(const u8 *__restrict__ blocks, u8 *__restrict__ parts, u32 per_wave)
{
    extern __shared__ __attribute__((aligned(16))) u8 dyn[];
    const int li = threadIdx.x;
    const u32 G = gridDim.x / WPS;
    const u32 w = blockIdx.x / WPS, sub = blockIdx.x % WPS;
    constexpr u32 NCH = (NU + U - 1) / U;
    constexpr u32 CPW = (NCH + WPS - 1) / WPS;  // chunks per sub-wave
    const u32 c0 = sub * CPW, c1 = c0 + CPW < NCH ? c0 + CPW : NCH;
    const u32 nch = c1 > c0 ? c1 - c0 : 0;
    const u32 ntask = per_wave * nch;
    // MAP 0 grid-stride, 1 contiguous per wave, 2 grid-stride with each wave's
    // chunk order rotated by 7w (concurrent waves at different offsets),
    // 3 grid-stride through an odd-multiplier permutation of the stripes
    auto stripe_of = [&](u32 j) {
        if constexpr (MAP == 1)
            return w * per_wave + j;
        else if constexpr (MAP == 3)
            return ((w + j * G) * 2654435761u) & (NS - 1);
        else
            return w + j * G;
    };
    auto chunk_of = [&](u32 t) { return MAP == 2 ? c0 + (t % nch + 7u * w) % nch : c0 + t % nch; };
    // MAP 4: compact front -- task t of wave w is global chunk t*G + w of the
    // batch's (stripe, chunk) sequence, so the chip's concurrent accesses sit
    // in a few adjacent stripes
    auto sc_of = [&](u32 t, u32 &s, u32 &c) {
        if constexpr (MAP == 4) {
            const u32 gc = t * G + w;
            s = gc / NCH;
            c = gc % NCH;
        } else {
            s = stripe_of(nch ? t / nch : 0);
            c = nch ? chunk_of(t) : c0;
        }
    };
    v4u d[2][U][CK];
    auto load = [&](v4u (&x)[U][CK], u32 t, int slot) {
        u32 s, c;
        sc_of(t, s, c);
        const bool ok = t < ntask && s < NS;
        const __amdgpu_buffer_rsrc_t r = rsrc(blocks + u64(ok ? s : 0) * CB, ok ? CB : 0u);
        if constexpr (LDMA) {
            u8 *dst = dyn + (u32(threadIdx.x >> 6) * 2 + slot) * (U * CK * 1024);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < CK; ++q) {
                    const u32 off = (c * U + u) * 5120u + q * 1024u + li * 16u;
                    const u8 *src = blocks + u64(ok ? s : 0) * CB + (ok && off < CB ? off : 0u);
                    __builtin_amdgcn_global_load_lds((const void *)src,
                                                     (__attribute__((address_space(3))) void *)(dst + (u * CK + q) * 1024),
                                                     16, 0, LPOL);
                }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < CK; ++q)
                    x[u][q] = bload<LPOL>(r, (c * U + u) * 5120u + q * 1024u + li * 16u);
        }
    };
    auto store = [&](v4u (&x)[U][CK], u32 t) {
        u32 s, c;
        sc_of(t, s, c);
        const bool ok = s < NS;
        const __amdgpu_buffer_rsrc_t r = rsrc(parts + u64(ok ? s : 0) * CN * CPP, ok ? CN * CPP : 0u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 row = (c * U + u) * 1024u + li * 16u;
#pragma unroll
            for (int i = 0; i < int(CN); ++i) {
                v4u v = x[u][i % CK];
                v.x ^= u32(i);
                u32 off;
                if constexpr (OUT == 0)
                    off = live_off(row < CPP, u32(i) * CPP + row);
                else
                    off = live_off((c * U + u) < NU, ((c * U + u) * CN + u32(i)) * 1024u + li * 16u);
                bstore<SPOL>(v, r, off);
            }
        }
    };
    if (!nch)
        return;
    load(d[0], 0, 0);
    for (u32 t = 0; t < ntask; t += 2) {
        load(d[1], t + 1, 1);
        if constexpr (LDMA) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * CK) : "memory");
            const u8 *src = dyn + (u32(threadIdx.x >> 6) * 2 + 0) * (U * CK * 1024);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < CK; ++q)
                    d[0][u][q] = *reinterpret_cast<const v4u *>(src + (u * CK + q) * 1024 + li * 16);
        }
        store(d[0], t);
        if (t + 1 >= ntask)
            break;
        load(d[0], t + 2, 0);
        if constexpr (LDMA) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * CK) : "memory");
            const u8 *src = dyn + (u32(threadIdx.x >> 6) * 2 + 1) * (U * CK * 1024);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < CK; ++q)
                    d[1][u][q] = *reinterpret_cast<const v4u *>(src + (u * CK + q) * 1024 + li * 16);
        }
        store(d[1], t + 1);
    }
}

// ------------------------------------------------------------------ streams
// grid-stride float4 streams over `bytes`: MODE 0 copy, 1 read-only, 2 write-only
template <int MODE>
__global__ __launch_bounds__(256) void k_stream(const v4u *__restrict__ a, v4u *__restrict__ b, u64 n16, u32 *sink)
{
    extern __shared__ __attribute__((aligned(16))) u8 dyn[];
    const u64 stride = u64(gridDim.x) * blockDim.x;
    v4u acc = {0, 0, 0, 0};
    for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride) {
        if constexpr (MODE == 0)
            b[i] = a[i];
        else if constexpr (MODE == 1)
            acc ^= a[i];
        else
            b[i] = v4u{u32(i), 1, 2, 3};
    }
    if (MODE == 1 && acc.x == 0x12345678u && acc.y == 7u)
        sink[0] = acc.z;
}

// copy with 4 x 16 B per lane in flight: workgroup-contiguous 16 KiB tiles
__global__ __launch_bounds__(256) void k_copy4(const v4u *__restrict__ a, v4u *__restrict__ b, u64 n16)
{
    const u64 tiles = n16 / 1024;
    for (u64 t = blockIdx.x; t < tiles; t += gridDim.x) {
        v4u x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            x[j] = a[t * 1024 + j * 256 + threadIdx.x];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            b[t * 1024 + j * 256 + threadIdx.x] = x[j];
    }
}

// mixed stream: per step a wave loads L KiB (contiguous, one 1 KiB run per
// instruction) and stores S KiB (contiguous); chunks grid-stride so the
// concurrent front is compact; next step's loads issued before this step's
// stores.  L = 0: write-only; S = 0: read-only.
template <int L, int S, int SPOL, bool SPREAD = false>
__global__ __launch_bounds__(64) void k_mix(const u8 *__restrict__ in, u8 *__restrict__ out, u32 nsteps, u32 *sink)
{
    extern __shared__ __attribute__((aligned(16))) u8 dyn[];
    const int li = threadIdx.x;
    const u32 G = gridDim.x;
    constexpr int LL = L ? L : 1;
    v4u d[2][LL];
    const __amdgpu_buffer_rsrc_t ri = rsrc(in, 0x7FFFFFFF);
    v4u acc = {0, 0, 0, 0};
    auto load = [&](v4u (&x)[LL], u32 t) {
        if constexpr (L > 0) {
            const u64 base = SPREAD ? (u64(blockIdx.x) * nsteps + t) * (L * 1024u) : (u64(t) * G + blockIdx.x) * (L * 1024u);
            const bool ok = t < nsteps;
            const u8 *p = in + (ok ? base : 0);
#pragma unroll
            for (int q = 0; q < L; ++q)
                x[q] = *reinterpret_cast<const v4u *>(p + q * 1024 + li * 16);
        }
    };
    auto store = [&](v4u (&x)[LL], u32 t) {
        if constexpr (S > 0) {
            u8 *p = out + (SPREAD ? (u64(blockIdx.x) * nsteps + t) : (u64(t) * G + blockIdx.x)) * (S * 1024u);
            const __amdgpu_buffer_rsrc_t ro = rsrc(p, S * 1024u);
#pragma unroll
            for (int q = 0; q < S; ++q) {
                v4u v = x[q % LL];
                v.x ^= u32(q) + t;
                bstore<SPOL>(v, ro, q * 1024u + li * 16u);
            }
        } else {
#pragma unroll
            for (int q = 0; q < LL; ++q)
                acc ^= x[q];
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
    if (S == 0 && acc.x == 0x12345678u && acc.y == 7u)
        sink[0] = acc.z;
    (void)ri;
}

// time-phased mix: every wave issues its loads only inside the read window
// of a chip-wide period read from the constant 100 MHz realtime clock, and
// its stores only outside it, so the HBM controllers see read phases and
// write phases instead of a steady 5:8 mix.  Per round a wave loads M x
// 5 KiB into LDS (global_load_lds), then stores M x 8 KiB read back from LDS.
template <int M>
__global__ __launch_bounds__(64) void k_phase(const u8 *__restrict__ in, u8 *__restrict__ out, u32 nrounds, u32 period,
                                              u32 rwin)
{
    extern __shared__ __attribute__((aligned(16))) u8 dyn[];
    const int li = threadIdx.x;
    const u32 G = gridDim.x;
    for (u32 r = 0; r < nrounds; ++r) {
        const u64 chunk = u64(r) * G + blockIdx.x;  // compact front
        if (period) {
            u64 now;
            do {
                now = __builtin_amdgcn_s_memrealtime();
            } while (u32(now % period) >= rwin);
        }
        const u8 *src = in + chunk * (M * 5120u);
#pragma unroll
        for (int q = 0; q < M * 5; ++q)
            __builtin_amdgcn_global_load_lds((const void *)(src + q * 1024 + li * 16),
                                             (__attribute__((address_space(3))) void *)(dyn + q * 1024), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (period) {
            u64 now;
            do {
                now = __builtin_amdgcn_s_memrealtime();
            } while (u32(now % period) < rwin);
        }
        u8 *dst = out + chunk * (M * 8192u);
#pragma unroll
        for (int q = 0; q < M * 8; ++q) {
            v4u v = *reinterpret_cast<const v4u *>(dyn + ((q / 8) * 5 + (q % 8) % 5) * 1024 + li * 16);
            v.x ^= u32(q);
            *reinterpret_cast<v4u *>(dst + q * 1024 + li * 16) = v;
        }
    }
}

// ------------------------------------------------------------------ harness
static int g_cus = 256;

template <class F>
static float timeit(F f, int reps)
{
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i)
        f();
    float ts[32];
    for (int r = 0; r < reps; ++r) {
        CHK(hipEventRecord(e0, 0));
        f();
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ts[r], e0, e1));
    }
    for (int a = 0; a < reps; ++a)
        for (int b = a + 1; b < reps; ++b)
            if (ts[b] < ts[a]) {
                const float t = ts[a];
                ts[a] = ts[b];
                ts[b] = t;
            }
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return ts[reps / 2];
}

// dynamic LDS that caps a 64-thread kernel at `per_cu` resident waves per CU
static size_t pad_for(int per_cu, size_t need)
{
    size_t p = 160 * 1024 / size_t(per_cu);
    if (p > 65536)
        p = 65536;
    return p < need ? need : p;
}

template <int U, int SPOL, int LPOL, int MAP, int WPS, int OUT, bool LDMA>
static void walk(const char *name, const u8 *in, u8 *out, int per_cu)
{
    const u32 waves = u32(g_cus) * u32(per_cu);
    const u32 G = waves / WPS;
    const u32 per_wave = (NS + G - 1) / G;
    const size_t need = LDMA ? 2 * U * CK * 1024 : 0;
    const size_t pad = pad_for(per_cu, need);
    auto kern = k_walk<U, SPOL, LPOL, MAP, WPS, OUT, LDMA>;
    CHK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64, pad));
    const float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(G * WPS), dim3(64), pad, 0, in, out, per_wave); }, 9);
    CHK(hipGetLastError());
    const double bytes = double(NS) * (CB + double(CN) * CPS);
    printf("%-44s %3d/CU(occ %2d)  %8.3f ms  %7.1f GB/s\n", name, per_cu, occ, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int L, int S, int SPOL = 0, bool SPREAD = false>
static void mix(const u8 *in, u8 *out, u32 *sink, int per_cu, size_t inb, size_t outb)
{
    const u32 G = u32(g_cus) * u32(per_cu);
    // steps so that neither buffer overflows: L*1024*G*steps <= inb etc.
    u64 steps = ~0ull;
    if (L)
        steps = inb / (u64(L) * 1024u * G);
    if (S) {
        const u64 s2 = outb / (u64(S) * 1024u * G);
        steps = s2 < steps ? s2 : steps;
    }
    const size_t pad = pad_for(per_cu, 0);
    auto kern = k_mix<L, S, SPOL, SPREAD>;
    CHK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    const float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(G), dim3(64), pad, 0, in, out, u32(steps), sink); }, 9);
    CHK(hipGetLastError());
    const double rb = double(L) * 1024 * G * steps, wb = double(S) * 1024 * G * steps;
    char name[64];
    snprintf(name, sizeof name, "mix L%d S%d pol%d%s", L, S, SPOL, SPREAD ? " spread" : "");
    printf("%-44s %3d/CU  %8.3f ms  %7.1f GB/s  (read %.2f GB, write %.2f GB)\n", name, per_cu, ms,
           (rb + wb) / (ms * 1e-3) / 1e9, rb / 1e9, wb / 1e9);
    fflush(stdout);
}

template <int M>
static void phase(const u8 *in, u8 *out, int per_cu, u32 period, u32 rwin, size_t inb, size_t outb)
{
    const u32 G = u32(g_cus) * u32(per_cu);
    u64 rounds = inb / (u64(M) * 5120u * G);
    const u64 r2 = outb / (u64(M) * 8192u * G);
    rounds = r2 < rounds ? r2 : rounds;
    const size_t pad = pad_for(per_cu, M * 5120);
    auto kern = k_phase<M>;
    CHK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    const float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(G), dim3(64), pad, 0, in, out, u32(rounds), period, rwin); }, 7);
    CHK(hipGetLastError());
    const double rb = double(M) * 5120 * G * rounds, wb = double(M) * 8192 * G * rounds;
    char name[80];
    snprintf(name, sizeof name, "phase M%d period %u rwin %u", M, period, rwin);
    printf("%-44s %3d/CU  %8.3f ms  %7.1f GB/s  (read %.2f GB, write %.2f GB)\n", name, per_cu, ms,
           (rb + wb) / (ms * 1e-3) / 1e9, rb / 1e9, wb / 1e9);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    hipDeviceProp_t pr;
    CHK(hipGetDeviceProperties(&pr, 0));
    g_cus = pr.multiProcessorCount;
    printf("device %s, %d CUs\n", pr.name, g_cus);
    const char *only = argc > 1 ? argv[1] : nullptr;
    u8 *in, *out;
    u32 *sink;
    const size_t inb = size_t(NS) * CB, outb = size_t(NS) * CN * CPP;
    CHK(hipMalloc(&in, inb));
    CHK(hipMalloc(&out, outb));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(in, 3, inb));
    CHK(hipMemset(out, 0, outb));

    auto copy4 = [&](const char *tag) {
        const u64 n16 = inb / 16;
        const float ms = timeit([&] { hipLaunchKernelGGL(k_copy4, dim3(g_cus * 8), dim3(256), 0, 0, (const v4u *)in, (v4u *)out, n16); }, 9);
        printf("%-44s %8.3f ms  %7.1f GB/s (r+w)\n", tag, ms, 2.0 * inb / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    copy4("copy4 8 GiB (start)");
    if (!only || !strcmp(only, "streams")) {
        const u64 n16 = inb / 16;
        const int grid = g_cus * 8;
        float ms = timeit([&] { hipLaunchKernelGGL(k_stream<0>, dim3(grid), dim3(256), 0, 0, (const v4u *)in, (v4u *)out, n16, sink); }, 9);
        printf("%-44s %8.3f ms  %7.1f GB/s (r+w)\n", "copy 8 GiB", ms, 2.0 * inb / (ms * 1e-3) / 1e9);
        ms = timeit([&] { hipLaunchKernelGGL(k_stream<1>, dim3(grid), dim3(256), 0, 0, (const v4u *)in, (v4u *)out, n16, sink); }, 9);
        printf("%-44s %8.3f ms  %7.1f GB/s\n", "read 8 GiB", ms, 1.0 * inb / (ms * 1e-3) / 1e9);
        const u64 o16 = outb / 16;
        ms = timeit([&] { hipLaunchKernelGGL(k_stream<2>, dim3(grid), dim3(256), 0, 0, (const v4u *)in, (v4u *)out, o16, sink); }, 9);
        printf("%-44s %8.3f ms  %7.1f GB/s\n", "write 13.8 GB", ms, 1.0 * outb / (ms * 1e-3) / 1e9);
        fflush(stdout);
    }
    if (!only || !strcmp(only, "mix")) {
        mix<8, 0>(in, out, sink, 8, inb, outb);
        mix<0, 8>(in, out, sink, 8, inb, outb);
        mix<8, 8>(in, out, sink, 8, inb, outb);
        mix<5, 8>(in, out, sink, 8, inb, outb);
        mix<4, 8>(in, out, sink, 8, inb, outb);
        mix<8, 0>(in, out, sink, 16, inb, outb);
        mix<0, 8>(in, out, sink, 16, inb, outb);
        mix<8, 8>(in, out, sink, 16, inb, outb);
        mix<5, 8>(in, out, sink, 16, inb, outb);
        mix<8, 8>(in, out, sink, 4, inb, outb);
        mix<5, 8>(in, out, sink, 4, inb, outb);
        mix<16, 16>(in, out, sink, 4, inb, outb);
        mix<10, 16>(in, out, sink, 4, inb, outb);
        mix<0, 8, 2>(in, out, sink, 8, inb, outb);
        mix<5, 8, 2>(in, out, sink, 8, inb, outb);
        mix<0, 8, 16>(in, out, sink, 8, inb, outb);
        mix<8, 0>(in, out, sink, 8, inb, outb);
        mix<0, 8>(in, out, sink, 8, inb, outb);
        mix<5, 8>(in, out, sink, 8, inb, outb);
    }
    if (!only || !strcmp(only, "phase")) {
        mix<5, 8>(in, out, sink, 8, inb, outb);
        phase<4>(in, out, 4, 0, 0, inb, outb);
        phase<4>(in, out, 8, 0, 0, inb, outb);
        phase<6>(in, out, 4, 0, 0, inb, outb);
        // per round chip-wide: 256 CUs x per_cu x M x 5 KiB read
        phase<4>(in, out, 4, 1000, 380, inb, outb);
        phase<4>(in, out, 4, 600, 230, inb, outb);
        phase<4>(in, out, 4, 400, 150, inb, outb);
        phase<6>(in, out, 4, 1500, 570, inb, outb);
        phase<6>(in, out, 4, 800, 300, inb, outb);
        phase<4>(in, out, 8, 1000, 380, inb, outb);
        phase<4>(in, out, 8, 2000, 760, inb, outb);
        phase<4>(in, out, 4, 1000, 300, inb, outb);
        phase<4>(in, out, 4, 1000, 450, inb, outb);
        mix<5, 8>(in, out, sink, 8, inb, outb);
    }
    if (!only || !strcmp(only, "front")) {
        mix<5, 8>(in, out, sink, 8, inb, outb);
        mix<5, 8, 0, true>(in, out, sink, 8, inb, outb);
        mix<5, 8>(in, out, sink, 16, inb, outb);
        mix<5, 8, 0, true>(in, out, sink, 16, inb, outb);
        walk<1, 0, 0, 0, 1, 0, false>("walk U1 stripe per wave", in, out, 8);
        walk<1, 0, 0, 0, 1, 0, false>("walk U1 stripe per wave", in, out, 16);
        walk<1, 0, 0, 4, 1, 0, false>("walk U1 compact front", in, out, 8);
        walk<1, 0, 0, 4, 1, 0, false>("walk U1 compact front", in, out, 16);
        walk<2, 0, 0, 4, 1, 0, false>("walk U2 compact front", in, out, 8);
        walk<1, 0, 0, 4, 1, 1, false>("walk U1 compact front, contiguous out", in, out, 8);
        walk<1, 2, 2, 4, 1, 0, false>("walk U1 compact front nt", in, out, 8);
        mix<5, 8>(in, out, sink, 8, inb, outb);
        walk<1, 0, 0, 0, 1, 0, false>("walk U1 stripe per wave", in, out, 8);
        walk<1, 0, 0, 4, 1, 0, false>("walk U1 compact front", in, out, 8);
    }
    if (!only || !strcmp(only, "walk")) {
        // <U, SPOL, LPOL, MAP, WPS, OUT, LDMA>
        walk<1, 0, 0, 0, 1, 0, false>("walk U1 grid-stride", in, out, 8);
        walk<1, 0, 0, 1, 1, 0, false>("walk U1 contiguous", in, out, 8);
        walk<1, 0, 0, 2, 1, 0, false>("walk U1 grid-stride rotated chunks", in, out, 8);
        walk<1, 0, 0, 3, 1, 0, false>("walk U1 permuted stripes", in, out, 8);
        walk<1, 0, 0, 1, 1, 0, false>("walk U1 contiguous", in, out, 4);
        walk<1, 0, 0, 1, 1, 0, false>("walk U1 contiguous", in, out, 6);
        walk<1, 0, 0, 1, 1, 0, false>("walk U1 contiguous", in, out, 12);
        walk<1, 0, 0, 1, 1, 0, false>("walk U1 contiguous", in, out, 16);
        walk<2, 0, 0, 1, 1, 0, false>("walk U2 contiguous", in, out, 8);
        walk<2, 0, 0, 1, 1, 0, false>("walk U2 contiguous", in, out, 4);
        walk<1, 0, 0, 2, 1, 0, false>("walk U1 rotated", in, out, 4);
        walk<1, 0, 0, 2, 1, 0, false>("walk U1 rotated", in, out, 16);
        walk<1, 0, 0, 3, 1, 0, false>("walk U1 permuted", in, out, 4);
        walk<1, 0, 0, 3, 1, 0, false>("walk U1 permuted", in, out, 16);
        walk<1, 2, 2, 1, 1, 0, false>("walk U1 contiguous nt ld+st", in, out, 8);
        walk<1, 0, 0, 1, 1, 1, false>("ideal contiguous-out, contiguous stripes", in, out, 8);
        walk<1, 0, 0, 1, 2, 0, false>("walk U1 contiguous 2 waves/stripe", in, out, 8);
        walk<1, 0, 0, 1, 4, 0, false>("walk U1 contiguous 4 waves/stripe", in, out, 16);
        walk<1, 0, 0, 2, 1, 0, true>("walk U1 rotated LDS-DMA", in, out, 8);
        walk<1, 0, 0, 1, 1, 0, false>("walk U1 contiguous (repeat)", in, out, 8);
        walk<1, 0, 0, 0, 1, 0, false>("walk U1 grid-stride (repeat)", in, out, 8);
    }
    copy4("copy4 8 GiB (end)");
    return 0;
}
