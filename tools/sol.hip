// tools/sol.hip -- speed-of-light probes for the shapes of this repo's hot
// kernels, arithmetic stripped (a XOR per 16 B), plus the issue cost of one
// XXH64 round.  Bytes counted = bytes read + bytes written (bench.py's
// roofline convention).
//   hipcc --offload-arch=gfx950 -O3 tools/sol.hip -o tools/sol && tools/sol
//
// Encode C2 (65,536 x 4 KiB -> 4 x 2 KiB), encode C3 (2,048 x 1 MiB -> 8 x
// 209,716 at a 209,920 pitch), decode C3 (5 x 209,716 -> 1 MiB).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ inline void st16(void *p, uint4 v, bool nt)
{
    const v4u x = {v.x, v.y, v.z, v.w};
    if (nt)
        __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(p));
    else
        *reinterpret_cast<v4u *>(p) = x;
}

__device__ inline uint4 mix(uint4 v, uint32_t p) { return make_uint4(v.x ^ p, v.y + p, v.z, v.w ^ (p << 3)); }

// ------------------------------------------------------------ encode C2
// wave = G stripes, one-shot (the whole stripe per wave).  PAT 0: lane loads
// 32 contiguous bytes per unit (16 rows, K = 2) -- each load instruction
// touches every other 16 B of a 2 KiB span; PAT 1: every load instruction
// is one contiguous 1 KiB run.  Stores: 1 KiB contiguous per part per unit.
constexpr uint32_t C2B = 4096, C2P = 2048, C2N = 4;

template <int G, int PAT, bool NT, int LDSPAD>
__global__ __launch_bounds__(64) void k_c2(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts)
{
    __shared__ uint4 pad[LDSPAD ? LDSPAD / 16 : 1];
    const int li = threadIdx.x;
    uint4 d[G][4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint8_t *b = blocks + size_t(blockIdx.x * G + g) * C2B;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const size_t off = PAT == 0 ? (u * 1024 + li * 16) * 2 + 16 * q : (u * 2 + q) * 1024 + li * 16;
                d[g][u * 2 + q] = *reinterpret_cast<const uint4 *>(b + off);
            }
    }
    if (LDSPAD) {
        pad[li] = d[0][0];
        __syncthreads();
        d[0][0].x ^= pad[(li + 1) & 63].y;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        uint8_t *p = parts + size_t(blockIdx.x * G + g) * C2N * C2P;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                st16(p + i * C2P + u * 1024 + li * 16, mix(d[g][u * 2 + (i & 1)], i), NT);
    }
}

// 256-thread workgroup, one stripe per wave (same per-wave shape as G = 1)
__global__ __launch_bounds__(256) void k_c2_wg4(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts)
{
    const int li = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint8_t *b = blocks + size_t(blockIdx.x * 4 + w) * C2B;
    uint4 d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        d[j] = *reinterpret_cast<const uint4 *>(b + j * 1024 + li * 16);
    uint8_t *p = parts + size_t(blockIdx.x * 4 + w) * C2N * C2P;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u)
            st16(p + i * C2P + u * 1024 + li * 16, mix(d[u * 2 + (i & 1)], i), false);
}

// persistent: the wave walks SPW stripes (G = 1 shape each), next stripe's
// loads issued before this stripe's stores
template <int SPW>
__global__ __launch_bounds__(64) void k_c2_persist(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts)
{
    const int li = threadIdx.x;
    uint4 d[4], nx[4];
    const uint32_t s0 = blockIdx.x * SPW;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        d[j] = *reinterpret_cast<const uint4 *>(blocks + size_t(s0) * C2B + j * 1024 + li * 16);
    for (int t = 0; t < SPW; ++t) {
        if (t + 1 < SPW)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                nx[j] = *reinterpret_cast<const uint4 *>(blocks + size_t(s0 + t + 1) * C2B + j * 1024 + li * 16);
        uint8_t *p = parts + size_t(s0 + t) * C2N * C2P;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                st16(p + i * C2P + u * 1024 + li * 16, mix(d[u * 2 + (i & 1)], i), false);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            d[j] = nx[j];
    }
}


// grid-stride persistent: wave b handles stripes b, b + NW, ... (NW = grid)
// so the resident waves cover a compact window of stripes at any time
template <int LDSPAD>
__global__ __launch_bounds__(64) void k_c2_gs(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts,
                                              uint32_t nstripes)
{
    __shared__ uint4 pad[LDSPAD ? LDSPAD / 16 : 1];
    const int li = threadIdx.x;
    if (LDSPAD) {
        pad[li] = make_uint4(li, 0, 0, 0);
        __syncthreads();
        if (pad[(li + 1) & 63].x == 1000)
            return;
    }
    uint4 d[4], nx[4];
    uint32_t s = blockIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        d[j] = *reinterpret_cast<const uint4 *>(blocks + size_t(s) * C2B + j * 1024 + li * 16);
    for (; s < nstripes; s += gridDim.x) {
        const uint32_t sn = s + gridDim.x;
        if (sn < nstripes)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                nx[j] = *reinterpret_cast<const uint4 *>(blocks + size_t(sn) * C2B + j * 1024 + li * 16);
        uint8_t *p = parts + size_t(s) * C2N * C2P;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                st16(p + i * C2P + u * 1024 + li * 16, mix(d[u * 2 + (i & 1)], i), false);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            d[j] = nx[j];
    }
}

// decode C2: 2 parts x 2 KiB -> 4 KiB, one stripe per wave; PAT 0 lane
// stores its 32 contiguous bytes (stride-32 store instructions), PAT 1
// contiguous 1 KiB per store instruction
template <int PAT, int LDSPAD>
__global__ __launch_bounds__(64) void k_d2(const uint8_t *__restrict__ parts, uint8_t *__restrict__ blocks)
{
    __shared__ uint4 pad[LDSPAD ? LDSPAD / 16 : 1];
    const int li = threadIdx.x;
    if (LDSPAD) {
        pad[li] = make_uint4(li, 0, 0, 0);
        __syncthreads();
        if (pad[(li + 1) & 63].x == 1000)
            return;
    }
    const uint8_t *p = parts + size_t(blockIdx.x) * C2N * C2P;
    uint4 d[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            d[u][c] = *reinterpret_cast<const uint4 *>(p + (c + 1) * C2P + u * 1024 + li * 16);
    uint8_t *b = blocks + size_t(blockIdx.x) * C2B;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const size_t off = PAT == 0 ? (u * 1024 + li * 16) * 2 + 16 * q : (u * 2 + q) * 1024 + li * 16;
            st16(b + off, mix(d[u][q], q), false);
        }
}

// ------------------------------------------------------------ encode C3
constexpr uint32_t C3B = 1048576, C3PS = 209716, C3PP = 209920, C3N = 8, C3K = 5;
constexpr uint32_t C3SL = (C3PS + 1023) / 1024;  // 1,024-row slices per stripe (205)

// one wave per (stripe, group of SL slices); PAT 0: lane loads 80 contiguous
// bytes (16 rows of 5), PAT 1: each load instruction one contiguous 1 KiB.
// DEPTH = slices of loads in flight per lane.
template <int SL, int PAT, int DEPTH, bool NT, int LDSPAD = 0>
__global__ __launch_bounds__(64) void k_c3(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts,
                                           uint32_t nstripes)
{
    __shared__ uint4 pad[LDSPAD ? LDSPAD / 16 : 1];
    const int li = threadIdx.x;
    if (LDSPAD) {
        pad[li] = make_uint4(li, 0, 0, 0);
        __syncthreads();
        if (pad[(li + 1) & 63].x == 1000)
            return;
    }
    constexpr uint32_t GPS = (C3SL + SL - 1) / SL;  // groups per stripe
    const uint32_t s = blockIdx.x / GPS, grp = blockIdx.x % GPS;
    const uint8_t *b = blocks + size_t(s) * C3B;
    uint8_t *p = parts + size_t(s) * C3N * C3PP;
    uint4 d[DEPTH][5];
    auto load = [&](uint4 (&x)[5], uint32_t sl) {
        const uint32_t r0 = sl * 1024;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const size_t off = PAT == 0 ? size_t(r0 + li * 16) * 5 + 16 * q : size_t(r0) * 5 + q * 1024 + li * 16;
            if (off + 16 <= C3B)
                x[q] = *reinterpret_cast<const uint4 *>(b + off);
        }
    };
    const uint32_t sl0 = grp * SL;
#pragma unroll
    for (int j = 0; j < DEPTH; ++j)
        if (j < SL && sl0 + j < C3SL)
            load(d[j], sl0 + j);
    for (int t = 0; t < SL; t += DEPTH) {
#pragma unroll
        for (int j = 0; j < DEPTH; ++j) {
            const uint32_t sl = sl0 + t + j;
            if (t + j >= SL || sl >= C3SL)
                break;
            uint4 v[5];
#pragma unroll
            for (int q = 0; q < 5; ++q)
                v[q] = d[j][q];
            if (t + j + DEPTH < SL && sl + DEPTH < C3SL)
                load(d[j], sl + DEPTH);
            const uint32_t r = sl * 1024 + li * 16;
            if (r + 16 <= C3PP)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    st16(p + i * C3PP + r, mix(v[i % 5], i), NT);
        }
    }
    (void)nstripes;
}


// walking: wave (stripe s, sub w) handles steps t = w, w + WPS, ... of its
// stripe, step t = slices [t*SPS, t*SPS + SPS); next step's loads issued
// before this step's stores; grid = nstripes * WPS (all stripes walk at once,
// the resident set limited by LDSPAD)
template <int SPS, int WPS, int LDSPAD, int BS = 64, int PAT = 1>
__global__ __launch_bounds__(BS) void k_walk(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts)
{
    __shared__ uint4 pad[LDSPAD ? LDSPAD / 16 : 1];
    const int li = threadIdx.x & 63;
    if (LDSPAD) {
        pad[threadIdx.x] = make_uint4(li, 0, 0, 0);
        __syncthreads();
        if (pad[(threadIdx.x + 1) & 63].x == 1000)
            return;
    }
    const uint32_t gw = blockIdx.x * (BS / 64) + threadIdx.x / 64;
    const uint32_t s = gw / WPS, w = gw % WPS;
    const uint8_t *b = blocks + size_t(s) * C3B;
    uint8_t *p = parts + size_t(s) * C3N * C3PP;
    constexpr uint32_t NSTEP = (C3SL + SPS - 1) / SPS;
    uint4 d[SPS][5], nx[SPS][5];
    auto load = [&](uint4 (&x)[SPS][5], uint32_t t) {
#pragma unroll
        for (int j = 0; j < SPS; ++j)
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const size_t off = PAT ? size_t(t * SPS + j) * 5120 + q * 1024 + li * 16
                                       : size_t(t * SPS + j) * 5120 + li * 80 + q * 16;
                if (off + 16 <= C3B)
                    x[j][q] = *reinterpret_cast<const uint4 *>(b + off);
            }
    };
    load(d, w);
    for (uint32_t t = w; t < NSTEP; t += WPS) {
        if (t + WPS < NSTEP)
            load(nx, t + WPS);
#pragma unroll
        for (int j = 0; j < SPS; ++j) {
            const uint32_t r = (t * SPS + j) * 1024 + li * 16;
            if (r + 16 <= C3PP)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    st16(p + i * C3PP + r, mix(d[j][i % 5], i), false);
        }
#pragma unroll
        for (int j = 0; j < SPS; ++j)
#pragma unroll
            for (int q = 0; q < 5; ++q)
                d[j][q] = nx[j][q];
    }
}

// C2 with 4 stripes per 256-thread workgroup (one per wave) and LDSPAD per WG
template <int LDSPAD>
__global__ __launch_bounds__(256) void k_c2_wg4p(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts)
{
    __shared__ uint4 pad[LDSPAD / 16];
    const int li = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint8_t *b = blocks + size_t(blockIdx.x * 4 + w) * C2B;
    uint4 d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        d[j] = *reinterpret_cast<const uint4 *>(b + j * 1024 + li * 16);
    pad[threadIdx.x] = d[0];
    __syncthreads();
    d[0].x ^= pad[(threadIdx.x + 1) & 255].y;
    uint8_t *p = parts + size_t(blockIdx.x * 4 + w) * C2N * C2P;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u)
            st16(p + i * C2P + u * 1024 + li * 16, mix(d[u * 2 + (i & 1)], i), false);
}

// ------------------------------------------------------------ decode C3
// wave per (stripe, group of SL slices): 5 x 1 KiB part loads per slice,
// rows packed back: PAT 0 lane stores its 80 contiguous bytes (5 stores at
// an 80-byte lane stride), PAT 1 each store instruction one contiguous
// 1 KiB run (the real kernel would need an LDS transpose for that).
template <int SL, int PAT, bool NT, int LDSPAD = 0>
__global__ __launch_bounds__(64) void k_d3(const uint8_t *__restrict__ parts, uint8_t *__restrict__ blocks)
{
    __shared__ uint4 pad[LDSPAD ? LDSPAD / 16 : 1];
    const int li = threadIdx.x;
    if (LDSPAD) {
        pad[li] = make_uint4(li, 0, 0, 0);
        __syncthreads();
        if (pad[(li + 1) & 63].x == 1000)
            return;
    }
    constexpr uint32_t GPS = (C3SL + SL - 1) / SL;
    const uint32_t s = blockIdx.x / GPS, grp = blockIdx.x % GPS;
    const uint8_t *p = parts + size_t(s) * C3N * C3PP;
    uint8_t *b = blocks + size_t(s) * C3B;
    uint4 d[5], nx[5];
    auto load = [&](uint4 (&x)[5], uint32_t sl) {
        const uint32_t r = sl * 1024 + li * 16;
#pragma unroll
        for (int c = 0; c < 5; ++c)
            if (r + 16 <= C3PP)
                x[c] = *reinterpret_cast<const uint4 *>(p + c * C3PP + r);
    };
    const uint32_t sl0 = grp * SL;
    load(d, sl0);
    for (int t = 0; t < SL && sl0 + t < C3SL; ++t) {
        const uint32_t sl = sl0 + t;
        if (t + 1 < SL && sl + 1 < C3SL)
            load(nx, sl + 1);
        const uint32_t r0 = sl * 1024;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const size_t off = PAT == 0 ? size_t(r0 + li * 16) * 5 + 16 * q : size_t(r0) * 5 + q * 1024 + li * 16;
            if (off + 16 <= C3B)
                st16(b + off, mix(d[q], q), NT);
        }
#pragma unroll
        for (int c = 0; c < 5; ++c)
            d[c] = nx[c];
    }
}

// ------------------------------------------------------------ XXH64 round
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull, XP2 = 0xC2B2AE3D27D4EB4Full;
__device__ inline uint64_t rotl31(uint64_t v)
{
    const uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
    return (uint64_t(__builtin_amdgcn_alignbit(hi, lo, 1)) << 32) | __builtin_amdgcn_alignbit(lo, hi, 1);
}
__device__ inline uint64_t xround(uint64_t acc, uint64_t w) { return rotl31(acc + w * XP2) * XP1; }

// CH independent chains per lane, NR rounds each; lanes >= ACTIVE idle
template <int ACTIVE, int CH>
__global__ __launch_bounds__(64) void k_xxh(uint64_t *out, int nr)
{
    const int li = threadIdx.x;
    if (li >= ACTIVE)
        return;
    uint64_t a[CH], w[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        a[c] = li * 7 + c;
        w[c] = (uint64_t(li) << 32) | c;
    }
    for (int r = 0; r < nr; ++r)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            a[c] = xround(a[c], w[c]);
            w[c] += 0x9E3779B97F4A7C15ull;
        }
    uint64_t x = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c)
        x ^= a[c];
    out[blockIdx.x * 64 + li] = x;
}

template <class F>
static float timeit(F f, int reps = 10)
{
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i)
        f();
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHK(hipEventRecord(e0, 0));
        f();
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    return best;
}

struct Res {
    const char *name;
    float v[5];
};

int main()
{
    // ---- XXH64 round issue cost
    if (getenv("SOL_XXH")) {
        uint64_t *o;
        CHK(hipMalloc(&o, 256 * 64 * 64 * 8));
        const int nr = 4096;
        struct X { const char *n; int act, ch, wps; } xs[] = {
            {"xxh 64 lanes, 1 chain, 1 wave/SIMD", 64, 1, 1}, {"xxh 64 lanes, 1 chain, 8 waves/SIMD", 64, 1, 8},
            {"xxh 64 lanes, 4 chains, 1 wave/SIMD", 64, 4, 1}, {"xxh 64 lanes, 4 chains, 8 waves/SIMD", 64, 4, 8},
            {"xxh 16 lanes, 4 chains, 8 waves/SIMD", 16, 4, 8}, {"xxh 32 lanes, 4 chains, 8 waves/SIMD", 32, 4, 8},
        };
        for (auto &x : xs) {
            const int grid = 256 * 4 * x.wps;
            float ms;
            if (x.act == 64 && x.ch == 1)
                ms = timeit([&] { hipLaunchKernelGGL((k_xxh<64, 1>), grid, 64, 0, 0, o, nr); }, 5);
            else if (x.act == 64)
                ms = timeit([&] { hipLaunchKernelGGL((k_xxh<64, 4>), grid, 64, 0, 0, o, nr); }, 5);
            else if (x.act == 32)
                ms = timeit([&] { hipLaunchKernelGGL((k_xxh<32, 4>), grid, 64, 0, 0, o, nr); }, 5);
            else
                ms = timeit([&] { hipLaunchKernelGGL((k_xxh<16, 4>), grid, 64, 0, 0, o, nr); }, 5);
            // cycles per round per SIMD at 2.4 GHz (rounds issued per SIMD = wps * ch * nr)
            const double cyc = ms * 1e-3 * 2.4e9 / (double(x.wps) * x.ch * nr);
            printf("%-42s %8.3f ms  %6.1f SIMD-cycles per wave-round\n", x.n, ms, cyc);
        }
        CHK(hipFree(o));
    }

    // ---- data-movement shapes
    const size_t c2S = 65536, c3S = 2048;
    uint8_t *in, *out;
    const size_t inb = c3S * C3B, outb = c3S * C3N * C3PP;
    CHK(hipMalloc(&in, inb));
    CHK(hipMalloc(&out, outb));
    CHK(hipMemset(in, 3, inb));
    CHK(hipMemset(out, 0, outb));
    const double c2bytes = double(c2S) * (C2B + C2N * C2P);
    const double c3bytes = double(c3S) * (C3B + C3N * double(C3PS));
    const double d2bytes = double(c2S) * (C2B + 2.0 * C2P);
    const double d3bytes = double(c3S) * (C3B + C3K * double(C3PS));
    constexpr int REPS = 5;
    Res res[64];
    int nv = 0;
    for (int rep = 0; rep < REPS; ++rep) {
        int i = 0;
#define RUN(NAME, BYTES, ...)                                                            \
    do {                                                                                 \
        const float ms = timeit([&] { __VA_ARGS__; });                                   \
        res[i].name = NAME;                                                              \
        res[i++].v[rep] = float((BYTES) / (ms * 1e-3) / 1e9);                            \
    } while (0)
        RUN("walk SPS1 WPS1 8/CU pat1", c3bytes, hipLaunchKernelGGL((k_walk<1, 1, 20480>), c3S, 64, 0, 0, in, out));
        RUN("walk SPS1 WPS1 8/CU pat0", c3bytes, hipLaunchKernelGGL((k_walk<1, 1, 20480, 64, 0>), c3S, 64, 0, 0, in, out));
        RUN("walk SPS2 WPS1 8/CU pat0", c3bytes, hipLaunchKernelGGL((k_walk<2, 1, 20480, 64, 0>), c3S, 64, 0, 0, in, out));
        nv = i;
    }
    for (int v = 0; v < nv; ++v) {
        float *r = res[v].v;
        for (int a = 0; a < REPS; ++a)
            for (int b = a + 1; b < REPS; ++b)
                if (r[b] < r[a]) {
                    const float t = r[a];
                    r[a] = r[b];
                    r[b] = t;
                }
        printf("%-40s median %7.1f  min %7.1f  max %7.1f GB/s\n", res[v].name, r[REPS / 2], r[0], r[REPS - 1]);
    }
    return 0;
}
