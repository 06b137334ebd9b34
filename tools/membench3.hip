// tools/membench3.hip -- the C2 encode's exact HBM access shape with the
// arithmetic stripped out, to find which aspect of the shape costs
// bandwidth.  65,536 stripes x 4 KiB blocks -> 4 parts x 2 KiB (N4K2).
// A wave owns SPW stripes; G of them are processed side by side (64/G lanes
// each); per chunk a lane handles U 16-row units (reads U x 32 B of the
// block, writes U x 16 B of each part, unit u at lane offset u*LP*16 so each
// instruction is contiguous across the stripe's lanes); next chunk's loads
// are issued before this chunk's stores (prefetch 1).  ONESHOT: every wave
// handles one chunk of its G stripes only (grid multiplied accordingly).
//   hipcc --offload-arch=gfx950 -O3 tools/membench3.hip -o tools/membench3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr uint32_t BLK = 4096, PS = 2048, N = 4, K = 2;

template <int G, int U, int SPW, bool ONESHOT>
__global__ __launch_bounds__(64) void k_shape(const uint8_t *__restrict__ blocks, uint8_t *__restrict__ parts,
                                              uint32_t nstripes)
{
    constexpr int LP = 64 / G;
    constexpr uint32_t R = LP * 16 * U;  // rows per stripe per chunk
    constexpr uint32_t CPS = PS / R;     // chunks per stripe
    const int lane = threadIdx.x, gi = lane / LP, li = lane % LP;
    uint32_t first_task, ntasks;         // task = (stripe group, chunk)
    if (ONESHOT) {
        first_task = blockIdx.x;
        ntasks = 1;
    } else {
        first_task = blockIdx.x * (SPW / G) * CPS;
        ntasks = (SPW / G) * CPS;
    }
    uint4 cur[U][2], nxt[U][2];
    auto load = [&](uint4 (&d)[U][2], uint32_t t) {
        const uint32_t grp = t / CPS, c = t % CPS;
        const uint32_t s = grp * G + gi;
        if (s >= nstripes)
            return;
        const uint8_t *b = blocks + size_t(s) * BLK + size_t(c) * R * K;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint4 *p = reinterpret_cast<const uint4 *>(b + (u * LP * 16 + li * 16) * K);
            d[u][0] = p[0];
            d[u][1] = p[1];
        }
    };
    load(cur, first_task);
    for (uint32_t i = 0; i < ntasks; ++i) {
        const uint32_t t = first_task + i;
        if (i + 1 < ntasks)
            load(nxt, t + 1);
        const uint32_t grp = t / CPS, c = t % CPS;
        const uint32_t s = grp * G + gi;
        if (s < nstripes) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int p = 0; p < int(N); ++p) {
                    uint4 v = cur[u][p & 1];
                    v.x ^= p; v.y += p;
                    *reinterpret_cast<uint4 *>(parts + (size_t(s) * N + p) * PS + size_t(c) * R + u * LP * 16 +
                                               li * 16) = v;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            cur[u][0] = nxt[u][0];
            cur[u][1] = nxt[u][1];
        }
    }
}

template <class F>
static float timeit(F f)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        f();
    float best = 1e30f;
    for (int r = 0; r < 10; ++r) {
        (void)hipEventRecord(e0, 0);
        f();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    return best;
}

int main()
{
    const uint32_t S = 65536;
    uint8_t *blocks, *parts;
    CHK(hipMalloc(&blocks, size_t(S) * BLK));
    CHK(hipMalloc(&parts, size_t(S) * N * PS));
    CHK(hipMemset(blocks, 3, size_t(S) * BLK));
    CHK(hipMemset(parts, 0, size_t(S) * N * PS));
    const double bytes = double(S) * (BLK + N * PS);
    // every shape REPS times, interleaved, median / min / max
    constexpr int REPS = 5, NV = 12;
    float res[NV][REPS];
    const char *names[NV];
#define RUN(IDX, G, U, SPW, ONE)                                                                                   \
    do {                                                                                                           \
        constexpr uint32_t R = (64 / G) * 16 * U, CPS = PS / R;                                                    \
        const uint32_t grid = ONE ? (S / G) * CPS : S / SPW;                                                       \
        float ms = timeit([&] { hipLaunchKernelGGL((k_shape<G, U, SPW, ONE>), grid, 64, 0, 0, blocks, parts, S); }); \
        res[IDX][rep] = float(bytes / (ms * 1e-3) / 1e9);                                                          \
        names[IDX] = "G=" #G " U=" #U " SPW=" #SPW " " #ONE;                                                      \
    } while (0)
    for (int rep = 0; rep < REPS; ++rep) {
        RUN(0, 4, 1, 4, false);  // today's encode shape
        RUN(1, 4, 1, 4, true);
        RUN(2, 4, 2, 4, false);
        RUN(3, 4, 4, 4, false);
        RUN(4, 4, 2, 4, true);
        RUN(5, 4, 4, 4, true);
        RUN(6, 2, 2, 2, false);
        RUN(7, 1, 1, 1, false);
        RUN(8, 1, 2, 1, false);
        RUN(9, 1, 2, 4, false);
        RUN(10, 1, 1, 1, true);
        RUN(11, 4, 1, 8, false);
    }
    for (int v = 0; v < NV; ++v) {
        float *r = res[v];
        for (int i = 0; i < REPS; ++i)
            for (int j = i + 1; j < REPS; ++j)
                if (r[j] < r[i]) {
                    float t = r[i];
                    r[i] = r[j];
                    r[j] = t;
                }
        printf("%-28s median %7.1f  min %7.1f  max %7.1f GB/s\n", names[v], r[REPS / 2], r[0], r[REPS - 1]);
    }
    return 0;
}
