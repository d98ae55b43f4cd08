// Experiment (not product code): the read+write ceiling of config 5's shape. Per file: the
// 448 B tile stream in (28 quads, non-temporal loads) and 47 u32 + 47 f64 template-major
// outputs plus 3 x (i32, f64) top-k outputs (non-temporal stores) -- 1,057 B/file, the
// algorithmic bytes of dice_prog_matrix4 -- with no scoring work in between.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_matrix tools/exp/probe_matrix.hip && /tmp/probe_matrix
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                    \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int WQ, int T, int K, bool WRITE>
__global__ __launch_bounds__(256) void probe(const uint4* __restrict__ f, long ntiles, long n, uint32_t* __restrict__ ov,
                                             double* __restrict__ sc, int32_t* __restrict__ ki, double* __restrict__ ks) {
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint4* p = f + tile * WQ * 64 + lane;
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
        u32x4 v = __builtin_nontemporal_load((const u32x4*)(p + q * 64));
        x += v.x ^ v.y ^ v.z ^ v.w;
    }
    const long file = tile * 64 + lane;
    if (!WRITE) {
        if (x == 0x12345678u) ov[file] = x;
        return;
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
        __builtin_nontemporal_store(x + t, ov + (long)t * n + file);
        __builtin_nontemporal_store((double)(x ^ t), sc + (long)t * n + file);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        __builtin_nontemporal_store((int32_t)(x + k), ki + (long)k * n + file);
        __builtin_nontemporal_store((double)(x + k), ks + (long)k * n + file);
    }
}

// Reads only, the sparse program's load schedule without its VALU: bursts of B quads, the next
// burst requested before this one is consumed (2B quads in flight at most), ORDER 0 = memory
// order, 1 = zipped (27, 0, 26, 1, ...); WPB waves per workgroup.
template <int WQ, int B, int ORDER>
__device__ __forceinline__ int qidx(int i) {
    if (ORDER == 0) return i;
    return (i & 1) ? (i >> 1) : WQ - 1 - (i >> 1);
}

template <int WQ, int B, int ORDER, int PADKB = 0>
__global__ __launch_bounds__(256) void bursts(const uint4* __restrict__ f, long ntiles, uint32_t* __restrict__ out) {
    // PADKB: LDS per workgroup only to cap the occupancy (40 KB: 4 workgroups = 4 waves per SIMD,
    // the sparse program's)
    __shared__ uint32_t pad[PADKB > 0 ? PADKB * 256 : 1];
    if (PADKB > 0 && threadIdx.x == 0 && ntiles < 0) pad[0] = 0;
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint4* p = f + tile * WQ * 64 + lane;
    constexpr int NB = (WQ + B - 1) / B;
    u32x4 cur[B], nxt[B];
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < B; ++j) cur[j] = j < WQ ? __builtin_nontemporal_load((const u32x4*)(p + qidx<WQ, B, ORDER>(j) * 64)) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int i = (b + 1) * B + j;
            nxt[j] = i < WQ ? __builtin_nontemporal_load((const u32x4*)(p + qidx<WQ, B, ORDER>(i) * 64)) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < B; ++j) x += cur[j].x ^ cur[j].y ^ cur[j].z ^ cur[j].w;
#pragma unroll
        for (int j = 0; j < B; ++j) cur[j] = nxt[j];
    }
    if (x == 0x12345678u) out[tile * 64 + lane] = x;
}

// LDS-DMA on top of the VGPR bursts: the first L quads of the tile go straight to a per-wave LDS
// buffer (global_load_lds_dwordx4: no VGPRs), so 2B + L quads are in flight at the start; the VGPR
// bursts then cover the rest. (40 KB of LDS per workgroup in total: 4 waves per SIMD.)
__device__ __forceinline__ void dma16(const uint4* src, uint4* dst) {
    __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WQ, int B, int L>
__global__ __launch_bounds__(256) void bursts_lds(const uint4* __restrict__ f, long ntiles, uint32_t* __restrict__ out) {
    __shared__ uint4 buf[4][L > 0 ? L : 1][64];
    __shared__ uint32_t pad[(40 * 256 - 4 * (L > 0 ? L : 1) * 64 * 4) > 0 ? (40 * 256 - 4 * (L > 0 ? L : 1) * 64 * 4) : 1];
    if (threadIdx.x == 0 && ntiles < 0) pad[0] = 0;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const long tile = (long)blockIdx.x * 4 + w;
    if (tile >= ntiles) return;
    const uint4* p = f + tile * WQ * 64 + lane;
#pragma unroll
    for (int j = 0; j < L; ++j) dma16(p + j * 64, &buf[w][j][0]);
    constexpr int R = WQ - L;
    constexpr int NB = (R + B - 1) / B;
    u32x4 cur[B], nxt[B];
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < B; ++j) cur[j] = j < R ? __builtin_nontemporal_load((const u32x4*)(p + (L + j) * 64)) : u32x4{0, 0, 0, 0};
    wait_vm<B>();   // the L DMAs (issued first) landed
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const uint4 v = buf[w][j][lane];
        x += v.x ^ v.y ^ v.z ^ v.w;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int i = (b + 1) * B + j;
            nxt[j] = i < R ? __builtin_nontemporal_load((const u32x4*)(p + (L + i) * 64)) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < B; ++j) x += cur[j].x ^ cur[j].y ^ cur[j].z ^ cur[j].w;
#pragma unroll
        for (int j = 0; j < B; ++j) cur[j] = nxt[j];
    }
    if (x == 0x12345678u) out[tile * 64 + lane] = x;
}

template <int B, int L>
static void time_bursts_lds(const uint4* f, long ntiles, uint32_t* out, long n) {
    const dim3 grid((unsigned)((ntiles + 3) / 4)), block(256);
    for (int w = 0; w < 5; ++w) bursts_lds<28, B, L><<<grid, block>>>(f, ntiles, out);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int r = 0; r < 50; ++r) bursts_lds<28, B, L><<<grid, block>>>(f, ntiles, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / 50;
    printf("bursts of %d + %d quads by LDS-DMA (4 waves/SIMD): %.1f us, %.2f TB/s\n", B, L, us, n * 448.0 / (us * 1e-6) / 1e12);
}

template <int B, int ORDER, int PADKB = 0>
static void time_bursts(const uint4* f, long ntiles, uint32_t* out, long n) {
    const dim3 grid((unsigned)((ntiles + 3) / 4)), block(256);
    for (int w = 0; w < 5; ++w) bursts<28, B, ORDER, PADKB><<<grid, block>>>(f, ntiles, out);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int r = 0; r < 50; ++r) bursts<28, B, ORDER, PADKB><<<grid, block>>>(f, ntiles, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / 50;
    printf("bursts of %d, order %d, lds pad %d KB: %.1f us, %.2f TB/s\n", B, ORDER, PADKB, us, n * 448.0 / (us * 1e-6) / 1e12);
}

int main() {
    constexpr int WQ = 28, T = 47, K = 3;
    const long n = 1000000, ntiles = (n + 63) / 64, np = ntiles * 64;
    uint4* f;
    uint32_t* ov;
    double *sc, *ks;
    int32_t* ki;
    CK(hipMalloc(&f, (size_t)ntiles * WQ * 64 * 16));
    CK(hipMalloc(&ov, (size_t)np * T * 4));
    CK(hipMalloc(&sc, (size_t)np * T * 8));
    CK(hipMalloc(&ki, (size_t)np * K * 4));
    CK(hipMalloc(&ks, (size_t)np * K * 8));
    CK(hipMemset(f, 1, (size_t)ntiles * WQ * 64 * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const dim3 grid((unsigned)((ntiles + 3) / 4)), block(256);
    for (int mode = 0; mode < 2; ++mode) {
        for (int w = 0; w < 5; ++w) {
            if (mode) probe<WQ, T, K, true><<<grid, block>>>(f, ntiles, np, ov, sc, ki, ks);
            else probe<WQ, T, K, false><<<grid, block>>>(f, ntiles, np, ov, sc, ki, ks);
        }
        CK(hipDeviceSynchronize());
        const int reps = 50;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) {
            if (mode) probe<WQ, T, K, true><<<grid, block>>>(f, ntiles, np, ov, sc, ki, ks);
            else probe<WQ, T, K, false><<<grid, block>>>(f, ntiles, np, ov, sc, ki, ks);
        }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / reps;
        const double bytes = (double)n * (448 + (mode ? 12.0 * T + 12.0 * K : 0.0));
        printf("%s: %.1f us per launch, %.2f TB/s of %.0f MB\n", mode ? "read + matrix writes" : "read only", us,
               bytes / (us * 1e-6) / 1e12, bytes / 1e6);
    }
    time_bursts<5, 1, 40>(f, ntiles, ov, n);
    time_bursts<7, 1, 40>(f, ntiles, ov, n);
    time_bursts<28, 0, 40>(f, ntiles, ov, n);
    time_bursts_lds<5, 0>(f, ntiles, ov, n);
    time_bursts_lds<5, 4>(f, ntiles, ov, n);
    time_bursts_lds<5, 8>(f, ntiles, ov, n);
    time_bursts_lds<5, 10>(f, ntiles, ov, n);
    time_bursts<3, 0>(f, ntiles, ov, n);
    time_bursts<5, 0>(f, ntiles, ov, n);
    time_bursts<5, 1>(f, ntiles, ov, n);
    time_bursts<7, 0>(f, ntiles, ov, n);
    time_bursts<10, 0>(f, ntiles, ov, n);
    time_bursts<14, 0>(f, ntiles, ov, n);
    return 0;
}
