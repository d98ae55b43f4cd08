// Experiment (not product code): tile-stream read rate under Dice-like compute, for load
// scheduling patterns (ring prefetch depth, bursts, non-temporal). 1M files x 28 quads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
constexpr int WQ = 28;
constexpr int NACC = 48;

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
    if (NT) { u32x4 v = __builtin_nontemporal_load((const u32x4*)p); return make_uint4(v.x, v.y, v.z, v.w); }
    return *p;
}

template <int OPS>
__device__ __forceinline__ void work(u32 (&acc)[NACC], uint4 v, int q) {
    const u32 f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < OPS / 2; ++k) {
        u32 t;
        asm volatile("v_and_b32 %1, %2, %3\n\tv_bcnt_u32_b32 %0, %1, %0" : "+v"(acc[(k + q * 7) % NACC]), "=&v"(t)
                     : "v"(f[k % 4]), "s"(0x9e3779b9u * (k + 1)));
    }
}

// ring: prefetch distance PD, one load issued per consumed quad (steps unrolled by template)
template <int PD, bool NT, int OPS, int Q>
__device__ __forceinline__ void ring_step(u32 (&acc)[NACC], uint4 (&r)[PD], const uint4* p) {
    if constexpr (Q < WQ) {
        const uint4 v = r[Q % PD];
        if constexpr (Q + PD < WQ) r[Q % PD] = ld<NT>(p + (Q + PD) * 64);
        __builtin_amdgcn_sched_barrier(0);
        work<OPS>(acc, v, Q);
        ring_step<PD, NT, OPS, Q + 1>(acc, r, p);
    }
}

template <int EPI>
__device__ __forceinline__ u32 epilogue(u32 (&acc)[NACC], u32 wf) {
    u32 best = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
        u32 d = acc[i] * 3u + wf;
#pragma unroll
        for (int k = 0; k < EPI; ++k) d = ((d & 0xffffffu) * (0x1234u + k)) ^ acc[i];
        best = best > d ? best : d;
    }
    return best;
}

template <int PD, bool NT, int OPS, int EPI>
__global__ __launch_bounds__(256) void ring(const uint4* __restrict__ fl, long ntiles, u32* out) {
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint4* p = fl + tile * WQ * 64 + lane;
    u32 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0;
    uint4 r[PD];
#pragma unroll
    for (int i = 0; i < PD; ++i) r[i] = ld<NT>(p + i * 64);
    __builtin_amdgcn_sched_barrier(0);
    ring_step<PD, NT, OPS, 0>(acc, r, p);
    out[tile * 64 + lane] = epilogue<EPI>(acc, lane);
}

// burst: groups of B quads, double-buffered (load group g+1, then compute group g)
template <int B, bool NT, int OPS, int EPI>
__global__ __launch_bounds__(256) void burst(const uint4* __restrict__ fl, long ntiles, u32* out) {
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint4* p = fl + tile * WQ * 64 + lane;
    u32 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0;
    constexpr int NG = (WQ + B - 1) / B;
    uint4 a[B], b[B];
#pragma unroll
    for (int i = 0; i < B; ++i) a[i] = i < WQ ? ld<NT>(p + i * 64) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const int q = (g + 1) * B + i;
            if (q < WQ) b[i] = ld<NT>(p + q * 64);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < B; ++i)
            if (g * B + i < WQ) work<OPS>(acc, a[i], g * B + i);
#pragma unroll
        for (int i = 0; i < B; ++i) a[i] = b[i];
    }
    out[tile * 64 + lane] = epilogue<EPI>(acc, lane);
}

// multi-tile burst: each wave scores NTILE consecutive tiles; the group stream runs across tile
// boundaries, so the next tile's first group is in flight during the previous epilogue.
template <int B, bool NT, int OPS, int EPI, int NTILE>
__global__ __launch_bounds__(256) void burst_mt(const uint4* __restrict__ fl, long ntiles, u32* out) {
    const int lane = threadIdx.x & 63;
    const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long t0 = w * NTILE;
    if (t0 >= ntiles) return;
    constexpr int NG = (WQ + B - 1) / B;
    uint4 a[B], b[B];
    const uint4* p = fl + t0 * WQ * 64 + lane;
#pragma unroll
    for (int i = 0; i < B; ++i) a[i] = i < WQ ? ld<NT>(p + i * 64) : make_uint4(0, 0, 0, 0);
    for (int tt = 0; tt < NTILE; ++tt) {
        const long tile = t0 + tt;
        if (tile >= ntiles) break;
        const bool more = tt + 1 < NTILE && tile + 1 < ntiles;
        const uint4* pn = p + WQ * 64;
        u32 acc[NACC];
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = 0;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            if (g + 1 < NG) {
#pragma unroll
                for (int i = 0; i < B; ++i) {
                    const int q = (g + 1) * B + i;
                    if (q < WQ) b[i] = ld<NT>(p + q * 64);
                }
            } else if (more) {
#pragma unroll
                for (int i = 0; i < B; ++i) b[i] = ld<NT>(pn + i * 64);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < B; ++i)
                if (g * B + i < WQ) work<OPS>(acc, a[i], g * B + i);
#pragma unroll
            for (int i = 0; i < B; ++i) a[i] = b[i];
        }
        out[tile * 64 + lane] = epilogue<EPI>(acc, lane);
        p = pn;
    }
}

int main(int argc, char** argv) {
    const long nfiles = argc > 1 ? atol(argv[1]) : 1000000;
    const long ntiles = (nfiles + 63) / 64;
    const size_t bytes = (size_t)ntiles * WQ * 64 * 16;
    uint4* f; u32* out;
    CK(hipMalloc(&f, bytes));
    CK(hipMalloc(&out, ntiles * 64 * 4));
    CK(hipMemset(f, 0x5a, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const unsigned g4 = (unsigned)((ntiles + 3) / 4);
    auto run = [&](const char* name, auto kern, int ntile = 1) {
        const unsigned g = (unsigned)((ntiles + 4 * ntile - 1) / (4 * ntile));
        hipFuncAttributes at; CK(hipFuncGetAttributes(&at, (const void*)kern));
        for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, f, ntiles, out);
        CK(hipDeviceSynchronize());
        const int it = 40;
        CK(hipEventRecord(a));
        for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, f, ntiles, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1000.0 / it;
        printf("%-24s vgpr %3d  %8.1f us  %6.3f TB/s\n", name, at.numRegs, us, bytes / us * 1e-6);
    };
    run("burst4_nt_ops96_e8", burst<4, true, 96, 8>);
    run("burst7_nt_ops96_e8", burst<7, true, 96, 8>);
    run("mt2_b4_nt_e8", burst_mt<4, true, 96, 8, 2>, 2);
    run("mt2_b7_nt_e8", burst_mt<7, true, 96, 8, 2>, 2);
    run("mt4_b4_nt_e8", burst_mt<4, true, 96, 8, 4>, 4);
    run("mt4_b7_nt_e8", burst_mt<7, true, 96, 8, 4>, 4);
    run("mt2_b4_e8", burst_mt<4, false, 96, 8, 2>, 2);
    run("mt2_b4_nt_e0", burst_mt<4, true, 96, 0, 2>, 2);
    return 0;
}
