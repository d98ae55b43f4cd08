// Experiment (not product code): HBM read-rate of access patterns shaped like the Dice tile
// stream (1M files x 28 quads x 16 B = 448 MiB), to pick the resident layout.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
    if (NT) { u32x4 v = __builtin_nontemporal_load((const u32x4*)p); return make_uint4(v.x, v.y, v.z, v.w); }
    return *p;
}

// A: wave = tile, reads its WQ contiguous 1 KiB rows (current layout [tile][q][lane])
template <int WQ, bool NT>
__global__ __launch_bounds__(256) void tile_major(const uint4* __restrict__ f, long ntiles, uint4* out) {
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint4* p = f + tile * WQ * 64 + lane;
    uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < WQ; ++q) { uint4 v = ld<NT>(p + q * 64); x.x ^= v.x; x.y += v.y; x.z ^= v.z; x.w += v.w; }
    out[tile * 64 + lane] = x;
}

// B: quad-major layout [q][tile][lane]
template <int WQ, bool NT>
__global__ __launch_bounds__(256) void quad_major(const uint4* __restrict__ f, long ntiles, uint4* out) {
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint4* p = f + tile * 64 + lane;
    uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < WQ; ++q) { uint4 v = ld<NT>(p + (long)q * ntiles * 64); x.x ^= v.x; x.y += v.y; x.z ^= v.z; x.w += v.w; }
    out[tile * 64 + lane] = x;
}

// C: chunked layout [chunk of C tiles][q][tile in chunk][lane]: a workgroup's 4 waves read
// one contiguous 4 KiB span per quad step
template <int WQ, bool NT>
__global__ __launch_bounds__(256) void chunk4(const uint4* __restrict__ f, long ntiles, uint4* out) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const long tile = (long)blockIdx.x * 4 + w;
    if (tile >= ntiles) return;
    const uint4* p = f + (long)blockIdx.x * 4 * WQ * 64 + w * 64 + lane;
    uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < WQ; ++q) { uint4 v = ld<NT>(p + q * 256); x.x ^= v.x; x.y += v.y; x.z ^= v.z; x.w += v.w; }
    out[tile * 64 + lane] = x;
}

// D: flat grid-stride float4 read (copy-benchmark shape)
template <bool NT>
__global__ __launch_bounds__(256) void flat(const uint4* __restrict__ f, long nq, uint4* out) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long stride = (long)gridDim.x * 256;
    uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll 8
    for (; i < nq; i += stride) { uint4 v = ld<NT>(f + i); x.x ^= v.x; x.y += v.y; x.z ^= v.z; x.w += v.w; }
    out[(long)blockIdx.x * 256 + threadIdx.x] = x;
}

int main(int argc, char** argv) {
    const long nfiles = argc > 1 ? atol(argv[1]) : 1000000;
    constexpr int WQ = 28;
    const long ntiles = (nfiles + 63) / 64;
    const long nq = ntiles * WQ * 64;
    const size_t bytes = nq * 16;
    uint4 *f, *out;
    CK(hipMalloc(&f, bytes));
    CK(hipMalloc(&out, ntiles * 64 * 16 + (1 << 24)));
    CK(hipMemset(f, 1, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        CK(hipDeviceSynchronize());
        const int it = 50;
        CK(hipEventRecord(a));
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1000.0 / it;
        printf("%-28s %8.1f us  %6.3f TB/s\n", name, us, bytes / us * 1e-6);
    };
    const unsigned g4 = (unsigned)((ntiles + 3) / 4);
    run("tile_major", [&] { tile_major<WQ, false><<<g4, 256>>>(f, ntiles, out); });
    run("tile_major_nt", [&] { tile_major<WQ, true><<<g4, 256>>>(f, ntiles, out); });
    run("quad_major", [&] { quad_major<WQ, false><<<g4, 256>>>(f, ntiles, out); });
    run("quad_major_nt", [&] { quad_major<WQ, true><<<g4, 256>>>(f, ntiles, out); });
    run("chunk4", [&] { chunk4<WQ, false><<<g4, 256>>>(f, ntiles, out); });
    run("chunk4_nt", [&] { chunk4<WQ, true><<<g4, 256>>>(f, ntiles, out); });
    for (int g : {1024, 2048, 4096, 8192}) {
        char nm[64]; snprintf(nm, sizeof nm, "flat_g%d", g);
        run(nm, [&] { flat<false><<<g, 256>>>(f, nq, out); });
        snprintf(nm, sizeof nm, "flat_nt_g%d", g);
        run(nm, [&] { flat<true><<<g, 256>>>(f, nq, out); });
    }
    return 0;
}
