// Host shim to compile the generated sparse-program kernels (dice_program.cpp) with g++
// for CPU tests. The driver runs one "lane" per call; wave votes are wave-wide: every wave is
// run twice, a vote pass (g_vote_phase = 0: __all records the lane's value and answers true)
// and the real pass (g_vote_phase = 1: __all answers the AND over the wave's 64 lanes), so a
// wave that mixes fast and slow lanes takes the slow path for all of them, as on the GPU.
#pragma once
#include <stdint.h>
#define __global__
#define __device__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __restrict__ __restrict
struct uint4 { unsigned x, y, z, w; };
static inline uint4 make_uint4(unsigned x, unsigned y, unsigned z, unsigned w) { return {x, y, z, w}; }
struct Dim3 { unsigned x; };
static Dim3 threadIdx, blockIdx;
static int g_vote_phase = 1;
static bool g_vote_all = true;
static long long g_slow_waves = 0;   // waves whose vote came out false (real pass)
static inline bool __all(bool v) {
    if (g_vote_phase == 0) {
        g_vote_all = g_vote_all && v;
        return true;
    }
    return g_vote_all;
}
#define __builtin_amdgcn_sched_barrier(x) ((void)0)
struct GridDim { unsigned x; };
static GridDim gridDim = {1};
