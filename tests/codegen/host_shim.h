// Host shim to compile the generated sparse-program kernels (dice_program.cpp) with g++
// for CPU tests: one "lane" per call, wave votes degenerate to the lane's own value.
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
static inline bool __all(bool v) { return v; }
#define __builtin_amdgcn_sched_barrier(x) ((void)0)
struct GridDim { unsigned x; };
static GridDim gridDim = {1};
