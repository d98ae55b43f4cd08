// Wave-level helpers shared by the large-corpus kernels (dice_post.hip, dice_prune.hip):
// the strict (score, later key) order of dice.rb:39 with 24-bit exact compares inside the fast
// envelope, wave argmax, DPP prefix sums.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dice_common.h"

namespace dice {

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// "a ranks at or above b" in score order. FAST: both overlaps < 2^11 and both denominators in
// [1, 2^21) with scores < 1024 (the file and corpus envelope checked by the caller), where
// the rational compare is exact in 24-bit multiplies and equals the double order (dice_common.h).
template <bool FAST>
__device__ __forceinline__ bool ge(uint32_t oa, int32_t da, uint32_t ob, int32_t db) {
    if (FAST) return __umul24(oa, (uint32_t)db) >= __umul24(ob, (uint32_t)da);
    return dice_ge(oa, da, ob, db);
}

template <bool FAST>
__device__ __forceinline__ bool outranks_t(int32_t ai, uint32_t ao, int32_t ad, int32_t bi, uint32_t bo, int32_t bd) {
    if (ai < 0) return false;
    if (bi < 0) return true;
    const bool g = ge<FAST>(ao, ad, bo, bd), l = ge<FAST>(bo, bd, ao, ad);
    return g && (!l || ai > bi);
}

// Wave-wide argmax of (idx, ov, den) under `outranks` (butterfly over all 64 lanes).
template <bool FAST = false>
__device__ __forceinline__ void wave_best(int32_t& bi, uint32_t& bo, int32_t& bd) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const int32_t oi = __shfl_xor(bi, m);
        const uint32_t oo = (uint32_t)__shfl_xor((int)bo, m);
        const int32_t od = __shfl_xor(bd, m);
        if (outranks_t<FAST>(oi, oo, od, bi, bo, bd)) { bi = oi; bo = oo; bd = od; }
    }
}

// The same argmax by DPP (no LDS traffic: __shfl_xor is ds_bpermute): the row shifts and row
// broadcasts of wave_incl_max, with lanes that have no source keeping the identity (index -1,
// which never outranks), leave lane 63 with the best; it is then read back to every lane as
// wave-uniform values. Every lane must be active. The order is a strict total order over the
// candidates (distinct template indices), so the result is the butterfly's.
template <bool FAST = false>
__device__ __forceinline__ void wave_best_dpp(int32_t& bi, uint32_t& bo, int32_t& bd) {
#define DICE_BEST_STEP(ctrl, rows)                                                                  \
    {                                                                                               \
        const int32_t oi = __builtin_amdgcn_update_dpp(-1, bi, ctrl, rows, 0xf, false);             \
        const uint32_t oo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)bo, ctrl, rows, 0xf, false); \
        const int32_t od = __builtin_amdgcn_update_dpp(1, bd, ctrl, rows, 0xf, false);              \
        if (outranks_t<FAST>(oi, oo, od, bi, bo, bd)) {                                             \
            bi = oi;                                                                                \
            bo = oo;                                                                                \
            bd = od;                                                                                \
        }                                                                                           \
    }
    DICE_BEST_STEP(0x111, 0xf)   // row_shr:1
    DICE_BEST_STEP(0x112, 0xf)   // row_shr:2
    DICE_BEST_STEP(0x114, 0xf)   // row_shr:4
    DICE_BEST_STEP(0x118, 0xf)   // row_shr:8
    DICE_BEST_STEP(0x142, 0xa)   // row_bcast:15
    DICE_BEST_STEP(0x143, 0xc)   // row_bcast:31
#undef DICE_BEST_STEP
    bi = __builtin_amdgcn_readlane(bi, kWave - 1);
    bo = (uint32_t)__builtin_amdgcn_readlane((int32_t)bo, kWave - 1);
    bd = __builtin_amdgcn_readlane(bd, kWave - 1);
}

// Inclusive prefix sum over the 64 lanes (DPP: row shifts within each 16-lane row, then the
// row-15 / row-31 broadcasts); every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t bal) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
}

// Wave max (u32, all lanes active): the same DPP row shifts and row broadcasts as
// wave_incl_scan, so lane 63 ends with the maximum over the wave.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

}  // namespace dice
