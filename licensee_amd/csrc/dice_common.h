// Shared device helpers for the Dice kernels (gfx950). Formula and selection rules follow
// lib/licensee/content_helper.rb:128-133,337-347 and lib/licensee/matchers/dice.rb:34-53.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dice {

constexpr int kWave = 64;            // CDNA wavefront
constexpr int kTopKMax = 16;

// Per-template scalar constants, one int4 per template:
//   x = |Lf| - |fields_normalized_set|   (content_helper.rb:130-131)
//   y = 5*max(fields_normalized.size, spdx_alt_segments) or -1 for the simple delta (:343-345)
//   z = template content_normalized.length
//   w = creative_commons? (license.rb:209-212)
struct TplConst {
    int32_t base, slack, len, cc;
};

// Denominator of the similarity: total + variation_adjusted_length_delta / 4, where the
// Ruby Integer division floors (the operand is never negative here).
__device__ __forceinline__ int32_t dice_den(const int4 c, uint32_t wf, int32_t lenf) {
    int32_t d = c.z - lenf;
    d = d < 0 ? -d : d;
    int32_t adj = c.y < 0 ? d : (d - c.y > 0 ? d - c.y : 0);
    return c.x + (int32_t)wf + adj / 4;
}

// IEEE-754 double similarity, exactly (overlap * 200.0) / den as Ruby evaluates it.
__device__ __forceinline__ double dice_score(uint32_t ov, int32_t den) {
    return ((double)ov * 200.0) / (double)den;
}

// "a ranks at or above b": a = (ov_a, den_a), b = (ov_b, den_b) in double-score order.
// Exact rational compare when both denominators are in [1, 2^21) and both scores < 1024:
// two distinct rationals with such denominators differ by > 2^-42 > ulp(1024), so their
// doubles differ and the rational order IS the double order (ties coincide too). Outside
// that range, compare the IEEE doubles themselves.
__device__ __forceinline__ bool dice_ge(uint32_t ov_a, int32_t den_a, uint32_t ov_b, int32_t den_b) {
    const bool exact = (den_a > 0) & (den_b > 0) & (den_a < (1 << 21)) & (den_b < (1 << 21)) &
                       ((uint64_t)ov_a * 200u < ((uint64_t)den_a << 10)) &
                       ((uint64_t)ov_b * 200u < ((uint64_t)den_b << 10));
    if (exact) return (uint64_t)ov_a * (uint64_t)den_b >= (uint64_t)ov_b * (uint64_t)den_a;
    return dice_score(ov_a, den_a) >= dice_score(ov_b, den_b);
}

// Running argmax over templates visited in increasing key order; ">=" makes the later
// template win exact ties (stable ascending sort + reverse, dice.rb:39).
struct Best {
    int32_t idx;
    uint32_t ov;
    int32_t den;
    __device__ __forceinline__ void init() { idx = -1; ov = 0; den = 1; }
    __device__ __forceinline__ void offer(int32_t t, uint32_t ov_t, int32_t den_t) {
        if (idx < 0 || dice_ge(ov_t, den_t, ov, den)) { idx = t; ov = ov_t; den = den_t; }
    }
};

// Candidate a outranks b in the final order: higher score, or equal score and later key
// (a strict total order over distinct templates: any reduction order gives the same winner).
__device__ __forceinline__ bool outranks(int32_t ai, uint32_t ao, int32_t ad, int32_t bi, uint32_t bo, int32_t bd) {
    if (ai < 0) return false;
    if (bi < 0) return true;
    const bool ge = dice_ge(ao, ad, bo, bd), le = dice_ge(bo, bd, ao, ad);
    return ge && (!le || ai > bi);
}

// Top-k over KM register slots, sorted best-first: rank-and-shift insertion with selects only
// (p = slots strictly outranking the candidate; a later template goes before equal-scored
// earlier ones, dice.rb:39). Slots past the caller's k hold lower-ranked valid entries.
template <int KM>
struct TopK {
    int32_t idx[KM];
    uint32_t ov[KM];
    int32_t den[KM];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < KM; ++j) { idx[j] = -1; ov[j] = 0; den[j] = 1; }
    }
    __device__ __forceinline__ void offer(int32_t t, uint32_t o, int32_t d) {
        int p = 0;
#pragma unroll
        for (int j = 0; j < KM; ++j) p += (idx[j] >= 0 && !dice_ge(o, d, ov[j], den[j])) ? 1 : 0;
#pragma unroll
        for (int j = KM - 1; j > 0; --j) {
            const bool mv = j > p;
            idx[j] = mv ? idx[j - 1] : idx[j];
            ov[j] = mv ? ov[j - 1] : ov[j];
            den[j] = mv ? den[j - 1] : den[j];
        }
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const bool put = j == p;
            idx[j] = put ? t : idx[j];
            ov[j] = put ? o : ov[j];
            den[j] = put ? d : den[j];
        }
    }
};

}  // namespace dice
