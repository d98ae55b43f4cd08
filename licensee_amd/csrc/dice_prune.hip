// Bound-pruned Dice#match for large template sets (kind 3, T > 64; BASELINE config 3).
//
// Same contract as every match kernel (dice.rb:8-14,34-48 over content_helper.rb:128-133,
// 337-347): per file the top template among the unmasked ones in the strict (score, later key)
// order, its overlap and f64 score, and the index when score >= threshold. Only the top
// template's score leaves the kernel, so a template whose score provably cannot reach the top
// need not be scored exactly (the MaxScore idea of inverted-index retrieval):
//
//   ov_t = |Lf_t ∩ W_F| <= m_t = sum over word groups g of min(|Lf_t ∩ g|, |W_F ∩ g|)
//
// with 16 groups of vocabulary u64 words (word p is in group (p mod 64) / 4, so a lane's words
// all fall in one group and the file's group counts are a 4-lane sum). The score is monotone
// in the overlap (den > 0), so bound_t = (m_t * 200.0) / den_t >= score_t in IEEE doubles.
// Per file (one wave): all T bounds (lanes = templates, packed u16 min/add over the groups),
// then repeatedly score exactly the template of largest bound -- its records {u64 word, mask}
// against the file's row in LDS, one lane per record -- and drop every template whose bound is
// below the best score so far, until none is left. A dropped template scores strictly below
// the winner, and every template tying or beating it has bound >= its score, so it is scored:
// the winner, overlap and score are those of the full scan. Ordering uses f32 bounds rounded
// UP (keys); only the drop test matters for correctness and it compares an upper bound of the
// bound against a lower bound of the best score. Templates with den <= 0 are never dropped.
//
// On the config-3 workload a file scores 1.4 templates exactly on average (p99 13, of 600):
// the per-file cost is the bound pass, not the overlap. Files that resemble no template (low
// best score, loose bounds) score more templates, at worst all of them -- the same records
// walk as the LDS kernel (dice_lds.hip); the results never change. Matrix/top-k mode keeps the
// postings kernels (dice_post.hip): it needs every score.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "dice_common.h"
#include "dice_internal.h"
#include "dice_wave.h"

namespace dice {

constexpr int kPruneWaves = 16;          // waves per workgroup
constexpr int kPruneGroups = 16;         // word groups of the bound
constexpr int kPruneMaxJ = 8;            // u64 words per lane: w64 <= 512 (V <= 32768)
constexpr int kPruneMaxT = 704;          // = kPostMaxTpad (the key's low 10 bits hold the template)
constexpr uint32_t kKeyLow = 1023u;
constexpr int32_t kPruneMaxEvals = 8;     // default: exact scores per file before it is deferred to the postings kernels



// The next file's independent loads, in flight while the wave works on the current file.
template <int J>
struct PruneNext {
    uint64_t w[J];
    uint32_t wf, cc;
    int32_t lf;
};

template <int J, bool TAIL2 = false>
__device__ __forceinline__ void prune_load(PruneNext<J>& nx, const uint64_t* __restrict__ rows, int64_t file,
                                           int32_t w64, const uint32_t* __restrict__ wfp,
                                           const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp,
                                           int lane) {
    const uint64_t* row = rows + file * w64;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        // TAIL2: w64 > 64 (J - 2), so only the last two word slots can run past the row
        const int32_t p = lane + j * kWave;
        nx.w[j] = (TAIL2 && j < J - 2) || p < w64 ? __builtin_nontemporal_load(row + p) : 0;
    }
    nx.wf = wfp[file];
    nx.lf = lenp[file];
    nx.cc = ccp[file];
}

// Key of a template: an f32 upper bound of (m * 200.0) / den rounded UP to the key grid, the
// template index + 1 in the low 10 bits (0 = no template). The relative error of the f32
// evaluation (conversions, v_rcp_f32, two products) is < 2^-20; the 1 + 2^-16 factor covers
// it. den == 0 gives +inf or NaN: never dropped (den < 0 cannot occur, see below).
__device__ __forceinline__ uint32_t bound_key(uint32_t m, int32_t den, uint32_t tp1) {
    const float fb = (float)m * (200.0f * 1.0000153f) * __builtin_amdgcn_rcpf((float)den);
    return ((__float_as_uint(fb) + kKeyLow) & ~kKeyLow) | tp1;
}

// Records of template ts: its first 128 (two per lane) are requested by records_head so their
// latency overlaps other work; score_template finishes the overlap -- one lane per record {u64
// word, mask} against the wave's file row in LDS -- takes the denominator and updates the running
// best in the strict (score, later key) order; llo becomes an f32 lower bound of the best score.
struct RecHead {
    uint4 a, b;
    uint32_t r0, r1;
};

__device__ __forceinline__ RecHead records_head(int32_t ts, const uint32_t* soff, const uint4* __restrict__ qrec,
                                                int lane) {
    RecHead h;
    h.r0 = rfl(soff[ts]);
    h.r1 = rfl(soff[ts + 1]);
    const uint32_t r = h.r0 + lane;
    h.a = r < h.r1 ? qrec[r] : make_uint4(0, 0, 0, 0);
    h.b = r + kWave < h.r1 ? qrec[r + kWave] : make_uint4(0, 0, 0, 0);
    return h;
}

__device__ __forceinline__ uint32_t rec_bits(const uint64_t* myrow, const uint4 a) {
    const uint64_t f = myrow[a.x];
    return (uint32_t)__builtin_popcount((uint32_t)f & a.y) + (uint32_t)__builtin_popcount((uint32_t)(f >> 32) & a.z);
}

__device__ __forceinline__ void score_template(int32_t ts, const RecHead& h, const uint4* __restrict__ qrec,
                                               const uint64_t* myrow, const uint4* stc, uint32_t wf, int32_t lf,
                                               bool fast, int lane, int32_t& bi, uint32_t& bo, int32_t& bd,
                                               float& llo) {
    uint32_t acc = rec_bits(myrow, h.a) + rec_bits(myrow, h.b);   // zero records read word 0, mask 0
    for (uint32_t r = h.r0 + 2 * kWave + lane; r < h.r1; r += 2 * kWave) {   // > 128 records
        const uint4 a = qrec[r];
        const uint4 b = r + kWave < h.r1 ? qrec[r + kWave] : make_uint4(0, 0, 0, 0);
        acc += rec_bits(myrow, a) + rec_bits(myrow, b);
    }
    const uint32_t ov = rfl(__builtin_amdgcn_readlane(wave_incl_scan(acc), kWave - 1));
    const uint4 c = stc[ts];
    const int32_t den = dice_den(make_int4((int32_t)(c.z & 0xFFFFu), (int32_t)c.w >> 16, (int32_t)c.x, 0), wf, lf);
    const bool better = fast ? outranks_t<true>(ts, ov, den, bi, bo, bd) : outranks_t<false>(ts, ov, den, bi, bo, bd);
    if (better) {
        bi = ts;
        bo = ov;
        bd = den;
        // f32 lower bound of the best score (relative error of the f32 evaluation < 2^-20, the
        // 1 - 2^-16 factor covers it); no dropping against a best with den <= 0
        llo = bd > 0 ? (float)bo * (200.0f * 0.99998474f) * __builtin_amdgcn_rcpf((float)bd) : -1.0f;
    }
}

// Per-template constants in LDS (uint4), padded to TJ * 64 templates:
//   x = length, y = -max(slack, 0) (u32), z = base (= |Lf| - |Fld|) | sum_g min(|Lf ∩ g|, 255) << 16,
//   w = keep bits (bit 0: kept for unflagged files, bit 1: for CC-flagged files; 0 = padding)
//       | slack << 16 (int16, -1 = simple delta)
// max(|len - len_F| - max(slack, 0), 0) equals the reference's adjusted delta for slack >= 0
// and the plain delta for slack = -1 (content_helper.rb:337-347; dice_den).
//
// Group-count bound m = sum_g min(A_g, F_g) (A_g = |Lf ∩ g|, F_g = |W_F ∩ g|). When every
// F_g <= 255 the byte-clamped A'_g = min(A_g, 255) give the same minima, and
// min(a, f) = (a + f - |a - f|) / 2 turns the sum into one v_sad_u8 per 4 groups:
//   m = (sum_g A'_g + sum_g F_g - sum_g |A'_g - F_g|) / 2          (16 B of table per template)
// A file with some F_g > 255 (thousands of vocabulary words) uses the looser m = |W_F ∩ V|
// (more templates are scored exactly; results are the same).
template <int J, int TJ, int NW, bool PF, int OCC, bool V2>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void dice_prune_match(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t T, const uint4* __restrict__ q8g, const uint4* __restrict__ tc, const uint32_t* __restrict__ qoff,
    const uint4* __restrict__ qrec, const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp,
    const uint8_t* __restrict__ ccp, double thr, int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out,
    double* __restrict__ score_out, bool corpus_fast, int32_t diag, int32_t* __restrict__ defer,
    uint32_t* __restrict__ ndefer, int32_t max_evals) {
    // diag (DICE_PRUNE_DIAG, diagnostics only -- results are wrong): 1 skips the bound pass (one
    // template scored), 2 skips exact scoring, 4 skips the row loads
    constexpr int kTP = TJ * kWave;   // padded template count
    // LDS: [waves][w64] file rows | [kTP] uint4 byte group counts | [kTP] constants | [T + 1]
    // record offsets (lane stride 16 B: conflict-free b128 reads)
    extern __shared__ uint64_t lds[];
    uint4* q8 = reinterpret_cast<uint4*>(lds + (size_t)NW * w64);
    uint4* stc = q8 + kTP;
    uint32_t* soff = reinterpret_cast<uint32_t*>(stc + kTP);
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    uint64_t* myrow = lds + (size_t)wave * w64;
    for (int i = threadIdx.x; i < kTP; i += NW * kWave) {
        q8[i] = q8g[i];
        stc[i] = tc[i];
    }
    for (int i = threadIdx.x; i <= T; i += NW * kWave) soff[i] = qoff[i];

    // files: wave-strided over the grid (persistent: ~2 workgroups per CU, tables loaded once)
    const int64_t f0 = (int64_t)blockIdx.x * NW + wave;
    const int64_t fstride = (int64_t)gridDim.x * NW;
    PruneNext<J> nx;
    if (PF && f0 < n) prune_load<J>(nx, rows, f0, w64, wfp, lenp, ccp, lane);
    __syncthreads();

    for (int64_t file = f0; file < n; file += fstride) {   // wave-uniform
        if (!PF) prune_load<J>(nx, rows, (diag & 4) ? (file & 63) : file, w64, wfp, lenp, ccp, lane);
        // the file's row into the wave's LDS row; per-lane bit counts
        uint32_t pc = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int32_t p = lane + j * kWave;
            if (p < w64) myrow[p] = nx.w[j];
            pc += (uint32_t)__builtin_popcountll(nx.w[j]);
        }
        const uint32_t wf = nx.wf;
        const int32_t lf = nx.lf;
        const uint32_t ccf = nx.cc != 0 ? 1u : 0u;
        if (PF && file + fstride < n) prune_load<J>(nx, rows, file + fstride, w64, wfp, lenp, ccp, lane);
        // group g = lane / 4: 4-lane sums (DPP quad_perm)
        const uint32_t pc0 = pc;
        pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
        pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
        uint32_t wv = 0, gmax = 0;
        uint32_t fb[4];   // the 16 group counts as bytes (meaningful while every count <= 255)
        if (V2) {
            // bytes packed in VGPRs by row shifts (lane 16k + 12 holds groups 4k..4k+3), then
            // 4 readlanes; |W_F ∩ V| and the largest group count by DPP reductions
            uint32_t x = pc << 24;
            x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x114, 0xf, 0xf, false) << 16;   // row_shr:4
            x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x118, 0xf, 0xf, false) << 8;    // row_shr:8
            x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x11C, 0xf, 0xf, false);         // row_shr:12
#pragma unroll
            for (int k = 0; k < 4; ++k) fb[k] = rfl(__builtin_amdgcn_readlane(x, 16 * k + 12));
            wv = rfl(__builtin_amdgcn_readlane(wave_incl_scan(pc0), kWave - 1));
            gmax = rfl(__builtin_amdgcn_readlane(wave_incl_max(pc), kWave - 1));
        } else {
            uint32_t gs[kPruneGroups];
#pragma unroll
            for (int g = 0; g < kPruneGroups; ++g) gs[g] = rfl(__builtin_amdgcn_readlane(pc, 4 * g));
#pragma unroll
            for (int g = 0; g < kPruneGroups; ++g) {
                wv += gs[g];
                gmax = max(gmax, gs[g]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                fb[k] = gs[4 * k] | (gs[4 * k + 1] << 8) | (gs[4 * k + 2] << 16) | (gs[4 * k + 3] << 24);
        }
        // a file outside the plain range (len_F < 0, |W_F| >= 2^30: never from real text) keeps
        // every template: all are scored exactly (int32 den stays as dice_den computes it)
        const bool plain = lf >= 0 && wf < (1u << 30);

        // bounds (lanes = templates t = lane + 64 j), branch-free over the padded table; each
        // lane keeps its two largest keys
        uint32_t key[TJ];
        uint32_t m1 = 0, m2 = 0;
        // uniform switches as masks (bitwise selects: no branches inside the unrolled pass, so
        // the LDS reads of later templates are issued early)
        const uint32_t bigm = gmax > 255 ? ~0u : 0u;
        const uint32_t plainm = plain ? ~0u : 0u;
        const uint32_t d1m = (diag & 1) ? ~0u : 0u;
        const float kplain = plain ? 200.0f * 1.0000153f : __builtin_inff();
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int32_t t = lane + j * kWave;
            const uint4 c = stc[t];
            const uint4 a = q8[t];
            uint32_t d = __builtin_amdgcn_sad_u8(a.x, fb[0], 0u);
            d = __builtin_amdgcn_sad_u8(a.y, fb[1], d);
            d = __builtin_amdgcn_sad_u8(a.z, fb[2], d);
            d = __builtin_amdgcn_sad_u8(a.w, fb[3], d);
            const uint32_t m = (wv & bigm) | ((((c.z >> 16) + wv - d) >> 1) & ~bigm);
            const int32_t adj = max((int32_t)__usad(c.x, (uint32_t)lf, c.y), 0);
            const int32_t den = (int32_t)((c.z & 0xFFFFu) + wf + ((uint32_t)adj >> 2));
            const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int32_t)c.w, ccf, 1);   // 0 or ~0
            const uint32_t tp1 = (uint32_t)t + 1u;
            uint32_t bk;
            if (V2) {   // a non-plain file: x inf = +inf (or NaN): never dropped
                const float fbd = fabsf((float)m * __builtin_amdgcn_rcpf((float)den)) * kplain;
                bk = ((__float_as_uint(fbd) + kKeyLow) & ~kKeyLow) | tp1;
            } else {
                bk = (bound_key(m, den, tp1) & plainm) | ((0x7F800000u | tp1) & ~plainm);
            }
            uint32_t k = keep & bk & ~d1m;
            if (j == 0) k |= (lane == 0 ? 0x7F800001u : 0u) & d1m;
            key[j] = k;
            m2 = max(m2, min(m1, k));
            m1 = max(m1, k);
        }
        // the file's row is read by other lanes below: LDS ops of a wave run in order
        __builtin_amdgcn_wave_barrier();

        const bool fast = corpus_fast && wf < (1u << 20) && lf >= 0 && lf < (1 << 21);
        int32_t bi = -1, bd = 1;
        uint32_t bo = 0;
        float llo = -1.0f;   // lower bound of the best score (f32); bounds below it are dropped
        // the largest key, scored first, and the second largest (keys are distinct): if the
        // second is below the first template's score, so is every other and the file is done
        const uint32_t K1 = rfl(__builtin_amdgcn_readlane(wave_incl_max(m1), kWave - 1));
        if (K1 != 0) {
            const int32_t t1 = (int32_t)(K1 & kKeyLow) - 1;
            const RecHead h1 = records_head(t1, soff, qrec, lane);   // in flight while K2 is found
            const uint32_t K2 = rfl(__builtin_amdgcn_readlane(wave_incl_max(m1 == K1 ? m2 : m1), kWave - 1));
            if (diag & 2) { bi = t1; bo = K2; } else
            score_template(t1, h1, qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
            if (!(diag & 2) && K2 != 0 && !(__uint_as_float(K2 & ~kKeyLow) < llo)) {
                // more templates may reach the top: drop the scored one, then score the largest
                // remaining key and drop every key below the best score, until none is left
                if (lane == (t1 & (kWave - 1))) {
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        if (j == (t1 >> 6)) key[j] = 0;
                }
                for (int32_t evals = 1;; ++evals) {
                    uint32_t km = 0;
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        if (__uint_as_float(key[j] & ~kKeyLow) < llo) key[j] = 0;
                        km = max(km, key[j]);
                    }
                    const uint32_t K = rfl(__builtin_amdgcn_readlane(wave_incl_max(km), kWave - 1));
                    if (K == 0) break;   // every template scored or dropped
                    if (evals == max_evals) {   // max_evals 0: never
                        // a file whose bounds stay loose (it resembles several templates or none:
                        // stacked licenses, long notices) goes to the postings kernels instead
                        if (lane == 0) defer[atomicAdd(ndefer, 1u)] = (int32_t)file;
                        bi = -2;
                        break;
                    }
                    const int32_t ts = (int32_t)(K & kKeyLow) - 1;
                    if (lane == (ts & (kWave - 1))) {
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            if (j == (ts >> 6)) key[j] = 0;
                    }
                    score_template(ts, records_head(ts, soff, qrec, lane), qrec, myrow, stc, wf, lf, fast, lane, bi,
                                   bo, bd, llo);
                }
            }
        }
        if (bi == -2) continue;   // deferred: its results come from the postings kernels
        if (lane == 0) {
            const double s = bi >= 0 ? dice_score(bo, bd) : 0.0;
            best_out[file] = (bi >= 0 && s >= thr) ? bi : -1;
            ov_out[file] = bo;
            score_out[file] = s;
        }
    }
}

// ---- v3: the default schedule ----------------------------------------------------------------
//
// Same bound and exactness argument as above, cheaper per (file, template) pair (16 VALU
// instead of ~28) and per file:
//   * per-template LDS constants C = {length, -max(slack, 0), 4 base - 3, sum_g A'_g}, so
//       m2 = sum_g A'_g + wv - sum_g |A'_g - F_g| = 2 m      (the v_sad_u8 chain starts at -wv:
//                                                             one v_sub_u32 after it)
//       D4 = 4 base - 3 + 4 wf + max(|len_t - len_F| - slack, 0) <= 4 den   (Ruby's floor /4)
//     and score = 200 ov / den <= 200 m / den <= 400 m2 / D4: the key is the f32 m2 / D4 with
//     its low 10 bits replaced by t + 1 (truncated, not rounded: the drop test's lower bound of
//     the best score carries the 2^-11 margin instead, so that per-pair work stays minimal);
//   * each lane keeps its two largest keys with v_med3_u32 + v_max_u32;
//   * files whose denominators could be 0 or whose scalars leave the plain range (len_F < 0,
//     |W_F| >= 2^28) go to the postings kernels, so the pass needs no special cases;
//   * a file whose every bound is 0 is resolved without an exact score (each kept template
//     scores 0.0 exactly; the later key wins the tie): files resembling nothing;
//   * after two exact scores, a file with more than `route_cands` templates still able to reach
//     the top goes to the postings kernels at once (stacked licenses, long notices) instead of
//     after max_evals exact scores (one file in twenty has a top-bound template that is not the
//     winner, so a count after the first score would defer many files the second score settles);
//   * each wave owns a contiguous block of files: results collect in lane (file mod 64) and leave
//     as one f64 division and three coalesced stores per 64 files.
constexpr float kLloScale = 0.499755859375f;   // 0.5 (1 - 2^-11): keys are in units of score / 400

// Phase-skip diagnostics of v3 (tools/build_variant.sh -DPRUNE3_DIAG=n; results are wrong):
// 1 skips the bound pass (template 0 is the only key), 2 skips exact scoring, 4 re-reads the
// block's first row instead of streaming (no HBM traffic).
#ifndef PRUNE3_DIAG
#define PRUNE3_DIAG 0
#endif
// 8: per-wave s_memtime totals of v4's phases (dice_prune4), printed by prune_launch_match
constexpr int kTPhases = 8;
struct PhaseClock {
    uint64_t acc[kTPhases];
    uint64_t last;
    __device__ __forceinline__ void init() {
        for (int k = 0; k < kTPhases; ++k) acc[k] = 0;
        last = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void mark(int k) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        acc[k] += now - last;
        last = now;
    }
};
#define PHASE(k) do { if (PRUNE3_DIAG & 8) pclk.mark(k); } while (0)

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// The exact denominator from the v3 constants (dice_den: content_helper.rb:128-133,337-347).
__device__ __forceinline__ int32_t den3(const uint4 c, uint32_t wf, uint32_t lf) {
    const int32_t x = max((int32_t)__usad(c.x, lf, c.y), 0);
    return (int32_t)((c.z + 3u) >> 2) + (int32_t)wf + (x >> 2);
}

// One pass over the lane's TJ templates (t = lane + 64 j): keys and the lane's two largest.
// BIG: some file group count exceeds a byte, m2 = 2 |W_F ∩ V| for every template. CC: the file
// is potential_false_positive? -- cc-* templates are masked (ccm = ~0 for them).
template <int TJ, bool BIG, bool CC, bool CLAMP>
__device__ __forceinline__ void bound_pass3(const uint4* q8, const uint4* stc, const uint32_t* ccm, int32_t T,
                                            const uint32_t (&fb)[4], uint32_t negwv, uint32_t m2big, uint32_t lf,
                                            uint32_t wf4, int lane, uint32_t (&key)[TJ], uint32_t& m1,
                                            uint32_t& m2) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int32_t t = lane + j * kWave;
        const uint4 c = stc[t];
        uint32_t mm;
        if (!BIG) {
            const uint4 a = q8[t];
            uint32_t d = __builtin_amdgcn_sad_u8(a.x, fb[0], negwv);
            d = __builtin_amdgcn_sad_u8(a.y, fb[1], d);
            d = __builtin_amdgcn_sad_u8(a.z, fb[2], d);
            d = __builtin_amdgcn_sad_u8(a.w, fb[3], d);
            mm = c.w - d;
        } else {
            mm = m2big;
        }
        // x = |len_t - len_F| - slack; without the clamp at 0 (|W_F| >= wf_noclamp: every D4 stays
        // >= 1) D4 is a smaller, still positive, lower bound of 4 den
        const uint32_t x0 = __usad(c.x, lf, c.y);
        const uint32_t x = CLAMP ? (uint32_t)max((int32_t)x0, 0) : x0;
        const uint32_t d4 = c.z + wf4 + x;
        const float q = (float)mm * __builtin_amdgcn_rcpf((float)d4);
        // the slot j + 1 in the low bits (a literal: no register per slot); the lane is recovered
        // from the lanes' maxima (key_lane)
        uint32_t k = (__float_as_uint(q) & ~kKeyLow) | (uint32_t)(j + 1);
        if (CC) k &= ~ccm[t];
        if (j >= TJ - 2 && (j + 1) * kWave > T) k = t < T ? k : 0u;   // padding (TJ - 2 < T / 64 by prune3_tj)
        key[j] = k;
        m2 = umed3(m1, m2, k);
        m1 = max(m1, k);
    }
}

// The template of the wave's largest key K (v3 keys hold the lane's slot j + 1): the lowest lane
// whose own maximum is K (keys of one lane are distinct; equal keys in several lanes are equal
// bounds, any of them may go first).
__device__ __forceinline__ int32_t key_template(uint32_t K, uint32_t lane_max, int32_t& kl) {
    kl = (int32_t)__builtin_ctzll(__ballot(lane_max == K));
    return kl + (int32_t)((K & kKeyLow) - 1) * kWave;
}

__device__ __forceinline__ void score_template3(int32_t ts, const RecHead& h, const uint4* __restrict__ qrec,
                                                const uint64_t* myrow, const uint4* __restrict__ tcg, uint32_t wf,
                                                uint32_t lf, bool fast, int lane, int32_t& bi, uint32_t& bo,
                                                int32_t& bd, float& llo) {
    // the template's constants by a scalar load (ts is uniform): the denominator and the order
    // compare run on the scalar unit while the records' bits are counted
    const uint4 c = tcg[ts];
    uint32_t acc = rec_bits(myrow, h.a) + rec_bits(myrow, h.b);   // zero records read word 0, mask 0
    for (uint32_t r = h.r0 + 2 * kWave + lane; r < h.r1; r += 2 * kWave) {   // > 128 records
        const uint4 a = qrec[r];
        const uint4 b = r + kWave < h.r1 ? qrec[r + kWave] : make_uint4(0, 0, 0, 0);
        acc += rec_bits(myrow, a) + rec_bits(myrow, b);
    }
    const uint32_t ov = rfl(__builtin_amdgcn_readlane(wave_incl_scan(acc), kWave - 1));
    const int32_t den = den3(c, wf, lf);
    const bool better = fast ? outranks_t<true>(ts, ov, den, bi, bo, bd) : outranks_t<false>(ts, ov, den, bi, bo, bd);
    if (better) {
        bi = ts;
        bo = ov;
        bd = den;
        // f32 lower bound of best / 400 with a 2^-11 margin (covers the keys' truncation and
        // every f32 rounding on both sides); den >= 1 on this path
        llo = (float)bo * __builtin_amdgcn_rcpf((float)bd) * kLloScale;
    }
}

template <int J, int TJ, int NW>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(8, 8))) void dice_prune3(
    const uint64_t* __restrict__ rows, int64_t n, int64_t per_wave, int32_t w64, int32_t T,
    const uint4* __restrict__ q8g, const uint4* __restrict__ tcg, const uint32_t* __restrict__ ccg,
    const uint32_t* __restrict__ qoff, const uint4* __restrict__ qrec, const uint32_t* __restrict__ wfp,
    const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp, double thr, int32_t* __restrict__ best_out,
    uint32_t* __restrict__ ov_out, double* __restrict__ score_out, bool corpus_fast, bool zero_base,
    uint32_t wf_noclamp, int32_t* __restrict__ defer, uint32_t* __restrict__ ndefer, int32_t max_evals,
    int32_t route_cands) {
    constexpr int kTP = TJ * kWave;
    // LDS: [waves][J * 64] file rows | [kTP] uint4 group bytes | [kTP] uint4 constants | [kTP] cc
    // masks | [T + 1] record offsets
    extern __shared__ uint64_t lds[];
    uint4* q8 = reinterpret_cast<uint4*>(lds + (size_t)NW * J * kWave);
    uint4* stc = q8 + kTP;
    uint32_t* ccm = reinterpret_cast<uint32_t*>(stc + kTP);
    uint32_t* soff = ccm + kTP;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    uint64_t* myrow = lds + (size_t)wave * J * kWave;
    for (int i = threadIdx.x; i < kTP; i += NW * kWave) {
        q8[i] = q8g[i];
        stc[i] = tcg[i];
        ccm[i] = ccg[i];
    }
    for (int i = threadIdx.x; i <= T; i += NW * kWave) soff[i] = qoff[i];

    // the wave's contiguous block of files
    const int64_t wbeg = ((int64_t)blockIdx.x * NW + wave) * per_wave;
    const int64_t wend = min(n, wbeg + per_wave);
    PruneNext<J> nx;
    if (wbeg < wend) prune_load<J, true>(nx, rows, wbeg, w64, wfp, lenp, ccp, lane);
    __syncthreads();

    int32_t ri = -2, rd = 1;   // lane l: result of file (block start + l); -2 = none, -3 = deferred
    uint32_t ro = 0;
    for (int64_t file = wbeg; file < wend; ++file) {   // wave-uniform
        const int slot = (int)((file - wbeg) & (kWave - 1));
        uint32_t pc = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {   // the row buffer holds J * 64 words: no bounds test
            myrow[lane + j * kWave] = nx.w[j];
            pc += (uint32_t)__builtin_popcountll(nx.w[j]);
        }
        const uint32_t wf = nx.wf;
        const int32_t lfi = nx.lf;
        const uint32_t lf = (uint32_t)lfi;
        const bool ccf = nx.cc != 0;
        // the row is in LDS and counted before the next row's loads reuse its registers (else the
        // scheduler hoists those loads above the LDS writes: 24 row VGPRs live, spills at 64)
        __builtin_amdgcn_sched_barrier(0);
        if (file + 1 < wend) prune_load<J, true>(nx, rows, (PRUNE3_DIAG & 4) ? wbeg : file + 1, w64, wfp, lenp, ccp, lane);

        int32_t bi = -1, bd = 1;
        uint32_t bo = 0;
        bool deferred = false;
        // outside the plain range, or a possible zero denominator: the postings kernels
        if (lfi < 0 || wf >= (1u << 28) || (zero_base && wf == 0)) {
            deferred = true;
        } else {
            const uint32_t pc0 = pc;
            pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
            pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
            const bool big = __ballot(pc > 255u) != 0;
            uint32_t fb[4] = {0, 0, 0, 0};
            uint32_t negwv = 0, m2big = 0;
            if (!big) {
                // group counts as bytes (lane 16k + 12 holds groups 4k..4k+3), |W_F ∩ V| by v_sad_u8
                uint32_t x = pc << 24;
                x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x114, 0xf, 0xf, false) << 16;   // row_shr:4
                x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x118, 0xf, 0xf, false) << 8;    // row_shr:8
                x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x11C, 0xf, 0xf, false);         // row_shr:12
#pragma unroll
                for (int k = 0; k < 4; ++k) fb[k] = rfl(__builtin_amdgcn_readlane(x, 16 * k + 12));
                uint32_t wv = __builtin_amdgcn_sad_u8(fb[0], 0u, 0u);
                wv = __builtin_amdgcn_sad_u8(fb[1], 0u, wv);
                wv = __builtin_amdgcn_sad_u8(fb[2], 0u, wv);
                wv = __builtin_amdgcn_sad_u8(fb[3], 0u, wv);
                negwv = 0u - wv;
            } else {
                m2big = 2u * rfl(__builtin_amdgcn_readlane(wave_incl_scan(pc0), kWave - 1));
            }
            const uint32_t wf4 = 4u * wf;
            uint32_t key[TJ];
            uint32_t m1 = 0, m2 = 0;
            if (PRUNE3_DIAG & 1) {
#pragma unroll
                for (int j = 0; j < TJ; ++j) key[j] = 0;
                key[0] = m1 = lane == 0 ? 0x3F800001u : 0u;
            } else if (!big && !ccf && wf >= wf_noclamp)
                bound_pass3<TJ, false, false, false>(q8, stc, ccm, T, fb, negwv, m2big, lf, wf4, lane, key, m1, m2);
            else if (!big && !ccf)
                bound_pass3<TJ, false, false, true>(q8, stc, ccm, T, fb, negwv, m2big, lf, wf4, lane, key, m1, m2);
            else if (!big)
                bound_pass3<TJ, false, true, true>(q8, stc, ccm, T, fb, negwv, m2big, lf, wf4, lane, key, m1, m2);
            else if (!ccf)
                bound_pass3<TJ, true, false, true>(q8, stc, ccm, T, fb, negwv, m2big, lf, wf4, lane, key, m1, m2);
            else
                bound_pass3<TJ, true, true, true>(q8, stc, ccm, T, fb, negwv, m2big, lf, wf4, lane, key, m1, m2);
            // the file's row is read by other lanes below: LDS ops of a wave run in order
            __builtin_amdgcn_wave_barrier();

            const bool fast = corpus_fast && wf < (1u << 20) && lf < (1u << 21);
            const uint32_t K1 = rfl(__builtin_amdgcn_readlane(wave_incl_max(m1), kWave - 1));
            if (K1 != 0) {   // 0: every template masked (CC filter)
                if ((K1 & ~kKeyLow) == 0) {
                    // every bound is 0: every kept template overlaps nothing and scores 0.0 (den >= 1);
                    // the later key wins the tie: the largest kept index (the highest lane in the
                    // highest slot whose key is nonzero)
                    const int32_t j1 = (int32_t)(K1 & kKeyLow) - 1;
                    const int32_t t1 = 63 - (int32_t)__builtin_clzll(__ballot(m1 == K1)) + j1 * kWave;
                    bi = t1;
                    bd = den3(tcg[t1], wf, lf);
                } else {
                    float llo = -1.0f;   // lower bound of best / 400 (f32); keys below it are dropped
                    int32_t l1;
                    const int32_t t1 = key_template(K1, m1, l1);
                    if (PRUNE3_DIAG & 2) {
                        bi = t1;
                        bd = 1;
                    } else {
                    const RecHead h1 = records_head(t1, soff, qrec, lane);   // in flight while K2 is found
                    score_template3(t1, h1, qrec, myrow, tcg, wf, lf, fast, lane, bi, bo, bd, llo);
                    // any other key still at or above the best score? (each lane's largest other
                    // key: a ballot, no wave reduction)
                    const uint32_t o1 = lane == l1 ? m2 : m1;
                    if (__ballot(o1 != 0 && !(__uint_as_float(o1) < llo)) != 0) {
                        // more templates may reach the top: score the largest remaining key and drop
                        // every key below the best score, until none is left
                        if (lane == l1) {
#pragma unroll
                            for (int j = 0; j < TJ; ++j)
                                if (j == (t1 >> 6)) key[j] = 0;
                        }
                        for (int32_t evals = 1;; ++evals) {
                            uint32_t km = 0, live = 0;
#pragma unroll
                            for (int j = 0; j < TJ; ++j) {
                                if (__uint_as_float(key[j]) < llo) key[j] = 0;
                                km = max(km, key[j]);
                                if (evals == 2) live += (uint32_t)__builtin_popcountll(__ballot(key[j] != 0));
                            }
                            const uint32_t K = rfl(__builtin_amdgcn_readlane(wave_incl_max(km), kWave - 1));
                            if (K == 0) break;   // every template scored or dropped
                            // a file whose bounds stay loose (it resembles several templates or none:
                            // stacked licenses, long notices) goes to the postings kernels: after two
                            // exact scores when more than route_cands templates can still reach the top,
                            // else after max_evals
                            if (evals == max_evals || (evals == 2 && (int32_t)live > route_cands)) {
                                deferred = true;
                                break;
                            }
                            int32_t ls;
                            const int32_t ts = key_template(K, km, ls);
                            if (lane == ls) {
#pragma unroll
                                for (int j = 0; j < TJ; ++j)
                                    if (j == (ts >> 6)) key[j] = 0;
                            }
                            score_template3(ts, records_head(ts, soff, qrec, lane), qrec, myrow, tcg, wf, lf, fast,
                                            lane, bi, bo, bd, llo);
                        }
                    }
                    }   // PRUNE3_DIAG & 2
                }
            }
        }
        if (deferred) bi = -3;
        if (lane == slot) {
            ri = bi;
            ro = bo;
            rd = bd;
        }
        if (slot == kWave - 1 || file + 1 == wend) {
            // the block's results: one division and three coalesced stores per 64 files; its
            // deferred files take one atomic for the block (a per-file atomic on the one counter
            // serialized: 2.8 ms for 250k deferred long files)
            const int64_t f = file - slot + lane;
            const bool mine = lane <= slot;
            if (mine && ri >= -1) {
                const double s = ri >= 0 ? dice_score(ro, rd) : 0.0;
                best_out[f] = (ri >= 0 && s >= thr) ? ri : -1;
                ov_out[f] = ro;
                score_out[f] = s;
            }
            const uint64_t dm = __ballot(mine && ri == -3);
            if (dm) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(ndefer, (uint32_t)__builtin_popcountll(dm));
                base = __builtin_amdgcn_readlane(base, 0);
                if (mine && ri == -3) defer[base + lane_rank(dm)] = (int32_t)f;
            }
            ri = -2;
        }
    }
}


// records_head for v4: one LDS read of srec[ts], srec[ts + 1] (template index | record offset
// << 10) gives the record range and the template index at once.
__device__ __forceinline__ RecHead records_head4(int32_t ts, const uint32_t* srec, const uint4* __restrict__ qrec,
                                                 int lane, int32_t& to) {
    RecHead h;
    const uint32_t e0 = rfl(srec[ts]), e1 = rfl(srec[ts + 1]);
    to = (int32_t)(e0 & 1023u);
    h.r0 = e0 >> 10;
    h.r1 = e1 >> 10;
    const uint32_t r = h.r0 + lane;
    h.a = r < h.r1 ? qrec[r] : make_uint4(0, 0, 0, 0);
    h.b = r + kWave < h.r1 ? qrec[r + kWave] : make_uint4(0, 0, 0, 0);
    return h;
}

// score_template3 for position-ordered tables: the order compare (later key wins ties) and the
// result use the template index `to`.
__device__ __forceinline__ void score_template4(int32_t ts, int32_t to, const RecHead& h, const uint4* __restrict__ qrec,
                                                const uint64_t* myrow, const uint4* stc,
                                                uint32_t wf, uint32_t lf, bool fast, int lane, int32_t& bi,
                                                uint32_t& bo, int32_t& bd, float& llo) {
    // constants from LDS (uniform address: a broadcast read; a scalar load would share lgkmcnt
    // with the row reads below and make them wait for it)
    const uint4 c = stc[ts];
    uint32_t acc = rec_bits(myrow, h.a) + rec_bits(myrow, h.b);   // zero records read word 0, mask 0
    for (uint32_t r = h.r0 + 2 * kWave + lane; r < h.r1; r += 2 * kWave) {   // > 128 records
        const uint4 a = qrec[r];
        const uint4 b = r + kWave < h.r1 ? qrec[r + kWave] : make_uint4(0, 0, 0, 0);
        acc += rec_bits(myrow, a) + rec_bits(myrow, b);
    }
    const uint32_t ov = rfl(__builtin_amdgcn_readlane(wave_incl_scan(acc), kWave - 1));
    const int32_t den = den3(c, wf, lf);
    const bool better = fast ? outranks_t<true>(to, ov, den, bi, bo, bd) : outranks_t<false>(to, ov, den, bi, bo, bd);
    if (better) {
        bi = to;
        bo = ov;
        bd = den;
        llo = (float)bo * __builtin_amdgcn_rcpf((float)bd) * kLloScale;
    }
}

// Row-only prefetch for v4 (the per-file scalars come per 64-file block, see dice_prune4): J2
// 16-byte loads per lane, lane l of load j holding words 2q, 2q + 1 of q = l + 64 j (a 1 KiB
// coalesced global_load_dwordx4 per wave instruction; rows are 16-byte aligned when w64 is
// even, which the host checks). The bound's word groups follow the layout: word p is in group
// ((p / 2) mod 64) / 4, so a lane's words sit in one group and group g is lanes 4g..4g+3.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// P4_ROW16 (A/B): 1 = 16-byte row loads, word groups ((w / 2) mod 64) / 4; 0 = 8-byte loads (two
// per uint4: words l + 128 j and l + 64 + 128 j of lane l), word groups (w mod 64) / 4
#ifndef P4_ROW16
#define P4_ROW16 0   // 16-byte loads measured 1.30 vs 0.98 ms (2 interleaved reps, one box): 8-byte
#endif

template <int J2>
__device__ __forceinline__ void row_load(uint4 (&w)[J2], const uint64_t* __restrict__ rows, int64_t file,
                                         int32_t w64, int lane) {
#if P4_ROW16
    const u32x4* row = reinterpret_cast<const u32x4*>(rows + file * w64);
    const int32_t w128 = w64 >> 1;
#pragma unroll
    for (int j = 0; j < J2; ++j) {
        const int32_t q = lane + j * kWave;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (q < w128) v = __builtin_nontemporal_load(row + q);
        w[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
#else
    const uint64_t* row = rows + file * w64;
#pragma unroll
    for (int j = 0; j < J2; ++j) {
        const int32_t p0 = lane + 2 * j * kWave, p1 = p0 + kWave;
        const uint64_t a = p0 < w64 ? __builtin_nontemporal_load(row + p0) : 0;
        const uint64_t b = p1 < w64 ? __builtin_nontemporal_load(row + p1) : 0;
        w[j] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
#endif
}

template <int J2>
__device__ __forceinline__ void row_store(uint64_t* myrow, const uint4 (&w)[J2], int lane) {
#pragma unroll
    for (int j = 0; j < J2; ++j) {
#if P4_ROW16
        reinterpret_cast<uint4*>(myrow)[lane + j * kWave] = w[j];
#else
        myrow[lane + 2 * j * kWave] = (uint64_t)w[j].x | ((uint64_t)w[j].y << 32);
        myrow[lane + (2 * j + 1) * kWave] = (uint64_t)w[j].z | ((uint64_t)w[j].w << 32);
#endif
    }
}

// ---- v4: slot-skipping (the default schedule) --------------------------------------------
//
// v3's per-pair bound, evaluated for few templates: the host sorts the templates by length
// (content_normalized.length) into the 64-template lane slots, so each slot covers a narrow
// length band, and keeps per slot {min length, max length, 4 min base - 3, max slack | max |Lf| << 16}.
// For every template t of slot j and any file,
//   D4_t = 4 base_t - 3 + 4 wf + max(|len_t - len_F| - slack_t, 0)
//       >= 4 bmin_j - 3 + 4 wf + max(dist(len_F, [Lmin_j, Lmax_j]) - smax_j, 0) = D4_j
//   m2_t <= 2 min(|Lf_t|, |W_F ∩ V|) <= 2 min(Mmax_j, wv)
// so SB_j = 2 min(Mmax_j, wv) / D4_j bounds every key of slot j (lanes = slots: one vector pass
// of ~13 VALU per file for all slots). Per file: the keys of the slot whose band holds len_F,
// its top template scored exactly, then only the slots with SB_j >= the best score (2.7 of 10
// on the config-3 files, numpy simulation over 4000 files: DESIGN.md) get per-template keys;
// the rest is v3 (drop / score the largest remaining key / defer). Templates of skipped slots
// score strictly below the best (SB_j, in f32 within 2^-21, < llo <= best (1 - 2^-11)).
// Tables are in position (sorted) order; orig[] maps a position to the template index that
// outputs and the tie rule (later key wins) use.
struct Prune4Args {
    const uint4* q8;       // [kTP] group bytes, by position
    const uint4* tc;       // [kTP] v3 constants, by position
    const uint32_t* ccm;   // [kTP] CC masks, by position
    const uint32_t* srec;  // [kTP + 1] template index | record offset << 10, by position
    const uint4* qrec;     // records, by position
    const uint4* slot;     // [TJ] slot bounds {Lmin, Lmax, 4 bmin - 3, smax | Mmax << 16}
    int32_t zkeep[2];      // last kept template index (file not / potential_false_positive?), -1 none
    int32_t zpos[2];       // its position
};

template <bool BIG, bool CC, bool CLAMP>
__device__ __forceinline__ uint32_t slot_key(const uint4* q8, const uint4* stc, const uint32_t* ccm, int32_t t,
                                             uint32_t tag, int32_t T, bool pad, const uint32_t (&fb)[4],
                                             uint32_t negwv, uint32_t m2big, uint32_t lf, uint32_t wf4) {
    const uint4 c = stc[t];
    uint32_t mm;
    if (!BIG) {
        const uint4 a = q8[t];
        uint32_t d = __builtin_amdgcn_sad_u8(a.x, fb[0], negwv);
        d = __builtin_amdgcn_sad_u8(a.y, fb[1], d);
        d = __builtin_amdgcn_sad_u8(a.z, fb[2], d);
        d = __builtin_amdgcn_sad_u8(a.w, fb[3], d);
        mm = c.w - d;
    } else {
        mm = m2big;
    }
    const uint32_t x0 = __usad(c.x, lf, c.y);
    const uint32_t x = CLAMP ? (uint32_t)max((int32_t)x0, 0) : x0;
    const uint32_t d4 = c.z + wf4 + x;
    const float q = (float)mm * __builtin_amdgcn_rcpf((float)d4);
    uint32_t k = (__float_as_uint(q) & ~kKeyLow) | tag;
    if (CC) k &= ~ccm[t];
    if (pad) k = t < T ? k : 0u;
    return k;
}

// Phases 1 and 2 of a file for one (BIG, CC, CLAMP) case: the keys of slot jstar, its top
// template scored exactly, then the keys of every slot whose bound reaches the best score.
// Returns with key[] filled (0 for skipped slots and the scored template) and llo / bi / bo / bd
// set; first_scored false when slot jstar had no template with a nonzero bound.
template <int TJ, bool BIG, bool CC, bool CLAMP>
__device__ __forceinline__ void prune4_keys(const uint4* q8, const uint4* stc, const uint32_t* ccm, const uint32_t* srec,
                                            const Prune4Args& pa, const uint64_t* myrow, int32_t T, int32_t jstar,
                                            uint32_t sbk, const uint32_t (&fb)[4], uint32_t negwv, uint32_t m2big,
                                            uint32_t lf, uint32_t wf, uint32_t wf4, bool fast, int lane,
                                            uint32_t (&key)[TJ], uint32_t& lane_max, float& llo, int32_t& bi,
                                            uint32_t& bo, int32_t& bd, PhaseClock& pclk) {
    const int32_t t0 = lane + jstar * kWave;
    uint32_t ks = slot_key<BIG, CC, CLAMP>(q8, stc, ccm, t0, (uint32_t)(jstar + 1), T, (jstar + 1) * kWave > T, fb,
                                           negwv, m2big, lf, wf4);
    __builtin_amdgcn_wave_barrier();   // the row (written above) is read by other lanes below
    const uint32_t K1 = rfl(__builtin_amdgcn_readlane(wave_incl_max(ks), kWave - 1));
    PHASE(2);
    if ((K1 & ~kKeyLow) != 0) {
        int32_t l1;
        const int32_t t1 = key_template(K1, ks, l1);
        if (PRUNE3_DIAG & 2) {
            bi = t1;
            bd = 1;
            llo = 1e30f;
        } else {
            int32_t to;
            const RecHead h = records_head4(t1, srec, pa.qrec, lane, to);
            score_template4(t1, to, h, pa.qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
        }
        if (lane == l1) ks = 0;
    }
    PHASE(3);
    // slots whose bound reaches the best score so far (every slot when nothing was scored)
    const uint64_t mask = __ballot(lane < TJ && !(__uint_as_float(sbk) < llo));
    lane_max = 0;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        if (j == jstar) key[j] = ks;
        else if ((mask >> j) & 1)
            key[j] = slot_key<BIG, CC, CLAMP>(q8, stc, ccm, lane + j * kWave, (uint32_t)(j + 1), T,
                                              j >= TJ - 2 && (j + 1) * kWave > T, fb, negwv, m2big, lf, wf4);
        else key[j] = 0;
        lane_max = max(lane_max, key[j]);
    }
    PHASE(4);
}

template <int J, int TJ, int NW>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(8, 8))) void dice_prune4(
    const uint64_t* __restrict__ rows, int64_t n, int64_t per_wave, int32_t w64, int32_t T, Prune4Args pa,
    const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp, double thr,
    int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out, double* __restrict__ score_out, bool corpus_fast,
    bool zero_base, uint32_t wf_noclamp, int32_t* __restrict__ defer, uint32_t* __restrict__ ndefer,
    int32_t max_evals, int32_t route_cands, uint64_t* __restrict__ diag_out) {
    constexpr int kTP = TJ * kWave;
    // route_cands packs the routing point: candidates | exact scores before the test << 16 (0: 2)
    const int32_t route_at = (route_cands >> 16) ? (route_cands >> 16) : 2;
    route_cands &= 0xFFFF;
    // LDS: the tables first (their per-slot addresses then fit the 16-bit instruction offsets: no
    // address registers per slot) -- [kTP] uint4 group bytes | [kTP] uint4 constants | [kTP] cc
    // masks | [64] slot bounds | [kTP + 1] template index | record offset << 10 -- then the
    // waves' rows of J2 * 128 words
    extern __shared__ uint64_t lds[];
    uint4* q8 = reinterpret_cast<uint4*>(lds);
    uint4* stc = q8 + kTP;
    uint32_t* ccm = reinterpret_cast<uint32_t*>(stc + kTP);
    uint4* ssb = reinterpret_cast<uint4*>(ccm + kTP);   // lanes >= TJ: empty slots
    uint32_t* srec = reinterpret_cast<uint32_t*>(ssb + kWave);
    uint64_t* rows0 = lds + (((size_t)kTP * 36 + kWave * 16 + ((size_t)kTP + 1) * 4 + 15) / 16) * 2;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    uint64_t* myrow = rows0 + (size_t)wave * ((J + 1) / 2) * 2 * kWave;
    PhaseClock pclk;
    if (PRUNE3_DIAG & 8) pclk.init();
    for (int i = threadIdx.x; i < kTP; i += NW * kWave) {
        q8[i] = pa.q8[i];
        stc[i] = pa.tc[i];
        ccm[i] = pa.ccm[i];
    }
    for (int i = threadIdx.x; i <= kTP; i += NW * kWave) srec[i] = pa.srec[i];
    if (threadIdx.x < kWave) ssb[threadIdx.x] = threadIdx.x < TJ ? pa.slot[threadIdx.x] : make_uint4(0x7FFFFFFFu, 0, 0, 0);

    const int64_t wbeg = ((int64_t)blockIdx.x * NW + wave) * per_wave;
    const int64_t wend = min(n, wbeg + per_wave);
    // per-file scalars by 64-file block: lane l holds file (block start + l), loaded one block ahead
    // by vector loads and read per file with v_readlane. (Scalar loads of the next file's |W_F| /
    // len_F share lgkmcnt with the LDS reads, whose waits then stalled on HBM latency every file.)
    // (Loads are unconditional, at clamped indices: an exec-masked load merges with the register's
    // old value, and the copy that merge needs makes the compiler wait for the load at once.)
    // cwf = min(|W_F|, 2^28) | cc << 31 (|W_F| >= 2^28 defers the file either way) and cln = len_F
    // of the current block; the next block's raw values (nwf, nln, ncc) are loaded at the block's
    // first file and packed at its last, long after they arrived.
    uint32_t cwf = 0, cln = 0, nwf = 0, nln = 0, ncc = 0;
    constexpr int J2 = (J + 1) / 2;
    uint32_t pc = 0;   // the current row's bit count per lane
    if (wbeg < wend) {
        const int64_t f0 = min(wbeg + lane, n - 1);
        cwf = min(wfp[f0], 1u << 28) | ((uint32_t)(ccp[f0] != 0) << 31);
        cln = (uint32_t)lenp[f0];
        uint4 w0[J2];
        row_load<J2>(w0, rows, wbeg, w64, lane);
        row_store<J2>(myrow, w0, lane);   // the row buffer holds J2 * 128 words: no bounds test
#pragma unroll
        for (int j = 0; j < J2; ++j)
            pc += (uint32_t)__builtin_popcount(w0[j].x) + (uint32_t)__builtin_popcount(w0[j].y) +
                  (uint32_t)__builtin_popcount(w0[j].z) + (uint32_t)__builtin_popcount(w0[j].w);
    }
    __syncthreads();

    int32_t ri = -2, rd = 1;   // lane l: result of file (block start + l); -2 = none, -3 = deferred
    uint32_t ro = 0;
    if (PRUNE3_DIAG & 8) pclk.mark(7);
    for (int64_t file = wbeg; file < wend; ++file) {   // wave-uniform
        const int slot = (int)((file - wbeg) & (kWave - 1));
        if (slot == 0) {   // the next block's scalars
            const int64_t nb = min(file + kWave + lane, n - 1);
            nwf = wfp[nb];
            nln = (uint32_t)lenp[nb];
            ncc = ccp[nb];
        }
        // the next file's row: loaded now, written to the LDS row buffer at the end of this file
        // (registers consumed in the iteration that loads them: no copies, no early wait)
        uint4 nw[J2];
        row_load<J2>(nw, rows, (PRUNE3_DIAG & 4) ? wbeg : min(file + 1, wend - 1), w64, lane);
        const uint32_t wfx = rfl(__builtin_amdgcn_readlane(cwf, slot));
        const uint32_t wf = wfx & 0x7FFFFFFFu;
        const bool ccf = (wfx >> 31) != 0;
        const int32_t lfi = (int32_t)rfl(__builtin_amdgcn_readlane(cln, slot));
        const uint32_t lf = (uint32_t)lfi;
        PHASE(0);

        int32_t bi = -1, bd = 1;
        uint32_t bo = 0;
        bool deferred = false;
        if (lfi < 0 || wf >= (1u << 28) || (zero_base && wf == 0)) {
            deferred = true;
        } else {
            const uint32_t pc0 = pc;
            pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
            pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
            const bool big = __ballot(pc > 255u) != 0;
            uint32_t fb[4] = {0, 0, 0, 0};
            uint32_t negwv = 0, m2big = 0, wv;
            if (!big) {
                uint32_t x = pc << 24;
                x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x114, 0xf, 0xf, false) << 16;   // row_shr:4
                x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x118, 0xf, 0xf, false) << 8;    // row_shr:8
                x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pc, 0x11C, 0xf, 0xf, false);         // row_shr:12
#pragma unroll
                for (int k = 0; k < 4; ++k) fb[k] = rfl(__builtin_amdgcn_readlane(x, 16 * k + 12));
                wv = __builtin_amdgcn_sad_u8(fb[0], 0u, 0u);
                wv = __builtin_amdgcn_sad_u8(fb[1], 0u, wv);
                wv = __builtin_amdgcn_sad_u8(fb[2], 0u, wv);
                wv = __builtin_amdgcn_sad_u8(fb[3], 0u, wv);
                negwv = 0u - wv;
            } else {
                wv = rfl(__builtin_amdgcn_readlane(wave_incl_scan(pc0), kWave - 1));
                m2big = 2u * wv;
            }
            if (wv == 0) {
                // no vocabulary word: every kept template overlaps nothing and scores 0.0 (den >= 1);
                // the later key wins the tie: the last kept template
                bi = pa.zkeep[ccf ? 1 : 0];
                if (bi >= 0) bd = den3(stc[pa.zpos[ccf ? 1 : 0]], wf, lf);
            } else {
                const uint32_t wf4 = 4u * wf;
                // slot bounds, lanes = slots
                const uint4 sb = ssb[lane];
                const int32_t dist = max(max((int32_t)sb.x - lfi, lfi - (int32_t)sb.y), 0);
                const uint32_t d4 = sb.z + wf4 + (uint32_t)max(dist - (int32_t)(sb.w & 0xFFFFu), 0);
                const uint32_t mmx = 2u * min(sb.w >> 16, wv);
                const uint32_t sbk = lane < TJ ? __float_as_uint((float)mmx * __builtin_amdgcn_rcpf((float)d4)) : 0u;
                // the slot whose length band holds len_F (the last slot starting at or below it)
                const uint64_t below = __ballot(lane < TJ && (int32_t)sb.x <= lfi);
                const int32_t jstar = below ? 63 - (int32_t)__builtin_clzll(below) : 0;
                const bool fast = corpus_fast && wf < (1u << 20) && lf < (1u << 21);
                float llo = -1.0f;
                uint32_t key[TJ], lmax;
                PHASE(1);
                if (!big && !ccf && wf >= wf_noclamp)
                    prune4_keys<TJ, false, false, false>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                         lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, pclk);
                else if (!big && !ccf)
                    prune4_keys<TJ, false, false, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                        lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, pclk);
                else if (!big)
                    prune4_keys<TJ, false, true, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                       lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, pclk);
                else if (!ccf)
                    prune4_keys<TJ, true, false, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                       lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, pclk);
                else
                    prune4_keys<TJ, true, true, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                      lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, pclk);
                // the largest remaining key, scored while it can reach the best score (most files:
                // no key is left at or above the best score, one compare per lane)
                if (__ballot(lmax != 0 && !(__uint_as_float(lmax) < llo)) != 0)
                for (int32_t evals = 1;; ++evals) {
                    uint32_t km = 0, live = 0;
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        if (__uint_as_float(key[j]) < llo) key[j] = 0;
                        km = max(km, key[j]);
                        if (evals == route_at) live += (uint32_t)__builtin_popcountll(__ballot(key[j] != 0));
                    }
                    if (__ballot(km != 0) == 0) break;   // every template scored or dropped
                    // a file whose bounds stay loose (it resembles several templates or none: stacked
                    // licenses, long notices) goes to the postings kernels: after two exact scores
                    // when more than route_cands templates can still reach the top, else after
                    // max_evals
                    if (evals == max_evals || (evals == route_at && (int32_t)live > route_cands)) {
                        deferred = true;
                        break;
                    }
                    const uint32_t K = rfl(__builtin_amdgcn_readlane(wave_incl_max(km), kWave - 1));
                    int32_t ls;
                    const int32_t ts = key_template(K, km, ls);
                    if (lane == ls) {
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            if (j == (ts >> 6)) key[j] = 0;
                    }
                    int32_t to;
                    const RecHead h = records_head4(ts, srec, pa.qrec, lane, to);
                    score_template4(ts, to, h, pa.qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
                }
                PHASE(5);
            }
        }
        if (deferred) bi = -3;
        if (lane == slot) {
            ri = bi;
            ro = bo;
            rd = bd;
        }
        if (slot == kWave - 1 || file + 1 == wend) {
            const int64_t f = file - slot + lane;
            const bool mine = lane <= slot;
            if (mine && ri >= -1) {
                const double s = ri >= 0 ? dice_score(ro, rd) : 0.0;
                best_out[f] = (ri >= 0 && s >= thr) ? ri : -1;
                ov_out[f] = ro;
                score_out[f] = s;
            }
            const uint64_t dm = __ballot(mine && ri == -3);
            if (dm) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(ndefer, (uint32_t)__builtin_popcountll(dm));
                base = __builtin_amdgcn_readlane(base, 0);
                if (mine && ri == -3) defer[base + lane_rank(dm)] = (int32_t)f;
            }
            ri = -2;
        }
        if (slot == kWave - 1) {   // the next block's scalars, packed (they arrived long ago)
            cwf = min(nwf, 1u << 28) | ((uint32_t)(ncc != 0) << 31);
            cln = nln;
        }
        // the next file's row into the LDS buffer (LDS ops of a wave run in order: this file's
        // reads of its row are done) and its bit counts
        pc = 0;
        row_store<J2>(myrow, nw, lane);
#pragma unroll
        for (int j = 0; j < J2; ++j)
            pc += (uint32_t)__builtin_popcount(nw[j].x) + (uint32_t)__builtin_popcount(nw[j].y) +
                  (uint32_t)__builtin_popcount(nw[j].z) + (uint32_t)__builtin_popcount(nw[j].w);
        PHASE(6);
    }
    if ((PRUNE3_DIAG & 8) && diag_out && lane == 0) {
        const int64_t gw = (int64_t)blockIdx.x * NW + wave;
        for (int k = 0; k < kTPhases; ++k) diag_out[gw * (kTPhases + 1) + k] = pclk.acc[k];
        diag_out[gw * (kTPhases + 1) + kTPhases] = (uint64_t)(wend > wbeg ? wend - wbeg : 0);
    }
}

// ---- host side ---------------------------------------------------------------------------

// the old schedules' padded template count (10 or 11 per lane), and v3's (ceil(T / 64) rounded
// to an instantiated width)
static int32_t prune_tj(int32_t T) { return T <= 640 ? 10 : (kPruneMaxT + kWave - 1) / kWave; }
static int32_t prune3_tj(int32_t T) {
    for (int32_t tj : {2, 4, 6, 8, 10}) if (T <= tj * kWave) return tj;
    return (kPruneMaxT + kWave - 1) / kWave;
}

static size_t prune_lds_bytes(int32_t nw, int32_t w64, int32_t T) {
    const size_t tp = (size_t)prune_tj(T) * kWave;
    return (size_t)nw * w64 * 8 + tp * 16 + tp * 16 + ((size_t)T + 1) * 4;
}
static int32_t prune3_j(int32_t w64) {
    const int32_t jw = (w64 + kWave - 1) / kWave;
    return jw <= 2 ? jw : jw <= 4 ? 4 : jw <= 6 ? 6 : 8;
}
// v4: rows of ((J + 1) / 2) * 128 words, the v3 tables and the position -> template map
static size_t prune4_lds_bytes(int32_t nw, int32_t w64, int32_t T) {
    const size_t tp = (size_t)prune3_tj(T) * kWave;
    return (size_t)nw * ((prune3_j(w64) + 1) / 2) * 2 * kWave * 8 +
           (tp * (16 + 16 + 4) + kWave * 16 + (tp + 1) * 4 + 15) / 16 * 16;
}
static size_t prune3_lds_bytes(int32_t nw, int32_t w64, int32_t T) {
    const size_t tp = (size_t)prune3_tj(T) * kWave;
    return (size_t)nw * prune3_j(w64) * kWave * 8 + tp * (16 + 16 + 4) + ((size_t)T + 1) * 4;
}

// candidates left after two exact scores above which a file is deferred (v3, v4; r3c A/B on
// config-3 files, 3 reps: 16 -> 0.845 ms, 32 -> 0.878, 64 -> 0.909; long/mixed files 2.08 /
// 2.13 / 2.12 ms per 250k)
constexpr int32_t kRouteCands = 16;

// v4 tables: the templates in position order (stable sort by length), the per-slot bounds and
// the position -> template map (dice_prune4).
static int prune4_setup(dice_ctx* c, const dice_templates* t, const std::vector<uint32_t>& q8,
                        const std::vector<uint4>& tc3, const std::vector<uint32_t>& cc3,
                        const std::vector<uint32_t>& qoff, const std::vector<uint4>& qrec) {
    const int32_t T = c->T;
    const size_t tp = (size_t)kPruneMaxT;
    std::vector<int32_t> pos2t((size_t)T);
    for (int32_t i = 0; i < T; ++i) pos2t[(size_t)i] = i;
    std::stable_sort(pos2t.begin(), pos2t.end(), [&](int32_t a, int32_t b) { return t->length[a] < t->length[b]; });
    std::vector<uint32_t> q8p(tp * 4, 0), ccp(tp, 0), offp((size_t)T + 1, 0), srec(tp + 1, 0);
    std::vector<uint4> tcp(tp, make_uint4(0, 0, 0, 0)), recp;
    recp.reserve(qrec.size());
    const int32_t w64 = c->w64;
    for (int32_t p = 0; p < T; ++p) {
        const int32_t i = pos2t[(size_t)p];
        // group counts in v4's word groups: word w in group ((w / 2) mod 64) / 4 (16-byte row loads)
        uint32_t gc[kPruneGroups] = {0};
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        for (int32_t w = 0; w < w64; ++w)
            gc[((P4_ROW16 ? w >> 1 : w) % kWave) / (kWave / kPruneGroups)] += (uint32_t)__builtin_popcountll(r[w]);
        uint32_t sum8 = 0;
        for (int g = 0; g < kPruneGroups; ++g) {
            const uint32_t a8 = std::min<uint32_t>(gc[g], 255u);
            sum8 += a8;
            q8p[(size_t)p * 4 + g / 4] |= a8 << (8 * (g % 4));
        }
        tcp[(size_t)p] = tc3[(size_t)i];
        tcp[(size_t)p].w = sum8;
        ccp[(size_t)p] = cc3[(size_t)i];
        recp.insert(recp.end(), qrec.begin() + qoff[(size_t)i], qrec.begin() + qoff[(size_t)i + 1]);
        offp[(size_t)p + 1] = (uint32_t)recp.size();
    }
    // template index | record offset << 10 per position (padding positions: empty ranges)
    if (recp.size() >= (1u << 22)) return fail(DICE_E_ARG, "too many template records for the pruned match");
    for (size_t p = 0; p <= tp; ++p) {
        const uint32_t off = offp[std::min<size_t>(p, (size_t)T)];
        srec[p] = (p < (size_t)T ? (uint32_t)pos2t[p] : 0u) | (off << 10);
    }
    if (recp.empty()) recp.push_back(make_uint4(0, 0, 0, 0));
    // slot bounds {Lmin, Lmax, 4 bmin - 3, smax | Mmax << 16}; an empty slot never holds len_F
    // and bounds nothing (Mmax 0)
    const int32_t nslot = prune3_tj(T);
    std::vector<uint4> slot((size_t)nslot, make_uint4(0x7FFFFFFFu, 0x7FFFFFFFu, 0, 0));
    for (int32_t j = 0; j < nslot; ++j) {
        int64_t lmin = INT64_MAX, lmax = 0, bmin = INT64_MAX, smax = 0, mmax = 0;
        for (int32_t p = j * kWave; p < std::min(T, (j + 1) * kWave); ++p) {
            const int32_t i = pos2t[(size_t)p];
            lmin = std::min<int64_t>(lmin, t->length[i]);
            lmax = std::max<int64_t>(lmax, t->length[i]);
            bmin = std::min<int64_t>(bmin, (int64_t)t->lf_size[i] - (int64_t)t->fields_set_size[i]);
            smax = std::max<int64_t>(smax, std::max(t->length_slack[i], 0));
            mmax = std::max<int64_t>(mmax, t->lf_size[i]);
        }
        if (lmin == INT64_MAX) continue;
        // post_feasible: |Lf| < 65535, slack <= 32767
        slot[(size_t)j] = make_uint4((uint32_t)lmin, (uint32_t)lmax, (uint32_t)(4 * bmin - 3),
                                     (uint32_t)smax | ((uint32_t)mmax << 16));
    }
    // the last kept template (the tie winner when every score is 0.0) for unflagged / CC-flagged files
    int32_t zk[2] = {-1, -1}, zp[2] = {-1, -1};
    for (int32_t p = 0; p < T; ++p) {
        const int32_t i = pos2t[(size_t)p];
        if (i > zk[0]) zk[0] = i, zp[0] = p;
        if (!t->is_cc[i] && i > zk[1]) zk[1] = i, zp[1] = p;
    }
    int rc;
    if ((rc = dalloc_bytes(&c->d_p4q8, q8p.size() * 4)) || (rc = dalloc_bytes(&c->d_p4tc, tcp.size() * 16)) ||
        (rc = dalloc_bytes(&c->d_p4cc, ccp.size() * 4)) || (rc = dalloc_bytes(&c->d_p4off, srec.size() * 4)) ||
        (rc = dalloc_bytes(&c->d_p4rec, recp.size() * 16)) || (rc = dalloc_bytes(&c->d_p4slot, slot.size() * 16)))
        return rc;
    if (hipMemcpy(c->d_p4q8, q8p.data(), q8p.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_p4tc, tcp.data(), tcp.size() * 16, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_p4cc, ccp.data(), ccp.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_p4off, srec.data(), srec.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_p4rec, recp.data(), recp.size() * 16, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_p4slot, slot.data(), slot.size() * 16, hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "pruned-match v4 plan upload failed");
    for (int k = 0; k < 2; ++k) {
        c->p4_zkeep[k] = zk[k];
        c->p4_zpos[k] = zp[k] < 0 ? 0 : zp[k];
    }
    return DICE_OK;
}

int prune_setup(dice_ctx* c, const dice_templates* t) {
    const char* e = getenv("DICE_POST_PRUNE");
    if (e && *e == '0') return DICE_OK;
    const int32_t T = c->T, w64 = c->w64;
    if (T > kPruneMaxT || w64 > kPruneMaxJ * kWave || prune_lds_bytes(kPruneWaves, w64, T) > 160 * 1024 ||
        prune4_lds_bytes(kPruneWaves, w64, T) > 160 * 1024)
        return DICE_OK;
    // every table padded to the largest template count (704): each schedule reads its prefix.
    // Group counts A_g = |Lf_t ∩ g| clamped to bytes; the old and the v3 constants; the v3 CC
    // masks; the records of the nonzero u64 words. Padding templates have keep bits 0.
    const size_t tp = (size_t)kPruneMaxT;
    std::vector<uint32_t> q8(tp * 4, 0);
    std::vector<uint4> tcv(tp, make_uint4(0, 0, 0, 0)), tc3(tp, make_uint4(0, 0, 0, 0));
    std::vector<uint32_t> cc3(tp, 0);
    std::vector<uint32_t> qoff((size_t)T + 1, 0);
    std::vector<uint4> qrec;
    bool zero_base = false;
    for (int32_t i = 0; i < T; ++i) {
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        uint32_t gc[kPruneGroups] = {0};
        for (int32_t p = 0; p < w64; ++p) {
            if (!r[p]) continue;
            gc[(p % kWave) / (kWave / kPruneGroups)] += (uint32_t)__builtin_popcountll(r[p]);
            qrec.push_back(make_uint4((uint32_t)p, (uint32_t)r[p], (uint32_t)(r[p] >> 32), 0));
        }
        uint32_t sum8 = 0;
        for (int g = 0; g < kPruneGroups; ++g) {
            const uint32_t a8 = std::min<uint32_t>(gc[g], 255u);
            sum8 += a8;
            q8[(size_t)i * 4 + g / 4] |= a8 << (8 * (g % 4));
        }
        qoff[(size_t)i + 1] = (uint32_t)qrec.size();
        const int32_t slack = t->length_slack[i];
        const uint32_t base = t->lf_size[i] - t->fields_set_size[i];   // post_feasible: 0 <= base < 2^16
        zero_base = zero_base || base == 0;
        tcv[(size_t)i] = make_uint4((uint32_t)t->length[i], (uint32_t)(-std::max(slack, 0)), base | (sum8 << 16),
                                    (t->is_cc[i] ? 1u : 3u) | ((uint32_t)(slack & 0xFFFF) << 16));
        tc3[(size_t)i] = make_uint4((uint32_t)t->length[i], (uint32_t)(-std::max(slack, 0)), 4u * base - 3u, sum8);
        cc3[(size_t)i] = t->is_cc[i] ? ~0u : 0u;
    }
    if (qrec.empty()) qrec.push_back(make_uint4(0, 0, 0, 0));
    int rc;
    if ((rc = dalloc_bytes(&c->d_q8, q8.size() * 4)) ||
        (rc = dalloc_bytes(&c->d_qoff, qoff.size() * 4)) ||
        (rc = dalloc_bytes(&c->d_qrec, qrec.size() * sizeof(uint4))) ||
        (rc = dalloc_bytes(&c->d_qtc, tcv.size() * sizeof(uint4))) ||
        (rc = dalloc_bytes(&c->d_q3tc, tc3.size() * sizeof(uint4))) ||
        (rc = dalloc_bytes(&c->d_q3cc, cc3.size() * 4)))
        return rc;
    if (hipMemcpy(c->d_q8, q8.data(), q8.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_qoff, qoff.data(), qoff.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_qrec, qrec.data(), qrec.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_qtc, tcv.data(), tcv.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_q3tc, tc3.data(), tc3.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_q3cc, cc3.data(), cc3.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "pruned-match plan upload failed");
    c->prune_records = (int64_t)qoff[(size_t)T];
    c->prune_zero_base = zero_base;
    // |W_F| from which D4 = 4 base - 3 + 4 wf + (|len_t - len_F| - slack) >= 1 for every template
    // without the clamp: 4 wf >= slack + 4 - 4 base
    int64_t wnc = 0;
    for (int32_t i = 0; i < T; ++i) {
        const int64_t base = (int64_t)t->lf_size[i] - (int64_t)t->fields_set_size[i];
        const int64_t need = (int64_t)std::max(t->length_slack[i], 0) + 4 - 4 * base;
        wnc = std::max<int64_t>(wnc, (need + 3) / 4);
    }
    c->prune_wf_noclamp = (uint32_t)std::min<int64_t>(wnc, 1u << 30);
    const char* sc = getenv("DICE_PRUNE_SCHED");
    c->prune_sched = sc && *sc ? atoi(sc) : 0;
    const char* me = getenv("DICE_PRUNE_MAX_EVALS");
    c->prune_max_evals = me && *me ? std::max(0, atoi(me)) : kPruneMaxEvals;
    const char* rt = getenv("DICE_PRUNE_ROUTE");
    c->prune_route = rt && *rt ? std::min(std::max(0, atoi(rt)), 0xFFFF) : kRouteCands;
    // A/B: DICE_PRUNE_ROUTE_AT = exact scores before the routing test (v4; default 2)
    const char* ra = getenv("DICE_PRUNE_ROUTE_AT");
    if (ra && *ra) c->prune_route |= std::min(std::max(1, atoi(ra)), 64) << 16;
    const char* dg = diag_env("DICE_PRUNE_DIAG");
    c->prune_diag = dg && *dg ? atoi(dg) : 0;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->n_cu < 1)
        c->n_cu = 256;
    if ((rc = prune4_setup(c, t, q8, tc3, cc3, qoff, qrec))) return rc;
    c->prune = true;
    return DICE_OK;
}

// Old schedules (DICE_PRUNE_SCHED 1-5, A/B against v3; instantiated for the config-3 shape
// only: 6 u64 words per lane, 10 or 11 templates per lane).
template <int J, int TJ, int NW, bool PF, int OCC, bool V2 = false>
static int launch_prune(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    const size_t lds = prune_lds_bytes(NW, c->w64, c->T);
    auto kern = dice_prune_match<J, TJ, NW, PF, OCC, V2>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(DICE_E_DEVICE, "hipFuncSetAttribute failed");
    // persistent grid: as many workgroups as are resident at once (LDS- and wave-limited)
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(32 / NW, (160 * 1024) / (int64_t)lds));
    const int64_t groups = std::min<int64_t>((b->n + NW - 1) / NW, per_cu * c->n_cu);
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(NW * kWave), lds, s, (const uint64_t*)b->d_rows,
                       b->n, c->w64, c->T, (const uint4*)c->d_q8, (const uint4*)c->d_qtc,
                       (const uint32_t*)c->d_qoff, (const uint4*)c->d_qrec, b->d_wf, b->d_len, b->d_cc, thr,
                       b->d_best, b->d_ov, b->d_score, c->post_fast, c->prune_diag, b->d_defer, b->d_ndefer,
                       c->prune_max_evals);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_prune_match launch failed");
}

// 1 = round 2's default (16-wave workgroups, next row prefetched, DPP-packed group counts, the
// non-plain case folded into the f32 key); 2 = 16-wave, row loads at the file; 3 = 8-wave
// workgroups, next row prefetched; 4 = 8-wave, row loads at the file; 5 = as 1 with readlane packing.
template <int TJ>
static int launch_prune_old(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    switch (c->prune_sched) {
        case 2: return launch_prune<6, TJ, 16, false, 8>(c, b, thr, s);
        case 3: return launch_prune<6, TJ, 8, true, 6>(c, b, thr, s);
        case 4: return launch_prune<6, TJ, 8, false, 8>(c, b, thr, s);
        case 5: return launch_prune<6, TJ, 16, true, 8, false>(c, b, thr, s);
        default: return launch_prune<6, TJ, 16, true, 8, true>(c, b, thr, s);
    }
}

template <int J, int TJ>
static int launch_prune3(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    constexpr int NW = kPruneWaves;
    const size_t lds = prune3_lds_bytes(NW, c->w64, c->T);
    auto kern = dice_prune3<J, TJ, NW>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(DICE_E_DEVICE, "hipFuncSetAttribute failed");
    // persistent: as many workgroups as are resident at once, each wave a contiguous block of files
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(32 / NW, (160 * 1024) / (int64_t)lds));
    const int64_t max_waves = per_cu * c->n_cu * NW;
    const int64_t per_wave = std::max<int64_t>(1, (b->n + max_waves - 1) / max_waves);
    const int64_t groups = ((b->n + per_wave - 1) / per_wave + NW - 1) / NW;
    const int32_t max_evals = c->prune_max_evals == 0 ? INT32_MAX : c->prune_max_evals;
    const int32_t route = c->prune_max_evals == 0 ? INT32_MAX : c->prune_route;
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(NW * kWave), lds, s, (const uint64_t*)b->d_rows, b->n,
                       per_wave, c->w64, c->T, (const uint4*)c->d_q8, (const uint4*)c->d_q3tc,
                       (const uint32_t*)c->d_q3cc, (const uint32_t*)c->d_qoff, (const uint4*)c->d_qrec, b->d_wf,
                       b->d_len, b->d_cc, thr, b->d_best, b->d_ov, b->d_score, c->post_fast, c->prune_zero_base,
                       c->prune_wf_noclamp, b->d_defer, b->d_ndefer, max_evals, route);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_prune3 launch failed");
}

template <int J, int TJ>
static int launch_prune4(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    constexpr int NW = kPruneWaves;
    const size_t lds = prune4_lds_bytes(NW, c->w64, c->T);
    auto kern = dice_prune4<J, TJ, NW>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(DICE_E_DEVICE, "hipFuncSetAttribute failed");
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(32 / NW, (160 * 1024) / (int64_t)lds));
    const int64_t max_waves = per_cu * c->n_cu * NW;
    const int64_t per_wave = std::max<int64_t>(1, (b->n + max_waves - 1) / max_waves);
    const int64_t groups = ((b->n + per_wave - 1) / per_wave + NW - 1) / NW;
    const int32_t max_evals = c->prune_max_evals == 0 ? INT32_MAX : c->prune_max_evals;
    const int32_t route = c->prune_max_evals == 0 ? INT32_MAX : c->prune_route;
    Prune4Args pa;
    pa.q8 = (const uint4*)c->d_p4q8;
    pa.tc = (const uint4*)c->d_p4tc;
    pa.ccm = (const uint32_t*)c->d_p4cc;
    pa.srec = (const uint32_t*)c->d_p4off;
    pa.qrec = (const uint4*)c->d_p4rec;
    pa.slot = (const uint4*)c->d_p4slot;
    for (int k = 0; k < 2; ++k) {
        pa.zkeep[k] = c->p4_zkeep[k];
        pa.zpos[k] = c->p4_zpos[k];
    }
    uint64_t* diag = nullptr;
    if (PRUNE3_DIAG & 8) {
        static uint64_t* dbuf = nullptr;
        if (!dbuf && hipMalloc(&dbuf, (size_t)groups * NW * (kTPhases + 1) * 8) != hipSuccess) dbuf = nullptr;
        diag = dbuf;
        if (diag) (void)hipMemsetAsync(diag, 0, (size_t)groups * NW * (kTPhases + 1) * 8, s);
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(NW * kWave), lds, s, (const uint64_t*)b->d_rows, b->n,
                       per_wave, c->w64, c->T, pa, b->d_wf, b->d_len, b->d_cc, thr, b->d_best, b->d_ov, b->d_score,
                       c->post_fast, c->prune_zero_base, c->prune_wf_noclamp, b->d_defer, b->d_ndefer, max_evals,
                       route, diag);
    if ((PRUNE3_DIAG & 8) && diag) {
        // diagnostic build only: per-phase shader-clock totals over all waves, per file
        std::vector<uint64_t> h((size_t)groups * NW * (kTPhases + 1));
        (void)hipMemcpyAsync(h.data(), diag, h.size() * 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        double tot[kTPhases + 1] = {0};
        for (size_t w = 0; w < (size_t)groups * NW; ++w)
            for (int k = 0; k <= kTPhases; ++k) tot[k] += (double)h[w * (kTPhases + 1) + k];
        fprintf(stderr, "[prune4 phases] cycles/file:");
        for (int k = 0; k < kTPhases; ++k) fprintf(stderr, " p%d=%.0f", k, tot[k] / std::max(1.0, tot[kTPhases]));
        fprintf(stderr, "  (files %.0f)\n", tot[kTPhases]);
    }
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_prune4 launch failed");
}

template <int J>
static int launch_prune3_j(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    if (c->prune_sched != 6 && (!P4_ROW16 || (c->w64 & 1) == 0)) {   // v4 (16-byte row loads: even w64) unless v3
        switch (prune3_tj(c->T)) {
            case 2: return launch_prune4<J, 2>(c, b, thr, s);
            case 4: return launch_prune4<J, 4>(c, b, thr, s);
            case 6: return launch_prune4<J, 6>(c, b, thr, s);
            case 8: return launch_prune4<J, 8>(c, b, thr, s);
            case 10: return launch_prune4<J, 10>(c, b, thr, s);
            default: return launch_prune4<J, (kPruneMaxT + kWave - 1) / kWave>(c, b, thr, s);
        }
    }
    switch (prune3_tj(c->T)) {
        case 2: return launch_prune3<J, 2>(c, b, thr, s);
        case 4: return launch_prune3<J, 4>(c, b, thr, s);
        case 6: return launch_prune3<J, 6>(c, b, thr, s);
        case 8: return launch_prune3<J, 8>(c, b, thr, s);
        case 10: return launch_prune3<J, 10>(c, b, thr, s);
        default: return launch_prune3<J, (kPruneMaxT + kWave - 1) / kWave>(c, b, thr, s);
    }
}

// Device buffers of the pruned match, allocated with the batch (dice_batch_create): deferred
// file list + count, and the postings pass's dense partials.
int prune_reserve(dice_ctx* c, dice_batch* b) {
    int rc;
    if (!b->d_defer && ((rc = dalloc_bytes((void**)&b->d_defer, (size_t)b->capacity * 4)) ||
                        (rc = dalloc_bytes((void**)&b->d_ndefer, 4))))
        return rc;
    return post_reserve(c, b);
}

// Dice#match over the batch, asynchronous on `s`: the pruned kernel, then the postings kernels
// over the files it deferred (their count stays on the device: persistent grids read it and
// exit at once when it is 0).
int prune_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    if (b->n == 0) return DICE_OK;
    int rc;
    if ((rc = prune_reserve(c, b))) return rc;
    if (hipMemsetAsync(b->d_ndefer, 0, 4, s) != hipSuccess) return fail(DICE_E_DEVICE, "hipMemsetAsync failed");
    const int32_t jw = (c->w64 + kWave - 1) / kWave;
    const bool old = c->prune_sched >= 1 && c->prune_sched <= 5 && (jw == 5 || jw == 6) && c->T > 576;
    if (old) {
        rc = c->T <= 640 ? launch_prune_old<10>(c, b, thr, s)
                         : launch_prune_old<(kPruneMaxT + kWave - 1) / kWave>(c, b, thr, s);
        if (rc) return rc;
        if (c->prune_max_evals == 0) return DICE_OK;   // the old schedules score every file in-kernel then
    } else {
        switch (jw) {
            case 1: rc = launch_prune3_j<1>(c, b, thr, s); break;
            case 2: rc = launch_prune3_j<2>(c, b, thr, s); break;
            case 3:
            case 4: rc = launch_prune3_j<4>(c, b, thr, s); break;
            case 5:
            case 6: rc = launch_prune3_j<6>(c, b, thr, s); break;
            default: rc = launch_prune3_j<8>(c, b, thr, s); break;
        }
        if (rc) return rc;
    }
    return post_launch_match_indexed(c, b, thr, b->d_defer, b->d_ndefer, s);
}

}  // namespace dice
