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
// in the overlap (den > 0), so bound_t = (m_t * 200.0) / den_t >= score_t. Per file (one wave):
// the bounds (keys) of the templates that can still matter, then repeatedly the template of
// largest key scored exactly -- its records {u64 word, mask} against the file's row in LDS, one
// lane per record -- dropping every template whose key is below the best score so far, until
// none is left. A dropped template scores strictly below the winner, and every template tying
// or beating it has key >= its score, so it is scored: the winner, overlap and score are those
// of the full scan. Files whose bounds stay loose go to the postings kernels (dice_post.hip),
// which score every pair. Matrix/top-k mode keeps the postings kernels: it needs every score.
//
// Round 4 retired the superseded generations (v1/v2 dice_prune_match, v3 dice_prune3, their
// schedule switch DICE_PRUNE_SCHED and the 16-byte row-load variant); the history keeps them and
// DESIGN.md §4 their measurements.
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

// The first 128 records of a template (two per lane) are requested by records_head so their
// latency overlaps other work; score_template finishes the overlap -- one lane per record {u64
// word, mask} against the wave's file row in LDS -- takes the denominator and updates the running
// best in the strict (score, later key) order; llo becomes an f32 lower bound of the best score.
struct RecHead {
    uint4 a, b;
    uint32_t r0, r1;
};

__device__ __forceinline__ uint32_t rec_bits(const uint64_t* myrow, const uint4 a) {
    const uint64_t f = myrow[a.x];
    return (uint32_t)__builtin_popcount((uint32_t)f & a.y) + (uint32_t)__builtin_popcount((uint32_t)(f >> 32) & a.z);
}

// Keys and the exactness margin:
//   * per-template LDS constants C = {length, -max(slack, 0), 4 base - 3, sum_g A'_g}, so
//       m2 = sum_g A'_g + wv - sum_g |A'_g - F_g| = 2 m      (the v_sad_u8 chain starts at -wv:
//                                                             one v_sub_u32 after it)
//       D4 = 4 base - 3 + 4 wf + max(|len_t - len_F| - slack, 0) <= 4 den   (Ruby's floor /4)
//     and score = 200 ov / den <= 200 m / den <= 400 m2 / D4: the key is the f32 m2 / D4 with
//     its low 10 bits replaced by the template's slot (truncated, not rounded: the drop test's
//     lower bound of the best score carries the 2^-11 margin instead);
//   * files whose denominators could be 0 or whose scalars leave the plain range (len_F < 0,
//     |W_F| >= 2^28) go to the postings kernels, so the pass needs no special cases;
//   * a file whose every bound is 0 is resolved without an exact score (each kept template
//     scores 0.0 exactly; the later key wins the tie): files resembling nothing;
//   * after two exact scores, a file with more than `route_cands` templates still able to reach
//     the top goes to the postings kernels at once (stacked licenses, long notices) instead of
//     after max_evals exact scores;
//   * each wave owns a contiguous block of files: results collect in lane (file mod 64) and leave
//     as one f64 division and three coalesced stores per 64 files.
constexpr float kLloScale = 0.499755859375f;   // 0.5 (1 - 2^-11): keys are in units of score / 400

// Compile-time diagnostics (tools/build_variant.sh -DPRUNE_DIAG=n; results are wrong for 1, 2,
// 4): 1 skips the bound pass, 2 skips exact scoring, 4 re-reads the block's first row instead of
// streaming (no HBM traffic), 8 per-wave s_memtime totals of the phases, printed by the launch.
#ifndef PRUNE_DIAG
#define PRUNE_DIAG 0
#endif
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
#define PHASE(k) do { if (PRUNE_DIAG & 8) pclk.mark(k); } while (0)

// The exact denominator from the constants (dice_den: content_helper.rb:128-133,337-347).
__device__ __forceinline__ int32_t den3(const uint4 c, uint32_t wf, uint32_t lf) {
    const int32_t x = max((int32_t)__usad(c.x, lf, c.y), 0);
    return (int32_t)((c.z + 3u) >> 2) + (int32_t)wf + (x >> 2);
}

// The template of the wave's largest key K (keys hold the lane's slot j + 1): the lowest lane
// whose own maximum is K (keys of one lane are distinct; equal keys in several lanes are equal
// bounds, any of them may go first).
__device__ __forceinline__ int32_t key_template(uint32_t K, uint32_t lane_max, int32_t& kl) {
    kl = (int32_t)__builtin_ctzll(__ballot(lane_max == K));
    return kl + (int32_t)((K & kKeyLow) - 1) * kWave;
}

// records_head: one LDS read of srec[ts], srec[ts + 1] (template index | record offset
// << 10) gives the record range and the template index at once.
__device__ __forceinline__ RecHead records_head(int32_t ts, const uint32_t* srec, const uint4* __restrict__ qrec,
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

// score_template over position-ordered tables: the order compare (later key wins ties) and the
// result use the template index `to`.
__device__ __forceinline__ void score_template(int32_t ts, int32_t to, const RecHead& h, const uint4* __restrict__ qrec,
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
        // (never below its starting value: the confidence mode's threshold floor)
        llo = fmaxf(llo, (float)bo * __builtin_amdgcn_rcpf((float)bd) * kLloScale);
    }
}

// The next file's row: J2 pairs of 8-byte loads per lane (words l + 128 j and l + 64 + 128 j of
// lane l: two coalesced 512-B wave loads per pair), non-temporal (each row is read once). Word
// groups follow the layout: word p is in group (p mod 64) / 4, so a lane's words sit in one group
// and group g is lanes 4g..4g+3. (16-byte loads measured 1.30 vs 0.98 ms: removed.)
template <int J2>
__device__ __forceinline__ void row_load(uint4 (&w)[J2], const uint64_t* __restrict__ rows, int64_t file,
                                         int32_t w64, int lane) {
    const uint64_t* row = rows + file * w64;
#pragma unroll
    for (int j = 0; j < J2; ++j) {
        const int32_t p0 = lane + 2 * j * kWave, p1 = p0 + kWave;
        const uint64_t a = p0 < w64 ? __builtin_nontemporal_load(row + p0) : 0;
        const uint64_t b = p1 < w64 ? __builtin_nontemporal_load(row + p1) : 0;
        w[j] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

template <int J2>
__device__ __forceinline__ void row_store(uint64_t* myrow, const uint4 (&w)[J2], int lane) {
#pragma unroll
    for (int j = 0; j < J2; ++j) {
        myrow[lane + 2 * j * kWave] = (uint64_t)w[j].x | ((uint64_t)w[j].y << 32);
        myrow[lane + (2 * j + 1) * kWave] = (uint64_t)w[j].z | ((uint64_t)w[j].w << 32);
    }
}

// ---- the kernel: slot skipping --------------------------------------------------------------
//
// The per-pair bound above, evaluated for few templates: the host sorts the templates by length
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
// then drop / score the largest remaining key / defer. Templates of skipped slots
// score strictly below the best (SB_j, in f32 within 2^-21, < llo <= best (1 - 2^-11)).
// Tables are in position (sorted) order; srec[] maps a position to the template index that
// outputs and the tie rule (later key wins) use.
struct Prune4Args {
    const uint4* q8;       // [kTP] group bytes, by position
    const uint4* tc;       // [kTP] constants, by position
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
                                            uint32_t& bo, int32_t& bd, uint32_t& nsc, PhaseClock& pclk) {
    const int32_t t0 = lane + jstar * kWave;
    uint32_t ks = slot_key<BIG, CC, CLAMP>(q8, stc, ccm, t0, (uint32_t)(jstar + 1), T, (jstar + 1) * kWave > T, fb,
                                           negwv, m2big, lf, wf4);
    __builtin_amdgcn_wave_barrier();   // the row (written above) is read by other lanes below
    const uint32_t K1 = rfl(__builtin_amdgcn_readlane(wave_incl_max(ks), kWave - 1));
    PHASE(2);
    if ((K1 & ~kKeyLow) != 0 && !(__uint_as_float(K1 & ~kKeyLow) < llo)) {
        int32_t l1;
        const int32_t t1 = key_template(K1, ks, l1);
        if (PRUNE_DIAG & 2) {
            bi = t1;
            bd = 1;
            llo = 1e30f;
        } else {
            int32_t to;
            const RecHead h = records_head(t1, srec, pa.qrec, lane, to);
            score_template(t1, to, h, pa.qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
            ++nsc;
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
    int32_t max_evals, int32_t route_cands, float llo0, bool conf, uint32_t* __restrict__ nscored,
    uint64_t* __restrict__ diag_out) {
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
    if (PRUNE_DIAG & 8) pclk.init();
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
    uint32_t nsc = 0;          // (file, template) pairs this wave scored exactly (wave-uniform)
    if (PRUNE_DIAG & 8) pclk.mark(7);
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
        row_load<J2>(nw, rows, (PRUNE_DIAG & 4) ? wbeg : min(file + 1, wend - 1), w64, lane);
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
                // llo0: -1 (the exact top score of every file), or the confidence mode's threshold
                // floor (only templates that can reach the threshold are scored)
                float llo = llo0;
                uint32_t key[TJ], lmax;
                PHASE(1);
                if (!big && !ccf && wf >= wf_noclamp)
                    prune4_keys<TJ, false, false, false>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                         lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, nsc, pclk);
                else if (!big && !ccf)
                    prune4_keys<TJ, false, false, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                        lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, nsc, pclk);
                else if (!big)
                    prune4_keys<TJ, false, true, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                       lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, nsc, pclk);
                else if (!ccf)
                    prune4_keys<TJ, true, false, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                       lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, nsc, pclk);
                else
                    prune4_keys<TJ, true, true, true>(q8, stc, ccm, srec, pa, myrow, T, jstar, sbk, fb, negwv, m2big,
                                                      lf, wf, wf4, fast, lane, key, lmax, llo, bi, bo, bd, nsc, pclk);
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
                    const RecHead h = records_head(ts, srec, pa.qrec, lane, to);
                    score_template(ts, to, h, pa.qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
                    ++nsc;
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
                const bool hit = ri >= 0 && s >= thr;
                best_out[f] = hit ? ri : -1;
                // confidence mode: Dice#confidence outputs, 0 / 0.0 without a match
                ov_out[f] = (conf && !hit) ? 0u : ro;
                score_out[f] = (conf && !hit) ? 0.0 : s;
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
    // the wave's exact-score count, one slot per wave (dice_batch_scored_pairs sums them: no atomics)
    if (lane == 0) nscored[(int64_t)blockIdx.x * NW + wave] = nsc;
    if ((PRUNE_DIAG & 8) && diag_out && lane == 0) {
        const int64_t gw = (int64_t)blockIdx.x * NW + wave;
        for (int k = 0; k < kTPhases; ++k) diag_out[gw * (kTPhases + 1) + k] = pclk.acc[k];
        diag_out[gw * (kTPhases + 1) + kTPhases] = (uint64_t)(wend > wbeg ? wend - wbeg : 0);
    }
}


// ---- host side ---------------------------------------------------------------------------

// templates per lane (ceil(T / 64) rounded to an instantiated width) and u64 row words per lane
static int32_t prune_tj(int32_t T) {
    for (int32_t tj : {2, 4, 6, 8, 10}) if (T <= tj * kWave) return tj;
    return (kPruneMaxT + kWave - 1) / kWave;
}
static int32_t prune_j(int32_t w64) {
    const int32_t jw = (w64 + kWave - 1) / kWave;
    return jw <= 2 ? jw : jw <= 4 ? 4 : jw <= 6 ? 6 : 8;
}
// rows of ((J + 1) / 2) * 128 words per wave, the tables and the position -> template map
static size_t prune_lds_bytes(int32_t nw, int32_t w64, int32_t T) {
    const size_t tp = (size_t)prune_tj(T) * kWave;
    return (size_t)nw * ((prune_j(w64) + 1) / 2) * 2 * kWave * 8 +
           (tp * (16 + 16 + 4) + kWave * 16 + (tp + 1) * 4 + 15) / 16 * 16;
}

// candidates left after two exact scores above which a file is deferred (r3c A/B on config-3
// files, 3 reps: 16 -> 0.845 ms, 32 -> 0.878, 64 -> 0.909; long/mixed files 2.08 / 2.13 / 2.12 ms
// per 250k)
constexpr int32_t kRouteCands = 16;
// The tables of dice_prune4, in position order (templates stably sorted by length): group bytes,
// constants {length, -max(slack, 0), 4 base - 3, sum of group bytes}, CC masks, template index |
// record offset << 10, the records {u64 word index, mask lo, mask hi, 0} of every nonzero u64
// word, the per-slot bounds and the last kept template per CC flag.
int prune_setup(dice_ctx* c, const dice_templates* t) {
    const char* e = getenv("DICE_POST_PRUNE");
    if (e && *e == '0') return DICE_OK;
    const int32_t T = c->T, w64 = c->w64;
    if (T > kPruneMaxT || w64 > kPruneMaxJ * kWave || prune_lds_bytes(kPruneWaves, w64, T) > 160 * 1024)
        return DICE_OK;
    const size_t tp = (size_t)kPruneMaxT;
    std::vector<int32_t> pos2t((size_t)T);
    for (int32_t i = 0; i < T; ++i) pos2t[(size_t)i] = i;
    std::stable_sort(pos2t.begin(), pos2t.end(), [&](int32_t a, int32_t b) { return t->length[a] < t->length[b]; });
    std::vector<uint32_t> q8p(tp * 4, 0), ccp(tp, 0), offp((size_t)T + 1, 0), srec(tp + 1, 0);
    std::vector<uint4> tcp(tp, make_uint4(0, 0, 0, 0)), recp;
    bool zero_base = false;
    for (int32_t p = 0; p < T; ++p) {
        const int32_t i = pos2t[(size_t)p];
        uint32_t gc[kPruneGroups] = {0};
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        for (int32_t w = 0; w < w64; ++w) {
            if (!r[w]) continue;
            gc[(w % kWave) / (kWave / kPruneGroups)] += (uint32_t)__builtin_popcountll(r[w]);
            recp.push_back(make_uint4((uint32_t)w, (uint32_t)r[w], (uint32_t)(r[w] >> 32), 0));
        }
        uint32_t sum8 = 0;
        for (int g = 0; g < kPruneGroups; ++g) {
            const uint32_t a8 = std::min<uint32_t>(gc[g], 255u);
            sum8 += a8;
            q8p[(size_t)p * 4 + g / 4] |= a8 << (8 * (g % 4));
        }
        const int32_t slack = t->length_slack[i];
        const uint32_t base = t->lf_size[i] - t->fields_set_size[i];   // post_feasible: 0 <= base < 2^16
        zero_base = zero_base || base == 0;
        tcp[(size_t)p] = make_uint4((uint32_t)t->length[i], (uint32_t)(-std::max(slack, 0)), 4u * base - 3u, sum8);
        ccp[(size_t)p] = t->is_cc[i] ? ~0u : 0u;
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
    const int32_t nslot = prune_tj(T);
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
        return fail(DICE_E_DEVICE, "pruned-match plan upload failed");
    for (int k = 0; k < 2; ++k) {
        c->p4_zkeep[k] = zk[k];
        c->p4_zpos[k] = zp[k] < 0 ? 0 : zp[k];
    }
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
    const char* me = getenv("DICE_PRUNE_MAX_EVALS");
    c->prune_max_evals = me && *me ? std::max(0, atoi(me)) : kPruneMaxEvals;
    const char* rt = getenv("DICE_PRUNE_ROUTE");
    c->prune_route = rt && *rt ? std::min(std::max(0, atoi(rt)), 0xFFFF) : kRouteCands;
    // A/B: DICE_PRUNE_ROUTE_AT = exact scores before the routing test (default 2)
    const char* ra = getenv("DICE_PRUNE_ROUTE_AT");
    if (ra && *ra) c->prune_route |= std::min(std::max(1, atoi(ra)), 64) << 16;
    // Batches of long files go to the postings kernels whole in dice_match (top template of every
    // file): a file with more words than the largest template resembles several templates or none,
    // its bounds stay loose and it is deferred after the prune pass anyway (long/mixed files: 1.87
    // ms per 250k through the pruned kernel, 1.63 on the postings kernels alone). Routed when at
    // least 1 / DICE_PRUNE_LONG_ROUTE of the batch's files are such (default 4; 0 = never): config-3
    // files: 0.13%, long/mixed: 72%. Results are identical either way (both exact).
    c->prune_max_lf = 0;
    for (int32_t i = 0; i < T; ++i) c->prune_max_lf = std::max<uint32_t>(c->prune_max_lf, t->lf_size[i]);
    const char* lr = getenv("DICE_PRUNE_LONG_ROUTE");
    c->prune_long_route = lr && *lr ? std::max(0, atoi(lr)) : 4;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->n_cu < 1)
        c->n_cu = 256;
    c->prune = true;
    return DICE_OK;
}

template <int J, int TJ>
static int launch_prune(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, float llo0, bool conf) {
    constexpr int NW = kPruneWaves;
    const size_t lds = prune_lds_bytes(NW, c->w64, c->T);
    auto kern = dice_prune4<J, TJ, NW>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(DICE_E_DEVICE, "hipFuncSetAttribute failed");
    // persistent: as many workgroups as are resident at once, each wave a contiguous block of files
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
    if (PRUNE_DIAG & 8) {
        static uint64_t* dbuf = nullptr;
        if (!dbuf && hipMalloc(&dbuf, (size_t)groups * NW * (kTPhases + 1) * 8) != hipSuccess) dbuf = nullptr;
        diag = dbuf;
        if (diag) (void)hipMemsetAsync(diag, 0, (size_t)groups * NW * (kTPhases + 1) * 8, s);
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(NW * kWave), lds, s, (const uint64_t*)b->d_rows, b->n,
                       per_wave, c->w64, c->T, pa, b->d_wf, b->d_len, b->d_cc, thr, b->d_best, b->d_ov, b->d_score,
                       c->post_fast, c->prune_zero_base, c->prune_wf_noclamp, b->d_defer, b->d_ndefer, max_evals,
                       route, llo0, conf, b->d_nscored, diag);
    b->prune_waves = groups * NW;
    if ((PRUNE_DIAG & 8) && diag) {
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
static int launch_prune_j(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, float llo0, bool conf) {
    switch (prune_tj(c->T)) {
        case 2: return launch_prune<J, 2>(c, b, thr, s, llo0, conf);
        case 4: return launch_prune<J, 4>(c, b, thr, s, llo0, conf);
        case 6: return launch_prune<J, 6>(c, b, thr, s, llo0, conf);
        case 8: return launch_prune<J, 8>(c, b, thr, s, llo0, conf);
        case 10: return launch_prune<J, 10>(c, b, thr, s, llo0, conf);
        default: return launch_prune<J, (kPruneMaxT + kWave - 1) / kWave>(c, b, thr, s, llo0, conf);
    }
}

// Device buffers of the pruned match, allocated with the batch (dice_batch_create): deferred
// file list + count, and the postings pass's dense partials.
int prune_reserve(dice_ctx* c, dice_batch* b) {
    int rc;
    // the device list of deferred files and its length
    if (!b->d_defer && ((rc = dalloc_bytes((void**)&b->d_defer, (size_t)b->capacity * 4)) ||
                        (rc = dalloc_bytes((void**)&b->d_ndefer, 4))))
        return rc;
    // one exact-score count per wave of each persistent grid (at most 32 waves per CU each)
    if (!b->d_nscored && (rc = dalloc_bytes((void**)&b->d_nscored, (size_t)std::max(c->n_cu, 1) * 64 * 4 + 128 * 4)))
        return rc;
    return post_reserve(c, b);
}

// Dice#match over the batch, asynchronous on `s`: the pruned kernel, then the postings kernels
// over the files it deferred (their count stays on the device: persistent grids read it and
// exit at once when it is 0).
//
// confidence (dice_batch_match_confidence: Dice#match + #confidence, dice.rb:8-14,52-54): a file
// that matches nothing reports confidence 0, not its top score, so only templates that can reach
// the threshold need an exact score -- the drop level starts at the threshold (keys are in units
// of score / 400; the 2^-11 margin covers the keys' f32 evaluation as for the best score).
int prune_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, bool confidence) {
    if (b->n == 0) return DICE_OK;
    int rc;
    if ((rc = prune_reserve(c, b))) return rc;
    if (hipMemsetAsync(b->d_ndefer, 0, 4, s) != hipSuccess) return fail(DICE_E_DEVICE, "hipMemsetAsync failed");
    const float llo0 = confidence && thr > 0 ? (float)(thr / 400.0 * (1.0 - 1.0 / 2048)) : -1.0f;
    switch ((c->w64 + kWave - 1) / kWave) {
        case 1: rc = launch_prune_j<1>(c, b, thr, s, llo0, confidence); break;
        case 2: rc = launch_prune_j<2>(c, b, thr, s, llo0, confidence); break;
        case 3:
        case 4: rc = launch_prune_j<4>(c, b, thr, s, llo0, confidence); break;
        case 5:
        case 6: rc = launch_prune_j<6>(c, b, thr, s, llo0, confidence); break;
        default: rc = launch_prune_j<8>(c, b, thr, s, llo0, confidence); break;
    }
    if (rc) return rc;
    return post_launch_match_indexed(c, b, thr, b->d_defer, b->d_ndefer, s, confidence);
}

}  // namespace dice
