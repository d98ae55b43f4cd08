// Postings scorer for large template sets (T > 64, BASELINE config 3: ~600 templates).
//
// Same contract as the other Dice kernels (dice.rb:34-53 over content_helper.rb:128-133,
// 337-347): per file the argmax template among the unmasked ones, its overlap and f64 score,
// or the full row of T overlaps/scores plus the top-k.
//
// Why: at T ~ 600 a template u64 word holds ~5 of its 64 bits, so the record kernel
// (dice_lds.hip) spends 8 LDS cycles and 8 VALU per (record, 2 files) on mostly-empty masks,
// and ~51k records per file at 600 templates. Most words are NARROW: they occur in a handful
// of templates. Scoring a file by its words instead -- each narrow word present in the file
// adds 1 to the counter of every template on its postings list (the inverted index of the
// template word sets) -- costs ~2k counter increments per file instead. The few WIDE words
// (in hundreds of templates) stay bitset-scored: the vocabulary's first D u64 words (the host
// packs the widest words first) are ANDed against dense template masks.
//
// One workgroup = 16 waves = one tile of 64 files:
//   phase 1 (dense prefix, lanes = files): wave w scores templates [w*TW, (w+1)*TW) over the
//            files' first D u64 words (template masks uniform: scalar loads), writing the
//            partial overlaps to a u16 counter matrix in LDS, [file][template] (row stride
//            tpad + 2 halves: conflict-free for both access patterns below);
//   phase 2 (narrow words, one file per wave): lanes read the file's remaining u64 words; each
//            set bit is a word whose postings rows (16 template ids per row, 0xFFFF padding)
//            are queued in a per-wave LDS list; a group of 16 lanes walks one queued word's
//            rows and adds 1 to each listed template's counter (ds_add_u32 on the u16 pair);
//   phase 3 (score, lanes = templates): t = lane + 64 j: overlap from LDS, denominator from
//            the template constants, running best per lane, then a wave reduction (the same
//            strict order as every other kernel: score, then later key); the matrix mode
//            writes the row-major [n][T] row and the top-k.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "dice_common.h"
#include "dice_internal.h"

namespace dice {

constexpr int kPostWaves = 16;
constexpr int kPostFiles = 64;           // files per workgroup (one tile)
constexpr int kPostMaxTpad = 768;        // LDS budget of the counter matrix
constexpr int kPostMaxDense = 16;        // dense prefix u64 words
constexpr int kRowW = 16;                // template ids per postings row
constexpr int kWordCap = 192;            // per-wave queue of (row start, rows)
constexpr uint16_t kNoTpl = 0xFFFF;

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-wide argmax of (idx, ov, den) under `outranks` (butterfly over all 64 lanes).
__device__ __forceinline__ void wave_best(int32_t& bi, uint32_t& bo, int32_t& bd) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const int32_t oi = __shfl_xor(bi, m);
        const uint32_t oo = (uint32_t)__shfl_xor((int)bo, m);
        const int32_t od = __shfl_xor(bd, m);
        if (outranks(oi, oo, od, bi, bo, bd)) { bi = oi; bo = oo; bd = od; }
    }
}

template <bool kMatrix, int KM>
__global__ __launch_bounds__(kPostWaves * kWave) void dice_post_kernel(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tpad,
    const uint64_t* __restrict__ dmask, const uint32_t* __restrict__ wrow, const uint16_t* __restrict__ prow,
    const int4* __restrict__ tc, const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp,
    const uint8_t* __restrict__ ccp, double thr, int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out,
    double* __restrict__ score_out, int32_t k, uint32_t* __restrict__ mov, double* __restrict__ msc,
    int32_t* __restrict__ tki, double* __restrict__ tks) {
    constexpr int kStrideMax = kPostMaxTpad + 2;
    __shared__ uint32_t cnt32[kPostFiles * kStrideMax / 2];   // u16 counters, [file][template]
    __shared__ int4 tcs[kPostMaxTpad];
    __shared__ uint2 wl[kPostWaves][kWordCap];                 // queued (first row, rows)
    uint16_t* cnt16 = reinterpret_cast<uint16_t*>(cnt32);
    // row stride tpad + 2 halves = 32m + 1 dwords: lanes = files (phase 1) hit 64 distinct banks
    const int32_t cstride = tpad + 2;

    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * kPostFiles;

    for (int i = threadIdx.x; i < T; i += kPostWaves * kWave) tcs[i] = tc[i];

    // ---- phase 1: dense prefix, lanes = files --------------------------------------------
    {
        const int64_t file = f0 + lane;
        const bool valid = file < n;
        uint64_t fd[kPostMaxDense];
#pragma unroll
        for (int d = 0; d < kPostMaxDense; ++d) fd[d] = (valid && d < D) ? rows[file * w64 + d] : 0;
        const int32_t tw = (T + kPostWaves - 1) / kPostWaves;
        const int32_t tb = wave * tw, te = min(T, tb + tw);
        uint16_t* crow = cnt16 + lane * cstride;
        for (int32_t t = tb; t < te; ++t) {
            const uint64_t* m = dmask + (int64_t)t * kPostMaxDense;
            uint32_t acc = 0;
#pragma unroll
            for (int d = 0; d < kPostMaxDense; ++d) {
                if (d < D) {
                    const uint64_t md = m[d];
                    acc += __builtin_popcount((uint32_t)fd[d] & (uint32_t)md) +
                           __builtin_popcount((uint32_t)(fd[d] >> 32) & (uint32_t)(md >> 32));
                }
            }
            crow[t] = (uint16_t)acc;
        }
    }
    __syncthreads();

    // ---- phases 2 + 3, one file per wave ----------------------------------------------------
    for (int fi = wave; fi < kPostFiles; fi += kPostWaves) {
        const int64_t file = f0 + fi;
        if (file >= n) break;   // wave-uniform
        const uint64_t* row = rows + file * w64;
        uint32_t* crow32 = cnt32 + (fi * cstride) / 2;
        uint32_t nq = 0;        // queued words (uniform)

        // walk queued words: 4 words per pass, 16 lanes per word, one row of 16 ids per lane group
        auto flush = [&]() {
            const int g = lane >> 4, sub = lane & 15;
            for (uint32_t e0 = 0; e0 < nq; e0 += 4) {
                const uint32_t e = e0 + g;
                uint2 q = make_uint2(0, 0);
                if (e < nq) q = wl[wave][e];
                for (uint32_t r = 0; r < q.y; ++r) {
                    const uint16_t id = prow[(int64_t)(q.x + r) * kRowW + sub];
                    if (id != kNoTpl) atomicAdd(&crow32[id >> 1], 1u << ((id & 1) * 16));
                }
            }
            nq = 0;
        };

        for (int32_t pb = D; pb < w64; pb += kWave) {
            const int32_t p = pb + lane;
            uint64_t x = p < w64 ? row[p] : 0;
            while (__any(x != 0)) {
                const bool has = x != 0;
                const int b = has ? __builtin_ctzll(x) : 0;
                x &= x - 1;
                const int64_t w = (int64_t)p * 64 + b;
                uint32_t r0 = 0, nr = 0;
                if (has) {
                    r0 = wrow[w];
                    nr = wrow[w + 1] - r0;
                }
                const bool put = nr != 0;
                const uint64_t bal = __ballot(put);
                const uint32_t pos = nq + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
                if (put) wl[wave][pos] = make_uint2(r0, nr);
                nq += (uint32_t)__builtin_popcountll(bal);
                if (nq > kWordCap - kWave) flush();
            }
        }
        flush();

        // ---- phase 3: score, lanes = templates -------------------------------------------------
        const uint32_t wf = wfp[file];
        const int32_t lf = lenp[file];
        const bool cc = ccp[file] != 0;
        const uint16_t* crow = cnt16 + fi * cstride;
        int32_t bi = -1, bd = 1;
        uint32_t bo = 0;
        TopK<KM> top;
        if (kMatrix) top.init();
        for (int32_t t = lane; t < T; t += kWave) {
            const uint32_t ov = crow[t];
            const int4 c = tcs[t];
            const int32_t den = dice_den(c, wf, lf);
            if (kMatrix) {
                mov[file * T + t] = ov;
                msc[file * T + t] = dice_score(ov, den);
            }
            if (!(c.w && cc)) {
                if (kMatrix) top.offer(t, ov, den);
                else if (bi < 0 || dice_ge(ov, den, bo, bd)) { bi = t; bo = ov; bd = den; }
            }
        }
        if (!kMatrix) {
            wave_best(bi, bo, bd);
            if (lane == 0) {
                const double s = bi >= 0 ? dice_score(bo, bd) : 0.0;
                best_out[file] = (bi >= 0 && s >= thr) ? bi : -1;
                ov_out[file] = bo;
                score_out[file] = s;
            }
        } else if (tki) {
            // k rounds of a wave argmax over the lanes' sorted heads
            int h = 0;
            for (int r = 0; r < k; ++r) {
                int32_t ci = -1, cd = 1;
                uint32_t co = 0;
#pragma unroll
                for (int j = 0; j < KM; ++j)
                    if (j == h) { ci = top.idx[j]; co = top.ov[j]; cd = top.den[j]; }
                int32_t wi = ci, wd = cd;
                uint32_t wo = co;
                wave_best(wi, wo, wd);
                if (wi >= 0 && wi == ci) ++h;          // the winning lane advances
                if (lane == 0) {
                    tki[file * k + r] = wi;
                    tks[file * k + r] = wi >= 0 ? dice_score(wo, wd) : -1.0;
                }
            }
        }
    }
}

// ---- host side ---------------------------------------------------------------------------

// Estimated per-file cost (wave instructions) of a dense prefix of D u64 words: the dense
// phase pays T*D*4/64 VALU; every narrow membership a file hits costs ~1/16 of a 6-instruction
// row walk. A file resembling template t holds t's words, so the expected narrow memberships
// per file are sum over narrow words of p_w^2 / T (p_w = postings length).
static int pick_dense(const std::vector<int64_t>& sq_per_u64, int32_t T, int32_t w64) {
    const char* e = getenv("DICE_POST_DENSE");
    if (e && *e) return std::max(0, std::min(std::min(kPostMaxDense, w64), atoi(e)));
    double rest = 0;
    for (int64_t v : sq_per_u64) rest += (double)v;
    int best_d = 0;
    double best_c = 0.4 * rest / T;
    double c_dense = 0;
    for (int d = 1; d <= std::min(kPostMaxDense, w64); ++d) {
        rest -= (double)sq_per_u64[d - 1];
        c_dense = (double)T * d * 4.0 / 64.0;
        const double c = c_dense + 0.4 * rest / T;
        if (c < best_c) { best_c = c; best_d = d; }
    }
    return best_d;
}

bool post_feasible(const dice_templates* t) {
    const int32_t tpad = (t->n_templates + 63) / 64 * 64;
    if (tpad > kPostMaxTpad) return false;
    for (int32_t i = 0; i < t->n_templates; ++i)
        if (t->lf_size[i] >= 65535u) return false;   // u16 counters
    return true;
}

int post_setup(dice_ctx* c, const dice_templates* t) {
    const int32_t T = c->T, w64 = c->w64, tpad = (T + 63) / 64 * 64;
    const int64_t nbits = (int64_t)w64 * 64;
    // postings lengths per word and the dense-prefix choice
    std::vector<int32_t> plen((size_t)nbits, 0);
    for (int32_t i = 0; i < T; ++i) {
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        for (int32_t p = 0; p < w64; ++p)
            for (uint64_t x = r[p]; x; x &= x - 1) ++plen[(size_t)p * 64 + __builtin_ctzll(x)];
    }
    std::vector<int64_t> sq((size_t)w64, 0);
    for (int64_t w = 0; w < nbits; ++w) sq[(size_t)(w / 64)] += (int64_t)plen[(size_t)w] * plen[(size_t)w];
    const int D = pick_dense(sq, T, w64);
    // postings rows of the narrow words (u64 words >= D), template ids ascending
    std::vector<uint32_t> wrow((size_t)nbits + 1, 0);
    uint32_t nrows = 0;
    for (int64_t w = 0; w < nbits; ++w) {
        wrow[(size_t)w] = nrows;
        if (w / 64 >= D) nrows += (uint32_t)((plen[(size_t)w] + kRowW - 1) / kRowW);
    }
    wrow[(size_t)nbits] = nrows;
    std::vector<uint16_t> prow((size_t)std::max<uint32_t>(nrows, 1) * kRowW, kNoTpl);
    std::vector<uint32_t> fill((size_t)nbits, 0);
    for (int32_t i = 0; i < T; ++i) {
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        for (int32_t p = D; p < w64; ++p)
            for (uint64_t x = r[p]; x; x &= x - 1) {
                const int64_t w = (int64_t)p * 64 + __builtin_ctzll(x);
                prow[(size_t)wrow[(size_t)w] * kRowW + fill[(size_t)w]++] = (uint16_t)i;
            }
    }
    // dense prefix masks, template-major [T][kPostMaxDense]; template constants
    std::vector<uint64_t> dm((size_t)T * kPostMaxDense, 0);
    for (int32_t i = 0; i < T; ++i)
        for (int d = 0; d < D; ++d) dm[(size_t)i * kPostMaxDense + d] = t->lf_bits[(size_t)i * w64 + d];
    std::vector<int4> tcv((size_t)T);
    for (int32_t i = 0; i < T; ++i)
        tcv[i] = make_int4((int32_t)t->lf_size[i] - (int32_t)t->fields_set_size[i], t->length_slack[i],
                           t->length[i], t->is_cc[i] ? 1 : 0);
    int rc;
    if ((rc = dalloc_bytes(&c->d_pwrow, wrow.size() * 4)) || (rc = dalloc_bytes(&c->d_prow, prow.size() * 2)) ||
        (rc = dalloc_bytes(&c->d_pdm, dm.size() * 8)) || (rc = dalloc_bytes(&c->d_ptc, tcv.size() * sizeof(int4))))
        return rc;
    if (hipMemcpy(c->d_pwrow, wrow.data(), wrow.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_prow, prow.data(), prow.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_pdm, dm.data(), dm.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_ptc, tcv.data(), tcv.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "postings plan upload failed");
    c->post_dense = D;
    c->post_tpad = tpad;
    c->post_rows = nrows;
    c->kind = 3;
    return DICE_OK;
}

template <bool kMatrix, int KM>
static int launch(dice_ctx* c, dice_batch* b, double thr, int32_t k, hipStream_t s) {
    const int64_t groups = (b->n + kPostFiles - 1) / kPostFiles;
    hipLaunchKernelGGL((dice_post_kernel<kMatrix, KM>), dim3((unsigned)groups), dim3(kPostWaves * kWave), 0, s,
                       (const uint64_t*)b->d_rows, b->n, c->w64, c->post_dense, c->T, c->post_tpad,
                       (const uint64_t*)c->d_pdm, (const uint32_t*)c->d_pwrow, (const uint16_t*)c->d_prow,
                       (const int4*)c->d_ptc, b->d_wf, b->d_len, b->d_cc, thr, b->d_best, b->d_ov, b->d_score, k,
                       b->d_mov, b->d_mscore, k > 0 ? b->d_tki : nullptr, b->d_tks);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_post_kernel launch failed");
}

int post_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    return launch<false, 1>(c, b, thr, 0, s);
}

int post_launch_matrix(dice_ctx* c, dice_batch* b, int32_t k, hipStream_t s) {
    return k <= 4 ? launch<true, 4>(c, b, 0.0, k, s) : launch<true, kTopKMax>(c, b, 0.0, k, s);
}

}  // namespace dice
