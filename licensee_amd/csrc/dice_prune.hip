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
constexpr int kPruneGroups = 16;         // word groups of the bound (u16 pairs: 8 dwords per template)
constexpr int kPruneMaxJ = 8;            // u64 words per lane: w64 <= 512 (V <= 32768)
constexpr int kPruneMaxT = 704;          // = kPostMaxTpad (the key's low 10 bits hold the template)
constexpr uint32_t kKeyLow = 1023u;

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}

__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}

// The next file's independent loads, in flight while the wave works on the current file.
template <int J>
struct PruneNext {
    uint64_t w[J];
    uint32_t wf, cc;
    int32_t lf;
};

template <int J>
__device__ __forceinline__ void prune_load(PruneNext<J>& nx, const uint64_t* __restrict__ rows, int64_t file,
                                           int32_t w64, const uint32_t* __restrict__ wfp,
                                           const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp,
                                           int lane) {
    const uint64_t* row = rows + file * w64;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int32_t p = lane + j * kWave;
        nx.w[j] = p < w64 ? __builtin_nontemporal_load(row + p) : 0;
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

// Exact overlap of template ts with the wave's file row (one lane per record {u64 word, mask},
// two records per lane in flight), its denominator and the running best in the strict
// (score, later key) order; llo becomes an f32 lower bound of the best score.
__device__ __forceinline__ void score_template(int32_t ts, const uint32_t* soff, const uint4* __restrict__ qrec,
                                               const uint64_t* myrow, const uint4* stc, uint32_t wf, int32_t lf,
                                               bool fast, int lane, int32_t& bi, uint32_t& bo, int32_t& bd,
                                               float& llo) {
    const uint32_t r0 = rfl(soff[ts]), r1 = rfl(soff[ts + 1]);
    uint32_t acc = 0;
    for (uint32_t r = r0 + lane; r < r1; r += 2 * kWave) {
        const uint4 a = qrec[r];
        const uint4 b = r + kWave < r1 ? qrec[r + kWave] : make_uint4(0, 0, 0, 0);
        const uint64_t fa = myrow[a.x], fb = myrow[b.x];
        acc += (uint32_t)__builtin_popcount((uint32_t)fa & a.y) + (uint32_t)__builtin_popcount((uint32_t)(fa >> 32) & a.z);
        acc += (uint32_t)__builtin_popcount((uint32_t)fb & b.y) + (uint32_t)__builtin_popcount((uint32_t)(fb >> 32) & b.z);
    }
    const uint32_t ov = rfl(__builtin_amdgcn_readlane(wave_incl_scan(acc), kWave - 1));
    const uint4 c = stc[ts];
    const int32_t den = dice_den(make_int4((int32_t)c.z, (int32_t)c.w >> 16, (int32_t)c.x, 0), wf, lf);
    const bool better = fast ? outranks_t<true>(ts, ov, den, bi, bo, bd) : outranks_t<false>(ts, ov, den, bi, bo, bd);
    if (better) {
        bi = ts;
        bo = ov;
        bd = den;
        const double s = dice_score(bo, bd);
        // f32 lower bound of s: (1 - 2^-16) s rounds to nearest below s; no dropping against a
        // non-positive or NaN best
        llo = s > 0.0 ? (float)(s * (1.0 - 1.0 / 65536.0)) : -1.0f;
    }
}

// Per-template constants in LDS (uint4), padded to TJ * 64 templates:
//   x = length, y = -max(slack, 0) (u32), z = base = |Lf| - |Fld|,
//   w = keep bits (bit 0: kept for unflagged files, bit 1: for CC-flagged files; 0 = padding)
//       | slack << 16 (int16, -1 = simple delta)
// max(|len - len_F| - max(slack, 0), 0) equals the reference's adjusted delta for slack >= 0
// and the plain delta for slack = -1 (content_helper.rb:337-347; dice_den).
template <int J, int TJ, int G, int NW, bool PF, int OCC>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void dice_prune_match(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t T, const uint32_t* __restrict__ qa,
    const uint4* __restrict__ tc, const uint32_t* __restrict__ qoff, const uint4* __restrict__ qrec,
    const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp, double thr,
    int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out, double* __restrict__ score_out, bool corpus_fast, int32_t diag) {
    // diag (DICE_PRUNE_DIAG, diagnostics only -- results are wrong): 1 skips the bound pass (one
    // template scored), 2 skips exact scoring, 4 skips the row loads
    constexpr int kTP = TJ * kWave;   // padded template count
    constexpr int kGW = G / 2;        // group-count dwords per template
    // LDS: [waves][w64] file rows | [kGW / 4][kTP] uint4 group counts (lane stride 16 B: no bank
    // conflicts) | [kTP] constants | [T + 1] record offsets
    extern __shared__ uint64_t lds[];
    uint32_t* sqa = reinterpret_cast<uint32_t*>(lds + (size_t)NW * w64);
    const uint4* sqa4 = reinterpret_cast<const uint4*>(sqa);
    uint4* stc = reinterpret_cast<uint4*>(sqa + (size_t)kTP * kGW);
    uint32_t* soff = reinterpret_cast<uint32_t*>(stc + kTP);
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    uint64_t* myrow = lds + (size_t)wave * w64;
    for (int i = threadIdx.x; i < kTP * kGW; i += NW * kWave) sqa[i] = qa[i];
    for (int i = threadIdx.x; i < kTP; i += NW * kWave) stc[i] = tc[i];
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
        // group g = lane / (64 / G): sums over 4 (8) lanes, two groups per dword
        pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
        pc += (uint32_t)__builtin_amdgcn_mov_dpp((int)pc, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
        if (G == 8) pc += (uint32_t)__builtin_amdgcn_ds_swizzle((int)pc, 0x101F);   // lane ^ 4
        uint32_t fg[kGW];
#pragma unroll
        for (int k = 0; k < kGW; ++k)
            fg[k] = rfl(__builtin_amdgcn_readlane(pc, 2 * k * (64 / G)) |
                        (__builtin_amdgcn_readlane(pc, (2 * k + 1) * (64 / G)) << 16));
        // a file outside the plain range (len_F < 0, |W_F| >= 2^30: never from real text) keeps
        // every template: all are scored exactly (int32 den stays as dice_den computes it)
        const bool plain = lf >= 0 && wf < (1u << 30);

        // bounds (lanes = templates t = lane + 64 j), branch-free over the padded table; each
        // lane keeps its two largest keys
        uint32_t key[TJ];
        uint32_t m1 = 0, m2 = 0;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            if (diag & 1) { key[j] = (j == 0 && lane == 0) ? 0x7F800001u : 0u; m1 = max(m1, key[j]); continue; }
            const int32_t t = lane + j * kWave;
            const uint4 c = stc[t];
            uint32_t mn[kGW];
#pragma unroll
            for (int q = 0; q < kGW; q += 4) {
                const uint4 a4 = sqa4[(q / 4) * kTP + t];
                mn[q] = pk_min(a4.x, fg[q]);
                mn[q + 1] = pk_min(a4.y, fg[q + 1]);
                mn[q + 2] = pk_min(a4.z, fg[q + 2]);
                mn[q + 3] = pk_min(a4.w, fg[q + 3]);
            }
#pragma unroll
            for (int h = kGW / 2; h >= 1; h /= 2)   // pairwise u16 sums (short dependency chains)
#pragma unroll
                for (int q = 0; q < h; ++q) mn[q] = pk_add(mn[q], mn[q + h]);
            const uint32_t m = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, mn[0]), (u16x2){1, 1}, 0u, false);
            const int32_t adj = max((int32_t)__usad(c.x, (uint32_t)lf, c.y), 0);
            const int32_t den = (int32_t)(c.z + wf + ((uint32_t)adj >> 2));
            const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int32_t)c.w, ccf, 1);   // 0 or ~0
            const uint32_t tp1 = (uint32_t)t + 1u;
            const uint32_t k = keep & (plain ? bound_key(m, den, tp1) : (0x7F800000u | tp1));
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
            const uint32_t K2 = rfl(__builtin_amdgcn_readlane(wave_incl_max(m1 == K1 ? m2 : m1), kWave - 1));
            if (diag & 2) { bi = (int32_t)(K1 & kKeyLow) - 1; bo = K2; } else
            score_template((int32_t)(K1 & kKeyLow) - 1, soff, qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
            if (!(diag & 2) && K2 != 0 && !(__uint_as_float(K2 & ~kKeyLow) < llo)) {
                // more templates may reach the top: drop the scored one, then score the largest
                // remaining key and drop every key below the best score, until none is left
                const int32_t t1 = (int32_t)(K1 & kKeyLow) - 1;
                if (lane == (t1 & (kWave - 1))) {
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        if (j == (t1 >> 6)) key[j] = 0;
                }
                for (;;) {
                    uint32_t km = 0;
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        if (__uint_as_float(key[j] & ~kKeyLow) < llo) key[j] = 0;
                        km = max(km, key[j]);
                    }
                    const uint32_t K = rfl(__builtin_amdgcn_readlane(wave_incl_max(km), kWave - 1));
                    if (K == 0) break;   // every template scored or dropped
                    const int32_t ts = (int32_t)(K & kKeyLow) - 1;
                    if (lane == (ts & (kWave - 1))) {
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            if (j == (ts >> 6)) key[j] = 0;
                    }
                    score_template(ts, soff, qrec, myrow, stc, wf, lf, fast, lane, bi, bo, bd, llo);
                }
            }
        }
        if (lane == 0) {
            const double s = bi >= 0 ? dice_score(bo, bd) : 0.0;
            best_out[file] = (bi >= 0 && s >= thr) ? bi : -1;
            ov_out[file] = bo;
            score_out[file] = s;
        }
    }
}

// ---- host side ---------------------------------------------------------------------------

static int32_t prune_tj(int32_t T) { return T <= 640 ? 10 : (kPruneMaxT + kWave - 1) / kWave; }

static size_t prune_lds_bytes(int32_t nw, int32_t w64, int32_t T, int32_t groups) {
    const size_t tp = (size_t)prune_tj(T) * kWave;
    return (size_t)nw * w64 * 8 + tp * (groups / 2) * 4 + tp * 16 + ((size_t)T + 1) * 4;
}

int prune_setup(dice_ctx* c, const dice_templates* t) {
    const char* e = getenv("DICE_POST_PRUNE");
    if (e && *e == '0') return DICE_OK;
    const char* eg = getenv("DICE_PRUNE_GROUPS");
    const int32_t G = eg && *eg && atoi(eg) == 8 ? 8 : kPruneGroups;
    const int32_t T = c->T, w64 = c->w64;
    if (T > kPruneMaxT || w64 > kPruneMaxJ * kWave || prune_lds_bytes(kPruneWaves, w64, T, G) > 160 * 1024)
        return DICE_OK;
    const size_t tp = (size_t)prune_tj(T) * kWave;
    // group counts |Lf_t ∩ g| (< 2^16: post_feasible bounds |Lf|) as u16 pairs, the constants,
    // records of the nonzero u64 words; padding templates have keep bits 0
    std::vector<uint32_t> qa(tp * (G / 2), 0);
    std::vector<uint4> tcv(tp, make_uint4(0, 0, 0, 0));
    std::vector<uint32_t> qoff((size_t)T + 1, 0);
    std::vector<uint4> qrec;
    for (int32_t i = 0; i < T; ++i) {
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        uint32_t gc[kPruneGroups] = {0};
        for (int32_t p = 0; p < w64; ++p) {
            if (!r[p]) continue;
            gc[(p % kWave) / (kWave / G)] += (uint32_t)__builtin_popcountll(r[p]);
            qrec.push_back(make_uint4((uint32_t)p, (uint32_t)r[p], (uint32_t)(r[p] >> 32), 0));
        }
        for (int k = 0; k < G / 2; ++k)   // [G / 8][tp] uint4 planes
            qa[((size_t)(k / 4) * tp + (size_t)i) * 4 + (k % 4)] = gc[2 * k] | (gc[2 * k + 1] << 16);
        qoff[(size_t)i + 1] = (uint32_t)qrec.size();
        const int32_t slack = t->length_slack[i];
        tcv[(size_t)i] = make_uint4((uint32_t)t->length[i], (uint32_t)(-std::max(slack, 0)),
                                    t->lf_size[i] - t->fields_set_size[i],
                                    (t->is_cc[i] ? 1u : 3u) | ((uint32_t)(slack & 0xFFFF) << 16));
    }
    if (qrec.empty()) qrec.push_back(make_uint4(0, 0, 0, 0));
    int rc;
    if ((rc = dalloc_bytes(&c->d_qa, qa.size() * 4)) || (rc = dalloc_bytes(&c->d_qoff, qoff.size() * 4)) ||
        (rc = dalloc_bytes(&c->d_qrec, qrec.size() * sizeof(uint4))) ||
        (rc = dalloc_bytes(&c->d_qtc, tcv.size() * sizeof(uint4))))
        return rc;
    if (hipMemcpy(c->d_qa, qa.data(), qa.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_qoff, qoff.data(), qoff.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_qrec, qrec.data(), qrec.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_qtc, tcv.data(), tcv.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "pruned-match plan upload failed");
    c->prune_records = (int64_t)qoff[(size_t)T];
    const char* sc = getenv("DICE_PRUNE_SCHED");
    c->prune_sched = sc && *sc ? atoi(sc) : 0;
    c->prune_groups = G;
    const char* dg = getenv("DICE_PRUNE_DIAG");
    c->prune_diag = dg && *dg ? atoi(dg) : 0;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->n_cu < 1)
        c->n_cu = 256;
    c->prune = true;
    return DICE_OK;
}

template <int J, int TJ, int G, int NW, bool PF, int OCC>
static int launch_prune(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    const size_t lds = prune_lds_bytes(NW, c->w64, c->T, G);
    auto kern = dice_prune_match<J, TJ, G, NW, PF, OCC>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(DICE_E_DEVICE, "hipFuncSetAttribute failed");
    // persistent grid: as many workgroups as are resident at once (LDS- and wave-limited)
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(32 / NW, (160 * 1024) / (int64_t)lds));
    const int64_t groups = std::min<int64_t>((b->n + NW - 1) / NW, per_cu * c->n_cu);
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(NW * kWave), lds, s, (const uint64_t*)b->d_rows,
                       b->n, c->w64, c->T, (const uint32_t*)c->d_qa, (const uint4*)c->d_qtc,
                       (const uint32_t*)c->d_qoff, (const uint4*)c->d_qrec, b->d_wf, b->d_len, b->d_cc, thr,
                       b->d_best, b->d_ov, b->d_score, c->post_fast, c->prune_diag);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_prune_match launch failed");
}

// Schedule variants (DICE_PRUNE_SCHED, A/B): 0 = 16-wave workgroups, row loads at the file;
// 1 = 16-wave workgroups, the next file's row prefetched in VGPRs; 2 = 8-wave workgroups,
// the next row prefetched (6 waves/SIMD); 3 = 8-wave workgroups, row loads at the file.
template <int J, int TJ, int G>
static int launch_prune_s(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    switch (c->prune_sched) {
        case 1: return launch_prune<J, TJ, G, 16, true, 8>(c, b, thr, s);
        case 2: return launch_prune<J, TJ, G, 8, true, 6>(c, b, thr, s);
        case 3: return launch_prune<J, TJ, G, 8, false, 8>(c, b, thr, s);
        default: return launch_prune<J, TJ, G, 16, false, 8>(c, b, thr, s);
    }
}

template <int J>
static int launch_prune_j(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    constexpr int kTJ11 = (kPruneMaxT + kWave - 1) / kWave;
    if (c->prune_groups == 8)
        return c->T <= 640 ? launch_prune_s<J, 10, 8>(c, b, thr, s) : launch_prune_s<J, kTJ11, 8>(c, b, thr, s);
    return c->T <= 640 ? launch_prune_s<J, 10, 16>(c, b, thr, s) : launch_prune_s<J, kTJ11, 16>(c, b, thr, s);
}

int prune_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    if (b->n == 0) return DICE_OK;
    switch ((c->w64 + kWave - 1) / kWave) {
        case 1: return launch_prune_j<1>(c, b, thr, s);
        case 2: return launch_prune_j<2>(c, b, thr, s);
        case 3:
        case 4: return launch_prune_j<4>(c, b, thr, s);
        case 5:
        case 6: return launch_prune_j<6>(c, b, thr, s);
        default: return launch_prune_j<8>(c, b, thr, s);
    }
}

}  // namespace dice
