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
// Two kernels per launch:
//   dice_post_dense_mfma (default): the files' first D u64 words against the template masks as a
//            binary matrix product on the matrix cores (FP4 block-scaled MFMA, or int8 with
//            DICE_POST_MFMA=1; persistent workgroups; see below), written as a row-major [n][tp]
//            u16 matrix; dice_post_dense (DICE_POST_MFMA=0,
//            lanes = files, 16 waves per 64-file tile): the same by v_bcnt, template masks by
//            scalar loads, through an LDS [file][template] u16 stage;
//   dice_post_narrow_{match,matrix} (one file per wave): the file's dense partials, widened,
//            start the wave's u32 counter row in LDS; its remaining u64 words are loaded
//            kChunks x 64 at a time and their set bits (narrow words) are queued in a per-wave
//            LDS list, slots assigned by a DPP wave prefix sum; walk_short gives each queued
//            word one lane, reads its 32-byte postings row (16 entries, each a byte offset
//            4*t into the counter row, 0xFFFF padding) and adds 1 to the first 8 listed
//            counters (ds_add_u32), words with 9-16 entries their other 8 too; longer ones
//            wait in a long queue walked by all 64 lanes from the plong array. Scoring
//            reads the row with lanes = templates (t = lane + 64 j), using the
//            packed template constants {len | cc << 31, base | slack << 16}: the same
//            denominator, IEEE score and strict order (score, then later key) as every other
//            kernel, 24-bit exact compares inside the fast envelope; match mode reduces over
//            the wave, matrix mode writes the row-major [n][T] row and a k-round top-k.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <vector>

#include "dice_common.h"
#include "dice_internal.h"
#include "dice_wave.h"

namespace dice {

#ifndef DENSE_TU
#define DENSE_TU 2
#endif
// Phase-skip diagnostics (tools/build_variant.sh -DPOST_DIAG=n; results are wrong): 1 skips the
// dense kernel, 2 the postings walk, 4 the narrow-word extraction, 8 scoring
#ifndef POST_DIAG
#define POST_DIAG 0
#endif
// Dense partials: [n][tp] u16 rows, or (u8 mode, DICE_POST_U8=1, A/B, the FP4 dense kernel) a u8
// row ([n][s8] u32 words of four partials, rows padded to 16 bytes) for every file whose prefix
// holds at most 255 words -- no prefix overlap can exceed its popcount -- and a u16 row for the
// others (17% of config-3 files at 20 prefix words), with a per-file flag (1: u16). Parity green,
// 42% fewer partial bytes, and slower: the dense kernel 0.546 vs 0.479 ms on 5-T600 (its stores
// are bound by store instructions, and mixed rows need both a u16 and a u8 store per piece), the
// narrow kernels within 1%; 5-T600 5.13 vs 5.01 ms, all pairs 3.49 vs 3.45 (3 interleaved reps,
// profiles/r5_dense_ab.txt). (Round 4's byte rows decided per file from the values, a vote over
// the VALU kernel's stage, and measured slower too.)
struct Partials {
    uint16_t* p16;   // [n][tp] u16 rows (files flagged 1)
    uint32_t* p8;    // [n][s8] u32 words of four u8 partials (files flagged 0)
    uint8_t* flag;   // [n] 1: the file's row is the u16 one; nullptr: every row is u16
};
// u32 words per u8 row: tp bytes rounded up to 16
__host__ __device__ __forceinline__ int32_t u8_row_words(int32_t tp) { return (tp + 15) / 16 * 4; }

// A/B: the dense kernel's file prefixes staged through LDS by coalesced loads (1) or loaded per lane (0)
#ifndef POST_DENSE_LDS_PREFIX
#define POST_DENSE_LDS_PREFIX 1
#endif
// The walk's padding entries go to per-lane sinks instead of exec-masked adds (count_or_sink; 0:
// the masked form, A/B)
// the walk's entries 12-15 behind their own ballot (A/B)
#ifndef POST_WALK_SPLIT12
#define POST_WALK_SPLIT12 0
#endif
#ifndef POST_WALK_SINK
#define POST_WALK_SINK 1
#endif
constexpr int kPostWaves = 16;
// Waves per workgroup of the narrow kernels: the match kernel 16 (two workgroups per CU, 8 waves
// per SIMD); the matrix kernel 8 at 6 waves per SIMD (three workgroups fit a CU's LDS; 5-T600
// 5.17 -> 5.09 ms, 2 interleaved reps; the match kernel measured 3.54 -> 3.60 ms that way)
#ifndef POST_NARROW_WAVES
#define POST_NARROW_WAVES 16
#endif
#ifndef POST_NARROW_OCC
#define POST_NARROW_OCC 8
#endif
#ifndef POST_MATRIX_WAVES
#define POST_MATRIX_WAVES 8
#endif
// matrix kernel A/B: the next file's partials and first word chunks loaded before this file's row
// stores, so their waits do not include the stores (1), or at the file's start (0, default): 1
// measured 5.45 vs 5.10 ms on 5-T600 (2 interleaved reps; 80 VGPRs, the chunks live across the
// scoring)
#ifndef POST_MATRIX_PREFETCH
#define POST_MATRIX_PREFETCH 0
#endif
template <bool kMatrix>
constexpr int narrow_waves() { return kMatrix ? POST_MATRIX_WAVES : POST_NARROW_WAVES; }
constexpr int kPostFiles = 64;           // files per workgroup (one tile)
constexpr int kPostMaxTpad = 704;        // LDS budget of the dense stage (T <= 704)
constexpr int kPostMaxDense = 16;        // dense prefix u64 words (20 / 24 measured slower at T = 600)
constexpr int kRowW = 16;                // template ids per postings row
// per-wave queue of narrow word ids: as long as the narrow kernel's LDS allows two workgroups
// per CU (counter rows for TPMAX templates beside it)
template <int TPMAX>
constexpr int word_cap() { return TPMAX <= 608 ? 416 : 320; }
constexpr uint16_t kNoTpl = 0xFFFF;      // empty row entry
constexpr uint16_t kMore = 0xFFFE;       // row entry 15: a long word (entries 0-1 offset, 2 length)
constexpr int kLongCap = 64;             // per-wave queue of long words (offset, length)
// 64-word chunks of a file loaded together (match / matrix kernel)
#ifndef POST_CHUNKS_MATCH
#define POST_CHUNKS_MATCH 6
#endif
#ifndef POST_CHUNKS_MATRIX
#define POST_CHUNKS_MATRIX 6
#endif

// Postings entries are byte offsets (4 * template) into the wave's u32 counter row.
__device__ __forceinline__ void count(uint32_t* crow32, uint32_t off) {
    atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(crow32) + off), 1u);
}

// LDS byte addresses as integers (address space 3 is 32-bit), and a counter add at one.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(uint32_t* p) { return (uint32_t)(uintptr_t)(lds_u32*)p; }
__device__ __forceinline__ void lds_inc(uint32_t a) {
    __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// A postings row entry added without a branch: the address min(counter row + entry, sink) is the
// template's counter for a real entry (byte offset < 4 * TPMAX) and the lane's own sink dword for
// padding (0xFFFF) and the long-word marker (0xFFFE) -- the sink lies past every counter row and
// less than 0xFFFE bytes above any of them (the narrow kernel's LDS layout, post_narrow_body), so
// an entry costs one v_add (SDWA half select) + one v_min + the ds_add, instead of a compare and
// an exec mask round trip per entry. Sinks are per lane (distinct banks: no same-address
// serialization) and are queue slots whose words were already read (walk_short).
__device__ __forceinline__ void count_or_sink(uint32_t cbase, uint32_t sink, uint32_t entry) {
    lds_inc(min(cbase + entry, sink));
}

// Long words (> 16 narrow postings): 64 lanes per word, 4 words' id loads in flight.
__device__ __forceinline__ void walk_long(const uint2* lq, uint32_t& nl, const uint16_t* __restrict__ plong,
                                          uint32_t* crow32, int lane) {
    constexpr int kB = 4;   // words whose id loads are in flight together
    for (uint32_t e0 = 0; e0 < nl; e0 += kB) {
        uint16_t id[kB];
        uint2 q[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            q[u] = e0 + u < nl ? lq[e0 + u] : make_uint2(0, 0);
            id[u] = lane < (int)q[u].y ? plong[(int64_t)q[u].x + lane] : kNoTpl;
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            if (id[u] != kNoTpl) count(crow32, id[u]);
            for (uint32_t r = kWave; r < q[u].y; r += kWave)   // > 64 postings (rare)
                if (r + lane < q[u].y) count(crow32, plong[(int64_t)q[u].x + r + lane]);
        }
    }
    nl = 0;
}

// Queued narrow words, one lane per word: its 32-byte row in two loads, then the first 8
// template ids (8 predicated counter adds) and, for words with 9-16 ids, the row's other 8
// right away (their half is already loaded: no second pass). Words past 16 ids wait in the
// long queue, walked once it holds >= 64 words so its passes run with (nearly) every lane busy.
__device__ __forceinline__ void load_rows(const uint32_t* wq, uint32_t nq, uint32_t e0, const uint16_t* __restrict__ prow,
                                          int lane, uint32_t& w, uint4& r0, uint4& r1) {
    const uint32_t e = e0 + lane;
    r0 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    r1 = r0;
    w = 0;
    if (e < nq) {
        w = wq[e];
        const uint4* rp = reinterpret_cast<const uint4*>(prow + (int64_t)w * kRowW);
        r0 = rp[0];
        r1 = rp[1];
    }
}

template <int WCAP>
__device__ __forceinline__ void walk_short(const uint32_t* wq, uint32_t nq, uint2* lq, uint32_t& nl,
                                           const uint16_t* __restrict__ prow,
                                           const uint16_t* __restrict__ plong, uint32_t* crow32, int lane) {
    uint32_t w;
    uint4 r0, r1;
    if (nq) load_rows(wq, nq, 0, prow, lane, w, r0, r1);
    for (uint32_t e0 = 0; e0 < nq; e0 += kWave) {
        // the next pass's rows are requested before this pass's counter adds
        uint32_t wn = 0;
        uint4 n0 = r0, n1 = r1;
        if (e0 + kWave < nq) load_rows(wq, nq, e0 + kWave, prow, lane, wn, n0, n1);
        const bool lng = (r1.w >> 16) == kMore;
        const bool mid = !lng && (r1.x & 0xFFFFu) != kNoTpl;
        const uint64_t bl = __ballot(lng);
        if (bl) {
            if (lng) lq[nl + lane_rank(bl)] = make_uint2(r0.x, r0.y & 0xFFFFu);   // (offset, length)
            nl = rfl(nl + (uint32_t)__builtin_popcountll(bl));
            if (lng) r0 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        }
#if POST_WALK_SINK
        // this pass's queue slots [e0, e0 + 64) were read a pass ago: lane l's sink is slot e0 + l,
        // or slot WCAP - 64 + l in a last pass that starts past WCAP - 64 (those slots were read
        // too, and no later pass exists: nq <= WCAP)
        const uint32_t cbase = lds_addr(crow32),
                       sink = lds_addr(const_cast<uint32_t*>(wq) + min(e0, (uint32_t)(WCAP - kWave))) + 4u * (uint32_t)lane;
        const uint32_t rr[4] = {r0.x, r0.y, r0.z, r0.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) count_or_sink(cbase, sink, (rr[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
        if (__ballot(mid)) {   // entries 8-15 (0xFFFF padding / the long marker for other words: sinks)
            const uint32_t r2[4] = {r1.x, r1.y, r1.z, r1.w};
#if POST_WALK_SPLIT12
            // entries 12-15 only when a lane's word has more than 12 (about two passes in three)
#pragma unroll
            for (int k = 0; k < 4; ++k) count_or_sink(cbase, sink, (r2[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
            if (__ballot(mid && (r1.z & 0xFFFFu) != kNoTpl)) {
#pragma unroll
                for (int k = 4; k < 8; ++k) count_or_sink(cbase, sink, (r2[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
            }
#else
#pragma unroll
            for (int k = 0; k < 8; ++k) count_or_sink(cbase, sink, (r2[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
#endif
        }
#else
        const uint32_t rr[4] = {r0.x, r0.y, r0.z, r0.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t id = (rr[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
            if (id < kMore) count(crow32, id);
        }
        if (__ballot(mid)) {   // words with 9-16 ids: entries 8-15 from the row's loaded second half
            const uint32_t r2[4] = {r1.x, r1.y, r1.z, r1.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t id = (r2[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
                if (mid && id < kMore) count(crow32, id);
            }
        }
#endif
        if (nl > kLongCap - kWave) walk_long(lq, nl, plong, crow32, lane);
        w = wn;
        r0 = n0;
        r1 = n1;
    }
}

// The stage's [file][template] u16 rows of a 64-file tile out to the [n][tp] u16 partials, one file
// per wave at a time (the VALU dense kernel writes u16 rows only).
__device__ __forceinline__ void stage_out(const uint32_t* stage32, int32_t cs, int32_t tp, int64_t f0, int64_t nn,
                                          int wave, int nwaves, int lane, const Partials& pt) {
    for (int fi = wave; fi < kPostFiles; fi += nwaves) {
        const int64_t file = f0 + fi;
        if (file >= nn) break;
        const uint32_t* src = stage32 + (fi * cs) / 2;
        uint32_t* dst = reinterpret_cast<uint32_t*>(pt.p16 + file * tp);
        for (int32_t j = lane; j < tp / 2; j += kWave) dst[j] = src[j];
    }
}

// Phase 1 (dense prefix, lanes = files): wave w scores templates [w*TW, (w+1)*TW) over the 64
// files' first D u64 words (DP = D rounded up to a multiple of 4; masks past D are zero). The
// template masks are wave-uniform scalar loads, the next template's issued before this one is
// scored. Partial overlaps go to an LDS [file][template] u16 stage (row stride tp + 2 halves:
// an odd number of dwords, so the 64 lanes hit 64 banks), then out as row-major [n][tp] u16.
// Occupancy: two workgroups per CU (8 waves per SIMD) while the stage fits twice in LDS
// (TPMAX 608); one at the 704 maximum.
template <int DP, int TPMAX>
__global__ __launch_bounds__(kPostWaves * kWave) __attribute__((amdgpu_waves_per_eu(TPMAX <= 608 ? 8 : 4, TPMAX <= 608 ? 8 : 4))) void dice_post_dense(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tp,
    const uint64_t* __restrict__ dmask, Partials pt, const int32_t* __restrict__ idx,
    const uint32_t* __restrict__ pn) {
    __shared__ uint32_t stage32[kPostFiles * (TPMAX + 2) / 2];   // <= 78 KiB at TPMAX 608: 2 per CU
    uint16_t* st = reinterpret_cast<uint16_t*>(stage32);
    const int32_t cs = tp + 2;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    // indexed (idx != NULL): the *pn files deferred by the pruned match, file i's row being
    // rows[idx[i]] (persistent grid, count read on the device); partials stay indexed by i
    const int64_t nn = idx ? (int64_t)*pn : n;
    for (int64_t f0 = (int64_t)blockIdx.x * kPostFiles; f0 < nn; f0 += (int64_t)gridDim.x * kPostFiles) {
    // the tile's file prefixes, staged through LDS: thread (file tid / 16, word tid % 16) loads one
    // u64 (each file's 128 B are one coalesced segment), then every wave reads its lanes' words
    // back. (Loaded per lane, each wave fetched all 64 files' prefixes with 16 loads of 64
    // scattered 8-byte pieces: 16 waves x 1024 L1 requests per tile.) Rows padded to 18 words:
    // lane l's 16-byte reads start at bank 36 l mod 64, conflict-free within each 16-lane group.
    constexpr int kPreStride = kPostMaxDense + 2;
    static_assert(kPostFiles * kPostMaxDense == kPostWaves * kWave, "one prefix word per thread");
    static_assert(kPostFiles * kPreStride * 2 <= kPostFiles * (TPMAX + 2) / 2, "prefixes fit the stage");
    uint64_t fd[DP];
    if (POST_DENSE_LDS_PREFIX) {
        {
            uint64_t* pre = reinterpret_cast<uint64_t*>(stage32);
            const int fi = (int)threadIdx.x / kPostMaxDense, d = (int)threadIdx.x % kPostMaxDense;
            const int64_t file = f0 + fi;
            uint64_t v = 0;
            if (file < nn && d < D) v = rows[(idx ? (int64_t)idx[file] : file) * w64 + d];
            pre[fi * kPreStride + d] = v;
        }
        __syncthreads();
        const uint64_t* pre = reinterpret_cast<const uint64_t*>(stage32) + lane * kPreStride;
#pragma unroll
        for (int d = 0; d < DP; ++d) fd[d] = pre[d];
        __syncthreads();   // every wave holds its prefixes before the partials overwrite the stage
    } else {
        const int64_t file = f0 + lane;
        const bool valid = file < nn;
        const int64_t rf = valid && idx ? (int64_t)idx[file] : file;
#pragma unroll
        for (int d = 0; d < DP; ++d) fd[d] = (valid && d < D) ? rows[rf * w64 + d] : 0;
    }
    {
        const int32_t tw = (T + kPostWaves - 1) / kPostWaves;
        const int32_t tb = wave * tw, te = min(T, tb + tw);
        uint16_t* crow = st + lane * cs;
        // template masks: wave-uniform scalar loads (scalar returns are unordered, so a prefetch
        // would be waited for with the current template's masks: no software pipelining; the
        // other waves of the SIMD cover the latency)
        // TU = 2 templates per iteration, word-major, so both templates' mask loads are in flight
        // before the first wait (1 -> 2: config 3 5.39 -> 5.26 ms)
        constexpr int TU = DENSE_TU;
        for (int32_t t0 = tb; t0 < te; t0 += TU) {
            uint32_t acc[TU][4];
            const uint64_t* m[TU];
#pragma unroll
            for (int u = 0; u < TU; ++u) {
                // the last iteration of an odd range repeats template te - 1 (same value)
                m[u] = dmask + (int64_t)(t0 + u < te ? t0 + u : te - 1) * kPostMaxDense;
                // four independent accumulator chains (a single v_bcnt chain stalls on its latency)
                acc[u][0] = acc[u][1] = acc[u][2] = acc[u][3] = 0;
            }
            // word-major over the TU templates: every template's masks are live together
#pragma unroll
            for (int d = 0; d < DP; ++d)
#pragma unroll
                for (int u = 0; u < TU; ++u) {
                    const uint64_t md = m[u][d];
                    acc[u][(2 * d) & 3] += __builtin_popcount((uint32_t)fd[d] & (uint32_t)md);
                    acc[u][(2 * d + 1) & 3] += __builtin_popcount((uint32_t)(fd[d] >> 32) & (uint32_t)(md >> 32));
                }
#pragma unroll
            for (int u = 0; u < TU; ++u) {
                const int32_t t = t0 + u < te ? t0 + u : te - 1;
                crow[t] = (uint16_t)(acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3]);
            }
        }
        for (int32_t t = T + (threadIdx.x >> 6); t < tp; t += kPostWaves) crow[t] = 0;   // row padding
    }
    __syncthreads();
    stage_out(stage32, cs, tp, f0, nn, wave, kPostWaves, lane, pt);
    __syncthreads();   // the stage is refilled by the next tile
    }
}

// The dense prefix on the matrix cores (dice_post_dense_mfma; DICE_POST_MFMA: 4 = FP4, the
// default, 1 = int8). The prefix overlap |W_F ∩ Lf_t ∩ prefix| is a binary matrix product -- files
// x prefix bits times prefix bits x templates -- so with bits widened to 0/1 operands an MFMA
// computes a 32-file x 32-template tile exactly: v_mfma_i32_32x32x32_i8 32 bits at a time, the
// FP4 v_mfma_scale_f32_32x32x64_f8f6f4 a whole u64 word (below; counts <= 1280, exact in f32). A persistent workgroup
// (one per CU) = NW waves over tiles of MT x 32 files (MT = 3 for T <= 640, else 2); wave w owns
// 1-2 N-tiles of 32 templates (the ceil(T / 32) tiles dealt so the SIMDs' shares differ by at
// most one; 12 waves at 3 per SIMD, 11 above 640 templates), and each template fragment serves
// the MT M-tiles. Per u64 prefix word q: the files' words from the LDS-staged prefixes, the
// templates' words from the word-major masks (staged in LDS once per workgroup; FP4: as low/high
// u32 planes), each lane's bits widened to the operand format (widen_half / widen_a, widen_b),
// then MT x NTW MFMAs per word or k-step. A and B place the same bit in the same fragment element, so the products pair the same
// bits whatever the hardware's k order inside a step. Accumulator register g of lane (h, c) is
// file 32 m + (g & 3) + 8 (g >> 2) + 4 h, template 32 j + c: transposed through a per-wave 16 x 64
// LDS slab and stored as 16-byte pieces of the [n][tp] u16 partial rows (a wave's 64 templates of
// one file are 128 contiguous bytes). The next tile's prefixes are loaded into registers while
// this tile is scored (LDS waits count lgkmcnt, so they fly across the tile) and written to the
// other LDS buffer before this tile's stores are issued (one barrier per tile). (5-T600 dense
// kernel: round 4 1.70 -> 0.68 ms, the VALU kernel 1.45, profiles/r4_mfma_dense.txt; round 5 FP4
// 0.58, then 0.46 ms, profiles/r5_dense_ab.txt.)
// timing splits only (tools/build_variant.sh -DPOST_DENSE_AB=n; results wrong): 1 = no partial
// stores, 2 = no k-loop, 3 = no store phase (no slab, no stores)
#ifndef POST_DENSE_AB
#define POST_DENSE_AB 0
#endif
#ifndef POST_DENSE_BIAS
// FP4 planes: accumulators start at 2^23 so the counts sit in the low bits of their encodings (no
// cvt) -- off: parity failed at T = 65, the scaled FP4 MFMA does not add 64 unit products to 2^23
// exactly (its accumulation is not a full-precision f32 add; from 0 the counts stay exact)
#define POST_DENSE_BIAS 0
#endif
#ifndef POST_DENSE_PLANES
#define POST_DENSE_PLANES 1   // FP4: u32 planes in LDS and shift-free widening (widen_a / widen_b)
#endif
constexpr int kMfmaNT = 2;       // N-tiles per wave (at most)
constexpr int kMfmaCols = 768;   // template columns of the word-major masks (>= 11 waves x 2 N-tiles x 32)
constexpr int kMfmaMaxDense = 20;   // prefix u64 words of the matrix-core kernels (the masks' LDS budget)
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// Bits to int8 0/1 bytes for one fragment: half h of the 32-bit value v (a u64 word's low or high
// dword = the k-step), dword k of the fragment = (v >> (4 h + k)) & 0x01010101, i.e. bytes = bits
// 4h+k, 4h+k+8, 4h+k+16, 4h+k+24 -- a permutation of the k order that A and B share, so every
// product still pairs the same bit; two VALU per dword (one for the first).
__device__ __forceinline__ v4i widen_half(uint32_t v, int h) {
    const uint32_t x = v >> (4 * h);
    v4i r;
    r.x = (int)(x & 0x01010101u);
    r.y = (int)((x >> 1) & 0x01010101u);
    r.z = (int)((x >> 2) & 0x01010101u);
    r.w = (int)((x >> 3) & 0x01010101u);
    return r;
}

// FP4 variant (DICE_POST_MFMA=4): the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1
// operands takes a whole u64 prefix word per instruction (K = 64: lane half h holds the word's
// bits [32 h, 32 h + 32) as 32 nibbles). Bit -> nibble: dword k of the fragment = (v >> k) &
// 0x11111111, i.e. nibble i = bit 4 i + k (one VALU per dword after the first shift; A and B
// share the permutation, so every product pairs one bit of the file with the same bit of the
// template). Nibble 0b0001 is e2m1 0.5 and both block scales are 2^1 (E8M0 0x80), so each
// product is exactly 1.0 and the f32 accumulator holds the integer count (<= 1024, exact). Half
// the widening VALU and half the MFMAs of the int8 form per prefix bit (the FP4 rate is twice
// the int8 rate per clock on gfx950: 32 cycles for 32 x 32 x 64).
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
__device__ __forceinline__ v8i widen_nibbles(uint32_t v) {
    v8i r;
    r[0] = (int)(v & 0x11111111u);
    r[1] = (int)((v >> 1) & 0x11111111u);
    r[2] = (int)((v >> 2) & 0x11111111u);
    r[3] = (int)((v >> 3) & 0x11111111u);
    r[4] = r[5] = r[6] = r[7] = 0;   // (fp4 operands use the first four registers)
    return r;
}
constexpr int kE8M0Two = 0x80808080;   // block scale 2^1 in every byte
constexpr int kE8M0One = 0x7F7F7F7F;   // block scale 2^0

// The planes form (POST_DENSE_PLANES, default 1): nibble i of fragment dword k still holds bit
// 4 i + k of the word, but left where a mask finds it, so the two operands carry different e2m1
// values per dword and each product is still exactly 1.0 at block scales 2^0:
//   dword   A (file prefix)          value   B (template mask)          value
//   0       v & 0x11111111           0.5     (v << 2) & 0x44444444      2.0
//   1       v & 0x22222222           1.0     v & 0x22222222             1.0
//   2       v & 0x44444444           2.0     (v >> 2) & 0x11111111      0.5
//   3       (v >> 1) & 0x44444444    2.0     (v >> 3) & 0x11111111      0.5
// (e2m1 0b0001 = 0.5, 0b0010 = 1.0, 0b0100 = 2.0): 5 VALU for A, 7 for B (8 each before), and A
// is widened MT times per word.
__device__ __forceinline__ v8i widen_a(uint32_t v) {
    v8i r;
    r[0] = (int)(v & 0x11111111u);
    r[1] = (int)(v & 0x22222222u);
    r[2] = (int)(v & 0x44444444u);
    r[3] = (int)((v >> 1) & 0x44444444u);
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}
__device__ __forceinline__ v8i widen_b(uint32_t v) {
    v8i r;
    r[0] = (int)((v << 2) & 0x44444444u);
    r[1] = (int)(v & 0x22222222u);
    r[2] = (int)((v >> 2) & 0x11111111u);
    r[3] = (int)((v >> 3) & 0x11111111u);
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}

// A tile's accumulators out to the [n][tp] u16 partials through the wave's LDS slab, one piece =
// (M-tile m, 16-file half sh: accumulator registers 8 sh .. 8 sh + 7) at a time: in as u16 (file
// row, template column) into a 16 x 64 slab (rows 128 B, unpadded: the b16 writes of one row are
// conflict-free), back as 16-byte row pieces. A wave with two N-tiles then stores 8 whole 128-byte
// row pieces per instruction (the b128 reads of 8 rows x 128 B are conflict-free); a wave with one
// stores 16 rows x 64 bytes (2-way conflicts on that one read). (2-byte stores straight from the
// accumulators: 1.04 ms vs 0.94; 64-byte pieces from a 32 x 32 slab: 549 vs 528 us, 5-T600.)
// BIASED: the accumulators started at 2^23 (dice_post_dense_mfma, FP4 planes form), so the low 16
// bits of their f32 encodings are the counts -- no conversion.
constexpr int kSlabCols = 64;   // u16 per slab row (one wave's two N-tiles)
template <int MT, bool BIASED, bool U8OK, class ACC>
__device__ __forceinline__ void mfma_store_tile(const ACC (&acc)[MT][2], uint16_t* slab, const Partials& pt,
                                                const uint32_t* fc, int64_t f0, int64_t nn, int32_t tb, int32_t te,
                                                int32_t tp, int wave, int lane) {
    uint16_t* __restrict__ part = pt.p16;
    constexpr bool u8 = U8OK;
    int32_t tpf = tp, lf = lane;
    asm volatile("" : "+s"(tpf), "+v"(lf));   // addresses formed here, per tile
    const int32_t rf = lf & 31, hf = lf >> 5;
    const int32_t nt = (te - tb) / 32;   // the wave's N-tiles (uniform: 0, 1 or 2)
    if (nt == 0) return;
    auto val = [&](int m, int j, int g) -> uint16_t {
        if constexpr (BIASED) return (uint16_t)__builtin_bit_cast(uint32_t, acc[m][j][g]);
        else return (uint16_t)(uint32_t)acc[m][j][g];
    };
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j < nt) {   // uniform
#pragma unroll
                    for (int gg = 0; gg < 8; ++gg) {
                        const int g = 8 * sh + gg;
                        slab[((g & 3) + 8 * ((g >> 2) & 1) + 4 * hf) * kSlabCols + 32 * j + rf] = val(m, j, g);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            // u8 mode: a file's row is u16 only when its prefix holds more than 255 words
            // (fc: the tile's prefix popcounts, dice_post_dense_mfma)
            const uint32_t* fcp = fc + 32 * m + 16 * sh;
            if (nt == 2) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int row = (lf >> 3) + 8 * i, piece = lf & 7;
                    const uint4 v = *reinterpret_cast<const uint4*>(slab + row * kSlabCols + piece * 8);
                    const int64_t file = f0 + 32 * m + 16 * sh + row;
                    const int32_t t = tb + piece * 8;
                    const bool w = !u8 || fcp[row] > 255u;
                    if (POST_DENSE_AB != 1 && w && t < tpf && file < nn) *reinterpret_cast<uint4*>(part + file * tpf + t) = v;
                }
            } else {
                const int row = lf >> 2, piece = lf & 3;
                const uint4 v = *reinterpret_cast<const uint4*>(slab + row * kSlabCols + piece * 8);
                const int64_t file = f0 + 32 * m + 16 * sh + row;
                const int32_t t = tb + piece * 8;
                const bool w = !u8 || fcp[row] > 255u;
                if (POST_DENSE_AB != 1 && w && t < tpf && file < nn) *reinterpret_cast<uint4*>(part + file * tpf + t) = v;
            }
            if (u8) {
                // the byte rows: lane = (file row lf >> 2, 16 templates lf & 3), 16 u16 from the slab
                // packed to 16 bytes (bytes 0 and 2 of each u16 pair); rows padded to 16 bytes, so a
                // piece that starts below tp may run into the padding
                const int row = lf >> 2, p16 = lf & 3;
                const uint4 a = *reinterpret_cast<const uint4*>(slab + row * kSlabCols + 16 * p16);
                const uint4 c = *reinterpret_cast<const uint4*>(slab + row * kSlabCols + 16 * p16 + 8);
                const uint4 v = make_uint4(__builtin_amdgcn_perm(a.y, a.x, 0x06040200u), __builtin_amdgcn_perm(a.w, a.z, 0x06040200u),
                                           __builtin_amdgcn_perm(c.y, c.x, 0x06040200u), __builtin_amdgcn_perm(c.w, c.z, 0x06040200u));
                const int64_t file = f0 + 32 * m + 16 * sh + row;
                const int32_t t = tb + 16 * p16;
                if (POST_DENSE_AB != 1 && fcp[row] <= 255u && t < te && t < tpf && file < nn)
                    *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(pt.p8 + file * u8_row_words(tpf)) + t) = v;
                if (wave == 0 && lf < 16 && f0 + 32 * m + 16 * sh + lf < nn)
                    pt.flag[f0 + 32 * m + 16 * sh + lf] = fcp[lf] > 255u ? 1 : 0;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int DP, int NTW, int NW, int MT, bool F4 = false, bool U8 = false>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(3, 3))) void dice_post_dense_mfma(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t tp,
    const uint64_t* __restrict__ dmask, const Partials pt, const int32_t* __restrict__ idx,
    const uint32_t* __restrict__ pn) {
    // MT 32-file M-tiles per tile; the prefix buffer is doubled when LDS allows (one barrier per
    // tile; every shipped shape since the 16 x 64 slabs), else one buffer and a second barrier
    static_assert(DP <= kMfmaMaxDense, "prefix wider than the masks' table");
    static_assert(NTW == 2, "two N-tiles per wave (the store slab)");
    constexpr int kTF = 32 * MT;                     // files per tile
    // DP + 1 u64 per file row (odd: the 32 lanes of a ds_read_b64 column read hit 64 distinct banks)
    constexpr int kPreStride = DP + 1;
    constexpr int kPreWords = kTF * DP;
    constexpr int kPer = (kPreWords + NW * kWave - 1) / (NW * kWave);   // prefix words per thread
    constexpr int kCols = NTW == 2 && NW == 12 ? 640 : NW * NTW * 32;   // the workgroup's template columns
    constexpr size_t kFixed = (size_t)DP * kCols * 8 + (size_t)NW * 16 * kSlabCols * 2 + 3 * (size_t)kTF * 4;
    constexpr int kBufs = kFixed + 2 * (size_t)kTF * kPreStride * 8 <= 160 * 1024 ? 2 : 1;
    __shared__ uint64_t pre[kBufs][kTF * kPreStride];
    __shared__ uint64_t bm[DP * kCols];              // template masks, word-major (<= 110 KiB at DP 20)
    __shared__ uint16_t tslab[NW][16 * kSlabCols];   // per-wave 16 x 64 transpose slab (2 KiB)
    // u8 mode: the prefix popcount of each file of a tile, a ring of three: tile i reads slot i % 3,
    // its store_pre adds the next tile's into slot (i + 1) % 3, and it zeroes slot (i + 2) % 3 -- each
    // step a barrier away from the last use of its slot
    __shared__ uint32_t fcnt[3][kTF];
    static_assert(sizeof(pre) + sizeof(bm) + sizeof(tslab) + sizeof(fcnt) <= 160 * 1024, "one workgroup's LDS");
    constexpr bool u8 = F4 && U8;   // byte rows (DICE_POST_U8=1): a separate instantiation
    constexpr bool kBiased = F4 && POST_DENSE_PLANES && POST_DENSE_BIAS;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int64_t nn = idx ? (int64_t)*pn : n;
    // the wave's N-tiles: the ceil(tp / 32) tiles dealt as evenly as the waves allow (wave w on SIMD
    // w mod 4: 19 tiles over 12 waves give the SIMDs 5, 5, 5, 4)
    const int32_t ntiles = (tp + 31) / 32, tbase = ntiles / NW, textra = ntiles % NW;
    const int32_t nw_tiles = tbase + (wave < textra ? 1 : 0);
    const int32_t tb = 32 * (wave * tbase + min(wave, textra));
    const int64_t stride = (int64_t)gridDim.x * kTF;
    int64_t f0 = (int64_t)blockIdx.x * kTF;
    if (f0 >= nn) return;
    // this thread's share of a tile's prefix words (file i / 16, word i % 16)
    auto load_pre = [&](int64_t fs, uint64_t (&pv)[kPer]) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = (int)threadIdx.x + k * NW * kWave;
            const int fi = i / DP, d = i % DP;
            const int64_t file = fs + fi;
            pv[k] = (i < kPreWords && file < nn && d < D) ? rows[(idx ? (int64_t)idx[file] : file) * w64 + d] : 0;
        }
    };
    auto store_pre = [&](int buf, const uint64_t (&pv)[kPer], int slot) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = (int)threadIdx.x + k * NW * kWave;
            if (i < kPreWords) {
                if (u8 && pv[k]) atomicAdd(&fcnt[slot][i / DP], (uint32_t)__builtin_popcountll(pv[k]));
                const int at = (i / DP) * kPreStride + i % DP;
                if constexpr (F4 && POST_DENSE_PLANES) {   // low and high dwords in two planes
                    uint32_t* p32 = reinterpret_cast<uint32_t*>(pre[buf]);
                    p32[at] = (uint32_t)pv[k];
                    p32[kTF * kPreStride + at] = (uint32_t)(pv[k] >> 32);
                } else {
                    pre[buf][at] = pv[k];
                }
            }
        }
    };
    // the masks once per (persistent) workgroup: LDS reads in the k-loop wait on lgkmcnt, so the
    // next tile's prefix loads (vmcnt) fly across the whole tile
    for (int i = threadIdx.x; i < DP * kCols; i += NW * kWave) {
        const uint64_t v = dmask[(i / kCols) * kMfmaCols + i % kCols];
        if constexpr (F4 && POST_DENSE_PLANES) {
            reinterpret_cast<uint32_t*>(bm)[i] = (uint32_t)v;
            reinterpret_cast<uint32_t*>(bm)[DP * kCols + i] = (uint32_t)(v >> 32);
        } else {
            bm[i] = v;
        }
    }
    if (u8 && threadIdx.x < kTF) {
        fcnt[0][threadIdx.x] = 0;
        fcnt[1][threadIdx.x] = 0;
    }
    if (u8) __syncthreads();
    uint64_t pv[kPer];
    load_pre(f0, pv);
    store_pre(0, pv, 0);
    __syncthreads();
    int slot = 0;   // fcnt slot of the current tile (uniform)
    v16f bias;   // 2^23: the accumulators' f32 encodings then hold the counts in their low bits
#pragma unroll
    for (int g = 0; g < 16; ++g) bias[g] = 8388608.0f;
    for (int buf = 0; f0 < nn; f0 += stride, buf = (buf + 1) % kBufs, slot = slot == 2 ? 0 : slot + 1) {
        // unconditional (zeros past the end): a load under `if (more)` left pending on the skip path
        // would make the loop head wait vmcnt(0) for this tile's stores
        load_pre(f0 + stride, pv);
        const int nslot = slot == 2 ? 0 : slot + 1, zslot = nslot == 2 ? 0 : nslot + 1;
        if (u8 && threadIdx.x < kTF) fcnt[zslot][threadIdx.x] = 0;
        using Acc = typename std::conditional<F4, v16f, v16i>::type;
        Acc acc[MT][NTW];
        if constexpr (!kBiased) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int j = 0; j < NTW; ++j) acc[m][j] = Acc{};
        }
        const uint64_t* pb = pre[buf];
        const uint64_t* bcol = bm + tb + r;
        // one prefix word (biased: the first word's MFMAs take C from `bias`; q = 0 is peeled)
        auto word = [&](int q, auto first) {
            uint64_t bw[NTW] = {}, a[MT] = {};
            if constexpr (!(F4 && POST_DENSE_PLANES)) {
#pragma unroll
                for (int j = 0; j < NTW; ++j) bw[j] = j < nw_tiles ? bcol[q * kCols + j * 32] : 0;   // (uniform: no read past bm)
#pragma unroll
                for (int m = 0; m < MT; ++m) a[m] = pb[(32 * m + r) * kPreStride + q];
            }
            if constexpr (F4 && POST_DENSE_PLANES) {
                // lane half h reads its dwords from plane h (no 64-bit shift; conflict-free b32 reads:
                // the prefix rows' stride is odd) and widens them without shifts where the nibble
                // class allows (widen_a / widen_b: products 1.0 at block scales 2^0)
                const uint32_t* pa = reinterpret_cast<const uint32_t*>(pb) + h * (kTF * kPreStride) + r * kPreStride + q;
                const uint32_t* pw = reinterpret_cast<const uint32_t*>(bm) + h * (DP * kCols) + q * kCols + tb + r;
                uint32_t bw32[NTW];
#pragma unroll
                for (int j = 0; j < NTW; ++j) bw32[j] = j < nw_tiles ? pw[j * 32] : 0;
                v8i fa[MT];
#pragma unroll
                for (int m = 0; m < MT; ++m) fa[m] = widen_a(pa[32 * m * kPreStride]);
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    if (j < nw_tiles) {   // uniform
                        const v8i fb = widen_b(bw32[j]);
#pragma unroll
                        for (int m = 0; m < MT; ++m)
                            acc[m][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                                fa[m], fb, kBiased && decltype(first)::value ? bias : acc[m][j], 4, 4, 0, kE8M0One, 0,
                                kE8M0One);
                    }
                }
            } else if constexpr (F4) {
                // one instruction per (M-tile, N-tile) and word: lane half h holds bits [32 h, 32 h + 32)
                v8i fa[MT];
#pragma unroll
                for (int m = 0; m < MT; ++m) fa[m] = widen_nibbles((uint32_t)(a[m] >> (32 * h)));
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    if (j < nw_tiles) {   // uniform
                        const v8i fb = widen_nibbles((uint32_t)(bw[j] >> (32 * h)));
#pragma unroll
                        for (int m = 0; m < MT; ++m)
                            acc[m][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[m], fb, acc[m][j], 4, 4, 0,
                                                                                         kE8M0Two, 0, kE8M0Two);
                    }
                }
            } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                v4i fa[MT];
#pragma unroll
                for (int m = 0; m < MT; ++m) fa[m] = widen_half((uint32_t)(a[m] >> (32 * ks)), h);
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    if (j < nw_tiles) {   // uniform
                        const v4i fb = widen_half((uint32_t)(bw[j] >> (32 * ks)), h);
#pragma unroll
                        for (int m = 0; m < MT; ++m)
                            acc[m][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m], fb, acc[m][j], 0, 0, 0);
                    }
                }
            }
            }
        };
        if (POST_DENSE_AB != 2) {
            word(0, std::true_type{});
#pragma unroll 2
            for (int q = 1; q < DP; ++q) word(q, std::false_type{});
        }
        if (kBufs == 1) __syncthreads();   // every wave is done with the one prefix buffer
        // the next tile's prefixes into LDS before this tile's stores are issued: the wait on their
        // loads (vmcnt counts stores too, in order) then finds only the previous tile's stores,
        // issued a whole k-loop ago, and this tile's stores drain under the next tile's MFMAs
        store_pre((buf + 1) % kBufs, pv, nslot);
        if (POST_DENSE_AB != 3)
            mfma_store_tile<MT, kBiased, u8>(acc, tslab[wave], pt, fcnt[slot], f0, nn, tb, tb + 32 * nw_tiles, tp, wave, lane);
        __syncthreads();   // the next tile's prefixes are complete (MT = 2: the other buffer)
    }
}

// The file's dense partials into its counter row (a plain copy, widened: this wave's postings
// adds for the file come after it; the copy writes every entry, so the row is never re-zeroed),
// one LDS address and immediate offsets. wide (uniform): part[] holds u16 pairs, else words of
// four u8 partials (one 16-byte LDS store each).
template <int PJ>
__device__ __forceinline__ void copy_in(uint32_t* crow32, const uint32_t (&part)[PJ], int32_t tp, bool wide, int lane) {
    if (wide) {
        uint2* dst = reinterpret_cast<uint2*>(crow32) + lane;
#pragma unroll
        for (int j = 0; j < PJ; ++j)
            if (lane + j * kWave < tp / 2) dst[j * kWave] = make_uint2(part[j] & 0xFFFFu, part[j] >> 16);
    } else {
        uint4* dst = reinterpret_cast<uint4*>(crow32) + lane;
#pragma unroll
        for (int j = 0; j < (PJ + 1) / 2; ++j) {
            const uint32_t v = part[j];
            if (lane + j * kWave < tp / 4) dst[j * kWave] = make_uint4(v & 0xFFu, (v >> 8) & 0xFFu, (v >> 16) & 0xFFu, v >> 24);
        }
    }
}

// A file's partials (u16 pairs or u8 quads, see copy_in). CLAMP: unconditional loads at clamped
// indices (copy_in masks the rest), else exec-masked ones.
template <int PJ, bool CLAMP>
__device__ __forceinline__ void load_partials(const Partials& pt, int64_t pos, int32_t tp, bool wide, int lane,
                                              uint32_t (&part)[PJ]) {
    const uint32_t* src = wide ? reinterpret_cast<const uint32_t*>(pt.p16 + pos * tp) : pt.p8 + pos * u8_row_words(tp);
    const int32_t nw = wide ? tp / 2 : tp / 4;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
        const int32_t i = lane + j * kWave;
        if (!wide && j >= (PJ + 1) / 2) {
            part[j] = 0;
        } else if (CLAMP) {
            part[j] = src[min(i, nw - 1)];
        } else {
            part[j] = i < nw ? src[i] : 0;
        }
    }
}

template <int kChunks>
__device__ __forceinline__ void load_chunks(const uint64_t* __restrict__ row, int32_t w64, int32_t pb, int lane,
                                            uint64_t (&xs)[kChunks]) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        const int32_t p = pb + c * kWave + lane;
        xs[c] = p < w64 ? row[p] : 0;
    }
}

// One round of kChunks x 64 file words: per chunk a wave prefix sum of the lanes' bit counts
// gives every lane its queue slots, and each lane writes its own words (a chunk of more than
// WCAP words -- a file holding most of the vocabulary -- goes round by round instead); a full
// queue is walked.
template <int WCAP, int kChunks>
__device__ __forceinline__ void queue_chunks(const uint64_t (&xs)[kChunks], int32_t pb, uint32_t* wq, uint32_t& nq,
                                             uint2* lq, uint32_t& nl, const uint16_t* __restrict__ prow,
                                             const uint16_t* __restrict__ plong, uint32_t* crow32, int lane) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        const uint32_t wbase = (uint32_t)(pb + c * kWave + lane) * 64u;
        uint64_t x = xs[c];
        const uint32_t cnt = (uint32_t)__builtin_popcountll(x);
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t total = rfl(__builtin_amdgcn_readlane(incl, kWave - 1));
        if (total == 0) continue;
        if (nq + total > WCAP) {
            if (!(POST_DIAG & 2)) walk_short<WCAP>(wq, nq, lq, nl, prow, plong, crow32, lane);
            nq = 0;
        }
        if (total <= WCAP) {
            uint32_t pos = nq + incl - cnt;
            while (x) {
                wq[pos++] = wbase + (uint32_t)__builtin_ctzll(x);
                x &= x - 1;
            }
            nq += total;
            continue;
        }
        while (__any(x != 0)) {
            const bool has = x != 0;
            const uint32_t w = wbase + (has ? (uint32_t)__builtin_ctzll(x) : 0u);
            x &= x - 1;
            const uint64_t bal = __ballot(has);
            if (has) wq[nq + lane_rank(bal)] = w;
            nq = rfl(nq + (uint32_t)__builtin_popcountll(bal));
            if (nq > WCAP - kWave) {
                if (!(POST_DIAG & 2)) walk_short<WCAP>(wq, nq, lq, nl, prow, plong, crow32, lane);
                nq = 0;
            }
        }
    }
}

// Phase 2 for one file: queue its narrow words (set bits of u64 words >= pb0) and walk their
// postings into the wave's counter row. LATE (matrix mode): the file's dense partials are loaded
// here, before its first word chunks, and copied in once those are requested -- instead of being
// prefetched into registers during the previous file's scoring, where the matrix kernel cannot
// afford them.
template <int WCAP, bool LATE, int PJ, int kChunks = LATE ? POST_CHUNKS_MATRIX : POST_CHUNKS_MATCH, bool PF = false>
__device__ __forceinline__ void file_postings(const uint64_t* __restrict__ row, int32_t w64, int32_t pb0,
                                              const Partials& pt, int64_t pos, bool wide, int32_t tp, uint32_t* wq,
                                              uint2* lq,
                                              const uint16_t* __restrict__ prow, const uint16_t* __restrict__ plong,
                                              uint32_t* crow32, int lane, const uint64_t (*xs0)[kChunks] = nullptr) {
    uint32_t nq = 0;           // queued narrow words (wave-uniform)
    uint32_t nl = 0;           // queued long words (uniform)
    // queue the file's narrow words (set bits of u64 words >= D), kChunks x 64 words loaded
    // together (queue_chunks). The first round is peeled so that LATE's partials are copied in
    // between its loads and their use and are dead for the rest of the file; with PF the first
    // round arrives prefetched (xs0: loaded before the previous file was scored).
    int32_t pb = pb0;
    uint64_t xs[kChunks];
    if (PF) {
        if (pb < w64) {
            queue_chunks<WCAP, kChunks>(*xs0, pb, wq, nq, lq, nl, prow, plong, crow32, lane);
            pb += kChunks * kWave;
        }
    } else if (LATE) {
        uint32_t part[PJ];
        load_partials<PJ, true>(pt, pos, tp, wide, lane, part);
        if (pb < w64) load_chunks<kChunks>(row, w64, pb, lane, xs);
        copy_in<PJ>(crow32, part, tp, wide, lane);
        if (pb < w64) {
            queue_chunks<WCAP, kChunks>(xs, pb, wq, nq, lq, nl, prow, plong, crow32, lane);
            pb += kChunks * kWave;
        }
    }
    for (; pb < w64; pb += kChunks * kWave) {
        load_chunks<kChunks>(row, w64, pb, lane, xs);
        queue_chunks<WCAP, kChunks>(xs, pb, wq, nq, lq, nl, prow, plong, crow32, lane);
    }
    if (!(POST_DIAG & 2)) walk_short<WCAP>(wq, nq, lq, nl, prow, plong, crow32, lane);
    walk_long(lq, nl, plong, crow32, lane);
}

// Phase 3 for one file: lanes = templates (t = lane + 64 j), overlap from the counter row
// (the next file's copy-in overwrites every entry), the shared denominator and order; match
// mode reduces over the wave, matrix mode writes the row and the top-k. Every lane keeps only
// its best template; the top-k is k rounds of a wave argmax in which the winning lane marks its
// template taken and rescans its other templates (from the LDS row) for its next best -- the
// order of k argmaxes with removal, i.e. Dice#matches_by_similarity's (dice.rb:34-41), with one
// candidate per lane instead of k sorted slots (the matrix kernel keeps the match kernel's
// register budget and occupancy).
template <bool FAST>
__device__ __forceinline__ void lane_best(const uint32_t* crow32, const uint2* tcs, int32_t t, uint32_t wf, int32_t lf,
                                          bool cc, int32_t& bi, uint32_t& bo, int32_t& bd, uint32_t& ov,
                                          int32_t& den) {
    ov = crow32[t];
    const uint2 pc = tcs[t];   // {len | cc << 31, base | slack << 16}
    const int4 c = make_int4((int32_t)(pc.y & 0xFFFFu), (int32_t)pc.y >> 16, (int32_t)(pc.x & 0x7FFFFFFFu),
                             (int32_t)(pc.x >> 31));
    den = dice_den(c, wf, lf);
    if (!(c.w && cc) && (bi < 0 || ge<FAST>(ov, den, bo, bd))) {
        bi = t;
        bo = ov;
        bd = den;
    }
}

// One template's overlap and denominator, and whether it counts (not a masked cc-* template).
template <bool FAST>
__device__ __forceinline__ bool lane_eval(const uint32_t* crow32, const uint2* tcs, int32_t t, uint32_t wf, int32_t lf,
                                          bool cc, uint32_t& ov, int32_t& den) {
    ov = crow32[t];
    const uint2 pc = tcs[t];
    const int4 c = make_int4((int32_t)(pc.y & 0xFFFFu), (int32_t)pc.y >> 16, (int32_t)(pc.x & 0x7FFFFFFFu),
                             (int32_t)(pc.x >> 31));
    den = dice_den(c, wf, lf);
    return !(c.w && cc);
}

// wave argmax: DPP row shifts (1) or the ds_bpermute butterfly (0)
#ifndef POST_DPP_BEST
#define POST_DPP_BEST 1
#endif
#if POST_DPP_BEST
#define WAVE_BEST wave_best_dpp
#else
#define WAVE_BEST wave_best
#endif

// Matrix top-k: each lane also keeps its second best, so the first time a lane's template is
// ranked its next candidate is that second one instead of a rescan of its templates from LDS
// (a lane ranked twice still rescans)
#ifndef POST_TOPK_SECOND
#define POST_TOPK_SECOND 1
#endif

#ifndef POST_SCORE_NODIV
#define POST_SCORE_NODIV 0
#endif
#ifndef POST_MATRIX_STORE
#define POST_MATRIX_STORE 3
#endif
#define DICE_STR(x) #x
#define DICE_UNROLL(n) _Pragma(DICE_STR(unroll n))
// scoring loop unroll (A/B: 1, 2, 5, 10 within 1% for the matrix kernel; the match kernel
// needs 57 instead of 64 VGPRs at 2)
#ifndef SCORE_UNROLL
#define SCORE_UNROLL kMatrix ? 10 : 2
#endif
// A global pointer every lane holds the same value of, as SGPRs (address space 1: an integer
// round trip would leave a generic pointer, and generic stores are flat stores, which count in
// lgkmcnt as well as vmcnt, so every LDS wait would also wait for them).
template <class E>
using gptr = __attribute__((address_space(1))) E*;
template <class E>
__device__ __forceinline__ gptr<E> uniform_ptr(E* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (gptr<E>)(lo | (hi << 32));
}

template <bool kMatrix, int TJ, bool FAST>
__device__ __forceinline__ void score_file_t(uint32_t* crow32, const uint2* tcs, int32_t T, int32_t ld, int64_t file, uint32_t wf,
                                             int32_t lf, bool cc, double thr, int32_t* __restrict__ best_out,
                                             uint32_t* __restrict__ ov_out, double* __restrict__ score_out, int32_t k,
                                             uint32_t* __restrict__ mov, double* __restrict__ msc,
                                             int32_t* __restrict__ tki, double* __restrict__ tks, int lane) {
    int32_t bi = -1, bd = 1, bi2 = -1, bd2 = 1;
    uint32_t bo = 0, bo2 = 0;
    // The file's row bases as SGPR values (readfirstlane: the compiler cannot fold a lane offset
    // into a hoisted per-lane 64-bit base) and the lane opaque per file: every store is SGPR base +
    // a 32-bit VGPR offset formed where it is used, so no per-lane address stays live across the
    // file loop (they spilled to scratch, and each reload's vmcnt(0) waited for every store
    // issued before it).
    gptr<uint32_t> orow = nullptr;
    gptr<double> srow = nullptr;
    uint32_t lo = (uint32_t)lane;
    if (kMatrix) {
        orow = uniform_ptr(mov + file * ld);
        srow = uniform_ptr(msc + file * ld);
        asm volatile("" : "+v"(lo));
    }
    constexpr int kUnroll = SCORE_UNROLL;
    DICE_UNROLL(kUnroll)
    for (int j = 0; j < TJ; ++j) {
        const int32_t t = (int32_t)lo + j * kWave;
        if (t < T) {
            uint32_t ov;
            int32_t den;
            if (kMatrix && POST_TOPK_SECOND) {
                // the lane's two best (t ascending within a lane: a later template that ties takes
                // the place, the strict (score, later key) order)
                if (lane_eval<FAST>(crow32, tcs, t, wf, lf, cc, ov, den)) {
                    const bool b1 = bi < 0 || ge<FAST>(ov, den, bo, bd);
                    const bool b2 = !b1 && (bi2 < 0 || ge<FAST>(ov, den, bo2, bd2));
                    bi2 = b1 ? bi : b2 ? t : bi2;
                    bo2 = b1 ? bo : b2 ? ov : bo2;
                    bd2 = b1 ? bd : b2 ? den : bd2;
                    bi = b1 ? t : bi;
                    bo = b1 ? ov : bo;
                    bd = b1 ? den : bd;
                }
            } else {
                lane_best<FAST>(crow32, tcs, t, wf, lf, cc, bi, bo, bd, ov, den);
            }
            if (kMatrix) {
#if POST_MATRIX_STORE == 3
                __builtin_nontemporal_store(ov, orow + t);
#if POST_SCORE_NODIV   // timing split only (results wrong): the score store without its division
                __builtin_nontemporal_store((double)ov * (double)den, srow + t);
#else
                __builtin_nontemporal_store(dice_score(ov, den), srow + t);
#endif
#else
                const double sc = dice_score(ov, den);
                // diagnostics (POST_MATRIX_STORE, A/B builds only): bit 0 / 1 store overlaps / scores
                // (a cleared bit still computes them), bit 2 plain stores instead of nontemporal
                if ((POST_MATRIX_STORE & 1) || ov == 0xFFFFFFFFu) {
                    if (POST_MATRIX_STORE & 4) orow[t] = ov;
                    else __builtin_nontemporal_store(ov, orow + t);
                }
                if ((POST_MATRIX_STORE & 2) || ov == 0xFFFFFFFFu) {
                    if (POST_MATRIX_STORE & 4) srow[t] = sc;
                    else __builtin_nontemporal_store(sc, srow + t);
                }
#endif
            }
        }
    }
    if (!kMatrix) {
        WAVE_BEST<FAST>(bi, bo, bd);
        if (lane == 0) {
            const double s = bi >= 0 ? dice_score(bo, bd) : 0.0;
            const bool hit = bi >= 0 && s >= thr;
            // match mode k = 1: Dice#confidence outputs (0 / 0.0 for a file without a match)
            best_out[file] = hit ? bi : -1;
            ov_out[file] = (k == 1 && !hit) ? 0u : bo;
            score_out[file] = (k == 1 && !hit) ? 0.0 : s;
        }
    } else if (tki) {
        uint32_t taken = 0;   // bit j: template lane + 64 j already ranked
        bool second = true;   // (POST_TOPK_SECOND) the lane's second best not yet promoted
        for (int r = 0; r < k; ++r) {
            int32_t wi = bi, wd = bd;
            uint32_t wo = bo;
            WAVE_BEST<FAST>(wi, wo, wd);
            if (lane == 0) {
                tki[file * k + r] = wi;
                tks[file * k + r] = wi >= 0 ? dice_score(wo, wd) : -1.0;
            }
            if (wi < 0) {   // every potential match ranked: pad the rest (wave-uniform)
                for (int q = r + 1 + lane; q < k; q += kWave) {
                    tki[file * k + q] = -1;
                    tks[file * k + q] = -1.0;
                }
                break;
            }
            if (r + 1 < k && wi == bi) {   // the owner lane: next best among its untaken templates
                taken |= 1u << (wi >> 6);
                const bool promote = POST_TOPK_SECOND && second;
                second = false;
                if (promote) {
                    bi = bi2;
                    bo = bo2;
                    bd = bd2;
                } else {
                    bi = -1;
                    bo = 0;
                    bd = 1;
                    for (int j = 0; j < TJ; ++j) {
                        const int32_t t = (int32_t)lo + j * kWave;
                        if (t < T && !((taken >> j) & 1u)) {
                            uint32_t ov;
                            int32_t den;
                            lane_best<FAST>(crow32, tcs, t, wf, lf, cc, bi, bo, bd, ov, den);
                        }
                    }
                }
            }
        }
    }
}

template <bool kMatrix, int KM, int TJ>
__device__ __forceinline__ void score_file(uint32_t* crow32, const uint2* tcs, int32_t T, int32_t ld, int64_t file, uint32_t wf,
                                           int32_t lf, bool cc, bool corpus_fast, double thr, int32_t* __restrict__ best_out,
                                           uint32_t* __restrict__ ov_out, double* __restrict__ score_out, int32_t k,
                                           uint32_t* __restrict__ mov, double* __restrict__ msc, int32_t* __restrict__ tki,
                                           double* __restrict__ tks, int lane) {
    // file inside the fast envelope (wave-uniform): 24-bit exact compares
    if (corpus_fast && wf < (1u << 20) && lf >= 0 && lf < (1 << 21))
        score_file_t<kMatrix, TJ, true>(crow32, tcs, T, ld, file, wf, lf, cc, thr, best_out, ov_out, score_out, k, mov,
                                        msc, tki, tks, lane);
    else
        score_file_t<kMatrix, TJ, false>(crow32, tcs, T, ld, file, wf, lf, cc, thr, best_out, ov_out, score_out, k, mov,
                                         msc, tki, tks, lane);
}

// A file's loads that do not depend on its walk -- dense partials, scalars, first word chunks --
// issued while the wave is still scoring the previous file (prefetch_file), so they are in
// flight during that file's scoring instead of heading this file's dependency chain.
template <int TPMAX>
constexpr int pairs_per_lane() { return (TPMAX / 2 + kWave - 1) / kWave; }   // u32 partial pairs per lane

// Phases 2 + 3, one file per wave (16 waves x 4 files per workgroup). Each wave owns one u32
// counter row in LDS (zero between files). Narrow words are queued from the file's u64 words
// >= D and walked (walk_short / walk_long) after the file's dense partials (from
// dice_post_dense) are copied in (every entry: no zeroing between files); scoring reads the counters and reduces over the
// wave. The LDS footprint (~74 KiB) and <= 64 VGPRs leave room for two workgroups per CU.
template <bool kMatrix, int KM, int TPMAX, bool U8>
__device__ __forceinline__ void post_narrow_body(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tp,
    const Partials pt, const uint16_t* __restrict__ prow, const uint16_t* __restrict__ plong,
    const uint2* __restrict__ tc, const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp,
    const uint8_t* __restrict__ ccp, double thr, int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out,
    double* __restrict__ score_out, int32_t k, uint32_t* __restrict__ mov, double* __restrict__ msc,
    int32_t* __restrict__ tki, double* __restrict__ tks, bool corpus_fast,
    const int32_t* __restrict__ idx, const uint32_t* __restrict__ pn, int32_t ld) {
    constexpr int kNarrowWaves = narrow_waves<kMatrix>();
    constexpr int kTJ = (TPMAX + kWave - 1) / kWave;           // templates per lane
    constexpr int kWCap = word_cap<TPMAX>();
    constexpr int kPJ = pairs_per_lane<TPMAX>();
    // u32 counters, one row per wave, then the queues of narrow word ids: one array, so the queue
    // slots (the walk's sinks, count_or_sink) lie past every counter row and within 64 KiB of it
    __shared__ uint32_t cntq[kNarrowWaves * TPMAX + kNarrowWaves * kWCap];
    // (wave w's sinks end 4 (16 TPMAX + (w + 1) WCAP) bytes in, its row starts at 4 w TPMAX: the
    // largest gap is wave 0's)
    static_assert(kWCap <= TPMAX && (kNarrowWaves * TPMAX + kWCap) * 4 <= 0xFFFE, "sinks within reach of every row");
    uint32_t* const cnt32 = cntq;
    uint32_t (*const wq)[kWCap] = reinterpret_cast<uint32_t (*)[kWCap]>(cntq + kNarrowWaves * TPMAX);
    __shared__ uint2 tcs[TPMAX];                               // packed template constants
    __shared__ uint2 lq[kNarrowWaves][kLongCap];                 // queued long words (offset, length)
    __shared__ uint2 tsc[kMatrix ? kNarrowWaves : 1][kPostFiles / kNarrowWaves];   // matrix: own files' {|W_F|, len_F}
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    uint32_t* crow32 = cnt32 + wave * TPMAX;
    for (int i = threadIdx.x; i < T; i += kNarrowWaves * kWave) tcs[i] = tc[i];
    for (int i = lane; i < TPMAX; i += kWave) crow32[i] = 0;
    __syncthreads();

    const int32_t pb0 = (POST_DIAG & 4) ? w64 : D;
    // indexed (idx != NULL, match mode): position i is the deferred file idx[i] of a pruned match
    // (its dense partials at i, its row, scalars and results at idx[i]); persistent tiles
    const int64_t nn = idx ? (int64_t)*pn : n;
    for (int64_t f0 = (int64_t)blockIdx.x * kPostFiles; f0 < nn; f0 += (int64_t)gridDim.x * kPostFiles) {
    if (kMatrix) asm volatile("" : "+s"(tp));   // (see Tf below)
    // the tile's file indices and scalars, lane l = tile file l, by vector loads; each file reads
    // them with v_readlane. (Scalar loads of the next file's |W_F| / len_F shared lgkmcnt with the
    // postings walk's LDS adds and reads, whose waits then stalled on HBM latency.)
    // files of this tile (uniform, 1..64): the tile's compares stay 32-bit scalar ones (64-bit
    // signed compares go to the VALU and keep a VGPR copy of nn)
    const int64_t rem64 = nn - f0;
    const int32_t nt = (rem64 >> 32) != 0 || (uint32_t)rem64 >= (uint32_t)kPostFiles ? kPostFiles : (int32_t)rem64;
    const int64_t tpos = f0 + min(lane, nt - 1);
    // (indexed mode only: the file of tile position l; otherwise position = file, no register)
    const uint32_t tfile = idx ? (uint32_t)idx[tpos] : (uint32_t)tpos;
    uint32_t twf = wfp[tfile];
    uint32_t tlen = (uint32_t)lenp[tfile];
    const uint64_t tcc = __ballot(ccp[tfile] != 0);   // the tile's CC flags, one bit per file
    if (kMatrix) {
        // matrix mode: the wave's own files' |W_F| and len_F parked in its LDS slots instead of two
        // VGPRs live across the whole tile (the scoring's registers need them)
        uint32_t lw = (uint32_t)lane;
        asm volatile("" : "+v"(lw));   // the slot address formed here, not hoisted out of the tile loop
        if ((lw & (kNarrowWaves - 1)) == (uint32_t)wave) tsc[wave][lw / kNarrowWaves] = make_uint2(twf, tlen);
    }
    // the tile's partial formats (bit l: position f0 + l has a u16 row)
    const uint64_t tov = U8 ? __ballot(pt.flag[f0 + min(lane, nt - 1)] != 0) : ~0ull;
    // match mode: the next file's dense partials, prefetched while the wave scores the previous
    // file (the matrix kernel loads them at the file's start: file_postings LATE); matrix mode with
    // POST_MATRIX_PREFETCH: the next file's partials and first word chunks, loaded before this
    // file's row stores -- so their waits do not wait for the stores (gfx950's vmcnt counts stores)
    constexpr bool kPF = kMatrix && POST_MATRIX_PREFETCH && TPMAX <= 608;   // (704-template rows: no VGPRs left)
    constexpr int kNC = kMatrix ? POST_CHUNKS_MATRIX : POST_CHUNKS_MATCH;
    uint32_t pre[kPJ];
    uint64_t xs0[kPF ? kNC : 1];
    // (U8 match mode loads them at the file's start, as the matrix kernel does: the prefetch's
    // registers beside the byte-row logic exceed 64 VGPRs)
    constexpr bool kEarly = (!kMatrix && !U8) || kPF;
    if (kEarly && wave < nt) load_partials<kPJ, U8>(pt, f0 + wave, tp, (tov >> wave) & 1, lane, pre);
    if (kPF && wave < nt && pb0 < w64) load_chunks<kNC>(rows + (f0 + wave) * w64, w64, pb0, lane, *reinterpret_cast<uint64_t (*)[kNC]>(xs0));
    for (int fi = wave; fi < kPostFiles; fi += kNarrowWaves) {
        const int64_t pos = f0 + fi;
        if (fi >= nt) break;   // wave-uniform
        const int64_t file = idx ? (int64_t)rfl(__builtin_amdgcn_readlane(tfile, fi)) : pos;
        const uint64_t* row = rows + file * w64;
        // T, tp and ld opaque per file: the per-lane masks (t < T, i < tp / 2) and LDS addresses
        // are then formed where they are used instead of being hoisted out of the file loop, where
        // they stayed live as ~30 SGPRs and several VGPRs and spilled (the matrix kernel to scratch)
        int32_t Tf = T, tpf = tp, ldf = ld;
        int lanef = lane;   // likewise every lane-derived constant (lane + 64 j, lane addresses)
        if (kMatrix || U8) asm volatile("" : "+s"(Tf), "+s"(tpf), "+s"(ldf), "+v"(lanef));
        // this file's dense partials start its counter row (matrix mode without prefetch: inside
        // file_postings)
        const bool wide = (tov >> fi) & 1;
        if (kEarly) copy_in<kPJ>(crow32, pre, tpf, wide, lanef);
        uint32_t wf;
        int32_t lf;
        if (kMatrix) {
            const uint2 sc = tsc[wave][fi / kNarrowWaves];   // uniform address: a broadcast read
            wf = rfl(sc.x);
            lf = (int32_t)rfl(sc.y);
        } else {
            wf = rfl(__builtin_amdgcn_readlane(twf, fi));
            lf = (int32_t)rfl(__builtin_amdgcn_readlane(tlen, fi));
        }
        const bool cc = ((tcc >> fi) & 1u) != 0;
        if (kPF) {
            file_postings<kWCap, true, kPJ, kNC, true>(row, w64, pb0, pt, pos, wide, tpf, wq[wave], lq[wave], prow,
                                                       plong, crow32, lanef,
                                                       reinterpret_cast<const uint64_t (*)[kNC]>(xs0));
        } else {
            file_postings<kWCap, !kEarly, kPJ, kNC>(row, w64, pb0, pt, pos, wide, tpf, wq[wave], lq[wave], prow, plong,
                                               crow32, lanef);
        }
        // the wave's next file's partials (and with kPF its first chunks) fly while this one is scored
        if (kEarly && fi + kNarrowWaves < nt)
            load_partials<kPJ, U8>(pt, pos + kNarrowWaves, tpf, (tov >> (fi + kNarrowWaves)) & 1, lane, pre);
        if (kPF && fi + kNarrowWaves < nt && pb0 < w64)
            load_chunks<kNC>(rows + (pos + kNarrowWaves) * w64, w64, pb0, lane, *reinterpret_cast<uint64_t (*)[kNC]>(xs0));

        if (POST_DIAG & 8) continue;
        score_file<kMatrix, KM, kTJ>(crow32, tcs, Tf, ldf, file, wf, lf, cc, corpus_fast, thr, best_out, ov_out, score_out,
                                            k, mov, msc, tki, tks, lanef);
    }
    }
}

// Match mode held to 64 VGPRs (8 waves per SIMD: two workgroups per CU); the matrix mode's
// top-k slots need more registers and run at the occupancy they get.
// U8: the partials come as byte rows where the prefix allows (Partials.flag); the u16-only form is a
// separate instantiation, so its registers are those of the rounds before byte rows
template <int TPMAX, bool U8>
__global__ __launch_bounds__(narrow_waves<false>() * kWave) __attribute__((amdgpu_waves_per_eu(POST_NARROW_OCC, POST_NARROW_OCC))) void dice_post_narrow_match(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tp,
    const Partials pt, const uint16_t* __restrict__ prow, const uint16_t* __restrict__ plong,
    const uint2* __restrict__ tc, const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp,
    const uint8_t* __restrict__ ccp, double thr, int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out,
    double* __restrict__ score_out, int32_t k, uint32_t* __restrict__ mov, double* __restrict__ msc,
    int32_t* __restrict__ tki, double* __restrict__ tks, bool corpus_fast,
    const int32_t* __restrict__ idx, const uint32_t* __restrict__ pn, int32_t ld) {
    post_narrow_body<false, 1, TPMAX, U8>(rows, n, w64, D, T, tp, pt, prow, plong, tc, wfp, lenp, ccp, thr, best_out, ov_out,
                               score_out, k, mov, msc, tki, tks, corpus_fast, idx, pn, ld);
}

// POST_MATRIX_OCC (A/B): waves per SIMD the matrix kernel is compiled for (6 with its 8-wave
// workgroups: three per CU; 8 with 16-wave workgroups: two workgroups
// per CU as in match mode, at 64 VGPRs)
#ifndef POST_MATRIX_OCC
#define POST_MATRIX_OCC 6
#endif
template <int KM, int TPMAX, bool U8>
__global__ __launch_bounds__(narrow_waves<true>() * kWave) __attribute__((amdgpu_waves_per_eu(POST_MATRIX_OCC, POST_MATRIX_OCC))) void dice_post_narrow_matrix(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tp,
    const Partials pt, const uint16_t* __restrict__ prow, const uint16_t* __restrict__ plong,
    const uint2* __restrict__ tc, const uint32_t* __restrict__ wfp, const int32_t* __restrict__ lenp,
    const uint8_t* __restrict__ ccp, double thr, int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out,
    double* __restrict__ score_out, int32_t k, uint32_t* __restrict__ mov, double* __restrict__ msc,
    int32_t* __restrict__ tki, double* __restrict__ tks, bool corpus_fast,
    const int32_t* __restrict__ idx, const uint32_t* __restrict__ pn, int32_t ld) {
    post_narrow_body<true, KM, TPMAX, U8>(rows, n, w64, D, T, tp, pt, prow, plong, tc, wfp, lenp, ccp, thr, best_out, ov_out,
                               score_out, k, mov, msc, tki, tks, corpus_fast, idx, pn, ld);
}

// ---- host side ---------------------------------------------------------------------------

// Estimated per-file cost (wave instructions) of a dense prefix of D u64 words: the dense
// phase pays T*D*wd per file (VALU kernel: 4/64 -- a v_bcnt pair per template, word and 64-file
// wave; the FP4 matrix-core kernel: 1/128, eight times less per word, which moves the optimum to
// the 20-word cap on the config-3 corpus, as measured: DESIGN.md 4); every narrow membership a
// file hits costs ~1/16 of a 6-instruction row walk. A file resembling template t holds t's
// words, so the expected narrow memberships per file are sum over narrow words of p_w^2 / T
// (p_w = postings length).
static int pick_dense(const std::vector<int64_t>& sq_per_u64, int32_t T, int32_t w64, int maxd, double wd) {
    const char* e = getenv("DICE_POST_DENSE");
    if (e && *e) return std::max(0, std::min(std::min(maxd, w64), atoi(e)));
    double rest = 0;
    for (int64_t v : sq_per_u64) rest += (double)v;
    int best_d = 0;
    double best_c = 0.4 * rest / T;
    double c_dense = 0;
    for (int d = 1; d <= std::min(maxd, w64); ++d) {
        rest -= (double)sq_per_u64[d - 1];
        c_dense = (double)T * d * wd;
        const double c = c_dense + 0.4 * rest / T;
        if (c < best_c) { best_c = c; best_d = d; }
    }
    return best_d;
}

bool post_feasible(const dice_templates* t) {
    const int32_t tpad = (t->n_templates + 63) / 64 * 64;
    if (tpad > kPostMaxTpad) return false;
    for (int32_t i = 0; i < t->n_templates; ++i) {
        // u16 dense partials, packed constants: base in 16 bits, slack in int16, length in 31 bits
        const int64_t base = (int64_t)t->lf_size[i] - (int64_t)t->fields_set_size[i];
        if (t->lf_size[i] >= 65535u || base < 0 || base > 65535 || t->length_slack[i] < -32768 ||
            t->length_slack[i] > 32767 || t->length[i] < 0)
            return false;
    }
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
    // the dense prefix on the matrix cores, FP4 form (4, default: config 3 all pairs 3.76 -> 3.59 ms,
    // 5-T600 5.33 -> 5.15 ms against the int8 form, 2 interleaved reps); 1: the int8 form; 0: the
    // VALU kernel (A/B)
    const char* mf = getenv("DICE_POST_MFMA");
    c->post_mfma = (mf && *mf == '0') ? 0 : (mf && *mf == '1') ? 1 : 4;
    // the dense phase runs D rounded up to a multiple of 4 anyway (kernel template): use them all;
    // up to 20 words on the matrix cores, 16 on the VALU kernel (their LDS budgets)
    const int maxd = c->post_mfma ? kMfmaMaxDense : kPostMaxDense;
    const double wd = c->post_mfma == 4 ? 1.0 / 128 : c->post_mfma ? 1.0 / 64 : 4.0 / 64;
    const int D = std::min(std::min(w64, maxd), (pick_dense(sq, T, w64, maxd, wd) + 3) / 4 * 4);
    // one 32-byte postings row per narrow word (u64 words >= D), indexed by word id: a SHORT word
    // (<= 16 templates) lists its template ids ascending, 0xFFFF padding; a LONG word stores its
    // offset into the flat `plong` id list in entries 0-1, its length in entry 2, 0xFFFE in 15
    std::vector<uint16_t> prow((size_t)nbits * kRowW, kNoTpl);
    std::vector<uint32_t> loff((size_t)nbits, 0);
    uint32_t nlong = 0;
    for (int64_t w = 0; w < nbits; ++w) {
        loff[(size_t)w] = nlong;
        if (w / 64 >= D && plen[(size_t)w] > kRowW) {
            nlong += (uint32_t)plen[(size_t)w];
            uint16_t* r = &prow[(size_t)w * kRowW];
            r[0] = (uint16_t)(loff[(size_t)w] & 0xFFFF);
            r[1] = (uint16_t)(loff[(size_t)w] >> 16);
            r[2] = (uint16_t)plen[(size_t)w];
            r[kRowW - 1] = kMore;
        }
    }
    std::vector<uint16_t> plong((size_t)std::max<uint32_t>(nlong, 1), kNoTpl);
    std::vector<uint32_t> fill((size_t)nbits, 0);
    for (int32_t i = 0; i < T; ++i) {
        const uint64_t* r = t->lf_bits + (size_t)i * w64;
        for (int32_t p = D; p < w64; ++p)
            for (uint64_t x = r[p]; x; x &= x - 1) {
                const int64_t w = (int64_t)p * 64 + __builtin_ctzll(x);
                const uint32_t j = fill[(size_t)w]++;
                if (plen[(size_t)w] <= kRowW) prow[(size_t)w * kRowW + j] = (uint16_t)(4 * i);
                else plong[(size_t)loff[(size_t)w] + j] = (uint16_t)(4 * i);
            }
    }
    // a short row's entries in a per-word pseudo-random order (default; DICE_POST_ROW_SHUFFLE=0
    // keeps them ascending): the walk adds entry k of 64 words in one ds_add, and a file's own
    // template sits at similar ranks of its words' ascending rows -- the same counter address in
    // many lanes of one instruction, whose adds the LDS serializes. Shuffled, that template's hits
    // spread evenly over the entry slots (config 3 all pairs 3.44 -> 3.37 ms, 3 interleaved reps)
    {
        const char* rs = getenv("DICE_POST_ROW_SHUFFLE");
        if (!(rs && *rs == '0'))
            for (int64_t w = (int64_t)D * 64; w < nbits; ++w) {
                const int32_t m = plen[(size_t)w];
                if (m < 2 || m > kRowW) continue;
                uint16_t* r = &prow[(size_t)w * kRowW];
                uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(w + 1);
                for (int32_t i = m - 1; i > 0; --i) {   // Fisher-Yates over the m entries
                    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
                    std::swap(r[i], r[(int32_t)(x % (uint64_t)(i + 1))]);
                }
            }
    }
    // dense prefix masks, template-major [T][kPostMaxDense]; template constants
    std::vector<uint64_t> dm((size_t)T * kPostMaxDense, 0);
    for (int32_t i = 0; i < T; ++i)
        for (int d = 0; d < std::min(D, kPostMaxDense); ++d) dm[(size_t)i * kPostMaxDense + d] = t->lf_bits[(size_t)i * w64 + d];
    // template constants packed for LDS: {length | cc << 31, base | slack << 16} (post_feasible
    // checks the ranges)
    std::vector<uint2> tcv((size_t)T);
    for (int32_t i = 0; i < T; ++i) {
        const uint32_t base = t->lf_size[i] - t->fields_set_size[i];
        tcv[i] = make_uint2((uint32_t)t->length[i] | (t->is_cc[i] ? 0x80000000u : 0u),
                            (base & 0xFFFFu) | ((uint32_t)(t->length_slack[i] & 0xFFFF) << 16));
    }
    int rc;
    if ((rc = dalloc_bytes(&c->d_prow, prow.size() * 2)) || (rc = dalloc_bytes(&c->d_povf, plong.size() * 2)) ||
        (rc = dalloc_bytes(&c->d_pdm, dm.size() * 8)) || (rc = dalloc_bytes(&c->d_ptc, tcv.size() * sizeof(uint2))))
        return rc;
    // the masks word-major for the MFMA kernels: [q][kMfmaCols], q < kMfmaMaxDense, zero for t >= T
    // and for q >= D
    std::vector<uint64_t> dmt((size_t)kMfmaMaxDense * kMfmaCols, 0);
    for (int32_t i = 0; i < T; ++i)
        for (int d = 0; d < D; ++d) dmt[(size_t)d * kMfmaCols + i] = t->lf_bits[(size_t)i * w64 + d];
    if ((rc = dalloc_bytes(&c->d_pdmt, dmt.size() * 8))) return rc;
    if (hipMemcpy(c->d_pdmt, dmt.data(), dmt.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "postings plan upload failed");
    if (hipMemcpy(c->d_povf, plong.data(), plong.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_prow, prow.data(), prow.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_pdm, dm.data(), dm.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_ptc, tcv.data(), tcv.size() * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "postings plan upload failed");
    c->post_dense = D;
    c->post_tpad = tpad;
    // the dense prefix on the matrix cores (dice_post_dense_mfma) unless DICE_POST_MFMA=0
    const char* mt = getenv("DICE_POST_MFMA_MT");   // 32-file M-tiles per MFMA tile (2 or 3; A/B)
    c->post_mfma_mt = (mt && *mt == '2') ? 2 : 3;
    const char* u8 = getenv("DICE_POST_U8");   // byte partial rows where the prefix allows (A/B: 1; slower)
    c->post_u8 = u8 && *u8 == '1';
    // corpus part of the 24-bit compare envelope: |Lf| < 2^11 (overlaps), 1 <= base < 2^18,
    // template lengths < 2^20 and 200 |Lf| < 1024 base (every fast-file score < 1024)
    c->post_fast = true;
    for (int32_t i = 0; i < T; ++i) {
        const int64_t base = (int64_t)t->lf_size[i] - (int64_t)t->fields_set_size[i];
        if (!(t->lf_size[i] < (1u << 11) && base >= 1 && base < (1 << 18) && t->length[i] >= 0 &&
              t->length[i] < (1 << 20) && 200 * (int64_t)t->lf_size[i] < 1024 * base))
            c->post_fast = false;
    }
    c->post_tp = (T + 7) / 8 * 8;
    // matrix rows of whole 128-byte lines ([n][ld] u32 and f64): no row shares a line with the next
    // file's (another wave's) -- partial-line writes cost read-modify-write traffic in HBM
    c->post_ld = (T + 31) / 32 * 32;
    c->post_rows = nlong;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->n_cu < 1)
        c->n_cu = 256;
    c->kind = 3;
    return DICE_OK;
}

// The batch's partials region: [capacity][tp] u16 rows | [capacity][s8] u32 words of u8 rows |
// [capacity] flags. u8: the launch writes byte rows where a file's prefix allows (the matrix-core
// dense kernels, DICE_POST_U8); otherwise flag = nullptr and every row is u16.
static int32_t partials_s8(const dice_ctx* c) { return u8_row_words(c->post_tp); }
static Partials partials_of(const dice_ctx* c, const dice_batch* b, bool u8) {
    char* base = reinterpret_cast<char*>(b->d_pdense);
    const size_t n16 = (size_t)b->capacity * c->post_tp * 2, n8 = (size_t)b->capacity * partials_s8(c) * 4;
    Partials pt;
    pt.p16 = reinterpret_cast<uint16_t*>(base);
    pt.p8 = reinterpret_cast<uint32_t*>(base + n16);
    pt.flag = u8 ? reinterpret_cast<uint8_t*>(base + n16 + n8) : nullptr;
    return pt;
}

template <int DP>
static void launch_dense(dice_ctx* c, dice_batch* b, hipStream_t s, int64_t groups, const int32_t* idx,
                         const uint32_t* pn, const Partials& pt) {
    if (c->post_mfma) {
        // kMfmaNT N-tiles of 32 templates per wave: 10 waves cover 640 templates (tp <= 640), 11 704;
        // persistent workgroups (one per CU: 10-11 waves at 3 per SIMD), the next tile's prefixes
        // loaded during this one
        const bool small = c->post_tp <= 640;
        auto kern = c->post_mfma == 4
                        ? (small ? (c->post_mfma_mt == 3 ? (pt.flag ? dice_post_dense_mfma<DP, kMfmaNT, 12, 3, true, true>
                                                                    : dice_post_dense_mfma<DP, kMfmaNT, 12, 3, true>)
                                                         : dice_post_dense_mfma<DP, kMfmaNT, 12, 2, true>)
                                 : dice_post_dense_mfma<DP, kMfmaNT, 11, 2, true>)
                        : (small ? (c->post_mfma_mt == 3 ? dice_post_dense_mfma<DP, kMfmaNT, 12, 3>
                                                         : dice_post_dense_mfma<DP, kMfmaNT, 12, 2>)
                                 : dice_post_dense_mfma<DP, kMfmaNT, 11, 2>);
        const int64_t mtiles = (b->n + 32 * c->post_mfma_mt - 1) / (32 * c->post_mfma_mt);
        const int64_t g = std::min<int64_t>(std::min<int64_t>(groups, mtiles), (int64_t)c->n_cu);
        hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3((small ? 12 : 11) * kWave), 0, s,
                           (const uint64_t*)b->d_rows, b->n, c->w64, c->post_dense, c->post_tp,
                           (const uint64_t*)c->d_pdmt, pt, idx, pn);
        return;
    }
    if constexpr (DP <= kPostMaxDense) {   // (the VALU kernel's prefix is capped at 16 words: post_setup)
        auto kern = c->post_tp <= 608 ? dice_post_dense<DP, 608> : dice_post_dense<DP, kPostMaxTpad>;
        hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(kPostWaves * kWave), 0, s,
                           (const uint64_t*)b->d_rows, b->n, c->w64, c->post_dense, c->T, c->post_tp,
                           (const uint64_t*)c->d_pdm, pt, idx, pn);
    }
}

int post_reserve(dice_ctx* c, dice_batch* b) {
    // u16 rows, u8 rows and flags (partials_of)
    const size_t need = (size_t)b->capacity * c->post_tp * 2 + (size_t)b->capacity * partials_s8(c) * 4 +
                        (size_t)b->capacity;
    if (b->pdense_bytes < need) {
        if (b->d_pdense) (void)hipFree(b->d_pdense);
        b->d_pdense = nullptr;
        b->pdense_bytes = 0;
        int rc = dalloc_bytes(&b->d_pdense, need);
        if (rc) return rc;
        b->pdense_bytes = need;
    }
    return DICE_OK;
}

// idx/pn (match mode only): score the *pn files idx[0..*pn) of the batch (the pruned match's
// deferred files) on persistent grids; nothing is read back on the host.
template <bool kMatrix, int KM>
static int launch(dice_ctx* c, dice_batch* b, double thr, int32_t k, hipStream_t s, const int32_t* idx = nullptr,
                  const uint32_t* pn = nullptr) {
    int rc = post_reserve(c, b);
    if (rc) return rc;
    const int64_t tiles = (b->n + kPostFiles - 1) / kPostFiles;
    // two workgroups per CU are resident in either kernel (LDS)
    // (the narrow kernel's workgroups resident per CU: two 16-wave, three 8-wave)
    constexpr int kNarrowWaves = narrow_waves<kMatrix>();
    const int64_t groups = idx ? std::min<int64_t>(tiles, (kNarrowWaves == 16 ? 2 : 3) * (int64_t)c->n_cu) : tiles;
    const bool dense = c->post_dense > 0 && !(POST_DIAG & 1);
    // (byte rows: the FP4 kernel at 3 M-tiles, tp <= 640, the one instantiated with them)
    const Partials pt = partials_of(c, b, dense && c->post_mfma == 4 && c->post_u8 && c->post_tp <= 640 &&
                                              c->post_mfma_mt == 3);
    if (!dense) {
        // no dense prefix: zero u16 partials
        const size_t rows = (size_t)(idx ? b->capacity : b->n);
        if (hipMemsetAsync(pt.p16, 0, rows * c->post_tp * 2, s) != hipSuccess)
            return fail(DICE_E_DEVICE, "hipMemsetAsync failed");
    } else {
        switch ((c->post_dense + 3) / 4) {
            case 1: launch_dense<4>(c, b, s, groups, idx, pn, pt); break;
            case 2: launch_dense<8>(c, b, s, groups, idx, pn, pt); break;
            case 3: launch_dense<12>(c, b, s, groups, idx, pn, pt); break;
            case 4: launch_dense<16>(c, b, s, groups, idx, pn, pt); break;
            default: launch_dense<20>(c, b, s, groups, idx, pn, pt); break;
        }
    }
    auto kern = pt.flag ? (c->post_tp <= 608 ? (kMatrix ? dice_post_narrow_matrix<KM, 608, true> : dice_post_narrow_match<608, true>)
                                             : (kMatrix ? dice_post_narrow_matrix<KM, kPostMaxTpad, true>
                                                        : dice_post_narrow_match<kPostMaxTpad, true>))
                        : (c->post_tp <= 608 ? (kMatrix ? dice_post_narrow_matrix<KM, 608, false> : dice_post_narrow_match<608, false>)
                                             : (kMatrix ? dice_post_narrow_matrix<KM, kPostMaxTpad, false>
                                                        : dice_post_narrow_match<kPostMaxTpad, false>));
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(kNarrowWaves * kWave), 0, s,
                       (const uint64_t*)b->d_rows, b->n, c->w64, c->post_dense, c->T, c->post_tp,
                       pt, (const uint16_t*)c->d_prow, (const uint16_t*)c->d_povf,
                       (const uint2*)c->d_ptc, b->d_wf, b->d_len, b->d_cc, thr, b->d_best, b->d_ov, b->d_score, k,
                       b->d_mov, b->d_mscore, k > 0 ? b->d_tki : nullptr, b->d_tks, c->post_fast, idx,
                       pn, c->post_ld);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_post kernels launch failed");
}

// confidence: Dice#confidence outputs (the match kernel's k argument, unused in match mode, = 1)
int post_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, bool confidence) {
    return launch<false, 1>(c, b, thr, confidence ? 1 : 0, s);
}

int post_launch_match_indexed(dice_ctx* c, dice_batch* b, double thr, const int32_t* idx, const uint32_t* pn,
                              hipStream_t s, bool confidence) {
    return launch<false, 1>(c, b, thr, confidence ? 1 : 0, s, idx, pn);
}

int post_launch_matrix(dice_ctx* c, dice_batch* b, int32_t k, hipStream_t s) {
    // any k <= 16: one candidate per lane, k wave argmax rounds (score_file_t)
    return launch<true, 1>(c, b, 0.0, k, s);
}

}  // namespace dice
