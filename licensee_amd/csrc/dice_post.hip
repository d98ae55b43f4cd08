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
//   dice_post_dense_mfma: the files' first D u64 words against the template masks as a binary
//            matrix product on the matrix cores (FP4 block-scaled MFMA, persistent workgroups; see
//            below), written as a row-major [n][tp] u16 matrix of partial overlaps;
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

// Phase-skip diagnostics (tools/build_variant.sh -DPOST_DIAG=n; results are wrong): 1 skips the
// dense kernel, 2 the postings walk, 4 the narrow-word extraction, 8 scoring. (Round 6's fusion-cost
// probe, 16 / 48, and the matrix kernel with walk and store waves are in the history:
// profiles/r6_fusion_probe.txt, profiles/r6_store_waves_ab.txt)
#ifndef POST_DIAG
#define POST_DIAG 0
#endif
// The walk's padding entries go to per-lane sinks instead of exec-masked adds (count_or_sink).
// Waves per workgroup of the narrow kernels: the match kernel 16 (two workgroups per CU, 8 waves
// per SIMD); the matrix kernel 8 at 6 waves per SIMD (three workgroups fit a CU's LDS; 5-T600
// 5.17 -> 5.09 ms, 2 interleaved reps; the match kernel measured 3.54 -> 3.60 ms that way)
constexpr int kNarrowWavesMatch = 16, kNarrowOccMatch = 8;
constexpr int kNarrowWavesMatrix = 8, kNarrowOccMatrix = 6;
template <bool kMatrix>
constexpr int narrow_waves() { return kMatrix ? kNarrowWavesMatrix : kNarrowWavesMatch; }
constexpr int kPostFiles = 64;           // files per workgroup (one tile)
constexpr int kPostMaxTpad = 704;        // templates of the largest instantiation (LDS budget)
constexpr int kRowW = 16;                // template ids per postings row
// per-wave queue of narrow word ids: as long as the narrow kernel's LDS allows two workgroups
// per CU (counter rows for TPMAX templates beside it)
template <int TPMAX>
constexpr int word_cap() { return TPMAX <= 608 ? 416 : 320; }
constexpr uint16_t kNoTpl = 0xFFFF;      // empty row entry
constexpr uint16_t kMore = 0xFFFE;       // row entry 15: a long word (entries 0-1 offset, 2 length)
constexpr int kLongCap = 64;             // per-wave queue of long words (offset, length)
// 64-word chunks of a file loaded together (match and matrix kernel)
constexpr int kChunks = 6;

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
#pragma unroll
            for (int k = 0; k < 8; ++k) count_or_sink(cbase, sink, (r2[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
        }
        if (nl > kLongCap - kWave) walk_long(lq, nl, plong, crow32, lane);
        w = wn;
        r0 = n0;
        r1 = n1;
    }
}

// The dense prefix on the matrix cores (dice_post_dense_mfma). The prefix overlap |W_F ∩ Lf_t ∩
// prefix| is a binary matrix product -- files x prefix bits times prefix bits x templates -- so
// with bits widened to 0/1 operands an MFMA computes a 32-file x 32-template tile exactly: the FP4
// v_mfma_scale_f32_32x32x64_f8f6f4 takes a whole u64 prefix word per instruction (K = 64: lane
// half h holds the word's bits [32 h, 32 h + 32) as 32 nibbles; counts <= 1280, exact in f32). A
// persistent workgroup (one per CU) = NW waves over tiles of MT x 32 files (MT = 3 for T <= 640,
// else 2); wave w owns 1-2 N-tiles of 32 templates (the ceil(T / 32) tiles dealt so the SIMDs'
// shares differ by at most one; 12 waves at 3 per SIMD, 11 above 640 templates), and each template
// fragment serves the MT M-tiles. Per u64 prefix word q: the files' words from the LDS-staged
// prefixes, the templates' words from the word-major masks (staged in LDS once per workgroup, as
// low/high u32 planes), each lane's bits widened to e2m1 nibbles (widen_a / widen_b), then MT x
// NTW MFMAs. A and B place the same bit in the same fragment element, so the products pair the
// same bits whatever the hardware's k order inside a step. Accumulator register g of lane (h, c)
// is file 32 m + (g & 3) + 8 (g >> 2) + 4 h, template 32 j + c: transposed through a per-wave
// 16 x 64 LDS slab and stored as 16-byte pieces of the [n][tp] u16 partial rows (a wave's 64
// templates of one file are 128 contiguous bytes). The next tile's prefixes are loaded into
// registers while this tile is scored (LDS waits count lgkmcnt, so they fly across the tile) and
// written to the other LDS buffer before this tile's stores are issued (one barrier per tile).
// (5-T600 dense kernel: round 4 1.70 -> 0.68 ms, the VALU kernel 1.45, profiles/r4_mfma_dense.txt;
// round 5 FP4 0.58, then 0.46 ms, profiles/r5_dense_ab.txt; the retired int8 and VALU forms are
// in DESIGN.md Appendix B.)
constexpr int kMfmaNT = 2;       // N-tiles per wave (at most)
constexpr int kMfmaCols = 768;   // template columns of the word-major masks (>= 11 waves x 2 N-tiles x 32)
constexpr int kMfmaMaxDense = 20;   // prefix u64 words (the masks' LDS budget)
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kE8M0One = 0x7F7F7F7F;   // block scale 2^0 in every byte

// Bits to e2m1 nibbles, one fragment dword k per bit class: nibble i of dword k holds bit 4 i + k
// of the word, left where a mask finds it, so the two operands carry different e2m1 values per
// dword and each product is still exactly 1.0 at block scales 2^0:
//   dword   A (file prefix)          value   B (template mask)          value
//   0       v & 0x11111111           0.5     (v << 2) & 0x44444444      2.0
//   1       v & 0x22222222           1.0     v & 0x22222222             1.0
//   2       v & 0x44444444           2.0     (v >> 2) & 0x11111111      0.5
//   3       (v >> 1) & 0x44444444    2.0     (v >> 3) & 0x11111111      0.5
// (e2m1 0b0001 = 0.5, 0b0010 = 1.0, 0b0100 = 2.0; bit 3 of a nibble is the sign): 5 VALU for A,
// 7 for B, and A is widened MT times per word. FP4 operands use the first four registers.
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
constexpr int kSlabCols = 64;   // u16 per slab row (one wave's two N-tiles)
template <int MT>
__device__ __forceinline__ void mfma_store_tile(const v16f (&acc)[MT][2], uint16_t* slab, uint16_t* __restrict__ part,
                                                int64_t f0, int64_t nn, int32_t tb, int32_t te, int32_t tp, int lane) {
    int32_t tpf = tp, lf = lane;
    asm volatile("" : "+s"(tpf), "+v"(lf));   // addresses formed here, per tile
    const int32_t rf = lf & 31, hf = lf >> 5;
    const int32_t nt = (te - tb) / 32;   // the wave's N-tiles (uniform: 0, 1 or 2)
    if (nt == 0) return;
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
                        slab[((g & 3) + 8 * ((g >> 2) & 1) + 4 * hf) * kSlabCols + 32 * j + rf] =
                            (uint16_t)(uint32_t)acc[m][j][g];
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (nt == 2) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int row = (lf >> 3) + 8 * i, piece = lf & 7;
                    const uint4 v = *reinterpret_cast<const uint4*>(slab + row * kSlabCols + piece * 8);
                    const int64_t file = f0 + 32 * m + 16 * sh + row;
                    const int32_t t = tb + piece * 8;
                    if (t < tpf && file < nn) *reinterpret_cast<uint4*>(part + file * tpf + t) = v;
                }
            } else {
                const int row = lf >> 2, piece = lf & 3;
                const uint4 v = *reinterpret_cast<const uint4*>(slab + row * kSlabCols + piece * 8);
                const int64_t file = f0 + 32 * m + 16 * sh + row;
                const int32_t t = tb + piece * 8;
                if (t < tpf && file < nn) *reinterpret_cast<uint4*>(part + file * tpf + t) = v;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int DP, int NTW, int NW, int MT>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(3, 3))) void dice_post_dense_mfma(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t tp,
    const uint64_t* __restrict__ dmask, uint16_t* __restrict__ part, const int32_t* __restrict__ idx,
    const uint32_t* __restrict__ pn) {
    // MT 32-file M-tiles per tile; the prefix buffer is doubled when LDS allows (one barrier per
    // tile; every shipped shape since the 16 x 64 slabs), else one buffer and a second barrier
    static_assert(DP <= kMfmaMaxDense, "prefix wider than the masks' table");
    static_assert(NTW == 2, "two N-tiles per wave (the store slab)");
    constexpr int kTF = 32 * MT;                     // files per tile
    // DP + 1 u64 per file row (odd: the 32 lanes of a column read hit distinct banks)
    constexpr int kPreStride = DP + 1;
    constexpr int kPreWords = kTF * DP;
    constexpr int kPer = (kPreWords + NW * kWave - 1) / (NW * kWave);   // prefix words per thread
    constexpr int kCols = NTW == 2 && NW == 12 ? 640 : NW * NTW * 32;   // the workgroup's template columns
    constexpr size_t kFixed = (size_t)DP * kCols * 8 + (size_t)NW * 16 * kSlabCols * 2;
    constexpr int kBufs = kFixed + 2 * (size_t)kTF * kPreStride * 8 <= 160 * 1024 ? 2 : 1;
    __shared__ uint64_t pre[kBufs][kTF * kPreStride];   // file prefixes as low / high u32 planes
    __shared__ uint64_t bm[DP * kCols];              // template masks, word-major planes (<= 100 KiB at DP 20)
    __shared__ uint16_t tslab[NW][16 * kSlabCols];   // per-wave 16 x 64 transpose slab (2 KiB)
    static_assert(sizeof(pre) + sizeof(bm) + sizeof(tslab) <= 160 * 1024, "one workgroup's LDS");
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
    // this thread's share of a tile's prefix words (file i / DP, word i % DP)
    auto load_pre = [&](int64_t fs, uint64_t (&pv)[kPer]) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = (int)threadIdx.x + k * NW * kWave;
            const int fi = i / DP, d = i % DP;
            const int64_t file = fs + fi;
            pv[k] = (i < kPreWords && file < nn && d < D) ? rows[(idx ? (int64_t)idx[file] : file) * w64 + d] : 0;
        }
    };
    auto store_pre = [&](int buf, const uint64_t (&pv)[kPer]) {
        uint32_t* p32 = reinterpret_cast<uint32_t*>(pre[buf]);
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = (int)threadIdx.x + k * NW * kWave;
            if (i < kPreWords) {   // low and high dwords in two planes
                const int at = (i / DP) * kPreStride + i % DP;
                p32[at] = (uint32_t)pv[k];
                p32[kTF * kPreStride + at] = (uint32_t)(pv[k] >> 32);
            }
        }
    };
    // the masks once per (persistent) workgroup: LDS reads in the k-loop wait on lgkmcnt, so the
    // next tile's prefix loads (vmcnt) fly across the whole tile
    for (int i = threadIdx.x; i < DP * kCols; i += NW * kWave) {
        const uint64_t v = dmask[(i / kCols) * kMfmaCols + i % kCols];
        reinterpret_cast<uint32_t*>(bm)[i] = (uint32_t)v;
        reinterpret_cast<uint32_t*>(bm)[DP * kCols + i] = (uint32_t)(v >> 32);
    }
    uint64_t pv[kPer];
    load_pre(f0, pv);
    store_pre(0, pv);
    __syncthreads();
    for (int buf = 0; f0 < nn; f0 += stride, buf = (buf + 1) % kBufs) {
        // unconditional (zeros past the end): a load under `if (more)` left pending on the skip path
        // would make the loop head wait vmcnt(0) for this tile's stores
        load_pre(f0 + stride, pv);
        v16f acc[MT][NTW];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int j = 0; j < NTW; ++j) acc[m][j] = v16f{};
        // lane half h reads its dwords from plane h (no 64-bit shift; conflict-free b32 reads: the
        // prefix rows' stride is odd) and widens them without shifts where the nibble class allows
        const uint32_t* pa0 = reinterpret_cast<const uint32_t*>(pre[buf]) + h * (kTF * kPreStride) + r * kPreStride;
        const uint32_t* pw0 = reinterpret_cast<const uint32_t*>(bm) + h * (DP * kCols) + tb + r;
#pragma unroll 2
        for (int q = 0; q < DP; ++q) {
            uint32_t bw32[NTW];
#pragma unroll
            for (int j = 0; j < NTW; ++j) bw32[j] = j < nw_tiles ? pw0[q * kCols + j * 32] : 0;   // (uniform: no read past bm)
            v8i fa[MT];
#pragma unroll
            for (int m = 0; m < MT; ++m) fa[m] = widen_a(pa0[32 * m * kPreStride + q]);
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                if (j < nw_tiles) {   // uniform
                    const v8i fb = widen_b(bw32[j]);
#pragma unroll
                    for (int m = 0; m < MT; ++m)
                        acc[m][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[m], fb, acc[m][j], 4, 4, 0,
                                                                                     kE8M0One, 0, kE8M0One);
                }
            }
        }
        if (kBufs == 1) __syncthreads();   // every wave is done with the one prefix buffer
        // the next tile's prefixes into LDS before this tile's stores are issued: the wait on their
        // loads (vmcnt counts stores too, in order) then finds only the previous tile's stores,
        // issued a whole k-loop ago, and this tile's stores drain under the next tile's MFMAs
        store_pre((buf + 1) % kBufs, pv);
        mfma_store_tile<MT>(acc, tslab[wave], part, f0, nn, tb, tb + 32 * nw_tiles, tp, lane);
        __syncthreads();   // the next tile's prefixes are complete (MT = 2: the other buffer)
    }
}

// The file's dense partials into its counter row (a plain copy, widened: this wave's postings
// adds for the file come after it; the copy writes every entry, so the row is never re-zeroed),
// one LDS address and immediate offsets; part[] holds u16 pairs.
template <int PJ>
__device__ __forceinline__ void copy_in(uint32_t* crow32, const uint32_t (&part)[PJ], int32_t tp, int lane) {
    uint2* dst = reinterpret_cast<uint2*>(crow32) + lane;
#pragma unroll
    for (int j = 0; j < PJ; ++j)
        if (lane + j * kWave < tp / 2) dst[j * kWave] = make_uint2(part[j] & 0xFFFFu, part[j] >> 16);
}

// A file's partials as u16 pairs. CLAMP: unconditional loads at clamped indices (copy_in masks the
// rest), else exec-masked ones.
template <int PJ, bool CLAMP>
__device__ __forceinline__ void load_partials(const uint16_t* __restrict__ part16, int64_t pos, int32_t tp, int lane,
                                              uint32_t (&part)[PJ]) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(part16 + pos * tp);
    const int32_t nw = tp / 2;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
        const int32_t i = lane + j * kWave;
        if (CLAMP) part[j] = src[min(i, nw - 1)];
        else part[j] = i < nw ? src[i] : 0;
    }
}

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
template <int WCAP>
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
template <int WCAP, bool LATE, int PJ>
__device__ __forceinline__ void file_postings(const uint64_t* __restrict__ row, int32_t w64, int32_t pb0,
                                              const uint16_t* __restrict__ part16, int64_t pos, int32_t tp, uint32_t* wq,
                                              uint2* lq, const uint16_t* __restrict__ prow,
                                              const uint16_t* __restrict__ plong, uint32_t* crow32, int lane) {
    uint32_t nq = 0;           // queued narrow words (wave-uniform)
    uint32_t nl = 0;           // queued long words (uniform)
    // queue the file's narrow words (set bits of u64 words >= D), kChunks x 64 words loaded
    // together (queue_chunks). The first round is peeled so that LATE's partials are copied in
    // between its loads and their use and are dead for the rest of the file.
    int32_t pb = pb0;
    uint64_t xs[kChunks];
    if (LATE) {
        uint32_t part[PJ];
        load_partials<PJ, true>(part16, pos, tp, lane, part);
        if (pb < w64) load_chunks(row, w64, pb, lane, xs);
        copy_in<PJ>(crow32, part, tp, lane);
        if (pb < w64) {
            queue_chunks<WCAP>(xs, pb, wq, nq, lq, nl, prow, plong, crow32, lane);
            pb += kChunks * kWave;
        }
    }
    for (; pb < w64; pb += kChunks * kWave) {
        load_chunks(row, w64, pb, lane, xs);
        queue_chunks<WCAP>(xs, pb, wq, nq, lq, nl, prow, plong, crow32, lane);
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

#define DICE_STR(x) #x
#define DICE_UNROLL(n) _Pragma(DICE_STR(unroll n))
// Matrix top-k: each lane also keeps its second best, so the first time a lane's template is
// ranked its next candidate is that second one instead of a rescan of its templates from LDS
// (a lane ranked twice still rescans). Scoring loop unroll (1, 2, 5, 10 within 1% for the matrix
// kernel; the match kernel needs 57 instead of 64 VGPRs at 2).
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
    constexpr int kUnroll = kMatrix ? 10 : 2;
    DICE_UNROLL(kUnroll)
    for (int j = 0; j < TJ; ++j) {
        const int32_t t = (int32_t)lo + j * kWave;
        if (t < T) {
            uint32_t ov;
            int32_t den;
            if (kMatrix) {
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
                __builtin_nontemporal_store(ov, orow + t);
                __builtin_nontemporal_store(dice_score(ov, den), srow + t);
            }
        }
    }
    if (!kMatrix) {
        wave_best_dpp<FAST>(bi, bo, bd);
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
        bool second = true;   // the lane's second best not yet promoted
        for (int r = 0; r < k; ++r) {
            int32_t wi = bi, wd = bd;
            uint32_t wo = bo;
            wave_best_dpp<FAST>(wi, wo, wd);
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
                const bool promote = second;
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

template <bool kMatrix, int TJ>
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

template <int TPMAX>
constexpr int pairs_per_lane() { return (TPMAX / 2 + kWave - 1) / kWave; }   // u32 partial pairs per lane

// Phases 2 + 3, one file per wave (a 64-file tile per workgroup). Each wave owns one u32 counter
// row in LDS. Narrow words are queued from the file's u64 words >= D and walked (walk_short /
// walk_long) after the file's dense partials (from dice_post_dense_mfma) are copied in (every
// entry: no zeroing between files); scoring reads the counters and reduces over the wave. Match
// mode prefetches the next file's partials while it scores this one (its loads do not depend on
// the walk); the matrix kernel loads them at the file's start (file_postings LATE). The match
// kernel's LDS footprint (~77 KiB) and <= 64 VGPRs leave room for two workgroups per CU.
template <bool kMatrix, int TPMAX>
__device__ __forceinline__ void post_narrow_body(
    const uint64_t* __restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tp,
    const uint16_t* __restrict__ part16, const uint16_t* __restrict__ prow, const uint16_t* __restrict__ plong,
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
    // match mode: the next file's dense partials, prefetched while the wave scores the previous file
    constexpr bool kEarly = !kMatrix;
    uint32_t pre[kPJ];
    if (kEarly && wave < nt) load_partials<kPJ, false>(part16, f0 + wave, tp, lane, pre);
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
        if (kMatrix) asm volatile("" : "+s"(Tf), "+s"(tpf), "+s"(ldf), "+v"(lanef));
        // this file's dense partials start its counter row (matrix mode: inside file_postings)
        if (kEarly) copy_in<kPJ>(crow32, pre, tpf, lanef);
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
        file_postings<kWCap, !kEarly, kPJ>(row, w64, pb0, part16, pos, tpf, wq[wave], lq[wave], prow, plong, crow32,
                                           lanef);
        // the wave's next file's partials fly while this one is scored
        if (kEarly && fi + kNarrowWaves < nt) load_partials<kPJ, false>(part16, pos + kNarrowWaves, tpf, lane, pre);

        if (POST_DIAG & 8) continue;
        score_file<kMatrix, kTJ>(crow32, tcs, Tf, ldf, file, wf, lf, cc, corpus_fast, thr, best_out, ov_out, score_out,
                                 k, mov, msc, tki, tks, lanef);
    }
    }
}

// Match mode held to 64 VGPRs (8 waves per SIMD: two workgroups per CU); the matrix mode's
// top-k slots need more registers and run at 6 waves per SIMD (three 8-wave workgroups per CU).
#define POST_NARROW_ARGS                                                                                              \
    const uint64_t *__restrict__ rows, int64_t n, int32_t w64, int32_t D, int32_t T, int32_t tp,                     \
        const uint16_t *__restrict__ part16, const uint16_t *__restrict__ prow, const uint16_t *__restrict__ plong,   \
        const uint2 *__restrict__ tc, const uint32_t *__restrict__ wfp, const int32_t *__restrict__ lenp,             \
        const uint8_t *__restrict__ ccp, double thr, int32_t *__restrict__ best_out, uint32_t *__restrict__ ov_out,   \
        double *__restrict__ score_out, int32_t k, uint32_t *__restrict__ mov, double *__restrict__ msc,              \
        int32_t *__restrict__ tki, double *__restrict__ tks, bool corpus_fast, const int32_t *__restrict__ idx,       \
        const uint32_t *__restrict__ pn, int32_t ld
template <int TPMAX>
__global__ __launch_bounds__(kNarrowWavesMatch * kWave) __attribute__((amdgpu_waves_per_eu(kNarrowOccMatch, kNarrowOccMatch))) void dice_post_narrow_match(POST_NARROW_ARGS) {
    post_narrow_body<false, TPMAX>(rows, n, w64, D, T, tp, part16, prow, plong, tc, wfp, lenp, ccp, thr, best_out, ov_out,
                                   score_out, k, mov, msc, tki, tks, corpus_fast, idx, pn, ld);
}

template <int TPMAX>
__global__ __launch_bounds__(kNarrowWavesMatrix * kWave) __attribute__((amdgpu_waves_per_eu(kNarrowOccMatrix, kNarrowOccMatrix))) void dice_post_narrow_matrix(POST_NARROW_ARGS) {
    post_narrow_body<true, TPMAX>(rows, n, w64, D, T, tp, part16, prow, plong, tc, wfp, lenp, ccp, thr, best_out, ov_out,
                                  score_out, k, mov, msc, tki, tks, corpus_fast, idx, pn, ld);
}

// ---- host side ---------------------------------------------------------------------------

// Estimated per-file cost (wave instructions) of a dense prefix of D u64 words: the matrix-core
// dense phase pays T*D/128 per file (an FP4 MFMA covers a u64 word of 32 files x 32 templates,
// plus its widening), which puts the optimum at the 20-word cap on the config-3 corpus, as
// measured; every narrow membership a file hits costs ~1/16 of a 6-instruction row
// walk. A file resembling template t holds t's words, so the expected narrow memberships per file
// are sum over narrow words of p_w^2 / T (p_w = postings length).
static int pick_dense(const std::vector<int64_t>& sq_per_u64, int32_t T, int32_t w64) {
    const int maxd = std::min(kMfmaMaxDense, w64);
    const char* e = getenv("DICE_POST_DENSE");
    if (e && *e) return std::max(0, std::min(maxd, atoi(e)));
    double rest = 0;
    for (int64_t v : sq_per_u64) rest += (double)v;
    int best_d = 0;
    double best_c = 0.4 * rest / T;
    for (int d = 1; d <= maxd; ++d) {
        rest -= (double)sq_per_u64[d - 1];
        const double c = (double)T * d / 128.0 + 0.4 * rest / T;
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
    // the dense kernel runs D rounded up to a multiple of 4 anyway (kernel template): use them all,
    // up to 20 words (the masks' LDS budget)
    const int D = std::min(std::min(w64, kMfmaMaxDense), (pick_dense(sq, T, w64) + 3) / 4 * 4);
    // one 32-byte postings row per narrow word (u64 words >= D), indexed by word id: a SHORT word
    // (<= 16 templates) lists its template ids, 0xFFFF padding; a LONG word stores its offset into
    // the flat `plong` id list in entries 0-1, its length in entry 2, 0xFFFE in 15
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
    // a short row's m entries in a per-word pseudo-random order (entries [0, m) move; the padding
    // stays in m..15, so the walk's entry-8 ballot still tells 9-16 entries from fewer): the walk
    // adds entry k of 64 words in one ds_add, and a file's own template sat at similar ranks of its
    // words' ascending rows -- the same counter address in many lanes of one instruction, whose adds
    // the LDS serializes. Shuffled, that template's hits spread evenly over the entry slots (config
    // 3 all pairs 3.44 -> 3.37 ms against ascending rows, 3 interleaved reps)
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
    // template constants packed for LDS: {length | cc << 31, base | slack << 16} (post_feasible
    // checks the ranges)
    std::vector<uint2> tcv((size_t)T);
    for (int32_t i = 0; i < T; ++i) {
        const uint32_t base = t->lf_size[i] - t->fields_set_size[i];
        tcv[i] = make_uint2((uint32_t)t->length[i] | (t->is_cc[i] ? 0x80000000u : 0u),
                            (base & 0xFFFFu) | ((uint32_t)(t->length_slack[i] & 0xFFFF) << 16));
    }
    // the dense-prefix masks word-major for the matrix-core kernel: [q][kMfmaCols], q < kMfmaMaxDense,
    // zero for t >= T and for q >= D
    std::vector<uint64_t> dmt((size_t)kMfmaMaxDense * kMfmaCols, 0);
    for (int32_t i = 0; i < T; ++i)
        for (int d = 0; d < D; ++d) dmt[(size_t)d * kMfmaCols + i] = t->lf_bits[(size_t)i * w64 + d];
    int rc;
    if ((rc = dalloc_bytes(&c->d_prow, prow.size() * 2)) || (rc = dalloc_bytes(&c->d_povf, plong.size() * 2)) ||
        (rc = dalloc_bytes(&c->d_ptc, tcv.size() * sizeof(uint2))) || (rc = dalloc_bytes(&c->d_pdmt, dmt.size() * 8)))
        return rc;
    if (hipMemcpy(c->d_pdmt, dmt.data(), dmt.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_povf, plong.data(), plong.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_prow, prow.data(), prow.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_ptc, tcv.data(), tcv.size() * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "postings plan upload failed");
    c->post_dense = D;
    c->post_tpad = tpad;
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

// kMfmaNT N-tiles of 32 templates per wave: 12 waves cover 640 templates at 3 M-tiles (tp <= 640),
// 11 waves 704 at 2; persistent workgroups (one per CU at 3 waves per SIMD), the next tile's
// prefixes loaded during this one
template <int DP>
static void launch_dense(dice_ctx* c, dice_batch* b, hipStream_t s, int64_t groups, const int32_t* idx,
                         const uint32_t* pn) {
    const bool small = c->post_tp <= 640;
    const int mt = small ? 3 : 2;
    auto kern = small ? dice_post_dense_mfma<DP, kMfmaNT, 12, 3> : dice_post_dense_mfma<DP, kMfmaNT, 11, 2>;
    const int64_t mtiles = (b->n + 32 * mt - 1) / (32 * mt);
    const int64_t g = std::min<int64_t>(std::min<int64_t>(groups, mtiles), (int64_t)c->n_cu);
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3((small ? 12 : 11) * kWave), 0, s, (const uint64_t*)b->d_rows,
                       b->n, c->w64, c->post_dense, c->post_tp, (const uint64_t*)c->d_pdmt,
                       reinterpret_cast<uint16_t*>(b->d_pdense), idx, pn);
}

// The batch's dense partials, [capacity][tp] u16 rows.
int post_reserve(dice_ctx* c, dice_batch* b) {
    const size_t need = (size_t)b->capacity * c->post_tp * 2;
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
template <bool kMatrix>
static int launch(dice_ctx* c, dice_batch* b, double thr, int32_t k, hipStream_t s, const int32_t* idx = nullptr,
                  const uint32_t* pn = nullptr) {
    int rc = post_reserve(c, b);
    if (rc) return rc;
    const int64_t tiles = (b->n + kPostFiles - 1) / kPostFiles;
    // (the narrow kernel's workgroups resident per CU: two 16-wave, three 8-wave)
    constexpr int kNarrowWaves = narrow_waves<kMatrix>();
    const int64_t groups = idx ? std::min<int64_t>(tiles, (kNarrowWaves == 16 ? 2 : 3) * (int64_t)c->n_cu) : tiles;
    uint16_t* part16 = reinterpret_cast<uint16_t*>(b->d_pdense);
    if (c->post_dense == 0 || (POST_DIAG & 1)) {
        // no dense prefix: zero partials
        const size_t rows = (size_t)(idx ? b->capacity : b->n);
        if (hipMemsetAsync(part16, 0, rows * c->post_tp * 2, s) != hipSuccess)
            return fail(DICE_E_DEVICE, "hipMemsetAsync failed");
    } else {
        switch ((c->post_dense + 3) / 4) {
            case 1: launch_dense<4>(c, b, s, groups, idx, pn); break;
            case 2: launch_dense<8>(c, b, s, groups, idx, pn); break;
            case 3: launch_dense<12>(c, b, s, groups, idx, pn); break;
            case 4: launch_dense<16>(c, b, s, groups, idx, pn); break;
            default: launch_dense<20>(c, b, s, groups, idx, pn); break;
        }
    }
    auto kern = c->post_tp <= 608 ? (kMatrix ? dice_post_narrow_matrix<608> : dice_post_narrow_match<608>)
                                  : (kMatrix ? dice_post_narrow_matrix<kPostMaxTpad> : dice_post_narrow_match<kPostMaxTpad>);
    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(kNarrowWaves * kWave), 0, s,
                       (const uint64_t*)b->d_rows, b->n, c->w64, c->post_dense, c->T, c->post_tp,
                       part16, (const uint16_t*)c->d_prow, (const uint16_t*)c->d_povf,
                       (const uint2*)c->d_ptc, b->d_wf, b->d_len, b->d_cc, thr, b->d_best, b->d_ov, b->d_score, k,
                       b->d_mov, b->d_mscore, k > 0 ? b->d_tki : nullptr, b->d_tks, c->post_fast, idx,
                       pn, c->post_ld);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_post kernels launch failed");
}

// confidence: Dice#confidence outputs (the match kernel's k argument, unused in match mode, = 1)
int post_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, bool confidence) {
    return launch<false>(c, b, thr, confidence ? 1 : 0, s);
}

int post_launch_match_indexed(dice_ctx* c, dice_batch* b, double thr, const int32_t* idx, const uint32_t* pn,
                              hipStream_t s, bool confidence) {
    return launch<false>(c, b, thr, confidence ? 1 : 0, s, idx, pn);
}

int post_launch_matrix(dice_ctx* c, dice_batch* b, int32_t k, hipStream_t s) {
    // any k <= 16: one candidate per lane, k wave argmax rounds (score_file_t)
    return launch<true>(c, b, 0.0, k, s);
}

}  // namespace dice
