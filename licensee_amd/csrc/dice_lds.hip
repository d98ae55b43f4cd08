// LDS-tiled sparse scorer for large template sets (T > 64, BASELINE config 3: ~600 templates).
//
// Same contract as dice_dense_match (dice.rb:34-53 over content_helper.rb:128-133,337-347):
// per file, the argmax template among the unmasked ones, its overlap and its f64 score.
//
// Why a second kernel: at T ~ 600 the dense formulation (every template x every vocabulary
// dword: 2 VALU per 32 (file, word) pairs) is VALU-bound, and ~79% of the template dwords are
// zero. Here only non-zero template words are visited:
//
//   * one workgroup = 2 tiles (128 files) x 16 waves; lane l of every wave serves file l of
//     both tiles;
//   * the tiles' bitsets are staged through LDS in slabs of 128 u64 words per file (128 KiB),
//     layout [pair][lane][tile] (a lane's words of both tiles: one 16-byte ds_read_b128);
//   * wave w owns a contiguous template group (<= G templates per pass, balanced by record
//     count on the host); its G x 2 accumulators stay in VGPRs for the whole pass;
//   * one record {LDS byte offset, mask lo, mask hi, 0} per non-zero template u64 word. A
//     wave's records for one slab are contiguous in the table (its templates are consecutive),
//     so they stream into a per-wave 2 x 64-record LDS ring by LDS-DMA (global_load_lds_dwordx4,
//     1 KiB per wave-instruction) and are read back with uniform-address ds_read_b128. Per
//     step of 4 records: one ring batch, one batch of 4 ds_read_b128 file words, 16 VALU. No
//     scalar load shares the LGKM counter with the file reads (the earlier scalar-record form
//     ran 3.5% slower: DESIGN.md section 4);
//   * after the last pass the per-wave winners (dice_ge, later template wins exact ties) are
//     merged across the 16 waves through LDS.
//
// Template sets larger than 16 * G run in several passes over the same files.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "dice_common.h"
#include "dice_internal.h"

namespace dice {

constexpr int kLdsWaves = 16;
constexpr int kLdsBytes = 128 * 1024;                   // slab (the per-wave winners reuse it)
constexpr int kTiles = 2;                               // 64-file tiles per workgroup (files per lane)
constexpr int kG = 16;                                  // templates per wave per pass
// one u64 word of every file of the workgroup ("pair") is 2 * 512 B, so a slab holds 128 words
// per file
constexpr int kPairBytes = kTiles * kWave * 8;
constexpr int kSlabPairs = kLdsBytes / kPairBytes;
constexpr int kRing = 128;                              // records per wave ring (2 halves of 64)
constexpr int kRingPad = 64;                            // zero records past the table end

__device__ __forceinline__ uint32_t readfirstlane(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// LDS byte address (the ds_* address operand) of a __shared__ object.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// The LDS reads are inline asm, each batch with its own wait inside the statement: an asm
// output counts as written at the statement, so a load still in flight must never leave it
// (the register allocator could copy or spill the register before the data lands).

// 4 records of the wave's ring (uniform address: every lane reads the same 16 B). ds_read_b128,
// not b96: the 12-byte form made the whole kernel 20% slower.
__device__ __forceinline__ void ring_load4(uint32_t addr, uint4 (&c)[4]) {
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
        "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3])
        : "v"(addr));
}

// File words of 4 records at precomputed LDS addresses; the slab layout is [pair][lane][tile], so
// a lane's words of both tiles are one 16-byte ds_read_b128 (two ds_read_b64 of a [pair][tile]
// [lane] slab measured 1% slower, 4 tiles per workgroup 10% slower: DESIGN.md Appendix B).
__device__ __forceinline__ void file_load4w(const uint32_t (&a)[4], uint4 (&v)[4]) {
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]));
}

// acc[f] += popcount(file word & mask) for both tiles: v_and_b32 + v_bcnt_u32_b32 accumulate.
// One asm block per record: the hazard recognizer pads every inline-asm boundary with an s_nop.
__device__ __forceinline__ void use_record(uint32_t& a0, uint32_t& a1, const uint2 v0, const uint2 v1, const uint4 c) {
    uint32_t t;
    asm volatile(
        "v_and_b32 %2, %3, %5\n\tv_bcnt_u32_b32 %0, %2, %0\n\t"
        "v_and_b32 %2, %4, %6\n\tv_bcnt_u32_b32 %0, %2, %0\n\t"
        "v_and_b32 %2, %3, %7\n\tv_bcnt_u32_b32 %1, %2, %1\n\t"
        "v_and_b32 %2, %4, %8\n\tv_bcnt_u32_b32 %1, %2, %1"
        : "+v"(a0), "+v"(a1), "=&v"(t)
        : "v"(c.y), "v"(c.z), "v"(v0.x), "v"(v0.y), "v"(v1.x), "v"(v1.y));
}

// Ring bookkeeping when the stream position p (a multiple of 4) starts 64-record chunk c: wait
// for chunk c's DMA, then refill the half chunk c - 1 used (all its reads have returned) with
// chunk c + 1. The slab prologue issued chunks 0 and 1, so at c = 0 only the first of the two
// must have landed. LDS-DMA and ds_read are ordered only by this wave's vmcnt.
__device__ __forceinline__ void ring_enter(int32_t p, int32_t nchunk, const uint4* src, uint4* ring, int lane) {
    if ((p & 63) != 0) return;
    const int32_t c = p >> 6;
    if (c == 0 && nchunk > 1) {
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (c >= 1 && c + 1 < nchunk)
            __builtin_amdgcn_global_load_lds(src + (c + 1) * 64 + lane, ring + ((c + 1) & 1) * 64, 16, 0, 0);
    }
}

template <int G>
__global__ __launch_bounds__(kLdsWaves * kWave) void dice_lds_match(
    const uint4* __restrict__ tiles, int64_t n, int32_t wq, int32_t nslab, int32_t T,
    const int32_t* __restrict__ rec, const uint4* __restrict__ ep, const int32_t* __restrict__ wave_t0,
    int32_t npass, const int4* __restrict__ tc, const uint32_t* __restrict__ wfp,
    const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp, double thr,
    int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out, double* __restrict__ score_out) {
    // one LDS object: the rings in the low 32 KiB (LDS-DMA addresses them through M0), the
    // slab [pair][tile][lane] above them
    constexpr int kSlabQuads = kSlabPairs / 2;   // uint4 rows of a tile per slab
    __shared__ uint4 lds_all[kLdsWaves * kRing + kLdsBytes / 16];
    uint4 (*ring)[kRing] = reinterpret_cast<uint4 (*)[kRing]>(lds_all);
    uint2* slab = reinterpret_cast<uint2*>(lds_all + kLdsWaves * kRing);

    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)readfirstlane(threadIdx.x >> 6);
    const int64_t n_tiles = (n + kWave - 1) / kWave;
    const int64_t tile0 = (int64_t)blockIdx.x * kTiles;

    // per-file |W_F|, len_F, CC flag
    uint32_t my_wf[kTiles];
    int32_t my_len[kTiles];
    bool my_cc[kTiles];
    Best best[kTiles];
#pragma unroll
    for (int f = 0; f < kTiles; ++f) {
        const int64_t file = (tile0 + f) * kWave + lane;
        const bool ok = file < n;
        my_wf[f] = ok ? wfp[file] : 0;
        my_len[f] = ok ? lenp[file] : 0;
        my_cc[f] = ok ? ccp[file] != 0 : false;
        best[f].init();
    }
    const uint32_t base = lds_addr(slab) + lane * 8 * kTiles;
    const uint32_t ring_base = lds_addr(&ring[wave][0]);

    for (int pass = 0; pass < npass; ++pass) {
        const int32_t tb = wave_t0[pass * (kLdsWaves + 1) + wave];
        const int32_t te = wave_t0[pass * (kLdsWaves + 1) + wave + 1];
        uint32_t acc[G][kTiles];
#pragma unroll
        for (int j = 0; j < G; ++j)
#pragma unroll
            for (int f = 0; f < kTiles; ++f) acc[j][f] = 0;

        for (int si = 0; si < nslab; ++si) {
            // snake order: odd passes walk the slabs backwards, so a pass starts on the slab the
            // previous one ended on, which is still in LDS (npass - 1 fewer stagings)
            const int s = (pass & 1) ? nslab - 1 - si : si;
            const bool restage = !(pass > 0 && si == 0);
            if (restage) {
                // stage slab s: rows r = wave + 16 i of (tile f = r / 64, quad q = r % 64); one
                // 1 KiB coalesced load per row, two ds_write_b64 per lane
                uint4 stage[kTiles * kSlabQuads / kLdsWaves];
#pragma unroll
                for (int i = 0; i < kTiles * kSlabQuads / kLdsWaves; ++i) {
                    const int r = wave + i * kLdsWaves;
                    const int f = r / kSlabQuads, q = r % kSlabQuads;
                    const int qg = s * kSlabQuads + q;
                    const bool ok = tile0 + f < n_tiles && qg < wq;
                    stage[i] = ok ? tiles[((tile0 + f) * wq + qg) * kWave + lane] : make_uint4(0, 0, 0, 0);
                }
                __syncthreads();   // the previous slab's readers are done
#pragma unroll
                for (int i = 0; i < kTiles * kSlabQuads / kLdsWaves; ++i) {
                    const int r = wave + i * kLdsWaves;
                    const int f = r / kSlabQuads, q = r % kSlabQuads;
                    slab[((2 * q) * kWave + lane) * kTiles + f] = make_uint2(stage[i].x, stage[i].y);
                    slab[((2 * q + 1) * kWave + lane) * kTiles + f] = make_uint2(stage[i].z, stage[i].w);
                }
            }
            // this wave's record stream for slab s: runs of templates [tb, te), contiguous; the
            // first two 64-record chunks go to the ring now
            const int32_t* rs = rec + (int64_t)s * T;
            const int32_t r0 = rs[tb], total = rs[te] - r0;
            const uint4* src = ep + r0;
            const int32_t nchunk = (total + 63) / 64;
            if (nchunk > 0) __builtin_amdgcn_global_load_lds(src + lane, &ring[wave][0], 16, 0, 0);
            if (nchunk > 1) __builtin_amdgcn_global_load_lds(src + 64 + lane, &ring[wave][64], 16, 0, 0);
            if (restage) __syncthreads();   // slab writes visible to every wave

            int32_t p = 0;     // stream position (records), a multiple of 4
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const int32_t t = tb + j;
                if (t < te) {
                    // run of (slab s, template t): a multiple of 4 records (zero-mask padding)
                    const int32_t cnt = rs[t + 1] - rs[t];
                    for (int32_t e = 0; e < cnt; e += 4, p += 4) {
                        ring_enter(p, nchunk, src, ring[wave], lane);
                        uint4 c[4];
                        ring_load4(ring_base + (uint32_t)(p & (kRing - 1)) * 16u, c);
                        uint32_t fa[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) fa[k] = base + c[k].x;
                        uint4 w[4];
                        file_load4w(fa, w);
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            use_record(acc[j][0], acc[j][1], make_uint2(w[k].x, w[k].y), make_uint2(w[k].z, w[k].w),
                                       c[k]);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int32_t t = tb + j;
            if (t < te) {
                const int4 c = tc[t];
#pragma unroll
                for (int f = 0; f < kTiles; ++f)
                    if (!(c.w && my_cc[f])) best[f].offer(t, acc[j][f], dice_den(c, my_wf[f], my_len[f]));
            }
        }
    }
    // merge the 16 per-wave winners of every file through LDS (the slab is free now)
    __syncthreads();
    int32_t* r_idx = reinterpret_cast<int32_t*>(slab);                 // [wave][tile][lane]
    uint32_t* r_ov = reinterpret_cast<uint32_t*>(r_idx + kLdsWaves * kTiles * kWave);
    int32_t* r_den = reinterpret_cast<int32_t*>(r_ov + kLdsWaves * kTiles * kWave);
#pragma unroll
    for (int f = 0; f < kTiles; ++f) {
        const int k = (wave * kTiles + f) * kWave + lane;
        r_idx[k] = best[f].idx;
        r_ov[k] = best[f].ov;
        r_den[k] = best[f].den;
    }
    __syncthreads();
    if (wave < kTiles) {
        const int f = wave;
        int32_t bi = -1, bd = 1;
        uint32_t bo = 0;
        for (int w = 0; w < kLdsWaves; ++w) {
            const int k = (w * kTiles + f) * kWave + lane;
            if (outranks(r_idx[k], r_ov[k], r_den[k], bi, bo, bd)) { bi = r_idx[k]; bo = r_ov[k]; bd = r_den[k]; }
        }
        const int64_t file = (tile0 + f) * kWave + lane;
        if (file < n) {
            const double sc = bi >= 0 ? dice_score(bo, bd) : 0.0;
            best_out[file] = (bi >= 0 && sc >= thr) ? bi : -1;
            ov_out[file] = bo;
            score_out[file] = sc;
        }
    }
}

// ---- host side -------------------------------------------------------------------------

// Contiguous split of templates [a, b) over kLdsWaves waves, <= G each, minimising the
// largest per-wave cost (binary search on the bound + greedy fill).
static std::vector<int32_t> split_waves(const std::vector<int64_t>& cost, int32_t a, int32_t b, int32_t G) {
    auto fill = [&](int64_t cap, std::vector<int32_t>* out) {
        int32_t t = a;
        if (out) out->assign(1, a);
        for (int w = 0; w < kLdsWaves; ++w) {
            int64_t load = 0;
            int32_t k = 0;
            while (t < b && k < G && (k == 0 || load + cost[t] <= cap)) {
                load += cost[t];
                ++t;
                ++k;
            }
            if (out) out->push_back(t);
        }
        return t == b;
    };
    int64_t lo = 0, hi = 0;
    for (int32_t t = a; t < b; ++t) hi += cost[t];
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (fill(mid, nullptr)) hi = mid;
        else lo = mid + 1;
    }
    std::vector<int32_t> out;
    fill(lo, &out);
    return out;
}

// Templates per wave per pass: 16 measured fastest at T = 600 (24: -0.4%, 12: -2.6%); 3 passes over
// the files there.
int lds_setup(dice_ctx* c, const dice_templates* t) {
    const int G = kG, nt = kTiles;
    const int32_t T = c->T, w64 = c->w64;
    const int32_t nslab = (w64 + kSlabPairs - 1) / kSlabPairs;
    std::vector<int32_t> rec((size_t)nslab * T + 1);
    std::vector<uint4> ep;
    std::vector<int64_t> cost(T, 0);
    for (int32_t s = 0; s < nslab; ++s) {
        const int32_t pb = s * kSlabPairs, pe = std::min(w64, pb + kSlabPairs);
        for (int32_t i = 0; i < T; ++i) {
            const uint64_t* r = t->lf_bits + (size_t)i * w64;
            const size_t start = ep.size();
            rec[(size_t)s * T + i] = (int32_t)start;
            for (int32_t p = pb; p < pe; ++p)
                if (r[p])
                    ep.push_back(make_uint4((uint32_t)(p - pb) * kPairBytes, (uint32_t)r[p], (uint32_t)(r[p] >> 32), 0));
            while (ep.size() % 4) ep.push_back(make_uint4(0, 0, 0, 0));   // zero masks: no-op records
            // per record: v_add + 2 ds_read_b64 + 8 VALU; per (slab, template): run setup
            cost[i] += (1 + 4 * nt) * (int64_t)(ep.size() - start) + 40;
        }
    }
    rec.back() = (int32_t)ep.size();
    // the last ring chunk of a stream is fetched whole
    for (int k = 0; k < kRingPad; ++k) ep.push_back(make_uint4(0, 0, 0, 0));

    const int32_t per_pass = kLdsWaves * G;
    const int32_t npass = (T + per_pass - 1) / per_pass;
    std::vector<int32_t> wt;
    for (int32_t p = 0; p < npass; ++p) {
        const int32_t a = (int32_t)((int64_t)T * p / npass), b = (int32_t)((int64_t)T * (p + 1) / npass);
        const std::vector<int32_t> w = split_waves(cost, a, b, G);
        wt.insert(wt.end(), w.begin(), w.end());
    }
    int rc;
    if ((rc = dalloc_bytes(&c->d_lrec, rec.size() * sizeof(int32_t))) ||
        (rc = dalloc_bytes(&c->d_lep, ep.size() * sizeof(uint4))) ||
        (rc = dalloc_bytes(&c->d_lwt, wt.size() * sizeof(int32_t))))
        return rc;
    if (hipMemcpy(c->d_lrec, rec.data(), rec.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_lep, ep.data(), ep.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_lwt, wt.data(), wt.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "lds plan upload failed");
    c->lds_nslab = nslab;
    c->lds_npass = npass;
    c->lds_entries = (int64_t)ep.size() - kRingPad;
    c->kind = 2;
    return DICE_OK;
}

int lds_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    const int64_t n_tiles = (b->n + kWave - 1) / kWave;
    const int64_t groups = (n_tiles + kTiles - 1) / kTiles;
    hipLaunchKernelGGL((dice_lds_match<kG>), dim3((unsigned)groups), dim3(kLdsWaves * kWave), 0, s, b->d_tiles, b->n,
                       c->wq, c->lds_nslab, c->T, (const int32_t*)c->d_lrec, (const uint4*)c->d_lep,
                       (const int32_t*)c->d_lwt, c->lds_npass, c->d_tc, b->d_wf, b->d_len, b->d_cc, thr, b->d_best,
                       b->d_ov, b->d_score);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_lds_match launch failed");
}

}  // namespace dice
