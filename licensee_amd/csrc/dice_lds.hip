// LDS-tiled sparse scorer for large template sets (T > 64, BASELINE config 3: ~600 templates).
//
// Same contract as dice_dense_match (dice.rb:34-53 over content_helper.rb:128-133,337-347):
// per file, the argmax template among the unmasked ones, its overlap and its f64 score.
//
// Why a second kernel: at T ~ 600 the dense formulation (every template x every vocabulary
// dword: 2 VALU per 32 (file, word) pairs) is VALU-bound, and ~79% of the template dwords are
// zero. Here only non-zero template words are visited:
//
//   * one workgroup = F tiles (64F files) x 16 waves; lane l of every wave serves file l of
//     each of the F tiles;
//   * the F tiles' bitsets are staged through LDS (128 KiB) in slabs of 128K/(F*512) u64 words
//     per file, layout [pair][tile][lane] (8 B per lane: conflict-free ds_write_b64 /
//     ds_read_b64);
//   * wave w owns a contiguous template group (<= G templates per pass, balanced by record
//     count on the host); its G x F accumulators stay in VGPRs for the whole pass;
//   * one record {LDS byte offset, mask lo, mask hi} per non-zero template u64 word, read by
//     scalar loads (masks are SGPR operands). A record serves F files: one v_add, F
//     ds_read_b64 (immediate offsets per tile) and 4F VALU (v_and + v_bcnt per half per file).
//     Several files per record is what keeps the scalar record stream (~1 MB per pass at
//     T=600) from bounding the kernel: its latency is covered by F x the vector work;
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
constexpr int kLdsBytes = 128 * 1024;   // slab buffer (the per-wave winners reuse it at the end)

// Variants (DICE_LDS_VARIANT): F tiles (files per lane) per workgroup x G templates per wave per
// pass. The slab holds kLdsBytes / (F * 512) u64 words per file.
template <int F>
struct Slab {
    static constexpr int pairs = kLdsBytes / (F * kWave * 8);
    static constexpr int quads = pairs / 2;
    static constexpr int pair_bytes = F * kWave * 8;
};

__device__ __forceinline__ uint32_t readfirstlane(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// acc += popcount(x & m), m uniform (SGPR): v_and_b32 + v_bcnt_u32_b32 accumulate.
__device__ __forceinline__ void acc_and(uint32_t& acc, uint32_t x, uint32_t m) {
    uint32_t t;
    asm volatile("v_and_b32 %1, %2, %3\n\tv_bcnt_u32_b32 %0, %1, %0" : "+v"(acc), "=&v"(t) : "s"(m), "v"(x));
}

// 4 consecutive records through the scalar path: the base is made opaque (no strength-reduced
// negative offsets, which SMEM cannot encode) and read as constant memory: s_load_dwordx8 x2.
__device__ __forceinline__ void load4(const uint4* nx, uint4& n0, uint4& n1, uint4& n2, uint4& n3) {
    uint64_t addr = reinterpret_cast<uint64_t>(nx);
    asm volatile("" : "+s"(addr));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(4))) u32x4* const_u32x4_ptr;
    const const_u32x4_ptr p = (const_u32x4_ptr)addr;
    const u32x4 a = p[0], b = p[1], c = p[2], d = p[3];
    n0 = make_uint4(a.x, a.y, a.z, a.w);
    n1 = make_uint4(b.x, b.y, b.z, b.w);
    n2 = make_uint4(c.x, c.y, c.z, c.w);
    n3 = make_uint4(d.x, d.y, d.z, d.w);
}

// LDS byte address (the ds_* address operand) of a __shared__ object.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// LDS word of tile f at byte address addr (v) + f*512: a plain ds_read_b64 (2 LDS cycles per
// wave). Written as asm so the compiler cannot pair the tiles into ds_read2st64_b64, which
// costs 8x; the caller waits with lgkmcnt(0) before using the results.
template <int f>
__device__ __forceinline__ uint2 lds_word(uint32_t addr) {
    uint2 v;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(f * kWave * 8));
    return v;
}

template <int F>
__device__ __forceinline__ void read_record(uint2 (&v)[F], uint32_t base, uint32_t off) {
    const uint32_t addr = base + off;
    v[0] = lds_word<0>(addr);
    if constexpr (F > 1) v[1] = lds_word<1>(addr);
    if constexpr (F > 2) v[2] = lds_word<2>(addr);
    if constexpr (F > 3) v[3] = lds_word<3>(addr);
}

// Accumulate one record into the F files' counters. One asm block per record: the hazard
// recognizer pads every inline-asm boundary with an s_nop, so the and/bcnt pairs of all F files
// go in a single block.
template <int F>
__device__ __forceinline__ void use_record(uint32_t (&a)[F], const uint2 (&v)[F], const uint4 c);

template <>
__device__ __forceinline__ void use_record<4>(uint32_t (&a)[4], const uint2 (&v)[4], const uint4 c) {
    uint32_t t;
    asm volatile(
        "v_and_b32 %4, %5, %7\n\tv_bcnt_u32_b32 %0, %4, %0\n\t"
        "v_and_b32 %4, %6, %8\n\tv_bcnt_u32_b32 %0, %4, %0\n\t"
        "v_and_b32 %4, %5, %9\n\tv_bcnt_u32_b32 %1, %4, %1\n\t"
        "v_and_b32 %4, %6, %10\n\tv_bcnt_u32_b32 %1, %4, %1\n\t"
        "v_and_b32 %4, %5, %11\n\tv_bcnt_u32_b32 %2, %4, %2\n\t"
        "v_and_b32 %4, %6, %12\n\tv_bcnt_u32_b32 %2, %4, %2\n\t"
        "v_and_b32 %4, %5, %13\n\tv_bcnt_u32_b32 %3, %4, %3\n\t"
        "v_and_b32 %4, %6, %14\n\tv_bcnt_u32_b32 %3, %4, %3"
        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "=&v"(t)
        : "s"(c.y), "s"(c.z), "v"(v[0].x), "v"(v[0].y), "v"(v[1].x), "v"(v[1].y), "v"(v[2].x), "v"(v[2].y),
          "v"(v[3].x), "v"(v[3].y));
}

template <>
__device__ __forceinline__ void use_record<2>(uint32_t (&a)[2], const uint2 (&v)[2], const uint4 c) {
    uint32_t t;
    asm volatile(
        "v_and_b32 %2, %3, %5\n\tv_bcnt_u32_b32 %0, %2, %0\n\t"
        "v_and_b32 %2, %4, %6\n\tv_bcnt_u32_b32 %0, %2, %0\n\t"
        "v_and_b32 %2, %3, %7\n\tv_bcnt_u32_b32 %1, %2, %1\n\t"
        "v_and_b32 %2, %4, %8\n\tv_bcnt_u32_b32 %1, %2, %1"
        : "+v"(a[0]), "+v"(a[1]), "=&v"(t)
        : "s"(c.y), "s"(c.z), "v"(v[0].x), "v"(v[0].y), "v"(v[1].x), "v"(v[1].y));
}

// One step of 4 records: 4F LDS reads in flight together; the next 4 records load meanwhile.
template <int F>
__device__ __forceinline__ void step4(uint32_t (&a)[F], uint32_t base, const uint4 c0, const uint4 c1,
                                      const uint4 c2, const uint4 c3, const uint4* __restrict__ nx,
                                      uint4& n0, uint4& n1, uint4& n2, uint4& n3) {
    uint2 v0[F], v1[F], v2[F], v3[F];
    read_record<F>(v0, base, c0.x);
    read_record<F>(v1, base, c1.x);
    read_record<F>(v2, base, c2.x);
    read_record<F>(v3, base, c3.x);
    // SMEM and LDS share lgkmcnt and scalar loads return out of order, so any wait for the LDS
    // reads also waits for every scalar load in flight: the next records are requested right
    // AFTER the wait, and have this step's VALU work to arrive before the next step's wait.
    asm volatile("s_waitcnt lgkmcnt(0)");
    load4(nx, n0, n1, n2, n3);
    use_record<F>(a, v0, c0);
    use_record<F>(a, v1, c1);
    use_record<F>(a, v2, c2);
    use_record<F>(a, v3, c3);
}

// Candidate a outranks b in the final order: higher score, or equal score and later key.
__device__ __forceinline__ bool outranks(int32_t ai, uint32_t ao, int32_t ad, int32_t bi, uint32_t bo, int32_t bd) {
    if (ai < 0) return false;
    if (bi < 0) return true;
    const bool ge = dice_ge(ao, ad, bo, bd), le = dice_ge(bo, bd, ao, ad);
    return ge && (!le || ai > bi);
}

template <int F, int G, bool R3>
__global__ __launch_bounds__(kLdsWaves * kWave) void dice_lds_match(
    const uint4* __restrict__ tiles, int64_t n, int32_t wq, int32_t nslab, int32_t T,
    const int32_t* __restrict__ rec, const uint4* __restrict__ ep, const int32_t* __restrict__ wave_t0,
    int32_t npass, const int4* __restrict__ tc, const uint32_t* __restrict__ wfp,
    const int32_t* __restrict__ lenp, const uint8_t* __restrict__ ccp, double thr,
    int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out, double* __restrict__ score_out) {
    constexpr int kF = F;
    constexpr int kSlabQuads = Slab<F>::quads;
    __shared__ uint2 slab[kLdsBytes / 8];   // [pair][tile][lane]

    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)readfirstlane(threadIdx.x >> 6);
    const int64_t n_tiles = (n + kWave - 1) / kWave;
    const int64_t tile0 = (int64_t)blockIdx.x * kF;

    uint32_t my_wf[kF];
    int32_t my_len[kF];
    bool my_cc[kF];
    Best best[kF];
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        const int64_t file = (tile0 + f) * kWave + lane;
        const bool ok = file < n;
        my_wf[f] = ok ? wfp[file] : 0;
        my_len[f] = ok ? lenp[file] : 0;
        my_cc[f] = ok ? ccp[file] != 0 : false;
        best[f].init();
    }
    const uint32_t base = lds_addr(slab) + lane * 8;

    for (int pass = 0; pass < npass; ++pass) {
        const int32_t tb = wave_t0[pass * (kLdsWaves + 1) + wave];
        const int32_t te = wave_t0[pass * (kLdsWaves + 1) + wave + 1];
        uint32_t acc[G][kF];
#pragma unroll
        for (int j = 0; j < G; ++j)
#pragma unroll
            for (int f = 0; f < kF; ++f) acc[j][f] = 0;

        for (int s = 0; s < nslab; ++s) {
            // stage slab s: rows r = wave + 16 i of (tile f = r / 32, quad q = r % 32); one
            // 1 KiB coalesced load per row, two ds_write_b64 per lane.
            uint4 stage[kF * kSlabQuads / kLdsWaves];
#pragma unroll
            for (int i = 0; i < kF * kSlabQuads / kLdsWaves; ++i) {
                const int r = wave + i * kLdsWaves;
                const int f = r / kSlabQuads, q = r % kSlabQuads;
                const int qg = s * kSlabQuads + q;
                const bool ok = tile0 + f < n_tiles && qg < wq;
                stage[i] = ok ? tiles[((tile0 + f) * wq + qg) * kWave + lane] : make_uint4(0, 0, 0, 0);
            }
            __syncthreads();   // the previous slab's readers are done
#pragma unroll
            for (int i = 0; i < kF * kSlabQuads / kLdsWaves; ++i) {
                const int r = wave + i * kLdsWaves;
                const int f = r / kSlabQuads, q = r % kSlabQuads;
                slab[((2 * q) * kF + f) * kWave + lane] = make_uint2(stage[i].x, stage[i].y);
                slab[((2 * q + 1) * kF + f) * kWave + lane] = make_uint2(stage[i].z, stage[i].w);
            }
            __syncthreads();
            // the slab writes above are complete for this wave before its asm reads (barrier)

            const int32_t* rs = rec + (int64_t)s * T;
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const int32_t t = tb + j;
                if (t < te) {
                    // run of (slab s, template t): a multiple of 4 records, 64-B aligned; the
                    // table is padded past its end, so look-ahead loads stay in bounds.
                    const int32_t e0 = rs[t], e1 = rs[t + 1];
                    const uint4* ee = ep + e0;
                    const int32_t cnt = e1 - e0;
                    uint4 c0, c1, c2, c3, d0, d1, d2, d3;
                    load4(ee, c0, c1, c2, c3);
                    int32_t e = 0;
                    if constexpr (R3) {
                        // three record sets in rotation: the records of step s + 2 are
                        // requested during step s, so a scalar load has two steps of vector
                        // work to arrive (the table is padded 8 records past every run end)
                        uint4 g0, g1, g2, g3;
                        load4(ee + 4, d0, d1, d2, d3);
                        for (; e + 12 <= cnt; e += 12) {
                            step4<F>(acc[j], base, c0, c1, c2, c3, ee + e + 8, g0, g1, g2, g3);
                            step4<F>(acc[j], base, d0, d1, d2, d3, ee + e + 12, c0, c1, c2, c3);
                            step4<F>(acc[j], base, g0, g1, g2, g3, ee + e + 16, d0, d1, d2, d3);
                        }
                        if (e < cnt) step4<F>(acc[j], base, c0, c1, c2, c3, ee + e + 8, g0, g1, g2, g3);
                        if (e + 4 < cnt) step4<F>(acc[j], base, d0, d1, d2, d3, ee + e + 12, c0, c1, c2, c3);
                    } else {
                        for (; e + 8 <= cnt; e += 8) {   // ping-pong: no SGPR copies
                            step4<F>(acc[j], base, c0, c1, c2, c3, ee + e + 4, d0, d1, d2, d3);
                            step4<F>(acc[j], base, d0, d1, d2, d3, ee + e + 8, c0, c1, c2, c3);
                        }
                        if (e < cnt) step4<F>(acc[j], base, c0, c1, c2, c3, ee + e + 4, d0, d1, d2, d3);
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
                for (int f = 0; f < kF; ++f)
                    if (!(c.w && my_cc[f])) best[f].offer(t, acc[j][f], dice_den(c, my_wf[f], my_len[f]));
            }
        }
    }
    // merge the 16 per-wave winners of every file through LDS (the slab is free now)
    __syncthreads();
    int32_t* r_idx = reinterpret_cast<int32_t*>(slab);                 // [wave][tile][lane]
    uint32_t* r_ov = reinterpret_cast<uint32_t*>(r_idx + kLdsWaves * kF * kWave);
    int32_t* r_den = reinterpret_cast<int32_t*>(r_ov + kLdsWaves * kF * kWave);
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        const int k = (wave * kF + f) * kWave + lane;
        r_idx[k] = best[f].idx;
        r_ov[k] = best[f].ov;
        r_den[k] = best[f].den;
    }
    __syncthreads();
    if (wave < kF) {
        const int f = wave;
        int32_t bi = -1, bd = 1;
        uint32_t bo = 0;
        for (int w = 0; w < kLdsWaves; ++w) {
            const int k = (w * kF + f) * kWave + lane;
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

struct Variant {
    int f, g;
    bool r3;
};
static const Variant kVariants[] = {{4, 16, false}, {4, 8, false}, {2, 16, false}, {2, 24, false},
                                    {4, 16, true}, {4, 8, true}, {2, 24, true}};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));

static int slab_pairs(int f) { return kLdsBytes / (f * kWave * 8); }

int lds_setup(dice_ctx* c, const dice_templates* t) {
    const char* ve = getenv("DICE_LDS_VARIANT");
    // default: 2 tiles x 24 templates per wave with the 3-set record rotation -- no scratch
    // spills (113 VGPRs; F=4 x G=16 spills 32 B/lane) and 2 passes instead of 3 at T = 600
    const int vi = ve && *ve ? std::max(0, std::min(kNumVariants - 1, atoi(ve))) : 6;
    const int F = kVariants[vi].f, G = kVariants[vi].g;
    const int32_t kSlabPairs = slab_pairs(F), kPairBytes = F * kWave * 8;
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
            // per record: v_add + F ds_read_b64 + 4F VALU; per (slab, template): run setup
            cost[i] += (1 + 4 * F) * (int64_t)(ep.size() - start) + 40;
        }
    }
    rec.back() = (int32_t)ep.size();
    for (int k = 0; k < 8; ++k) ep.push_back(make_uint4(0, 0, 0, 0));   // look-ahead padding

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
    c->lds_entries = (int64_t)ep.size() - 8;
    c->lds_variant = vi;
    c->kind = 2;
    return DICE_OK;
}

template <int F, int G, bool R3>
static void launch(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    const int64_t n_tiles = (b->n + kWave - 1) / kWave;
    const int64_t groups = (n_tiles + F - 1) / F;
    hipLaunchKernelGGL((dice_lds_match<F, G, R3>), dim3((unsigned)groups), dim3(kLdsWaves * kWave), 0, s, b->d_tiles,
                       b->n, c->wq, c->lds_nslab, c->T, (const int32_t*)c->d_lrec, (const uint4*)c->d_lep,
                       (const int32_t*)c->d_lwt, c->lds_npass, c->d_tc, b->d_wf, b->d_len, b->d_cc, thr,
                       b->d_best, b->d_ov, b->d_score);
}

int lds_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    switch (c->lds_variant) {
        case 0: launch<4, 16, false>(c, b, thr, s); break;
        case 1: launch<4, 8, false>(c, b, thr, s); break;
        case 2: launch<2, 16, false>(c, b, thr, s); break;
        case 3: launch<2, 24, false>(c, b, thr, s); break;
        case 4: launch<4, 16, true>(c, b, thr, s); break;
        case 5: launch<4, 8, true>(c, b, thr, s); break;
        default: launch<2, 24, true>(c, b, thr, s); break;
    }
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_lds_match launch failed");
}

}  // namespace dice
