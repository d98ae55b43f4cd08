// Matchers::Exact on the device.
//
// Reference: lib/licensee/matchers/exact.rb:6-12 --
//   potential_matches.find { |potential_match| potential_match.wordset == file.wordset }
// over License.all(hidden: true, psuedo: false) in key order (matcher.rb), where a template's
// wordset is Lf ∪ its field words (content_helper.rb:108-110,323-335). Sets are equal iff the
// sizes are equal and one holds the other, so for file F and template t
//   W_t == W_F  <=>  |W_t| == |W_F|  and  R_t ⊆ row_F  and  need_t ⊆ fmask_F
// with R_t = W_t ∩ V (Lf_t and the field words that are vocabulary words, as bitset records)
// and need_t the field words outside the vocabulary (bits of the host's field-word numbering,
// licensee_host.h lh_template_field_masks; fmask_F from lh_prep_files). Words of W_t outside
// both are impossible: Lf_t ⊆ V.
//
// Kernel: one lane per file. The templates are sorted by (|W_t|, key index) on the host; a
// lane binary-searches |W_F| among the sorted sizes (in LDS); the few templates of that size are
// checked in key order by the whole wave, one (file, template) pair at a time -- most files have
// none, so the pass reads 4 B (|W_F|) + 8 B (field mask) and writes 4 B per file, plus the row
// words of the size-equal candidates.
#include <algorithm>
#include <string>
#include <vector>

#include "dice_common.h"
#include "dice_internal.h"

namespace dice {

namespace {

// sorted position k: {|W_t|, t, first record, end record}. One lane per file finds its size-equal
// templates (binary search over the sizes in LDS); the wave then checks the pending (file,
// template) pairs one at a time with all 64 lanes -- lanes = the template's records (coalesced
// 1 KiB loads), each reading its word of that one file's row -- so a pair costs two dependent
// loads instead of a record loop in one lane while the other 63 wait.
__global__ __launch_bounds__(256) void dice_exact_kernel(const uint64_t* __restrict__ rows, int64_t n, int32_t w64,
                                                         const uint32_t* __restrict__ wf,
                                                         const uint64_t* __restrict__ fmask,
                                                         const uint4* __restrict__ tbl,
                                                         const uint64_t* __restrict__ need,
                                                         const uint4* __restrict__ rec, int32_t T,
                                                         int32_t* __restrict__ out) {
    extern __shared__ uint32_t sz[];
    for (int i = threadIdx.x; i < T; i += blockDim.x) sz[i] = tbl[i].x;
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = f < n;
    const uint32_t w = valid ? wf[f] : 0xFFFFFFFFu;
    int32_t lo = 0, hi = T;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (sz[mid] < w) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t fm = valid && fmask ? fmask[f] : 0ull;
    int32_t res = -1;
    int32_t kc = valid && lo < T && sz[lo] == w ? lo : -1;   // this lane's next candidate position
    // skip candidates whose non-vocabulary field words the file lacks (lane-local)
    while (kc >= 0 && (need[kc] & ~fm) != 0) kc = kc + 1 < T && sz[kc + 1] == w ? kc + 1 : -1;
    for (uint64_t pend = __ballot(kc >= 0); pend; pend = __ballot(kc >= 0)) {
        const int src = (int)__builtin_ctzll(pend);
        const int32_t k = __builtin_amdgcn_readlane(kc, src);
        const int64_t fs = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~(kWave - 1)) + src;
        const uint64_t* row = rows + fs * (int64_t)w64;
        const uint4 e = tbl[k];
        bool ok = true;
        for (uint32_t r0 = e.z; r0 < e.w; r0 += kWave) {
            const uint32_t r = r0 + (uint32_t)lane;
            bool bad = false;
            if (r < e.w) {
                const uint4 q = rec[r];
                const uint64_t m = (uint64_t)q.y | ((uint64_t)q.z << 32);
                bad = (row[q.x] & m) != m;
            }
            if (__ballot(bad)) {
                ok = false;
                break;
            }
        }
        if (lane == src) {
            if (ok) {
                res = (int32_t)e.y;
                kc = -1;
            } else {
                do kc = kc + 1 < T && sz[kc + 1] == w ? kc + 1 : -1;
                while (kc >= 0 && (need[kc] & ~fm) != 0);
            }
        }
    }
    if (valid) out[f] = res;
}

struct Guard {
    int prev = -1;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

hipStream_t stream_of(dice_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }

}  // namespace

void exact_free(dice_ctx* c) {
    for (void* p : {c->d_ex_tbl, c->d_ex_need, c->d_ex_rec})
        if (p) (void)hipFree(p);
    c->d_ex_tbl = c->d_ex_need = c->d_ex_rec = nullptr;
    c->exact_ready = false;
}

}  // namespace dice

using dice::fail;

extern "C" {

int dice_exact_setup(dice_ctx* c, const uint32_t* wordset_size, const uint64_t* field_bits,
                     const uint64_t* field_need) {
    if (!c || !wordset_size) return fail(DICE_E_ARG, "NULL ctx/wordset_size");
    if (!c->h_lf.size()) return fail(DICE_E_STATE, "ctx holds no template bitsets");
    const int32_t T = c->T, w64 = c->w64;
    std::vector<int32_t> order((size_t)T);
    for (int32_t t = 0; t < T; ++t) order[(size_t)t] = t;
    // (|W_t|, key index): the first template of a size run that passes is the first in key order
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return wordset_size[a] < wordset_size[b]; });
    std::vector<uint4> tbl((size_t)T), rec;
    std::vector<uint64_t> need((size_t)T);
    for (int32_t k = 0; k < T; ++k) {
        const int32_t t = order[(size_t)k];
        const uint32_t r0 = (uint32_t)rec.size();
        for (int32_t p = 0; p < w64; ++p) {
            uint64_t m = c->h_lf[(size_t)t * w64 + p];
            if (field_bits) m |= field_bits[(size_t)t * w64 + p];
            if (m) rec.push_back(make_uint4((uint32_t)p, (uint32_t)m, (uint32_t)(m >> 32), 0u));
        }
        tbl[(size_t)k] = make_uint4(wordset_size[t], (uint32_t)t, r0, (uint32_t)rec.size());
        need[(size_t)k] = field_need ? field_need[t] : 0ull;
    }
    if (rec.empty()) rec.push_back(make_uint4(0, 0, 0, 0));
    dice::Guard g(c->device);
    dice::exact_free(c);
    int rc;
    if ((rc = dice::dalloc_bytes(&c->d_ex_tbl, tbl.size() * 16)) ||
        (rc = dice::dalloc_bytes(&c->d_ex_need, need.size() * 8)) ||
        (rc = dice::dalloc_bytes(&c->d_ex_rec, rec.size() * 16)))
        return rc;
    if (hipMemcpy(c->d_ex_tbl, tbl.data(), tbl.size() * 16, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_ex_need, need.data(), need.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_ex_rec, rec.data(), rec.size() * 16, hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "exact table upload failed");
    c->exact_ready = true;
    return DICE_OK;
}

int dice_batch_exact(dice_batch* b, const uint64_t* file_field_mask, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (!c->exact_ready) return fail(DICE_E_STATE, "dice_exact_setup was not called");
    dice::Guard g(c->device);
    int rc;
    if (!b->d_exact && (rc = dice::dalloc_bytes((void**)&b->d_exact, (size_t)b->capacity * 4))) return rc;
    if (!b->d_fmask && (rc = dice::dalloc_bytes((void**)&b->d_fmask, (size_t)b->capacity * 8))) return rc;
    if (b->n == 0) return DICE_OK;
    hipStream_t s = dice::stream_of(c, stream);
    if (file_field_mask &&
        hipMemcpyAsync(b->d_fmask, file_field_mask, (size_t)b->n * 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(DICE_E_DEVICE, "field mask upload failed");
    // dice_batch_upload_text built the masks on the device
    const bool masks = file_field_mask != nullptr || b->fmask_device;
    const unsigned grid = (unsigned)((b->n + 255) / 256);
    hipLaunchKernelGGL(dice::dice_exact_kernel, dim3(grid), dim3(256), (size_t)c->T * 4, s,
                       (const uint64_t*)b->d_rows, b->n, c->w64, (const uint32_t*)b->d_wf,
                       masks ? (const uint64_t*)b->d_fmask : nullptr, (const uint4*)c->d_ex_tbl,
                       (const uint64_t*)c->d_ex_need, (const uint4*)c->d_ex_rec, c->T, b->d_exact);
    return hipGetLastError() == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "dice_exact_kernel launch failed");
}

int dice_batch_download_exact(dice_batch* b, int32_t* exact, void* stream) {
    if (!b || !exact) return fail(DICE_E_ARG, "NULL batch/output");
    if (b->n && !b->d_exact) return fail(DICE_E_STATE, "dice_batch_exact was not run");
    dice::Guard g(b->ctx->device);
    hipStream_t s = dice::stream_of(b->ctx, stream);
    if (b->n && hipMemcpyAsync(exact, b->d_exact, (size_t)b->n * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return fail(DICE_E_DEVICE, "exact download failed");
    return hipStreamSynchronize(s) == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "hipStreamSynchronize failed");
}

int dice_exact(dice_ctx* c, const dice_files* f, const uint64_t* file_field_mask, int32_t* exact) {
    if (!c || !f || !exact) return fail(DICE_E_ARG, "NULL ctx/files/output");
    if (f->n_files == 0) return DICE_OK;
    dice_batch* b = nullptr;
    int rc;
    if ((rc = dice::scratch_for(c, f->n_files, &b))) return rc;
    if ((rc = dice_batch_upload(b, f, nullptr))) return rc;
    if ((rc = dice_batch_exact(b, file_field_mask, nullptr))) return rc;
    return dice_batch_download_exact(b, exact, nullptr);
}

}  // extern "C"
