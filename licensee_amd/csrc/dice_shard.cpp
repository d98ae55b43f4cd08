// One call, several devices: dice_match_sharded / dice_similarity_matrix_sharded
// (include/licensee_dice.h). The per-file loop of Dice#matches_by_similarity
// (lib/licensee/matchers/dice.rb:34-41) has no cross-file state, so the files of a call are
// split into contiguous shards, one per ctx; each shard runs on its ctx's device from its own
// host thread and stream (upload, kernel, download) and only results move.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/licensee_dice.h"
#include "dice_internal.h"

using dice::fail;

namespace {

struct Shard {
    int64_t lo = 0, hi = 0;
    int rc = DICE_OK;
    std::string err;
};

int check_ctxs(dice_ctx* const* ctxs, int32_t n_ctx, const dice_files* f, int32_t gather) {
    if (!ctxs || n_ctx < 1 || !f) return fail(DICE_E_ARG, "NULL ctxs/files or n_ctx < 1");
    if (gather != DICE_GATHER_HOST && gather != DICE_GATHER_DEVICE) return fail(DICE_E_ARG, "unknown gather_mode");
    for (int32_t i = 0; i < n_ctx; ++i) {
        if (!ctxs[i]) return fail(DICE_E_ARG, "NULL ctx in ctxs");
        if (ctxs[i]->T != ctxs[0]->T || ctxs[i]->V != ctxs[0]->V)
            return fail(DICE_E_ARG, "ctxs hold different corpora (T or V differ)");
        // each shard thread uses its ctx's scratch batch and stream: one ctx twice would race
        for (int32_t j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return fail(DICE_E_ARG, "the same ctx appears twice in ctxs");
    }
    if (f->n_files < 0) return fail(DICE_E_ARG, "n_files < 0");
    return DICE_OK;
}

dice_files slice(const dice_files* f, int64_t lo, int64_t hi, int32_t w64) {
    dice_files s;
    s.n_files = hi - lo;
    s.bits = f->bits + (size_t)lo * w64;
    s.wordset_size = f->wordset_size + lo;
    s.length = f->length + lo;
    s.cc_false_positive = f->cc_false_positive + lo;
    return s;
}

// Runs fn(i, shard) for every ctx on its own thread (device set per thread) and returns the
// first failing shard's status, its message moved to the calling thread's dice_last_error.
template <class F>
int run_shards(dice_ctx* const* ctxs, int32_t n_ctx, int64_t n, F&& fn) {
    std::vector<Shard> sh((size_t)n_ctx);
    for (int32_t i = 0; i < n_ctx; ++i) {
        sh[i].lo = n * i / n_ctx;
        sh[i].hi = n * (i + 1) / n_ctx;
    }
    auto body = [&](int32_t i) {
        // the shard's launch checks read HIP's per-thread last error: start from a clean one
        // (shard 0 runs on the caller's thread, which may hold a stale error of its own)
        (void)hipGetLastError();
        if (hipSetDevice(ctxs[i]->device) != hipSuccess) {
            sh[i].rc = DICE_E_DEVICE;
            sh[i].err = "hipSetDevice failed";
            return;
        }
        sh[i].rc = sh[i].hi > sh[i].lo ? fn(i, sh[i]) : DICE_OK;
        if (sh[i].rc != DICE_OK) sh[i].err = dice::last_error();
    };
    std::vector<std::thread> th;
    for (int32_t i = 1; i < n_ctx; ++i) th.emplace_back(body, i);
    int prev = -1;
    (void)hipGetDevice(&prev);
    body(0);
    for (auto& t : th) t.join();
    if (prev >= 0) (void)hipSetDevice(prev);
    for (auto& s : sh)
        if (s.rc != DICE_OK) return fail(s.rc, s.err);
    return DICE_OK;
}

thread_local int32_t g_last_gather_peer = -1;

// Page-locked memory? (the runtime DMAs it directly; pageable memory goes through its bounce
// buffers, which the shard threads of one call would share)
bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable: clear the sticky error
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

constexpr size_t kStageBytes = (size_t)32 << 20;   // per staging buffer (two per ctx)

// Shard upload: the bitset rows from pageable caller memory go through the ctx's two pinned
// staging buffers (memcpy of chunk i + 1 overlaps the DMA of chunk i); pinned or small inputs
// are handed to dice_batch_upload as they are.
int upload_shard(dice_ctx* c, dice_batch* b, const dice_files* part) {
    const size_t row = (size_t)c->w64 * 8, bytes = (size_t)part->n_files * row;
    if (bytes < 2 * kStageBytes || is_pinned(part->bits)) return dice_batch_upload(b, part, nullptr);
    if (!c->h_stage_bytes) {
        // all four resources or none: a partial set is freed, so the next call retries cleanly
        bool ok = true;
        for (int i = 0; i < 2 && ok; ++i)
            ok = (c->h_stage[i] || hipHostMalloc(&c->h_stage[i], kStageBytes, hipHostMallocDefault) == hipSuccess) &&
                 (c->stage_ev[i] || hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming) == hipSuccess);
        if (!ok) {
            (void)hipGetLastError();
            for (int i = 0; i < 2; ++i) {
                if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
                if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
                c->h_stage[i] = nullptr;
                c->stage_ev[i] = nullptr;
            }
            return fail(DICE_E_NOMEM, "pinned staging allocation failed");
        }
        c->h_stage_bytes = kStageBytes;
    }
    if (part->n_files > b->capacity) return fail(DICE_E_ARG, "n_files exceeds batch capacity");
    const int64_t per = (int64_t)(c->h_stage_bytes / row);
    if (per < 1) return dice_batch_upload(b, part, nullptr);
    const char* src = reinterpret_cast<const char*>(part->bits);
    char* dst = reinterpret_cast<char*>(b->d_rows);
    int k = 0;
    for (int64_t f0 = 0; f0 < part->n_files; f0 += per, k ^= 1) {
        const size_t nb = (size_t)std::min<int64_t>(per, part->n_files - f0) * row;
        if (hipEventSynchronize(c->stage_ev[k]) != hipSuccess) return fail(DICE_E_DEVICE, "staging wait failed");
        std::memcpy(c->h_stage[k], src + (size_t)f0 * row, nb);
        if (hipMemcpyAsync(dst + (size_t)f0 * row, c->h_stage[k], nb, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
            hipEventRecord(c->stage_ev[k], c->stream) != hipSuccess)
            return fail(DICE_E_DEVICE, "staged H2D failed");
    }
    // the per-file scalars (9 B per file) and the tile repack, behind the rows on the stream
    return dice::upload_rows_resident(b, part, c->stream);
}

// Peer access from device `from` to device `to` (tolerating an earlier enable); true when the
// results of a shard on `from` can be written straight into `to`'s memory over xGMI.
bool enable_peer(dice_ctx* from, int to) {
    if (from->device == to) return true;
    if (from->peer_mask >> to & 1) return true;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, from->device, to) != hipSuccess || !can) return false;
    int prev = -1;
    (void)hipGetDevice(&prev);
    bool ok = hipSetDevice(from->device) == hipSuccess;
    if (ok) {
        const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
        ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
        // any non-success return (AlreadyEnabled included) leaves HIP's per-thread last error
        // set; the shard launch checks on this thread would read it as their own failure
        if (e != hipSuccess) (void)hipGetLastError();
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    if (ok) from->peer_mask |= 1ull << to;
    return ok;
}

// Before a device gather: peer access from every shard's device to ctxs[0]'s; records whether
// all of them have it (dice_last_gather_peer: 1 / 0), or -1 when every ctx sits on ctxs[0]'s
// device -- no shard crosses devices, so the call says nothing about a peer path.
void prepare_device_gather(dice_ctx* const* ctxs, int32_t n_ctx) {
    bool all = true, remote = false;
    for (int32_t i = 1; i < n_ctx; ++i) {
        if (ctxs[i]->device == ctxs[0]->device) continue;
        remote = true;
        all = enable_peer(ctxs[i], ctxs[0]->device) && all;
    }
    g_last_gather_peer = !remote ? -1 : all ? 1 : 0;
}

// Device gather buffer on ctxs[0]'s device: `bytes` bytes, freed by the caller.
int gather_alloc(dice_ctx* c0, size_t bytes, void** p) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(c0->device) != hipSuccess) return fail(DICE_E_DEVICE, "hipSetDevice failed");
    const hipError_t e = hipMalloc(p, bytes ? bytes : 1);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(DICE_E_NOMEM, "gather buffer allocation failed");
    }
    return DICE_OK;
}

// One D2H per output array from the device gather buffer (regions laid out back to back).
int gather_d2h(dice_ctx* c0, const std::vector<std::pair<void*, size_t>>& outs, char* dev) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(c0->device) != hipSuccess) return fail(DICE_E_DEVICE, "hipSetDevice failed");
    size_t off = 0;
    hipError_t e = hipSuccess;
    for (auto& o : outs) {
        if (o.first && e == hipSuccess) e = hipMemcpyAsync(o.first, dev + off, o.second, hipMemcpyDeviceToHost, c0->stream);
        off += o.second;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c0->stream);
    if (prev >= 0) (void)hipSetDevice(prev);
    return e == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, std::string("gather D2H: ") + hipGetErrorString(e));
}

}  // namespace

static int match_sharded(dice_ctx* const* ctxs, int32_t n_ctx, const dice_files* f, double thr, int32_t gather,
                         int32_t* best, uint32_t* ov, double* score, bool confidence) {
    int rc = check_ctxs(ctxs, n_ctx, f, gather);
    if (rc) return rc;
    const int64_t n = f->n_files;
    if (n == 0) return DICE_OK;
    if (!f->bits || !f->wordset_size || !f->length || !f->cc_false_positive) return fail(DICE_E_ARG, "NULL file arrays");
    const int32_t w64 = ctxs[0]->w64;
    char* dev = nullptr;
    g_last_gather_peer = -1;
    if (gather == DICE_GATHER_DEVICE) {
        if ((rc = gather_alloc(ctxs[0], (size_t)n * 16, (void**)&dev))) return rc;
        prepare_device_gather(ctxs, n_ctx);
    }
    // device gather layout: best [n] i32 | overlap [n] u32 | score [n] f64
    int32_t* g_best = dev ? (int32_t*)dev : nullptr;
    uint32_t* g_ov = dev ? (uint32_t*)(dev + (size_t)n * 4) : nullptr;
    double* g_score = dev ? (double*)(dev + (size_t)n * 8) : nullptr;
    rc = run_shards(ctxs, n_ctx, n, [&](int32_t i, Shard& s) {
        dice_ctx* c = ctxs[i];
        dice_batch* b = nullptr;
        int r = dice::scratch_for(c, s.hi - s.lo, &b);
        if (r) return r;
        const dice_files part = slice(f, s.lo, s.hi, w64);
        if ((r = upload_shard(c, b, &part)) ||
            (r = confidence ? dice_batch_match_confidence(b, thr, nullptr) : dice_batch_match(b, thr, nullptr)))
            return r;
        if (dev)
            return dice::download_match_to(b, best ? g_best + s.lo : nullptr, ov ? g_ov + s.lo : nullptr,
                                           score ? g_score + s.lo : nullptr, c->stream, hipMemcpyDefault);
        return dice::download_match_to(b, best ? best + s.lo : nullptr, ov ? ov + s.lo : nullptr,
                                       score ? score + s.lo : nullptr, c->stream, hipMemcpyDeviceToHost);
    });
    if (rc == DICE_OK && dev)
        rc = gather_d2h(ctxs[0], {{best, (size_t)n * 4}, {ov, (size_t)n * 4}, {score, (size_t)n * 8}}, dev);
    if (dev) (void)hipFree(dev);
    return rc;
}

extern "C" {

int dice_match_sharded(dice_ctx* const* ctxs, int32_t n_ctx, const dice_files* f, double thr, int32_t gather,
                       int32_t* best, uint32_t* ov, double* score) {
    return match_sharded(ctxs, n_ctx, f, thr, gather, best, ov, score, false);
}

int dice_match_sharded_confidence(dice_ctx* const* ctxs, int32_t n_ctx, const dice_files* f, double thr,
                                  int32_t gather, int32_t* best, uint32_t* ov, double* score) {
    return match_sharded(ctxs, n_ctx, f, thr, gather, best, ov, score, true);
}

int dice_similarity_matrix_sharded(dice_ctx* const* ctxs, int32_t n_ctx, const dice_files* f, int32_t gather,
                                   uint32_t* ov, double* score, int32_t k, int32_t* tki, double* tks) {
    int rc = check_ctxs(ctxs, n_ctx, f, gather);
    if (rc) return rc;
    if (k < 0 || k > DICE_TOPK_MAX) return fail(DICE_E_ARG, "k out of range");
    if (k > 0 && (!tki || !tks)) return fail(DICE_E_ARG, "top-k outputs required when k > 0");
    const int64_t n = f->n_files;
    if (n == 0) return DICE_OK;
    if (!f->bits || !f->wordset_size || !f->length || !f->cc_false_positive) return fail(DICE_E_ARG, "NULL file arrays");
    const int32_t w64 = ctxs[0]->w64, T = ctxs[0]->T;
    if (k == 0) tki = nullptr, tks = nullptr;
    // device gather layout (row-major, as the ABI): overlap [n][T] u32 | score [n][T] f64 |
    // top-k index [n][k] i32 | top-k score [n][k] f64
    const size_t b_ov = (size_t)n * T * 4, b_sc = (size_t)n * T * 8, b_ki = (size_t)n * k * 4, b_ks = (size_t)n * k * 8;
    char* dev = nullptr;
    g_last_gather_peer = -1;
    if (gather == DICE_GATHER_DEVICE) {
        if ((rc = gather_alloc(ctxs[0], b_ov + b_sc + b_ki + b_ks, (void**)&dev))) return rc;
        prepare_device_gather(ctxs, n_ctx);
    }
    rc = run_shards(ctxs, n_ctx, n, [&](int32_t i, Shard& s) {
        dice_ctx* c = ctxs[i];
        dice_batch* b = nullptr;
        int r = dice::scratch_for(c, s.hi - s.lo, &b);
        if (r) return r;
        const dice_files part = slice(f, s.lo, s.hi, w64);
        if ((r = upload_shard(c, b, &part)) || (r = dice_batch_matrix(b, k, nullptr))) return r;
        const size_t lo = (size_t)s.lo;
        if (dev) {
            uint32_t* d_ov = (uint32_t*)dev;
            double* d_sc = (double*)(dev + b_ov);
            int32_t* d_ki = (int32_t*)(dev + b_ov + b_sc);
            double* d_ks = (double*)(dev + b_ov + b_sc + b_ki);
            return dice::download_matrix_to(b, ov ? d_ov + lo * T : nullptr, score ? d_sc + lo * T : nullptr,
                                            tki ? d_ki + lo * k : nullptr, tks ? d_ks + lo * k : nullptr, c->stream,
                                            hipMemcpyDefault);
        }
        return dice::download_matrix_to(b, ov ? ov + lo * T : nullptr, score ? score + lo * T : nullptr,
                                        tki ? tki + lo * k : nullptr, tks ? tks + lo * k : nullptr, c->stream,
                                        hipMemcpyDeviceToHost);
    });
    if (rc == DICE_OK && dev)
        rc = gather_d2h(ctxs[0], {{ov, b_ov}, {score, b_sc}, {tki, b_ki}, {tks, b_ks}}, dev);
    if (dev) (void)hipFree(dev);
    return rc;
}

int32_t dice_last_gather_peer(void) { return g_last_gather_peer; }

}  // extern "C"
