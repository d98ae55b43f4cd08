// Internal definitions shared by dice.hip and dice_program.cpp (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/licensee_dice.h"
#include "dice_program.h"

namespace dice {

constexpr int32_t kProgramMaxTemplates = 64;   // sparse program kernel for T <= 64

// thread-local last-error text (dice_last_error)
std::string& last_error();

inline int fail(int code, const std::string& msg) {
    last_error() = msg;
    return code;
}

// Diagnostic switches (DICE_*_DIAG) make results wrong by design (phase-skip and timing
// builds). They are honoured only by a library built with -DDICE_DIAG; the
// shipped library ignores them and says so once on stderr, so a stray variable in a production
// environment cannot corrupt Dice#match output.
inline const char* diag_env(const char* name) {
    const char* v = getenv(name);
    if (!v || !*v) return nullptr;
#ifdef DICE_DIAG
    return v;
#else
    static bool warned = false;
    if (!warned) {
        warned = true;
        fprintf(stderr, "liblicensee_dice: %s=%s ignored (diagnostic switches need a -DDICE_DIAG build)\n", name, v);
    }
    return nullptr;
#endif
}

inline int dalloc_bytes(void** p, size_t bytes) {
    if (hipMalloc(p, bytes ? bytes : 1) != hipSuccess) {
        *p = nullptr;
        return fail(DICE_E_NOMEM, "hipMalloc failed");
    }
    return DICE_OK;
}

}  // namespace dice

struct dice_ctx {
    int device = 0;
    int32_t T = 0, V = 0, w64 = 0, wq = 0, tpad = 0;
    hipStream_t stream = nullptr;
    uint4* d_tq = nullptr;  // [wq][tpad] template quads (dense kernel)
    int4* d_tc = nullptr;   // [tpad] TplConst (dense kernel)
    int32_t kind = 0;       // 0 dense, 1 sparse program, 2 LDS-tiled records, 3 postings (T > 64)
    dice::Program prog;     // sparse program (kind 1)
    hipModule_t module = nullptr;
    hipFunction_t prog_match = nullptr;
    hipFunction_t prog_matrix = nullptr;    // top-k <= 4
    hipFunction_t prog_matrix16 = nullptr;  // top-k <= 16
    int32_t* d_qperm = nullptr;             // sparse program tile slot -> vocabulary quad (kind 1)
    dice_batch* scratch = nullptr;  // reused by the host-buffer calls
    // kind 2 plan (dice_lds.hip): per-(slab, template) entry runs, entries, wave split
    void* d_lrec = nullptr;
    void* d_lep = nullptr;
    void* d_les = nullptr;
    void* d_lwt = nullptr;
    int32_t lds_nslab = 0, lds_npass = 0;
    int64_t lds_entries = 0;
    // kind 3 plan (dice_post.hip): postings rows of the narrow words, dense-prefix masks
    void* d_pdmt = nullptr;    // [20][kMfmaCols] u64 dense-prefix masks, word-major, zero-padded (MFMA kernel)
    void* d_prow = nullptr;    // [64*w64][16] u16 postings row per word (short ids / long word ref)
    void* d_povf = nullptr;    // flat u16 template ids of the long words
    void* d_ptc = nullptr;     // [T] int4 template constants
    int32_t post_dense = 0, post_tpad = 0, post_tp = 0, post_ld = 0;
    bool post_fast = false;
    int64_t post_rows = 0;
    // kind 3 match mode, bound-pruned (dice_prune.hip): tables in position (length-sorted) order --
    // group bytes, constants, CC masks, template index | record offset, records, slot bounds
    bool prune = false, prune_zero_base = false;
    uint32_t prune_max_lf = 0;       // largest template |Lf| (the long-file test of dice_match's routing)
    int32_t prune_long_route = 4;    // dice_match: postings kernels when >= 1/N of a batch's files are long (0: never)
    uint32_t prune_wf_noclamp = 0;   // |W_F| from which the bound's length term needs no clamp
    void *d_p4q8 = nullptr, *d_p4tc = nullptr, *d_p4cc = nullptr, *d_p4off = nullptr, *d_p4rec = nullptr,
         *d_p4slot = nullptr;
    int32_t p4_zkeep[2] = {-1, -1}, p4_zpos[2] = {0, 0};
    int32_t n_cu = 256, prune_max_evals = 8, prune_route = 16;
    // sharded calls (dice_shard.cpp): devices this ctx's device has peer access to (bit d), and
    // two page-locked staging buffers for shard uploads from pageable caller memory
    uint64_t peer_mask = 0;
    void* h_stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    size_t h_stage_bytes = 0;
    // Exact matcher (dice_exact.hip): host copy of the Lf bitsets; templates sorted by |W_t|
    // {|W_t|, t, record range}, need masks, records of W_t ∩ V
    std::vector<uint64_t> h_lf;
    // small host-buffer calls (n <= kSmallFiles, dice.hip): a batch whose inputs and results are
    // each one device region, mirrored by page-locked host regions -- one H2D and one D2H per call
    dice_batch* small = nullptr;
    void *h_small_in = nullptr, *h_small_out = nullptr;
    void *d_ex_tbl = nullptr, *d_ex_need = nullptr, *d_ex_rec = nullptr;
    bool exact_ready = false;
    // device wordset scan (dice_words.hip): the vocabulary table -- tagged slots, keys, lengths,
    // word offsets and bytes (for long words' tails)
    void *d_wslots = nullptr, *d_wkeys = nullptr, *d_wlen = nullptr, *d_woff = nullptr, *d_wtxt = nullptr;
    uint32_t words_bmask = 0, words_id_bits = 0, words_extra = 0;
    bool words_ready = false;
};

namespace dice {
int lds_setup(dice_ctx* c, const dice_templates* t);
int lds_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s);
bool post_feasible(const dice_templates* t);
int post_setup(dice_ctx* c, const dice_templates* t);
// confidence: Dice#confidence outputs (overlap 0 and score 0.0 for a file without a match)
int post_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, bool confidence = false);
int post_launch_matrix(dice_ctx* c, dice_batch* b, int32_t k, hipStream_t s);
// the deferred files idx[0 .. *pn) of a pruned match (count on the device; no host read-back)
int post_launch_match_indexed(dice_ctx* c, dice_batch* b, double thr, const int32_t* idx, const uint32_t* pn,
                              hipStream_t s, bool confidence = false);
// the batch's dense-partial buffer ([capacity][tp] u16)
int post_reserve(dice_ctx* c, dice_batch* b);
int prune_setup(dice_ctx* c, const dice_templates* t);
int prune_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s, bool confidence = false);
// the pruned match's device buffers for batch b (called by dice_batch_create)
int prune_reserve(dice_ctx* c, dice_batch* b);
// dice_batch_upload's tail (scalars, repack) for rows already copied to b->d_rows on `s`
int upload_rows_resident(dice_batch* b, const dice_files* f, hipStream_t s);
// the ctx's reusable batch for the host-buffer calls (grown on demand)
int scratch_for(dice_ctx* ctx, int64_t n, dice_batch** out);
// result downloads to host memory or (kind hipMemcpyDefault) another device's memory;
// synchronize `s`
int download_match_to(dice_batch* b, int32_t* best, uint32_t* ov, double* score, hipStream_t s,
                      hipMemcpyKind kind);
int download_matrix_to(dice_batch* b, uint32_t* ov, double* score, int32_t* tki, double* tks, hipStream_t s,
                       hipMemcpyKind kind);
// the Exact tables (dice_exact.hip)
void exact_free(dice_ctx* c);
// the device wordset tables (dice_words.hip)
void words_free(dice_ctx* c);
// dice_batch_upload's tail: per-file scalars (wf == NULL: already on the device, b->n_long set),
// padding, and the tile repack (dice.hip)
int upload_tail(dice_batch* b, int64_t n, const uint32_t* wf, const int32_t* len, const uint8_t* cc, hipStream_t s);
// the tile-layout kernels' repack of b->d_rows (no-op for the postings kernels)
int repack(dice_batch* b, hipStream_t s);
}  // namespace dice

struct dice_batch {
    dice_ctx* ctx = nullptr;
    int64_t capacity = 0, n = 0, n_tiles_cap = 0;
    uint64_t* d_rows = nullptr;     // staging [capacity][w64]
    uint4* d_tiles = nullptr;       // [n_tiles][wq][64]
    uint32_t* d_wf = nullptr;
    int32_t* d_len = nullptr;
    uint8_t* d_cc = nullptr;
    int32_t* d_best = nullptr;
    uint32_t* d_ov = nullptr;
    double* d_score = nullptr;
    // matrix results (lazily allocated)
    int64_t mat_cap = 0;
    int32_t mat_k = 0;
    int32_t k_used = 0;
    bool mat_rowmajor = false;      // kind 3 writes [n][ld] / [n][k] directly (no transpose)
    int32_t mat_ld = 0;             // row stride (templates) of the row-major matrix
    uint32_t* d_mov = nullptr;      // template-major [T][capacity] (coalesced stores)
    double* d_mscore = nullptr;     // template-major [T][capacity]
    int32_t* d_tki = nullptr;
    double* d_tks = nullptr;
    void* d_stage = nullptr;        // row-major staging for downloads
    void* d_pdense = nullptr;       // kind 3: dense-prefix partial overlaps [capacity][tp] u16
    void* d_ids = nullptr;          // dice_batch_upload_ids staging: the id list ...
    size_t ids_bytes = 0;
    int64_t* d_offs = nullptr;      // ... and its [capacity + 1] offsets
    size_t pdense_bytes = 0;
    size_t stage_bytes = 0;
    // pruned match (dice_prune.hip): files deferred to the postings kernels
    int32_t* d_defer = nullptr;     // [capacity] file indices dice_prune4 deferred
    uint32_t* d_ndefer = nullptr;   // their count
    uint32_t* d_nscored = nullptr;  // per wave of the last pruned launch: (file, template) pairs scored exactly
    int64_t prune_waves = 0;        // waves of that launch (entries of d_nscored)
    int32_t last_match = 0;         // last match call: 0 none, 1 every pair scored, 2 bound-pruned
    int64_t n_long = 0;             // files of the upload with |W_F| above every template's |Lf| (-1: unknown)
    // Exact matcher (dice_batch_exact, lazily allocated): per-file result, field masks
    int32_t* d_exact = nullptr;
    uint64_t* d_fmask = nullptr;
    bool fmask_device = false;      // d_fmask holds the last upload's masks (dice_batch_upload_text)
    // dice_batch_upload_text (dice_words.hip): texts, their offsets and lengths, per-file status,
    // counters {overflowed files, long files}
    uint8_t* d_text = nullptr;
    size_t text_cap = 0;
    int64_t* d_toff = nullptr;
    int32_t* d_tlen = nullptr;
    uint8_t* d_wstat = nullptr;
    uint32_t* d_wcnt = nullptr;
    // small-call batch: d_wf/d_len/d_cc/d_rows carved from d_in, results from d_out
    void *d_in = nullptr, *d_out = nullptr;
};
