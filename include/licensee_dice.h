/*
 * licensee_dice.h -- C-ABI of the MI355X-native Dice scorer (gfx950 / HIP).
 *
 * Drop-in boundary for licensee's Dice matching hot path. The reference has no FFI for
 * this path (it is pure Ruby); every entry point below replaces a Ruby method and is what
 * a Ruby FFI binding attaches. Citations are to /root/reference:
 *
 *   dice_create / dice_destroy      replace the process-wide memoized template corpus:
 *                                   License.all(hidden: true, psuedo: false)   lib/licensee/license.rb:20-36
 *                                   + per-template wordset_fieldless / fields_normalized(_set) /
 *                                   length / spdx_alt_segments   lib/licensee/content_helper.rb:108-117,323-335
 *                                   lib/licensee/license.rb:273-283
 *   dice_match                      Dice#match + #confidence + the score loop of
 *                                   #matches_by_similarity        lib/licensee/matchers/dice.rb:8-14,34-53
 *                                   over License#similarity        lib/licensee/content_helper.rb:128-133,337-347
 *                                   with the CC filter of #potential_matches  dice.rb:23-31
 *   dice_similarity_matrix          Dice#matches_by_similarity / #licenses_by_similarity (full N x T
 *                                   scores + sorted top-k, no threshold cut)  dice.rb:34-41;
 *                                   also `licensee detect` "closest licenses" lib/licensee/commands/detect.rb:96-106
 *   dice_*_sharded                  the same two calls with the files sharded over several
 *                                   devices of one node (the dice.rb:34-41 loop is per file)
 *   dice_batch_*                    device-resident batch variants of the two calls above
 *                                   (inputs as bitsets or as word-id lists)
 *   dice_last_error                 replaces the Ruby exceptions of the path (license.rb:258,
 *                                   content_helper.rb:230,310) with status codes + message
 *
 * Conventions
 *   - Caller owns every host buffer; the library owns all device memory inside a ctx/batch.
 *   - Every call returns DICE_OK (0) or a negative DICE_E_* code; dice_last_error() gives a
 *     thread-local message for the last failing call on this thread.
 *   - One ctx per host thread (no internal locking). Host-buffer calls are synchronous.
 *   - `stream` arguments are hipStream_t passed as void* (NULL = the ctx's own stream).
 *   - Bitsets: bit v of a word-set bitset is word-id v of the template vocabulary
 *     (word v lives in uint64 word v/64, bit v%64). Vocabulary = union of the templates'
 *     wordset_fieldless; words outside it cannot overlap and only count in |W_F|.
 *   - Results are bit-exact with the reference: overlap counts are exact integers, scores are
 *     IEEE-754 double (overlap*200.0)/denominator with Ruby's Integer floor division inside
 *     the denominator. Exact score ties (parity-unpinned in the reference, whose sort is not
 *     stable) resolve to the template LATER in key order.
 */
#ifndef LICENSEE_DICE_H
#define LICENSEE_DICE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DICE_OK 0
#define DICE_E_ARG (-1)       /* invalid argument / shape */
#define DICE_E_DEVICE (-2)    /* HIP runtime error or no usable gfx950 device */
#define DICE_E_NOMEM (-3)     /* host or device allocation failed */
#define DICE_E_STATE (-4)     /* call not valid in the current state */

#define DICE_TOPK_MAX 16

typedef struct dice_ctx dice_ctx;
typedef struct dice_batch dice_batch;

/* One entry per template, in License.all(hidden: true, psuedo: false) key order. */
typedef struct dice_templates {
    int32_t n_templates;            /* T (>= 1)                                              */
    int32_t n_vocab;                /* V, bits per bitset (>= 1)                              */
    const uint64_t *lf_bits;        /* [T][dice_words64(V)]: wordset_fieldless (Lf) bitsets  */
    const uint32_t *lf_size;        /* [T] |Lf|            (content_helper.rb:130)            */
    const uint32_t *fields_set_size;/* [T] |fields_normalized_set| (content_helper.rb:131)    */
    const int32_t *length_slack;    /* [T] 5*max(fields_normalized.size, spdx_alt_segments)  */
                                    /*     (content_helper.rb:345); < 0 selects the simple   */
                                    /*     delta used when self is not a License (:343)      */
    const int32_t *length;          /* [T] content_normalized.length (characters)           */
    const uint8_t *is_cc;           /* [T] creative_commons? (license.rb:209-212)             */
} dice_templates;

/* A batch of candidate files (host memory). */
typedef struct dice_files {
    int64_t n_files;
    const uint64_t *bits;           /* [n][dice_words64(V)] row-major wordset bitsets        */
    const uint32_t *wordset_size;   /* [n] |W_F|: all distinct words, in or out of vocabulary */
    const int32_t *length;          /* [n] content_normalized.length (characters)            */
    const uint8_t *cc_false_positive; /* [n] potential_false_positive? (license_file.rb:80-82) */
} dice_files;

/* Number of uint64 words per bitset for a vocabulary of n_vocab words. */
int32_t dice_words64(int32_t n_vocab);

/* Upload a template corpus to `device` (HIP ordinal). Selects the kernel for the corpus
 * (template-specialized sparse program for T <= 64; postings kernels, LDS record kernel or
 * dense tiles above). */
int dice_create(const dice_templates *templates, int32_t device, dice_ctx **out);
void dice_destroy(dice_ctx *ctx);

/* Introspection: T, V, kernel kind (0 = dense, 1 = sparse program, 2 = LDS records,
 * 3 = postings), program entries. */
int dice_ctx_info(const dice_ctx *ctx, int32_t *n_templates, int32_t *n_vocab,
                  int32_t *kernel_kind, int32_t *program_entries);
/* Introspection: the kernel dice_match / dice_batch_match run -- the kernel kind above, or
 * 4 = bound-pruned match (kind 3 corpora; DICE_POST_PRUNE=0 keeps the postings kernels) --
 * or -1 for a NULL ctx. Results are identical whichever runs. */
int32_t dice_ctx_match_kernel(const dice_ctx *ctx);

/* Dice#match / #confidence for every file, synchronous, host buffers.
 *   best[i]    index of the matched template, or -1 (Dice#match nil) when the top
 *              score is below `threshold` or every template is CC-filtered;
 *   overlap[i] |Lf ∩ W_F| of the top-ranked template (0 if none);
 *   score[i]   similarity of the top-ranked template (0.0 if none) -- equals
 *              Dice#confidence when best[i] >= 0.
 * Any of the three output pointers may be NULL. */
int dice_match(dice_ctx *ctx, const dice_files *files, double threshold,
               int32_t *best, uint32_t *overlap, double *score);
/* Dice#match and Dice#confidence exactly as a caller of the matcher sees them
 * (dice.rb:8-14, 51-53): best[i] as dice_match; score[i] = Dice#confidence, i.e. the matched
 * template's similarity, or 0.0 when best[i] == -1; overlap[i] the matched template's overlap or 0.
 * The top-ranked template of an unmatched file is not computed, so the bound-pruned kernel
 * (T > 64) drops every template whose bound is below the threshold from the start. Equal to
 * dice_match's outputs on every matched file. */
int dice_match_confidence(dice_ctx *ctx, const dice_files *files, double threshold,
                          int32_t *best, uint32_t *overlap, double *score);

/* Full N x T similarity matrix + per-file top-k (Dice#matches_by_similarity order).
 *   overlap/score: [n][T] row-major, every template (CC filter NOT applied), may be NULL;
 *   topk_index/topk_score: [n][k] best-first among potential_matches (CC filter applied),
 *   -1 / -1.0 padding; k in [0, DICE_TOPK_MAX]. */
int dice_similarity_matrix(dice_ctx *ctx, const dice_files *files,
                           uint32_t *overlap, double *score,
                           int32_t k, int32_t *topk_index, double *topk_score);

/* ---- one node, several devices: the files of one call sharded over contexts ----------
 * The loop of Dice#matches_by_similarity (dice.rb:34-41) is independent per file, so a call
 * splits its files into n_ctx contiguous shards (shard i = files [n*i/n_ctx, n*(i+1)/n_ctx)),
 * each scored by ctxs[i] on its own device, host thread and stream; templates are replicated
 * (every ctx must hold the same corpus: same T and V, checked; same bitsets, not checked).
 * Only results move:
 *   DICE_GATHER_HOST    every device copies its results straight into its disjoint slice of
 *                       the caller's buffers (parallel D2H);
 *   DICE_GATHER_DEVICE  every device copies its results into one buffer on ctxs[0]'s device
 *                       (peer copies over xGMI), then one D2H from there.
 * The device gather enables peer access (hipDeviceEnablePeerAccess) from every shard's device
 * to ctxs[0]'s first; where two devices have none the runtime stages the copy instead.
 * Shard rows given in pageable memory are staged through two page-locked buffers per ctx
 * (each shard thread copies its own slice), so the shards do not share the runtime's bounce
 * buffers. Several ctxs may share a device (tests on a one-GPU box); the same ctx twice is
 * DICE_E_ARG. Results are bit-identical to the single-ctx calls. Outputs as dice_match /
 * dice_similarity_matrix. */
#define DICE_GATHER_HOST 0
#define DICE_GATHER_DEVICE 1
int dice_match_sharded(dice_ctx *const *ctxs, int32_t n_ctx, const dice_files *files, double threshold,
                       int32_t gather_mode, int32_t *best, uint32_t *overlap, double *score);
/* dice_match_confidence's outputs (Dice#match + #confidence, dice.rb:8-14, 51-53), sharded. */
int dice_match_sharded_confidence(dice_ctx *const *ctxs, int32_t n_ctx, const dice_files *files,
                                  double threshold, int32_t gather_mode, int32_t *best, uint32_t *overlap,
                                  double *score);
int dice_similarity_matrix_sharded(dice_ctx *const *ctxs, int32_t n_ctx, const dice_files *files,
                                   int32_t gather_mode, uint32_t *overlap, double *score, int32_t k,
                                   int32_t *topk_index, double *topk_score);
/* The last sharded call on this thread: 1 = device gather, every shard on another device wrote
 * into ctxs[0]'s device through peer access; 0 = device gather with at least one such shard
 * through the runtime's staged copy; -1 = no peer path exercised: a host gather, a device gather
 * whose contexts all sit on ctxs[0]'s device, or no sharded call yet. */
int32_t dice_last_gather_peer(void);

/* ---- device-resident batches (inputs and results stay in HBM) ---------------------- */
int dice_batch_create(dice_ctx *ctx, int64_t capacity, dice_batch **out);
void dice_batch_destroy(dice_batch *batch);
/* H2D copy + on-device repack of host files into the kernel's tile layout. */
int dice_batch_upload(dice_batch *batch, const dice_files *files, void *stream);
/* The same files given as word-id lists instead of bitsets (CSR): file i's ids are
 * ids[offsets[i] .. offsets[i+1]) as uint16 (id_bytes 2) or uint32 (id_bytes 4) values; the
 * bitsets are built on the device. Ids >= n_vocab are ignored (words outside the template
 * vocabulary cannot overlap; they count only in wordset_size), duplicates are harmless.
 * offsets[0] = 0, non-decreasing (checked). For large vocabularies this moves a fraction of
 * the bitset bytes over the host link (600 synthetic templates: ~0.6 KB of u16 ids vs 2.9 KB
 * of bitset per file). Same entry point of the reference as dice_batch_upload. */
int dice_batch_upload_ids(dice_batch *batch, int64_t n_files, const int64_t *offsets, const void *ids,
                          int32_t id_bytes, const uint32_t *wordset_size, const int32_t *length,
                          const uint8_t *cc_false_positive, void *stream);
/* Kernel-only scoring of the resident batch, asynchronous on `stream`: no host synchronization
 * and no device-to-host copy inside (capturable in a hipGraph). For T > 64 corpora this is the
 * bound-pruned kernel followed by the postings kernels over the files it deferred; their count
 * stays on the device. */
int dice_batch_match(dice_batch *batch, double threshold, void *stream);
/* dice_match_confidence's semantics for a device batch (same asynchrony and capture contract). */
int dice_batch_match_confidence(dice_batch *batch, double threshold, void *stream);
/* Introspection after dice_batch_match (synchronizes `stream`): files the bound-pruned kernel
 * deferred to the postings kernels in the last call (0 for other kernels). */
int dice_batch_deferred(dice_batch *batch, int64_t *deferred, void *stream);
/* Introspection after dice_batch_match / dice_batch_match_confidence (synchronizes `stream`): the
 * (file, template) pairs whose overlap the last call computed exactly -- n * T for every kernel
 * but the bound-pruned one (T > 64 match), which scores only the templates whose bound reaches
 * the running best (or the threshold, confidence mode) and every pair of the files it deferred.
 * The pairs the bound rules out are decided without a score (dice.rb:34-48 only reads the top). */
int dice_batch_scored_pairs(dice_batch *batch, int64_t *pairs, void *stream);
/* Device-resident matrix results are template-major ([T][n] overlap/score, [k][n] top-k) so
 * every store is coalesced; dice_batch_download_matrix returns them row-major. */
int dice_batch_matrix(dice_batch *batch, int32_t k, void *stream);
/* D2H of results (synchronizes `stream`); NULL outputs are skipped.
 * dice_batch_download_matrix: overlap/score are [n][T]; topk_index/topk_score are [n][k] and
 * `k` must equal the k of the last dice_batch_matrix call on this batch (DICE_E_ARG
 * otherwise, so a caller's buffer is never written past its [n][k] extent). */
int dice_batch_download_match(dice_batch *batch, int32_t *best, uint32_t *overlap,
                              double *score, void *stream);
int dice_batch_download_matrix(dice_batch *batch, uint32_t *overlap, double *score, int32_t k,
                               int32_t *topk_index, double *topk_score, void *stream);
/* Device pointers of the match results (int32 best, uint32 overlap, double score). */
int dice_batch_result_ptrs(dice_batch *batch, void **best, void **overlap, void **score);
/* Diagnostic: stream-read the resident tiles with trivial compute (read-ceiling probe). */
int dice_batch_stream_probe(dice_batch *batch, void *stream);
/* Bytes of the resident tile layout per file (the kernel's algorithmic input stream). */
int64_t dice_batch_bytes_per_file(const dice_batch *batch);

/* ---- Matchers::Exact on the device --------------------------------------------------
 * Exact#match (exact.rb:6-12): the first template in key order (License.all, no CC filter)
 * whose wordset (content_helper.rb:108-110: Lf plus the field words, :323-335) equals the
 * file's. dice_exact_setup gives per template |wordset| ([T]), the field words that are
 * vocabulary words as bits (field_bits [T][dice_words64(V)], NULL = none) and the field words
 * outside the vocabulary as bits of the caller's numbering (field_need [T], NULL = none;
 * licensee_host.h lh_template_field_masks). Per file, file_field_mask[i] (host, [n]; NULL =
 * all zero) holds the same numbering's bits of the file's wordset (lh_prep_files).
 * exact[i] = template index or -1. The kernel reads the batch's row-major bitsets (the
 * stream probe overwrites them). dice_batch_exact is asynchronous on `stream`: the field masks
 * are copied from host memory on that stream, so they must stay valid until it has run. */
int dice_exact_setup(dice_ctx *ctx, const uint32_t *wordset_size, const uint64_t *field_bits,
                     const uint64_t *field_need);
int dice_batch_exact(dice_batch *batch, const uint64_t *file_field_mask, void *stream);
int dice_batch_download_exact(dice_batch *batch, int32_t *exact, void *stream);
int dice_exact(dice_ctx *ctx, const dice_files *files, const uint64_t *file_field_mask, int32_t *exact);

/* ---- ContentHelper#wordset on the device ----------------------------------------------
 * The wordset scan (content_helper.rb:108-110: /(?:[\w\/-](?:'s|(?<=s)')?)+/, ASCII \w) and its
 * interning into the batch's bitset rows, for texts already normalized (content_normalized,
 * content_helper.rb:153-168; licensee_host.h lh_normalize_files), so the host threads skip the
 * scan. dice_vocab_setup gives the context its vocabulary words in id order (n_words must equal
 * the V of dice_create; ASCII, distinct) and up to 64 extra words: the template field words
 * outside the vocabulary, numbered as licensee_host.h lh_template_field_masks numbers them, which
 * the scan reports as field-mask bits (what lh_prep_files' field_mask holds) instead of row bits. */
int dice_vocab_setup(dice_ctx *ctx, int32_t n_words, const char *const *words, int32_t n_extra,
                     const char *const *extra);
/* text[0, text_bytes): the batch's normalized texts as bytes (every non-ASCII character one byte
 * >= 0x80), file i at text[offsets[i], offsets[i] + text_len[i]), offsets 16-byte aligned;
 * length[i] = content_normalized.length in characters and cc_false_positive[i] as in dice_files.
 * The device builds each file's row, |W_F| (every distinct word, in the vocabulary or not) and
 * field mask (dice_batch_exact with file_field_mask = NULL reads them). Synchronizes `stream`.
 * status[i] (host, [n]) = 1 for a file with more distinct non-vocabulary words than the device
 * set holds (192); *n_overflow (may be NULL) counts them. Such a file's row is left empty: the
 * caller prepares it on the host (lh_prep_files) and sends it with dice_batch_set_rows before
 * scoring. Same entry point of the reference as dice_batch_upload (LicenseFile#wordset). */
int dice_batch_upload_text(dice_batch *batch, int64_t n_files, const uint8_t *text, int64_t text_bytes,
                           const int64_t *offsets, const int32_t *text_len, const int32_t *length,
                           const uint8_t *cc_false_positive, uint8_t *status, int64_t *n_overflow,
                           void *stream);
/* Overwrite the rows, |W_F| and field masks (NULL: zero) of files index[0..k) of the resident
 * batch (bits: [k][dice_words64(V)]); synchronizes `stream`. */
int dice_batch_set_rows(dice_batch *batch, int64_t k, const int64_t *index, const uint64_t *bits,
                        const uint32_t *wordset_size, const uint64_t *field_mask, void *stream);
/* Page-locked host memory (hipHostMalloc) for upload buffers -- texts, bitsets -- so their H2D
 * copies run at the link's rate and overlap the host; free with dice_host_free. */
int dice_host_alloc(int64_t bytes, void **out);
void dice_host_free(void *ptr);
/* D2H of the resident rows ([n][dice_words64(V)]), |W_F| and field masks (NULL outputs skipped;
 * the masks are those of the last dice_batch_upload_text / dice_batch_exact); synchronizes. */
int dice_batch_download_rows(dice_batch *batch, uint64_t *bits, uint32_t *wordset_size, uint64_t *field_mask,
                             void *stream);

/* Build step (no device needed): generate + compile the corpus-specialized sparse program
 * with hiprtc for gfx950 and store it in the code-object cache; writes the cache path. */
int dice_precompile(const dice_templates *templates, char *path, int32_t path_cap);
/* Generated HIP source of the sparse program (introspection/tests). Returns its length,
 * writes at most cap-1 bytes + NUL when buf != NULL, or -1 on bad input. */
int64_t dice_program_source(const dice_templates *templates, char *buf, int64_t cap);

const char *dice_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LICENSEE_DICE_H */
