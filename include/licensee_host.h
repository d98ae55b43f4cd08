/*
 * licensee_host.h -- C-ABI of the native host preparation library (liblicensee_host.so).
 *
 * Host side of the Dice path: turns raw license files into the
 * dice_files inputs of licensee_dice.h, in host threads. Replaces, for bulk use:
 *   ProjectFile#initialize decode + universal newline   lib/licensee/project_files/project_file.rb:37-45
 *   ContentHelper#content_normalized / #wordset          lib/licensee/content_helper.rb:108-110,144-168,219-321
 *   LicenseFile#potential_false_positive?                lib/licensee/project_files/license_file.rb:80-82
 *   Matchers::Copyright#match                            lib/licensee/matchers/copyright.rb:12-17
 *   Matchers::Exact#match                                lib/licensee/matchers/exact.rb:6-12
 * and packs the template vocabulary for the device bitsets (word ids are free: the overlap
 * of content_helper.rb:129 counts set members, so any order gives identical scores).
 * The regular expressions are supplied by the caller (licensee_amd/content_helper.py passes
 * its compiled patterns), so host paths share one pattern source. Texts outside the native
 * envelope (non-ASCII letters, HTML) report status 1 and are prepared by the caller.
 */
#ifndef LICENSEE_HOST_H
#define LICENSEE_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lh_ctx lh_ctx;

/* Patterns (name, Python-re source, re flags I|M|S), the spelling map and the vocabulary
 * (word id = position). Returns NULL and writes err on failure. */
lh_ctx *lh_create(int32_t n_patterns, const char *const *names, const char *const *patterns,
                  const int32_t *flags, int32_t n_spell, const char *const *spell_from,
                  const char *const *spell_to, int32_t n_vocab, const char *const *vocab,
                  char *err, int32_t errcap);
void lh_destroy(lh_ctx *ctx);

/* Exact-matcher data: [T][words64(V)] Lf bitsets, |wordset| and the field words. */
int lh_set_templates(lh_ctx *ctx, int32_t n_templates, const uint64_t *lf_bits,
                     const uint32_t *wordset_size, const int32_t *field_off,
                     const char *const *field_words);
/* The template field words outside the vocabulary, numbered in first-appearance order: need[t]
 * (if not NULL, [T]) gets bit k for each of template t's. Returns their count, -1 above 64.
 * These masks and lh_prep_files' field_mask feed dice_exact_setup / dice_batch_exact. */
int32_t lh_template_field_masks(lh_ctx *ctx, uint64_t *need);

/* Unicode tables, so texts with non-ASCII letters stay native (without them the native
 * envelope is ASCII letters only). lower_*: every non-ASCII code point whose Python
 * str.lower() is a different single code point; word_lo/hi: sorted inclusive ranges of the
 * non-ASCII code points with str.isalnum() True (Python's \w for \b). The caller derives
 * both from its own Unicode database (licensee_amd/native_host.py). 0 or -1 on bad input. */
int lh_set_unicode(lh_ctx *ctx, int32_t n_lower, const uint32_t *lower_from, const uint32_t *lower_to,
                   int32_t n_word, const uint32_t *word_lo, const uint32_t *word_hi);

/* content_normalized of one text (UTF-8 out); -1 = outside the native envelope. */
int64_t lh_normalize(lh_ctx *ctx, const char *data, int64_t len, const char *filename,
                     int32_t is_file, char *out, int64_t cap);

/* Batched preparation of n LicenseFiles into dice_files arrays + matcher flags.
 * exact may be NULL (Exact then runs on the device: dice_batch_exact); field_mask, if not
 * NULL, gets per file bit k = its wordset holds non-vocabulary field word k (-1 when the
 * templates have more than 64 such words). */
int lh_prep_files(lh_ctx *ctx, int64_t n, const char *const *data, const int64_t *lens,
                  const char *const *filenames, int32_t nthreads, uint64_t *bits, uint32_t *wf,
                  int32_t *length, uint8_t *cc, uint8_t *copyright, int32_t *exact,
                  uint8_t *status, uint64_t *field_mask);

/* Batched content_normalized (content_helper.rb:153-168) for the device wordset scan
 * (licensee_dice.h dice_batch_upload_text): file i's normalized text as bytes -- every
 * non-ASCII character one byte 0x80, since the wordset's [\w/-] is ASCII -- at
 * out[off[i], off[i] + tlen[i]), offsets 16-byte aligned, files placed in completion order in
 * the caller's `cap` bytes; length[i] = the text's length in characters (len_F), cc /
 * copyright as lh_prep_files. status[i]: 0 ok; 1 outside the native envelope (the caller
 * normalizes that file itself, off[i] = -1); 3 no room left in `out` (retry with room).
 * Returns the bytes of `out` used (-1 on bad arguments). */
int64_t lh_normalize_files(lh_ctx *ctx, int64_t n, const char *const *data, const int64_t *lens,
                           const char *const *filenames, int32_t nthreads, char *out, int64_t cap,
                           int64_t *off, int32_t *tlen, int32_t *length, uint8_t *cc,
                           uint8_t *copyright, uint8_t *status);

/* Vocabulary packing (csrc/vocab_pack.cpp): local search over word swaps between bins of
 * bin_bits (32: sparse-program (template, dword) instruction pairs; 64: LDS-kernel
 * (template, u64) records), starting from `init` (a permutation of 0..V-1). sig is
 * [V][sig_words] template-membership bitsets (bit t = word in template t's Lf). Writes the
 * new order (position -> word id of `sig`) to out; returns its cost, or -1 on bad input.
 * Deterministic for a given seed. */
int64_t lh_vocab_pack(const uint64_t *sig, int32_t n_vocab, int32_t sig_words, int32_t n_templates,
                      const int32_t *init, int32_t bin_bits, int64_t iters, uint64_t seed,
                      int32_t *out);

#ifdef __cplusplus
}
#endif

#endif /* LICENSEE_HOST_H */
