// Synthetic perturbed license corpus generator (measurement harness input, host C++).
//
// Files are generated directly in normalized space: a normalized template
// is a sequence of space-separated tokens; a token contributes its scan words
// (content_helper.rb:109 -- words never span a space) and its characters to the length.
// Perturbations follow the reference's own tests:
//   * insert k random ipsum words  (spec_helper.rb:82-91 add_random_words, default 5;
//     vendored_license_spec.rb:41 uses 75),
//   * drop / replace 0-5% of tokens,
//   * profile 1 ("long/mixed COPYING", BASELINE config 4): 2-6 templates concatenated plus
//     an appended notice of 50-300 ipsum words (dice_matcher_spec.rb:43-54 stacks MIT+GPL).
// Every file is a pure function of (seed, global index), so ranks generate disjoint shards
// without communication and tests can replay any file's token sequence (synth_tokens).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {  // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
};

}  // namespace

extern "C" {

typedef struct synth_spec {
    int32_t n_tokens;
    const int32_t *tok_len;        // [n_tokens] characters
    const int32_t *tok_word_off;   // [n_tokens+1] CSR into tok_words
    const int32_t *tok_words;      // extended word ids: [0, n_vocab) in vocabulary, [n_vocab, n_ext) not
    int32_t n_templates;
    const int64_t *tpl_off;        // [T+1] CSR into tpl_tokens
    const int32_t *tpl_tokens;
    int32_t n_ipsum;
    const int32_t *ipsum_tokens;
    int32_t n_vocab;
    int32_t n_ext;
    int32_t profile;               // 0: perturbed single template, 1: long/mixed
} synth_spec;

}  // extern "C"

namespace {

// The per-file recipe. Visitor gets (token, insert_pos) where insert_pos = -1 for tokens
// appended in order, >= 0 for insertions into the current sequence.
template <class Visit>
void recipe(const synth_spec *sp, uint64_t seed, int64_t index, Visit &&visit, uint8_t *cc_out,
            int32_t *src_out) {
    Rng r(seed ^ ((uint64_t)index * 0xD1B54A32D192ED03ULL + 0x2545F4914F6CDD1DULL));
    r.next();
    int64_t count = 0;
    auto emit_template = [&](int32_t t, uint32_t drop_permille) {
        for (int64_t i = sp->tpl_off[t]; i < sp->tpl_off[t + 1]; ++i) {
            uint64_t x = r.next();
            if ((uint32_t)(x % 1000) < drop_permille) {
                if ((x >> 32) & 1) {  // replace with a random ipsum word
                    visit(sp->ipsum_tokens[r.below(sp->n_ipsum)], -1);
                    ++count;
                }
                continue;
            }
            visit(sp->tpl_tokens[i], -1);
            ++count;
        }
    };
    int32_t src = 0;
    uint32_t inserts = 0;
    if (sp->profile == 1) {
        const uint32_t parts = 2 + r.below(5);  // 2..6 templates
        src = (int32_t)r.below(sp->n_templates);
        emit_template(src, 0);
        for (uint32_t p = 1; p < parts; ++p) emit_template((int32_t)r.below(sp->n_templates), 0);
        const uint32_t notice = 50 + r.below(251);
        for (uint32_t j = 0; j < notice; ++j) { visit(sp->ipsum_tokens[r.below(sp->n_ipsum)], -1); ++count; }
    } else {
        src = (int32_t)r.below(sp->n_templates);
        const uint32_t mode = r.below(100);
        uint32_t drop = 0;
        if (mode < 50) {
            inserts = r.below(6);
        } else if (mode < 90) {
            inserts = r.below(6);
            drop = r.below(51);
        } else {
            inserts = 75;
        }
        emit_template(src, drop);
    }
    for (uint32_t j = 0; j < inserts; ++j) {
        const int32_t tok = sp->ipsum_tokens[r.below(sp->n_ipsum)];
        const int64_t pos = (int64_t)(r.next() % (uint64_t)(count + 1));
        visit(tok, pos);
        ++count;
    }
    const bool cc = r.below(100) == 0;  // 1% potential CC false positives
    if (cc_out) *cc_out = cc ? 1 : 0;
    if (src_out) *src_out = src;
}

}  // namespace

extern "C" {

// Generates files [first, first+n) into row-major bitsets over the vocabulary (w64 words
// per file), |W_F| (distinct in- and out-of-vocabulary words), len_F and the CC flag.
int synth_generate(const synth_spec *sp, uint64_t seed, int64_t first, int64_t n, int32_t nthreads,
                   uint64_t *bits, uint32_t *wf, int32_t *len, uint8_t *cc, int32_t *src) {
    if (!sp || n < 0 || sp->n_templates < 1 || sp->n_ipsum < 1 || sp->n_vocab < 1 || sp->n_ext < sp->n_vocab)
        return -1;
    const int32_t w64 = (sp->n_vocab + 63) / 64;
    const int32_t e64 = (sp->n_ext + 63) / 64;
    if (nthreads < 1) nthreads = 1;
    auto work = [&](int64_t lo, int64_t hi) {
        std::vector<uint64_t> ext((size_t)e64);
        for (int64_t k = lo; k < hi; ++k) {
            std::fill(ext.begin(), ext.end(), 0);
            int64_t chars = 0, ntok = 0;
            auto visit = [&](int32_t tok, int64_t) {
                chars += sp->tok_len[tok];
                ++ntok;
                for (int32_t w = sp->tok_word_off[tok]; w < sp->tok_word_off[tok + 1]; ++w) {
                    const int32_t id = sp->tok_words[w];
                    ext[(size_t)id >> 6] |= 1ULL << (id & 63);
                }
            };
            recipe(sp, seed, first + k, visit, cc ? cc + k : nullptr, src ? src + k : nullptr);
            uint32_t distinct = 0;
            for (int32_t i = 0; i < e64; ++i) distinct += (uint32_t)__builtin_popcountll(ext[(size_t)i]);
            uint64_t *row = bits + (size_t)k * w64;
            memcpy(row, ext.data(), sizeof(uint64_t) * (size_t)w64);
            if (sp->n_vocab & 63) row[w64 - 1] &= (1ULL << (sp->n_vocab & 63)) - 1;
            wf[k] = distinct;
            len[k] = (int32_t)(ntok ? chars + ntok - 1 : 0);
        }
    };
    std::vector<std::thread> th;
    const int64_t chunk = (n + nthreads - 1) / nthreads;
    for (int32_t i = 0; i < nthreads; ++i) {
        const int64_t lo = (int64_t)i * chunk, hi = std::min<int64_t>(n, lo + chunk);
        if (lo >= hi) break;
        th.emplace_back(work, lo, hi);
    }
    for (auto &t : th) t.join();
    return 0;
}

// Replays file `index`'s token sequence (for tests). Returns the token count (may exceed
// cap; only the first cap tokens are written) or -1.
int64_t synth_tokens(const synth_spec *sp, uint64_t seed, int64_t index, int32_t *out, int64_t cap,
                     uint8_t *cc, int32_t *src) {
    if (!sp) return -1;
    std::vector<int32_t> seq;
    auto visit = [&](int32_t tok, int64_t pos) {
        if (pos < 0) seq.push_back(tok);
        else seq.insert(seq.begin() + pos, tok);
    };
    recipe(sp, seed, index, visit, cc, src);
    for (int64_t i = 0; i < (int64_t)seq.size() && i < cap; ++i) out[i] = seq[(size_t)i];
    return (int64_t)seq.size();
}

}  // extern "C"
