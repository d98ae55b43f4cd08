// Vocabulary packing for the device bitsets (host interner, corpus.vocabulary_order).
//
// Word ids are free: any bijection of the template vocabulary gives the same overlaps
// (content_helper.rb:129 counts set members, not positions). The order only decides how
// the scoring kernels pay for each template:
//   * bin_bits = 32, sparse program (T <= 64): one instruction pair per (template, dword)
//     the template touches -- v_and (literal mask) + v_bcnt -- or a lone v_bcnt when the
//     template owns all 32 words of the dword. Cost of a dword = sum over the templates in
//     the union of its words' signatures of (2, or 1 if full).
//   * bin_bits = 64, LDS kernel (T > 64): one record per (template, u64 word) touched.
// Minimizing that is a clustering problem (pack words into fixed-size bins so that few
// templates touch each bin). This is a deterministic local search over word swaps between
// bins, started from the caller's order (signature groups chained by Hamming distance),
// with per-bin template counts updated incrementally: a swap only touches the templates in
// sig(i) xor sig(j), so one attempt costs a handful of operations.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/licensee_host.h"

namespace {

struct Rng {  // xorshift64*: same sequence on every host
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed ? seed : 0x9E3779B97F4A7C15ULL) {}
    uint64_t next() {
        s ^= s >> 12;
        s ^= s << 25;
        s ^= s >> 27;
        return s * 0x2545F4914F6CDD1DULL;
    }
};

// Per-bin template state as bitsets over templates, so the cost delta of a swap is a few
// popcounts per signature word: present (count > 0), single (count == 1), full (count ==
// bin size, 32-bit bins only) and almost (count == 31 in a 32-word bin).
struct Packer {
    int32_t V, W, bin, nbins, T;
    const uint64_t* sig;           // [V][W]
    std::vector<int32_t> ord;      // position -> word
    std::vector<int32_t> pos;      // word -> position
    std::vector<uint16_t> cnt;     // [nbins][T]
    std::vector<int32_t> bsize;    // words per bin (the last may be short)
    std::vector<uint64_t> present, single, full, almost;   // [nbins][W]

    void refresh(int32_t b, int32_t t) {
        const uint16_t c = cnt[(size_t)b * T + t];
        const size_t k = (size_t)b * W + t / 64;
        const uint64_t bit = 1ULL << (t % 64);
        const bool counted = bin == 32 && bsize[b] == 32;
        present[k] = c > 0 ? present[k] | bit : present[k] & ~bit;
        single[k] = c == 1 ? single[k] | bit : single[k] & ~bit;
        full[k] = counted && c == 32 ? full[k] | bit : full[k] & ~bit;
        almost[k] = counted && c == 31 ? almost[k] | bit : almost[k] & ~bit;
    }
    int64_t total() const {
        int64_t s = 0;
        for (int32_t b = 0; b < nbins; ++b)
            for (int k = 0; k < W; ++k) {
                const size_t i = (size_t)b * W + k;
                s += (bin == 32 ? 2 : 1) * __builtin_popcountll(present[i]) - __builtin_popcountll(full[i]);
            }
        return s;
    }
    // cost delta of bin b losing the templates `lose` and gaining `gain` (one signature word k)
    int delta(int32_t b, int k, uint64_t lose, uint64_t gain) const {
        const size_t i = (size_t)b * W + k;
        if (bin == 64) return __builtin_popcountll(gain & ~present[i]) - __builtin_popcountll(lose & single[i]);
        return 2 * __builtin_popcountll(gain & ~present[i]) - 2 * __builtin_popcountll(lose & single[i]) +
               __builtin_popcountll(lose & full[i]) - __builtin_popcountll(gain & almost[i]);
    }
    int swap_delta(int32_t p, int32_t q) const {
        const int32_t a = p / bin, b = q / bin;
        const uint64_t* x = sig + (size_t)ord[p] * W;
        const uint64_t* y = sig + (size_t)ord[q] * W;
        int d = 0;
        for (int k = 0; k < W; ++k) {
            const uint64_t xa = x[k] & ~y[k], ya = y[k] & ~x[k];
            if (xa | ya) d += delta(a, k, xa, ya) + delta(b, k, ya, xa);
        }
        return d;
    }
    void apply_swap(int32_t p, int32_t q) {
        const int32_t a = p / bin, b = q / bin;
        const uint64_t* x = sig + (size_t)ord[p] * W;
        const uint64_t* y = sig + (size_t)ord[q] * W;
        for (int k = 0; k < W; ++k) {
            for (uint64_t m = x[k] & ~y[k]; m; m &= m - 1) {   // leaves a, joins b
                const int t = k * 64 + __builtin_ctzll(m);
                --cnt[(size_t)a * T + t];
                ++cnt[(size_t)b * T + t];
                refresh(a, t);
                refresh(b, t);
            }
            for (uint64_t m = y[k] & ~x[k]; m; m &= m - 1) {   // leaves b, joins a
                const int t = k * 64 + __builtin_ctzll(m);
                --cnt[(size_t)b * T + t];
                ++cnt[(size_t)a * T + t];
                refresh(a, t);
                refresh(b, t);
            }
        }
        std::swap(ord[p], ord[q]);
        pos[ord[p]] = p;
        pos[ord[q]] = q;
    }
};

// uniform integer in [0, n) from 32 random bits (multiply-high, no division)
inline uint32_t below(uint32_t r, uint32_t n) { return (uint32_t)(((uint64_t)r * n) >> 32); }

}  // namespace

extern "C" int64_t lh_vocab_pack(const uint64_t* sig, int32_t n_vocab, int32_t sig_words, int32_t n_templates,
                                 const int32_t* init, int32_t bin_bits, int64_t iters, uint64_t seed,
                                 int32_t* out) {
    if (!sig || !init || !out || n_vocab < 1 || sig_words < 1 || n_templates < 1 ||
        n_templates > sig_words * 64 || (bin_bits != 32 && bin_bits != 64) || iters < 0)
        return -1;
    Packer P;
    P.V = n_vocab;
    P.W = sig_words;
    P.bin = bin_bits;
    P.nbins = (n_vocab + bin_bits - 1) / bin_bits;
    P.T = n_templates;
    P.sig = sig;
    P.ord.assign(init, init + n_vocab);
    {   // init must be a permutation
        std::vector<uint8_t> seen(n_vocab, 0);
        for (int32_t w : P.ord) {
            if (w < 0 || w >= n_vocab || seen[w]) return -1;
            seen[w] = 1;
        }
    }
    P.cnt.assign((size_t)P.nbins * P.T, 0);
    P.bsize.assign(P.nbins, 0);
    for (int32_t p = 0; p < n_vocab; ++p) {
        const int32_t b = p / bin_bits;
        ++P.bsize[b];
        const uint64_t* x = sig + (size_t)P.ord[p] * P.W;
        for (int k = 0; k < P.W; ++k)
            for (uint64_t m = x[k]; m; m &= m - 1) ++P.cnt[(size_t)b * P.T + k * 64 + __builtin_ctzll(m)];
    }
    for (auto* v : {&P.present, &P.single, &P.full, &P.almost}) v->assign((size_t)P.nbins * P.W, 0);
    for (int32_t b = 0; b < P.nbins; ++b)
        for (int32_t t = 0; t < P.T; ++t) P.refresh(b, t);
    P.pos.assign(n_vocab, 0);
    for (int32_t p = 0; p < n_vocab; ++p) P.pos[P.ord[p]] = p;
    // words of each template (CSR): targeted moves bring a word next to another word of one
    // of its templates
    std::vector<int32_t> toff(P.T + 1, 0), twords;
    for (int32_t w = 0; w < n_vocab; ++w)
        for (int k = 0; k < P.W; ++k)
            for (uint64_t m = sig[(size_t)w * P.W + k]; m; m &= m - 1) ++toff[k * 64 + __builtin_ctzll(m) + 1];
    for (int32_t t = 0; t < P.T; ++t) toff[t + 1] += toff[t];
    twords.resize(toff[P.T]);
    {
        std::vector<int32_t> fill(toff.begin(), toff.end() - 1);
        for (int32_t w = 0; w < n_vocab; ++w)
            for (int k = 0; k < P.W; ++k)
                for (uint64_t m = sig[(size_t)w * P.W + k]; m; m &= m - 1) twords[fill[k * 64 + __builtin_ctzll(m)]++] = w;
    }
    int64_t cost = P.total();
    if (P.nbins > 1) {
        Rng rng(seed);
        for (int64_t it = 0; it < iters; ++it) {
            const uint64_t r = rng.next();
            const int32_t p = (int32_t)below((uint32_t)r, (uint32_t)n_vocab);
            int32_t q;
            const uint64_t r2 = rng.next();
            const uint64_t* x = sig + (size_t)P.ord[p] * P.W;
            if ((r >> 32) % 4 != 0) {
                // targeted: a random template t of word p, a random word of t, a random slot of
                // that word's bin
                int nb = 0;
                for (int k = 0; k < P.W; ++k) nb += __builtin_popcountll(x[k]);
                if (nb == 0) continue;
                int pick = (int)below((uint32_t)(r >> 32), (uint32_t)nb), t = -1;
                for (int k = 0; k < P.W && t < 0; ++k) {
                    const int c = __builtin_popcountll(x[k]);
                    if (pick < c) {
                        uint64_t m = x[k];
                        for (int i = 0; i < pick; ++i) m &= m - 1;
                        t = k * 64 + __builtin_ctzll(m);
                    } else {
                        pick -= c;
                    }
                }
                const int32_t nw = toff[t + 1] - toff[t];
                const int32_t other = twords[toff[t] + (int32_t)below((uint32_t)r2, (uint32_t)nw)];
                const int32_t qb = P.pos[other] / bin_bits;
                q = qb * bin_bits + (int32_t)below((uint32_t)(r2 >> 32), (uint32_t)P.bsize[qb]);
            } else {
                q = (int32_t)below((uint32_t)r2, (uint32_t)n_vocab);
            }
            if (p / bin_bits == q / bin_bits) continue;
            const int d = P.swap_delta(p, q);
            if (d <= 0) {   // accept (zero-delta moves walk plateaus)
                P.apply_swap(p, q);
                cost += d;
            }
        }
    }
    memcpy(out, P.ord.data(), sizeof(int32_t) * (size_t)n_vocab);
    return cost;
}
