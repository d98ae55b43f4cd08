// Vector scans over UTF-32 text for the host normalizer (normalize.cpp) and the regex engine's
// candidate search (rx.cpp): first occurrence of any of a few code points, first '  ' pair, and
// in-place compaction of whitespace runs. AVX2 (the host library is built for x86-64-v3) with a
// scalar tail; scalar everywhere when built without AVX2 (e.g. the sanitizer build).
#pragma once

#include <stddef.h>
#include <stdint.h>

#if defined(__AVX2__)
#include <immintrin.h>
#endif

namespace scan {

inline bool ws(char32_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }   // [ \t\n\v\f\r]

#if defined(__AVX2__)
// kCompact.idx[m]: the set lanes of the 8-bit mask m, in order, then zeros (a permutevar8x32
// control that packs the kept lanes of a block to its front)
struct Compact8 {
    int32_t idx[256][8];
    constexpr Compact8() : idx() {
        for (int m = 0; m < 256; ++m) {
            int k = 0;
            for (int l = 0; l < 8; ++l)
                if (m >> l & 1) idx[m][k++] = l;
        }
    }
};
inline constexpr Compact8 kCompact{};

inline uint32_t lanes(__m256i cmp) { return (uint32_t)_mm256_movemask_ps(_mm256_castsi256_ps(cmp)); }
inline __m256i ws_lanes(__m256i v) {
    const __m256i sp = _mm256_cmpeq_epi32(v, _mm256_set1_epi32(' '));
    const __m256i ctl = _mm256_and_si256(_mm256_cmpgt_epi32(v, _mm256_set1_epi32('\t' - 1)),
                                         _mm256_cmpgt_epi32(_mm256_set1_epi32('\r' + 1), v));
    return _mm256_or_si256(sp, ctl);
}
#endif

// first i in [from, n) with p[i] one of set[0..k) (1 <= k <= 8), or n
inline size_t find_any(const char32_t* p, size_t from, size_t n, const char32_t* set, int k) {
    size_t i = from;
#if defined(__AVX2__)
    __m256i v[8];
    for (int j = 0; j < k; ++j) v[j] = _mm256_set1_epi32((int)set[j]);
    for (; i + 8 <= n; i += 8) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(p + i));
        __m256i hit = _mm256_cmpeq_epi32(x, v[0]);
        for (int j = 1; j < k; ++j) hit = _mm256_or_si256(hit, _mm256_cmpeq_epi32(x, v[j]));
        const uint32_t m = lanes(hit);
        if (m) return i + (size_t)__builtin_ctz(m);
    }
#endif
    for (; i < n; ++i)
        for (int j = 0; j < k; ++j)
            if (p[i] == set[j]) return i;
    return n;
}

inline size_t find_char(const char32_t* p, size_t from, size_t n, char32_t c) { return find_any(p, from, n, &c, 1); }

// first i in [from, last] with p[i] in {a0, a1} and p[i + d] in {b0, b1}, or last + 1 (the
// candidate filter of a literal search: its first and last characters, d = length - 1)
inline size_t find_pair(const char32_t* p, size_t from, size_t last, size_t d, char32_t a0, char32_t a1, char32_t b0,
                        char32_t b1) {
    size_t i = from;
#if defined(__AVX2__)
    const __m256i va0 = _mm256_set1_epi32((int)a0), va1 = _mm256_set1_epi32((int)a1);
    const __m256i vb0 = _mm256_set1_epi32((int)b0), vb1 = _mm256_set1_epi32((int)b1);
    for (; i + 8 <= last + 1; i += 8) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(p + i));
        const __m256i y = _mm256_loadu_si256((const __m256i*)(p + i + d));
        const __m256i a = _mm256_or_si256(_mm256_cmpeq_epi32(x, va0), _mm256_cmpeq_epi32(x, va1));
        const __m256i b = _mm256_or_si256(_mm256_cmpeq_epi32(y, vb0), _mm256_cmpeq_epi32(y, vb1));
        const uint32_t m = lanes(_mm256_and_si256(a, b));
        if (m) return i + (size_t)__builtin_ctz(m);
    }
#endif
    for (; i <= last; ++i)
        if ((p[i] == a0 || p[i] == a1) && (p[i + d] == b0 || p[i + d] == b1)) return i;
    return last + 1;
}

// index of the second character of the first "  " pair at or after from, or n
inline size_t find_double_space(const char32_t* p, size_t from, size_t n) {
    size_t i = from;
#if defined(__AVX2__)
    const __m256i sp = _mm256_set1_epi32(' ');
    for (; i + 9 <= n; i += 8) {
        const uint32_t m = lanes(_mm256_and_si256(_mm256_cmpeq_epi32(_mm256_loadu_si256((const __m256i*)(p + i)), sp),
                                                  _mm256_cmpeq_epi32(_mm256_loadu_si256((const __m256i*)(p + i + 1)), sp)));
        if (m) return i + (size_t)__builtin_ctz(m) + 1;
    }
#endif
    for (; i + 1 < n; ++i)
        if (p[i] == ' ' && p[i + 1] == ' ') return i + 1;
    return n;
}

// In place over p[r, n), with p[0, w) (w <= r) already kept: drop every run character whose
// predecessor in the input was a run character too (prev_run: the one before p[r] was), and
// write every kept run character as ' '. Run characters are ' ' (squeeze(' ')) or, with
// all_ws, every [ \t\n\v\f\r] (gsub(/\s+/, ' ')). Returns the new length.
inline size_t squeeze_runs(char32_t* p, size_t w, size_t r, size_t n, bool prev_run, bool all_ws) {
#if defined(__AVX2__)
    const __m256i sp = _mm256_set1_epi32(' ');
    uint32_t prev = prev_run ? 1u : 0u;
    for (; r + 8 <= n; r += 8) {
        __m256i v = _mm256_loadu_si256((const __m256i*)(p + r));
        const __m256i run = all_ws ? ws_lanes(v) : _mm256_cmpeq_epi32(v, sp);
        if (all_ws) v = _mm256_blendv_epi8(v, sp, run);
        const uint32_t m = lanes(run);
        const uint32_t keep = ~(m & ((m << 1) | prev)) & 0xFFu;
        prev = m >> 7;
        const __m256i ctl = _mm256_loadu_si256((const __m256i*)kCompact.idx[keep]);
        _mm256_storeu_si256((__m256i*)(p + w), _mm256_permutevar8x32_epi32(v, ctl));   // w + 8 <= r + 8 <= n
        w += (size_t)__builtin_popcount(keep);
    }
    prev_run = prev != 0;
#endif
    for (; r < n; ++r) {
        const char32_t ch = p[r];
        const bool run = all_ws ? ws(ch) : ch == ' ';
        if (!(run && prev_run)) p[w++] = run ? U' ' : ch;
        prev_run = run;
    }
    return w;
}


// Bit j of the result: p[j] is an ASCII word character [A-Za-z0-9_] (with kSlashDash also '/'
// or '-'), for j < k <= 64 (higher bits 0). Non-ASCII positions are reported in *hi.
template <bool kSlashDash = false>
inline uint64_t ascii_word_mask(const char32_t* p, size_t k, uint64_t* hi) {
    uint64_t m = 0, h = 0;
    size_t j = 0;
#if defined(__AVX2__)
    const __m256i c20 = _mm256_set1_epi32(0x20), ca = _mm256_set1_epi32('a' - 1), cz = _mm256_set1_epi32('z' + 1);
    const __m256i c0 = _mm256_set1_epi32('0' - 1), c9 = _mm256_set1_epi32('9' + 1), cu = _mm256_set1_epi32('_');
    const __m256i c127 = _mm256_set1_epi32(127);
    for (; j + 8 <= k; j += 8) {
        const __m256i v = _mm256_loadu_si256((const __m256i*)(p + j));
        const __m256i lc = _mm256_or_si256(v, c20);
        const __m256i alpha = _mm256_and_si256(_mm256_cmpgt_epi32(lc, ca), _mm256_cmpgt_epi32(cz, lc));
        const __m256i digit = _mm256_and_si256(_mm256_cmpgt_epi32(v, c0), _mm256_cmpgt_epi32(c9, v));
        __m256i w = _mm256_or_si256(_mm256_or_si256(alpha, digit), _mm256_cmpeq_epi32(v, cu));
        if (kSlashDash)
            w = _mm256_or_si256(w, _mm256_or_si256(_mm256_cmpeq_epi32(v, _mm256_set1_epi32('/')),
                                                   _mm256_cmpeq_epi32(v, _mm256_set1_epi32('-'))));
        m |= (uint64_t)lanes(w) << j;
        h |= (uint64_t)lanes(_mm256_cmpgt_epi32(v, c127)) << j;
    }
#endif
    for (; j < k; ++j) {
        const char32_t c = p[j], lc = c | 0x20;
        const bool w = (lc >= 'a' && lc <= 'z') || (c >= '0' && c <= '9') || c == '_' || (kSlashDash && (c == '/' || c == '-'));
        m |= (uint64_t)w << j;
        h |= (uint64_t)(c > 127) << j;
    }
    m &= ~h;   // c | 0x20 of a non-ASCII code point is never ASCII, but keep the contract explicit
    *hi = h;
    return m;
}

}  // namespace scan
