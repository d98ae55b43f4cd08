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

// ---- the same scans over ASCII bytes (the byte path of normalize.cpp / rx.cpp: a text whose
// every character is ASCII is normalized as a std::string, one byte per character) ----------

#if defined(__AVX2__)
inline uint32_t bytes(__m256i cmp) { return (uint32_t)_mm256_movemask_epi8(cmp); }
#endif

inline size_t find_any(const char* p, size_t from, size_t n, const char32_t* set, int k) {
    size_t i = from;
#if defined(__AVX2__)
    __m256i v[8];
    int kk = 0;
    for (int j = 0; j < k; ++j)
        if (set[j] < 128) v[kk++] = _mm256_set1_epi8((char)set[j]);   // (non-ASCII members never occur)
    if (kk == 0) return n;
    for (; i + 32 <= n; i += 32) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(p + i));
        __m256i hit = _mm256_cmpeq_epi8(x, v[0]);
        for (int j = 1; j < kk; ++j) hit = _mm256_or_si256(hit, _mm256_cmpeq_epi8(x, v[j]));
        const uint32_t m = bytes(hit);
        if (m) return i + (size_t)__builtin_ctz(m);
    }
#endif
    for (; i < n; ++i)
        for (int j = 0; j < k; ++j)
            if ((char32_t)(unsigned char)p[i] == set[j]) return i;
    return n;
}

inline size_t find_char(const char* p, size_t from, size_t n, char32_t c) { return find_any(p, from, n, &c, 1); }

inline size_t find_pair(const char* p, size_t from, size_t last, size_t d, char32_t a0, char32_t a1, char32_t b0,
                        char32_t b1) {
    size_t i = from;
    if (a0 >= 128 && a1 >= 128) return last + 1;
    if (b0 >= 128 && b1 >= 128) return last + 1;
#if defined(__AVX2__)
    // (a non-ASCII member is replaced by an ASCII one of the same pair: it never occurs in the text)
    const __m256i va0 = _mm256_set1_epi8((char)(a0 < 128 ? a0 : a1)), va1 = _mm256_set1_epi8((char)(a1 < 128 ? a1 : a0));
    const __m256i vb0 = _mm256_set1_epi8((char)(b0 < 128 ? b0 : b1)), vb1 = _mm256_set1_epi8((char)(b1 < 128 ? b1 : b0));
    for (; i + 32 <= last + 1; i += 32) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(p + i));
        const __m256i y = _mm256_loadu_si256((const __m256i*)(p + i + d));
        const __m256i a = _mm256_or_si256(_mm256_cmpeq_epi8(x, va0), _mm256_cmpeq_epi8(x, va1));
        const __m256i b = _mm256_or_si256(_mm256_cmpeq_epi8(y, vb0), _mm256_cmpeq_epi8(y, vb1));
        const uint32_t m = bytes(_mm256_and_si256(a, b));
        if (m) return i + (size_t)__builtin_ctz(m);
    }
#endif
    for (; i <= last; ++i) {
        const char32_t x = (unsigned char)p[i], y = (unsigned char)p[i + d];
        if ((x == a0 || x == a1) && (y == b0 || y == b1)) return i;
    }
    return last + 1;
}

inline size_t find_double_space(const char* p, size_t from, size_t n) {
    size_t i = from;
#if defined(__AVX2__)
    const __m256i sp = _mm256_set1_epi8(' ');
    for (; i + 33 <= n; i += 32) {
        const uint32_t m = bytes(_mm256_and_si256(_mm256_cmpeq_epi8(_mm256_loadu_si256((const __m256i*)(p + i)), sp),
                                                  _mm256_cmpeq_epi8(_mm256_loadu_si256((const __m256i*)(p + i + 1)), sp)));
        if (m) return i + (size_t)__builtin_ctz(m) + 1;
    }
#endif
    for (; i + 1 < n; ++i)
        if (p[i] == ' ' && p[i + 1] == ' ') return i + 1;
    return n;
}

// squeeze_runs over bytes: 32-byte blocks without two adjacent run characters are copied (or
// left in place) whole, the others character by character.
inline size_t squeeze_runs(char* p, size_t w, size_t r, size_t n, bool prev_run, bool all_ws) {
#if defined(__AVX2__)
    const __m256i sp = _mm256_set1_epi8(' ');
    const __m256i t0 = _mm256_set1_epi8('\t' - 1), r1 = _mm256_set1_epi8('\r' + 1);
    for (; r + 32 <= n;) {
        const __m256i v = _mm256_loadu_si256((const __m256i*)(p + r));
        const __m256i is_sp = _mm256_cmpeq_epi8(v, sp);
        const __m256i run = all_ws ? _mm256_or_si256(is_sp, _mm256_and_si256(_mm256_cmpgt_epi8(v, t0), _mm256_cmpgt_epi8(r1, v)))
                                   : is_sp;
        const uint32_t m = bytes(run);
        if ((m & ((m << 1) | (prev_run ? 1u : 0u))) == 0 && (!all_ws || (m & ~bytes(is_sp)) == 0)) {
            // nothing to drop and nothing to rewrite: the block as it is
            if (w != r) _mm256_storeu_si256((__m256i*)(p + w), v);
            w += 32;
            r += 32;
            prev_run = (m >> 31) != 0;
            continue;
        }
        for (const size_t e = r + 32; r < e; ++r) {
            const char ch = p[r];
            const bool rn = all_ws ? ws((unsigned char)ch) : ch == ' ';
            if (!(rn && prev_run)) p[w++] = rn ? ' ' : ch;
            prev_run = rn;
        }
    }
#endif
    for (; r < n; ++r) {
        const char ch = p[r];
        const bool rn = all_ws ? ws((unsigned char)ch) : ch == ' ';
        if (!(rn && prev_run)) p[w++] = rn ? ' ' : ch;
        prev_run = rn;
    }
    return w;
}

// ascii_word_mask over bytes (every byte is ASCII on the byte path: *hi is 0)
template <bool kSlashDash = false>
inline uint64_t ascii_word_mask(const char* p, size_t k, uint64_t* hi) {
    uint64_t m = 0;
    size_t j = 0;
#if defined(__AVX2__)
    const __m256i c20 = _mm256_set1_epi8(0x20), ca = _mm256_set1_epi8('a' - 1), cz = _mm256_set1_epi8('z' + 1);
    const __m256i c0 = _mm256_set1_epi8('0' - 1), c9 = _mm256_set1_epi8('9' + 1), cu = _mm256_set1_epi8('_');
    for (; j + 32 <= k; j += 32) {
        const __m256i v = _mm256_loadu_si256((const __m256i*)(p + j));
        const __m256i lc = _mm256_or_si256(v, c20);
        const __m256i alpha = _mm256_and_si256(_mm256_cmpgt_epi8(lc, ca), _mm256_cmpgt_epi8(cz, lc));
        const __m256i digit = _mm256_and_si256(_mm256_cmpgt_epi8(v, c0), _mm256_cmpgt_epi8(c9, v));
        __m256i w = _mm256_or_si256(_mm256_or_si256(alpha, digit), _mm256_cmpeq_epi8(v, cu));
        if (kSlashDash)
            w = _mm256_or_si256(w, _mm256_or_si256(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('/')),
                                                   _mm256_cmpeq_epi8(v, _mm256_set1_epi8('-'))));
        m |= (uint64_t)bytes(w) << j;
    }
#endif
    for (; j < k; ++j) {
        const unsigned char c = (unsigned char)p[j], lc = c | 0x20;
        const bool w = (lc >= 'a' && lc <= 'z') || (c >= '0' && c <= '9') || c == '_' || (kSlashDash && (c == '/' || c == '-'));
        m |= (uint64_t)w << j;
    }
    *hi = 0;
    return m;
}

}  // namespace scan
