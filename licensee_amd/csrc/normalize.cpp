// Native host normalizer + interner: licensee's
// ContentHelper#content_normalized (lib/licensee/content_helper.rb:144-168, 219-321) and
// #wordset (:108-110), the LicenseFile decode (project_file.rb:37-45), the Copyright matcher
// (copyright.rb:12-17), the Exact matcher (exact.rb:6-12) and potential_false_positive?
// (license_file.rb:80-82), batched over host threads.
//
// The op sequence mirrors licensee_amd/content_helper.py one for one; the regular
// expressions themselves are handed over from that module's compiled patterns at lh_create
// time and run on rx (rx.h), so both host paths share a single pattern source.
// Texts containing characters whose Python case mapping or \b / \w semantics could differ
// from the ASCII rules implemented here (non-ASCII letters/digits) -- and HTML files -- are
// reported as status 1 and normalized by the Python path instead, as are texts whose match
// would nest deeper than the regex engine's frame limit (rx::TooDeep; e.g. thousands of
// consecutive copyright lines under the copyright pattern's repeated group).
#include <immintrin.h>
#include <malloc.h>
#include <cstdio>
#include <cstdlib>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "rx.h"
#include "scan.h"

using rx::Regex;
using rx::Str;
using rx::Str8;

// Per-pass timing (diagnostic builds only: -DLH_PASS_TIMING, tools/host_prep_passes.py). PASS
// wraps one step of the pipeline and adds its wall time to a per-thread table.
#ifdef LH_PASS_TIMING
#include <chrono>
#include <mutex>
namespace {
struct PassTable {
    std::vector<std::pair<const char*, double>> t;
    void add(const char* name, double s) {
        for (auto& e : t)
            if (e.first == name) { e.second += s; return; }
        t.emplace_back(name, s);
    }
};
std::mutex g_pass_mu;
PassTable g_pass_total;
thread_local PassTable tl_pass;
inline double pass_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void pass_flush() {
    std::lock_guard<std::mutex> g(g_pass_mu);
    for (auto& e : tl_pass.t) g_pass_total.add(e.first, e.second);
    tl_pass.t.clear();
}
}  // namespace
#define PASS(name, ...)                      \
    do {                                     \
        const double t0_ = pass_now();       \
        __VA_ARGS__;                         \
        tl_pass.add(name, pass_now() - t0_); \
    } while (0)
#else
#define PASS(name, ...) \
    do {                \
        __VA_ARGS__;    \
    } while (0)
#endif

namespace {

const char32_t kSpace = U' ';

// ASCII \w ([A-Za-z0-9_]) as a table
constexpr struct AsciiWord {
    uint8_t t[128];
    constexpr AsciiWord() : t() {
        for (int c = 0; c < 128; ++c)
            t[c] = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
    }
    constexpr uint8_t operator[](char32_t c) const { return t[c]; }
} kAsciiWord;

constexpr int kSpellSyms = 40;   // alphabet of the spelling keys + 1 (a-z, ' ', '-' in practice)

// spelling prefilter slot of a \w run: its first and last characters and its length (15 bits)
inline uint32_t spell_tok_slot(char32_t first, char32_t last, size_t len) {
    return (first & 31u) | (last & 31u) << 5 | (uint32_t)std::min<size_t>(len, 31) << 10;
}

bool is_strip_char(char32_t c) { return c == 0 || c == ' ' || (c >= '\t' && c <= '\r'); }

// Texts are normalized as UTF-32 (Str) or, when every character is ASCII, as bytes (Str8: the
// same passes over a quarter of the memory). cp: a text character as a code point; LIT: a
// literal in the text's character type.
inline char32_t cp(char32_t c) { return c; }
inline char32_t cp(char c) { return (unsigned char)c; }
template <class C>
constexpr const C* lit_of(const char* a, const char32_t* u) {
    if constexpr (sizeof(C) == 1) return a;
    else return u;
}
#define LIT(x) lit_of<C>(x, U##x)

template <class S>
S ruby_strip(const S& s) {
    size_t a = 0, b = s.size();
    while (a < b && is_strip_char(cp(s[a]))) ++a;
    while (b > a && is_strip_char(cp(s[b - 1]))) --b;
    return s.substr(a, b - a);
}

// Literal search: a vector scan for positions holding the literal's first and last characters,
// then a compare at each candidate (basic_string::find steps one character at a time).
template <class C>
size_t find_lit(const std::basic_string<C>& s, const C* lit, size_t from = 0) {
    const size_t m = std::char_traits<C>::length(lit), n = s.size();
    if (m == 0) return from <= n ? from : std::basic_string<C>::npos;
    if (n < m || from > n - m) return std::basic_string<C>::npos;
    const C* p = s.data();
    const char32_t c0 = cp(lit[0]), c1 = cp(lit[m - 1]);
    const size_t last = n - m;   // last candidate start
    for (size_t i = scan::find_pair(p, from, last, m - 1, c0, c0, c1, c1); i <= last;
         i = scan::find_pair(p, i + 1, last, m - 1, c0, c0, c1, c1))
        if (std::char_traits<C>::compare(p + i, lit, m) == 0) return i;
    return std::basic_string<C>::npos;
}

template <class C>
bool contains(const std::basic_string<C>& s, const C* lit) { return find_lit(s, lit) != std::basic_string<C>::npos; }

// non-ASCII code points whose Python semantics match the ASCII rules used here: no case
// mapping, not \w (str.isalnum() is False) -- punctuation, symbols, spaces, BOM.
bool safe_nonascii(char32_t c) {
    if (c >= 0xA0 && c <= 0xBF) return !(c == 0xAA || c == 0xB2 || c == 0xB3 || c == 0xB5 || c == 0xB9 || c == 0xBA ||
                                         (c >= 0xBC && c <= 0xBE));
    if (c == 0xD7 || c == 0xF7) return true;
    if (c >= 0x2000 && c <= 0x206F) return true;   // general punctuation
    if (c >= 0x20A0 && c <= 0x20CF) return true;   // currency
    if (c >= 0x2190 && c <= 0x22FF) return true;   // arrows, math operators
    if (c >= 0x2500 && c <= 0x25FF) return true;   // box drawing, blocks, shapes
    if (c == 0xFEFF || c == 0xFFFD || c == 0x3000) return true;
    return false;
}

// With the Unicode tables installed, the only texts left to the Python path are those with a
// character whose Python semantics are not a per-character table lookup: the letters re.I
// equates with ASCII ones (U+0130 İ, U+0131 ı, U+017F ſ, U+212A Kelvin K; U+0130 also lowers
// to two characters) and U+03A3 Σ (str.lower() applies the Final_Sigma context rule).
bool python_only(char32_t c) { return (c == 0x130) | (c == 0x131) | (c == 0x17F) | (c == 0x212A) | (c == 0x3A3); }

// Word keys for the wordset scan (content_helper.rb:109). Tokens are ASCII ([\w/-] with ASCII
// \w, and apostrophes), so a token's first 16 characters pack into two 64-bit words (one byte
// each); equal (lo, hi, len) is equality for tokens of <= 16 characters, longer ones also
// compare their tails. The hash mixes the packed words (and an FNV-1a of a long token's tail).
struct WordKey {
    uint64_t lo = 0, hi = 0, h = 0;
    uint32_t len = 0;
};

constexpr struct ByteMasks {
    uint64_t lo[17], hi[17];   // [min(len, 16)]: the packed bytes that belong to the token
    constexpr ByteMasks() : lo(), hi() {
        for (int l = 0; l <= 16; ++l) {
            lo[l] = l >= 8 ? ~0ull : (1ull << (8 * l)) - 1;
            hi[l] = l >= 16 ? ~0ull : l <= 8 ? 0 : (1ull << (8 * (l - 8))) - 1;
        }
    }
} kByteMasks;

inline uint64_t key_mix(uint64_t lo, uint64_t hi, uint64_t len, uint64_t tail) {
    // one multiply; its high half (well mixed) folded into the low bits the tables index by
    const uint64_t p = (lo ^ (hi * 0xC2B2AE3D27D4EB4FULL) ^ (len << 56) ^ tail) * 0x9E3779B97F4A7C15ULL;
    return p ^ (p >> 32);
}

template <class C>
inline uint64_t tail_hash(const C* p, size_t n) {   // FNV-1a over characters 16.. (long tokens)
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 16; i < n; ++i) {
        h ^= (uint64_t)(uint32_t)p[i];
        h *= 1099511628211ULL;
    }
    return h;
}

// key of p[0, n); `room` = characters readable from p (>= n): with >= 16 the packing reads a
// full 16-character window and masks it
inline WordKey word_key(const char32_t* p, size_t n, size_t room) {
    WordKey k;
    k.len = (uint32_t)n;
    const size_t m = n < 16 ? n : 16;
#if defined(__AVX2__)
    if (room >= 16) {
        const __m256i x = _mm256_packus_epi32(_mm256_loadu_si256((const __m256i*)p), _mm256_loadu_si256((const __m256i*)(p + 8)));
        const __m256i y = _mm256_permute4x64_epi64(x, 0xD8);
        const __m128i z = _mm_packus_epi16(_mm256_castsi256_si128(y), _mm256_extracti128_si256(y, 1));
        k.lo = (uint64_t)_mm_cvtsi128_si64(z) & kByteMasks.lo[m];
        k.hi = (uint64_t)_mm_extract_epi64(z, 1) & kByteMasks.hi[m];
    } else
#endif
    {
        (void)room;
        for (size_t i = 0; i < m; ++i) {
            const uint64_t b = (uint64_t)(p[i] < 255 ? p[i] : 255);
            if (i < 8) k.lo |= b << (8 * i);
            else k.hi |= b << (8 * (i - 8));
        }
    }
    k.h = key_mix(k.lo, k.hi, n, n > 16 ? tail_hash(p, n) : 0);
    return k;
}

inline WordKey word_key(const std::string& w) {
    WordKey k;
    const size_t n = w.size(), m = n < 16 ? n : 16;
    k.len = (uint32_t)n;
    for (size_t i = 0; i < m; ++i) {
        const uint64_t b = (unsigned char)w[i];
        if (i < 8) k.lo |= b << (8 * i);
        else k.hi |= b << (8 * (i - 8));
    }
    k.h = key_mix(k.lo, k.hi, n, n > 16 ? tail_hash(w.data(), n) : 0);
    return k;
}

// key of the ASCII bytes p[0, n) (the byte path; the same key as the code points')
inline WordKey word_key(const char* p, size_t n, size_t room) {
    WordKey k;
    k.len = (uint32_t)n;
    const size_t m = n < 16 ? n : 16;
    if (room >= 16) {
        memcpy(&k.lo, p, 8);
        memcpy(&k.hi, p + 8, 8);
        k.lo &= kByteMasks.lo[m];
        k.hi &= kByteMasks.hi[m];
    } else {
        for (size_t i = 0; i < m; ++i) {
            const uint64_t b = (unsigned char)p[i];
            if (i < 8) k.lo |= b << (8 * i);
            else k.hi |= b << (8 * (i - 8));
        }
    }
    k.h = key_mix(k.lo, k.hi, n, n > 16 ? tail_hash((const unsigned char*)p, n) : 0);
    return k;
}

template <class C>
inline bool tail_equal(const std::string& w, const C* p) {
    for (size_t i = 16; i < w.size(); ++i)
        if ((char32_t)(unsigned char)w[i] != cp(p[i])) return false;
    return true;
}

// The template vocabulary: buckets of 8 32-bit slots (id + 1 in the low id_bits, a hash tag
// above; 0 = empty), 32 KiB at the vendored corpus's 3.5k words so it stays in L1; a lookup
// compares a whole bucket's tags in one vector compare (almost every token is a hit, so there
// is no probe loop to mispredict), then the packed key of the one candidate (keys in id order);
// words kept for the tail compare of long words. A full bucket overflows into the next one.
struct VocabTable {
    struct Key {
        uint64_t lo, hi;
        uint32_t len;
    };
    static constexpr size_t kBucket = 8;
    std::vector<uint32_t> slot;   // [n_buckets][8], 32-byte aligned rows (see build)
    std::vector<Key> key;
    std::vector<std::string> words;
    size_t bmask = 0, base = 0;   // buckets - 1; first aligned slot in `slot`
    int id_bits = 1;
    uint32_t id_mask = 1;
    uint32_t tag(uint64_t h) const { return (uint32_t)(h >> 40) << id_bits; }
    const uint32_t* bucket(size_t b) const { return slot.data() + base + b * kBucket; }
    void build(int32_t n, const char* const* vocab) {
        size_t nb = 2;
        while (nb * kBucket < 2 * (size_t)n + 1) nb <<= 1;
        id_bits = 1;
        while (((uint64_t)1 << id_bits) <= (uint64_t)n + 1) ++id_bits;
        if (id_bits > 28) throw std::runtime_error("vocabulary too large for the host word table");
        id_mask = (1u << id_bits) - 1;
        slot.assign(nb * kBucket + kBucket, 0);
        base = (size_t)((32 - ((uintptr_t)slot.data() & 31)) & 31) / sizeof(uint32_t);
        bmask = nb - 1;
        key.resize((size_t)n);
        words.assign(vocab, vocab + n);
        for (int32_t i = 0; i < n; ++i) {
            const WordKey k = word_key(words[i]);
            key[(size_t)i] = Key{k.lo, k.hi, k.len};
            for (size_t b = k.h & bmask;; b = (b + 1) & bmask) {
                uint32_t* r = slot.data() + base + b * kBucket;
                size_t j = 0;
                while (j < kBucket && r[j]) ++j;
                if (j < kBucket) {
                    r[j] = tag(k.h) | (uint32_t)(i + 1);
                    break;
                }
            }
        }
    }
    template <class C>
    int32_t find(const WordKey& k, const C* p) const {
        if (key.empty()) return -1;
        const uint32_t t = tag(k.h);
        for (size_t b = k.h & bmask;; b = (b + 1) & bmask) {
            const uint32_t* r = bucket(b);
            uint32_t hit, empty;
#if defined(__AVX2__)
            const __m256i v = _mm256_loadu_si256((const __m256i*)r);   // aligned when the table was built in place
            hit = scan::lanes(_mm256_cmpeq_epi32(_mm256_and_si256(v, _mm256_set1_epi32((int)~id_mask)),
                                                 _mm256_set1_epi32((int)t)));
            empty = scan::lanes(_mm256_cmpeq_epi32(v, _mm256_setzero_si256()));
#else
            hit = empty = 0;
            for (size_t j = 0; j < kBucket; ++j) {
                hit |= (uint32_t)(r[j] && (r[j] & ~id_mask) == t) << j;
                empty |= (uint32_t)(r[j] == 0) << j;
            }
#endif
            hit &= ~empty;
            while (hit) {
                const int32_t id = (int32_t)(r[__builtin_ctz(hit)] & id_mask) - 1;
                const Key& e = key[(size_t)id];
                if (e.lo == k.lo && e.hi == k.hi && e.len == k.len && (k.len <= 16 || tail_equal(words[(size_t)id], p)))
                    return id;
                hit &= hit - 1;
            }
            if (empty) return -1;
        }
    }
};

// A file's distinct non-vocabulary words: open addressing over packed keys (start, len into
// the text for the tail compare), reused by a thread across files (an epoch stamp marks the
// live slots, so nothing is cleared per file); doubles when half full.
struct WordSet {
    struct Slot {
        uint64_t lo, hi;
        uint32_t start, len, epoch, hash;
    };
    std::vector<Slot> slot;
    uint32_t cur = 0;
    size_t count = 0, mask = 0;
    const char32_t* t32 = nullptr;   // the file's text (one of the two)
    const char* t8 = nullptr;
    template <class C>
    void reset(const C* text) {
        if constexpr (sizeof(C) == 1) t8 = text, t32 = nullptr;
        else t32 = text, t8 = nullptr;
        if (slot.empty()) slot.assign(1024, Slot{0, 0, 0, 0, 0, 0});
        mask = slot.size() - 1;
        if (++cur == 0) {   // epoch wrapped: clear once
            for (auto& e : slot) e.epoch = 0;
            cur = 1;
        }
        count = 0;
    }
    void grow() {
        std::vector<Slot> old;
        old.swap(slot);
        slot.assign(old.size() * 2, Slot{0, 0, 0, 0, 0, 0});
        mask = slot.size() - 1;
        for (const Slot& e : old) {
            if (e.epoch != cur) continue;
            size_t j = e.hash & mask;
            while (slot[j].epoch == cur) j = (j + 1) & mask;
            slot[j] = e;
        }
    }
    // true when the token [a, a + k.len) is a new word
    template <class C>
    bool insert(const C* text, size_t a, const WordKey& k) {
        for (size_t j = k.h & mask;; j = (j + 1) & mask) {
            Slot& s = slot[j];
            if (s.epoch != cur) {
                s = Slot{k.lo, k.hi, (uint32_t)a, k.len, cur, (uint32_t)k.h};
                if (2 * ++count > slot.size()) grow();
                return true;
            }
            if (s.lo == k.lo && s.hi == k.hi && s.len == k.len &&
                (k.len <= 16 || std::char_traits<C>::compare(text + s.start, text + a, k.len) == 0))
                return false;
        }
    }
    bool contains(const std::string& w) const {
        const WordKey k = word_key(w);
        for (size_t j = k.h & mask;; j = (j + 1) & mask) {
            const Slot& s = slot[j];
            if (s.epoch != cur) return false;
            if (s.lo == k.lo && s.hi == k.hi && s.len == k.len &&
                (k.len <= 16 || (t8 ? tail_equal(w, t8 + s.start) : tail_equal(w, t32 + s.start))))
                return true;
        }
    }
};

#ifndef LH_TEDDY_BYTES
#define LH_TEDDY_BYTES 4
#endif
constexpr int kTeddyBytes = LH_TEDDY_BYTES;   // key bytes in the spelling prefix fingerprint

struct Ctx {
    std::map<std::string, Regex> re;
    std::vector<std::pair<Str, Str>> spell;
    std::vector<Str8> spell_to8;   // the replacements as bytes (byte path; all ASCII when ascii_path)
    bool ascii_path = true;        // ASCII texts take the byte path
    // spelling keys as a trie over a small alphabet (spell_sym: ASCII -> 1..kSpellSyms-1, 0 = not
    // in any key); node 0 is the root, child 0 = none; spell_key: key index ending at a node
    uint8_t spell_sym[128] = {};
    std::vector<int32_t> spell_trie;
    std::vector<int32_t> spell_key;
    uint64_t spell_tok[(1u << 15) / 64] = {};   // spell_tok_slot of every key's first \w run
    // the keys by that slot (first in union order, then a chain), and each key's first eight
    // characters packed as bytes with the mask of those it has: a start's run may only match a
    // key whose slot and first characters it shares (checked before the trie walk)
    std::vector<int16_t> spell_tok_first = std::vector<int16_t>(1u << 15, -1);
    std::vector<int16_t> spell_tok_next;
    std::vector<uint64_t> spell_pre8, spell_pre8_mask;
    // byte path: the keys' first four bytes as a nibble fingerprint (spell_prefix_mask): 8
    // buckets; teddy[k][0|1][nibble] = the buckets with a key whose byte k has that low | high
    // nibble (16 entries repeated for both 128-bit lanes)
    alignas(32) uint8_t teddy[kTeddyBytes][2][32] = {};
    bool teddy_ok = true;
    // Unicode tables (lh_set_unicode): Python str.lower() of non-ASCII code points
    bool unicode = false;
    std::unordered_map<char32_t, char32_t> lower;
    std::vector<uint64_t> lower_bmp;   // BMP code points with an entry in `lower` (8 KiB)
    bool has_lower(char32_t ch) const {
        return ch >= 0x10000 || ((lower_bmp[ch >> 6] >> (ch & 63)) & 1);
    }
    VocabTable vocab;
    int32_t n_vocab = 0, w64 = 0;
    // templates (Exact)
    int32_t n_templates = 0;
    std::vector<uint64_t> lf_bits;                  // [T][w64]
    std::vector<uint32_t> full_size;                // |wordset|
    std::vector<std::vector<std::string>> fields;   // field words in the wordset
    std::vector<std::vector<int32_t>> field_ids;    // their vocabulary ids, or -1
    // field words outside the vocabulary, numbered in first-appearance order (bit k of a file's
    // field mask / a template's need mask; at most 64 are numbered)
    std::vector<std::string> nv_fields;
    std::vector<uint64_t> field_need;               // [T]
    std::string err;

    const Regex& R(const char* name) const { return re.at(name); }
};

template <class S>
struct Normalizer {
    using C = typename S::value_type;
    const Ctx& c;
    S cur;
    bool clean = false;   // cur is already squeezed and stripped (a strip op without a match is a no-op)

    // squeeze(' ').strip in place (String#squeeze / #strip: only ' ' runs, \0\t\n\v\f\r ends)
    void squeeze_strip() {
        C* p = cur.data();
        const size_t n = cur.size();
        const size_t r = scan::find_double_space(p, 0, n);   // nothing to squeeze before it
        if (r < n) cur.resize(scan::squeeze_runs(p, r, r, n, true, false));
        strip_ends();
    }
    void strip_ends() {
        size_t b = cur.size();
        while (b > 0 && is_strip_char(cp(cur[b - 1]))) --b;
        cur.resize(b);
        size_t a = 0;
        while (a < cur.size() && is_strip_char(cp(cur[a]))) ++a;
        if (a) cur.erase(0, a);
    }
    // strip(re): gsub(re, ' ').squeeze(' ').strip (content_helper.rb:223-236)
    void strip_re(const Regex& r) {
        if (!r.sub_into(cur, S(LIT(" "))) && clean) return;
        squeeze_strip();
        clean = true;
    }
    void sub_re(const Regex& r, const C* repl) {
        if (r.sub_into(cur, S(repl))) clean = false;
    }

    void strip_title() {
        const Regex& t = c.R("title");
        std::vector<long> caps;
        while (t.search(cur, 0, caps)) strip_re(t);
    }
    void strip_copyright() {
        const Regex& t = c.R("strip_copyright");
        std::vector<long> caps;
        while (t.search(cur, 0, caps)) strip_re(t);
    }
    // strip_comments (content_helper.rb:263-267): when every line of String#split("\n") (trailing
    // empty fields dropped) matches comment_markup ^[ \t\n\v\f\r]*?[/*]{1,2} -- on a line: its
    // first character outside [ \t\v\f\r] is '/' or '*' -- and there is not exactly one line
    static bool comment_line(const C* p, size_t a, size_t b) {
        while (a < b && (p[a] == ' ' || p[a] == '\t' || p[a] == '\v' || p[a] == '\f' || p[a] == '\r')) ++a;
        return a < b && (p[a] == '/' || p[a] == '*');
    }
    void strip_comments() {
        const C* p = cur.data();
        size_t end = cur.size();
        while (end > 0 && p[end - 1] == '\n') --end;   // trailing empty fields
        if (end > 0 && scan::find_char(p, 0, end, U'\n') == end) return;   // one line
        for (size_t a = 0; a < end;) {
            const size_t e = scan::find_char(p, a, end, U'\n');
            if (!comment_line(p, a, e)) return;
            a = e + 1;
        }
        strip_re(c.R("comment_markup"));
    }

    // hyphenated (content_helper.rb:40) can only match a '-' followed by [ \t\v\f\r]* and '\n'
    static bool has_hyphen_break(const S& s) {
        for (size_t i = scan::find_char(s.data(), 0, s.size(), U'-'); i < s.size();
             i = scan::find_char(s.data(), i + 1, s.size(), U'-')) {
            size_t j = i + 1;
            while (j < s.size() && (s[j] == ' ' || s[j] == '\t' || s[j] == '\v' || s[j] == '\f' || s[j] == '\r')) ++j;
            if (j < s.size() && s[j] == '\n') return true;
        }
        return false;
    }

    // normalize_spelling (content_helper.rb:314-316): /\b(?:k1|k2|...)\b/ with ordered
    // alternatives, tried only where \b can hold before a letter (a word start); text on this
    // path has ASCII word characters only, so \b is the ASCII boundary.
    void spelling() {
        const size_t n = cur.size();
        const C* p = cur.data();
        auto word = [](char32_t ch) {   // Python \b's \w
            return ch < 128 ? kAsciiWord[ch] != 0 : rx::is_word_char(ch);
        };
        // the key matching at word start i, or -1: the keys are walked in a trie and, of the
        // keys ending at a \b, the first in union order wins (Regexp.union alternation order)
        auto match_at = [&](size_t i, size_t& klen) -> int {
            int node = 0, best = -1;
            for (size_t j = i; j < n; ++j) {
                const char32_t cj = cp(p[j]);
                const int sym = cj < 128 ? c.spell_sym[cj] : 0;
                if (!sym) break;
                node = c.spell_trie[(size_t)node * kSpellSyms + sym];
                if (node <= 0) break;
                const int ki = c.spell_key[node];
                if (ki >= 0 && (best < 0 || ki < best) && (j + 1 == n || !word(cp(p[j + 1])))) {
                    best = ki;
                    klen = j + 1 - i;
                }
            }
            return best;
        };
        // Every key starts with a letter, so \b(?:key) matches only at a word start, and the
        // \w run starting there equals the key's first \w run (keys end in a letter, and \b
        // follows). Word starts come from 64-character \w masks; a start is tried only when
        // its run's (first, last, length) is that of some key's first run (spell_tok).
        S out;
        size_t copied = 0;   // cur[0, copied) is in out (or there is no match yet)
        uint64_t prev_word = 0;
        for (size_t b0 = 0; b0 < n; b0 += 64) {
            const size_t k = std::min<size_t>(64, n - b0);
            uint64_t hi;
            uint64_t w = scan::ascii_word_mask(p + b0, k, &hi);
            while (hi) {
                const int j = __builtin_ctzll(hi);
                hi &= hi - 1;
                if (rx::is_word_char(cp(p[b0 + (size_t)j]))) w |= 1ull << j;
            }
            uint64_t starts = w & ~((w << 1) | prev_word);
            prev_word = w >> 63;
#if defined(__AVX2__)
            if constexpr (sizeof(C) == 1) {
                if (c.teddy_ok && starts) starts &= spell_prefix_mask(p + b0, n - b0);
            } else if (c.teddy_ok && starts) {   // the characters narrowed to bytes (non-ASCII: 0xFF, in no key)
                alignas(32) char nar[64 + kTeddyBytes];
                const size_t m = std::min<size_t>(64 + kTeddyBytes - 1, n - b0);
                for (size_t j = 0; j < m; ++j) nar[j] = p[b0 + j] < 128 ? (char)p[b0 + j] : (char)0xFF;
                starts &= spell_prefix_mask(nar, m);
            }
#endif
            // (first, last, length) of every start's run, branch-free: a mask of the starts worth
            // a trie walk -- few -- instead of a mispredicted branch per start
            uint64_t hits = 0;
            for (uint64_t st = starts; st; st &= st - 1) {
                const unsigned off = (unsigned)__builtin_ctzll(st);
                const uint64_t rest = ~w >> off;
                const size_t len = rest ? (size_t)__builtin_ctzll(rest) : 1;
                const size_t s0 = b0 + off, e = std::min(s0 + len, n) - 1;
                hits |= (uint64_t)(rest == 0 || spell_tok_hit(cp(p[s0]), cp(p[e]), len)) << off;
            }
            starts = hits;   // (a run reaching past the block is checked below)
            while (starts) {
                const size_t off = (size_t)__builtin_ctzll(starts);
                starts &= starts - 1;
                const size_t s0 = b0 + off;
                if (s0 < copied) continue;
                const uint64_t rest = ~w >> off;   // bit 0 clear: p[s0] is a word character
                size_t len;
                if (rest) {
                    len = (size_t)__builtin_ctzll(rest);
                    if (s0 + len > n) len = n - s0;
                } else {
                    len = 64 - off;
                    while (s0 + len < n && word(cp(p[s0 + len]))) ++len;
                }
                if (!spell_tok_hit(cp(p[s0]), cp(p[s0 + len - 1]), len)) continue;
                if (!spell_pre_hit(p, s0, n, spell_tok_slot(cp(p[s0]), cp(p[s0 + len - 1]), len))) continue;
                size_t klen = 0;
                const int key = match_at(s0, klen);
                if (key < 0) continue;
                if (out.empty() && copied == 0) out.reserve(n + 16);
                out.append(cur, copied, s0 - copied);
                if constexpr (sizeof(C) == 1) out += c.spell_to8[(size_t)key];
                else out += c.spell[(size_t)key].second;
                copied = s0 + klen;
            }
        }
        if (copied == 0 && out.empty()) return;   // no varietal word: nothing to rebuild
        out.append(cur, copied, S::npos);
        cur.swap(out);
        clean = false;
    }
#if defined(__AVX2__)
    // Bit j: some key could start at q[j] -- its first four bytes pass the nibble fingerprint
    // (no false negatives; bytes past the text read as 0, which no key holds).
    uint64_t spell_prefix_mask(const char* q, size_t avail) const {
        alignas(32) char pad[96];
        if (avail < 64 + kTeddyBytes - 1) {
            memset(pad, 0, sizeof pad);
            memcpy(pad, q, avail);
            q = pad;
        }
        const __m256i nib = _mm256_set1_epi8(0x0f);
        uint64_t m = 0;
        for (int h = 0; h < 64; h += 32) {
            __m256i r = _mm256_set1_epi8(-1);
            for (int k = 0; k < kTeddyBytes; ++k) {
                const __m256i x = _mm256_loadu_si256((const __m256i*)(q + h + k));
                const __m256i lo = _mm256_shuffle_epi8(_mm256_load_si256((const __m256i*)c.teddy[k][0]), _mm256_and_si256(x, nib));
                const __m256i hi = _mm256_shuffle_epi8(_mm256_load_si256((const __m256i*)c.teddy[k][1]),
                                                       _mm256_and_si256(_mm256_srli_epi16(x, 4), nib));
                r = _mm256_and_si256(r, _mm256_and_si256(lo, hi));
            }
            m |= (uint64_t)(uint32_t)~_mm256_movemask_epi8(_mm256_cmpeq_epi8(r, _mm256_setzero_si256())) << h;
        }
        return m;
    }
#endif
    // some key with this first-run slot has the first (up to) eight characters at p[s0]
    bool spell_pre_hit(const C* p, size_t s0, size_t n, uint32_t slot) const {
        uint64_t x = 0;
        const size_t m = std::min<size_t>(8, n - s0);
        if constexpr (sizeof(C) == 1) {
            if (m == 8) memcpy(&x, p + s0, 8);
            else
                for (size_t j = 0; j < m; ++j) x |= (uint64_t)(unsigned char)p[s0 + j] << (8 * j);
        } else {
            for (size_t j = 0; j < m; ++j) x |= (uint64_t)(p[s0 + j] < 128 ? p[s0 + j] : 0xFF) << (8 * j);
        }
        for (int k = c.spell_tok_first[slot]; k >= 0; k = c.spell_tok_next[(size_t)k])
            if ((x & c.spell_pre8_mask[(size_t)k]) == c.spell_pre8[(size_t)k]) return true;
        return false;
    }
    bool spell_tok_hit(char32_t first, char32_t last, size_t len) const {
        const uint32_t h = spell_tok_slot(first, last, len);
        return (c.spell_tok[h >> 6] >> (h & 63)) & 1;
    }

    // Vector part of the downcase/quote pass: 8-character blocks of ASCII only are downcased,
    // '"' and '`' become '\'', and '&' are counted; stops at the first block holding a non-ASCII
    // character (ascii_done_: where the scalar loop continues).
    size_t ascii_done_ = 0;
    void downcase_quote_ascii(size_t& amps) {
        size_t i = 0;
#if defined(__AVX2__)
        if constexpr (sizeof(C) == 1) {   // the byte path: every block is ASCII
            char* p = cur.data();
            const size_t n = cur.size();
            const __m256i A1 = _mm256_set1_epi8('A' - 1), Z1 = _mm256_set1_epi8('Z' + 1), c32 = _mm256_set1_epi8(32);
            const __m256i dq = _mm256_set1_epi8('"'), bt = _mm256_set1_epi8('`'), sq = _mm256_set1_epi8('\'');
            const __m256i amp = _mm256_set1_epi8('&');
            for (; i + 32 <= n; i += 32) {
                __m256i v = _mm256_loadu_si256((const __m256i*)(p + i));
                const __m256i up = _mm256_and_si256(_mm256_cmpgt_epi8(v, A1), _mm256_cmpgt_epi8(Z1, v));
                v = _mm256_add_epi8(v, _mm256_and_si256(up, c32));
                v = _mm256_blendv_epi8(v, sq, _mm256_or_si256(_mm256_cmpeq_epi8(v, dq), _mm256_cmpeq_epi8(v, bt)));
                amps += (size_t)__builtin_popcount(scan::bytes(_mm256_cmpeq_epi8(v, amp)));
                _mm256_storeu_si256((__m256i*)(p + i), v);
            }
            ascii_done_ = i;
            return;
        } else {
        char32_t* p = cur.data();
        const size_t n = cur.size();
        const __m256i A1 = _mm256_set1_epi32('A' - 1), Z1 = _mm256_set1_epi32('Z' + 1), c32 = _mm256_set1_epi32(32);
        const __m256i dq = _mm256_set1_epi32('"'), bt = _mm256_set1_epi32('`'), sq = _mm256_set1_epi32('\'');
        const __m256i amp = _mm256_set1_epi32('&'), c127 = _mm256_set1_epi32(127);
        for (; i + 8 <= n; i += 8) {
            __m256i v = _mm256_loadu_si256((const __m256i*)(p + i));
            if (scan::lanes(_mm256_cmpgt_epi32(v, c127))) {   // a block with non-ASCII: one at a time
                for (size_t k = i; k < i + 8; ++k) downcase_one(cur[k], amps);
                continue;
            }
            const __m256i up = _mm256_and_si256(_mm256_cmpgt_epi32(v, A1), _mm256_cmpgt_epi32(Z1, v));
            v = _mm256_add_epi32(v, _mm256_and_si256(up, c32));
            v = _mm256_blendv_epi8(v, sq, _mm256_or_si256(_mm256_cmpeq_epi32(v, dq), _mm256_cmpeq_epi32(v, bt)));
            amps += (size_t)__builtin_popcount(scan::lanes(_mm256_cmpeq_epi32(v, amp)));
            _mm256_storeu_si256((__m256i*)(p + i), v);
        }
        }
#endif
        (void)amps;
        ascii_done_ = i;
    }

    // one character of the downcase/quote pass (content_helper.rb:34-41; Python str.lower())
    void downcase_one(C& ch, size_t& amps) const {
        if (cp(ch) < 128) {
            if (ch >= 'A' && ch <= 'Z') ch += 32;
            else if (ch == '"' || ch == '`') ch = '\'';
            else if (ch == '&') ++amps;
        } else if constexpr (sizeof(C) == 4) {
            if (ch == 0x2018 || ch == 0x2019 || ch == 0x201C || ch == 0x201D) {
                ch = '\'';
            } else if (c.unicode && c.has_lower(ch)) {
                auto it = c.lower.find(ch);
                if (it != c.lower.end()) ch = it->second;
            }
        }
    }

    // border_markup ^[*-](.*?)[*-]$ -> \1 (content_helper.rb:17, :98): '.' stops at '\n' and '$' holds
    // only before '\n' or at the end, so a match is a whole line of >= 2 characters that starts and
    // ends with '*' or '-', and the replacement drops those two characters. Line starts holding
    // '*' / '-' are found by a vector pair search; lines that match are then compacted in place.
    void strip_borders() {
        C* p = cur.data();
        const size_t n = cur.size();
        if (n < 2) return;
        auto border = [](C ch) { return ch == '*' || ch == '-'; };
        std::vector<std::pair<size_t, size_t>> lines;   // matching lines [a, e)
        auto check = [&](size_t a) {
            const size_t e = scan::find_char(p, a, n, U'\n');
            if (e - a >= 2 && border(p[e - 1])) lines.emplace_back(a, e);
            return e;
        };
        size_t from = 0;
        if (border(p[0])) from = check(0);
        while (from + 1 < n) {
            const size_t i = scan::find_pair(p, from, n - 2, 1, U'\n', U'\n', U'*', U'-');
            if (i > n - 2) break;
            from = check(i + 1);
        }
        if (lines.empty()) return;
        size_t w = lines[0].first;
        for (size_t j = 0; j < lines.size(); ++j) {
            const size_t a = lines[j].first, e = lines[j].second;
            const size_t next = j + 1 < lines.size() ? lines[j + 1].first : n;
            memmove(p + w, p + a + 1, (e - a - 2) * sizeof(C));   // the line without its borders
            w += e - a - 2;
            memmove(p + w, p + e, (next - e) * sizeof(C));        // '\n' and the lines up to the next match
            w += next - e;
        }
        cur.resize(w);
        clean = false;
    }

    // strip(:whitespace): gsub(/\s+/, ' ').squeeze(' ').strip, in place
    void collapse_whitespace() {
        cur.resize(scan::squeeze_runs(cur.data(), 0, 0, cur.size(), false, true));
        strip_ends();   // no ' ' runs are left, so squeeze(' ') is the identity: strip only
        clean = true;
    }

    // content_without_title_and_version + content_normalized (content_helper.rb:144-168)
    S run(const S& content) {
        PASS("strip", cur = ruby_strip(content));
        PASS("hrs", strip_re(c.R("hrs")));
        PASS("comments", strip_comments());
        PASS("markdown_headings", strip_re(c.R("markdown_headings")));
        // \[(.+?)\]\(.+?\) needs a literal "](": without one the lazy scans from every '[' are wasted
        PASS("link_markup", if (contains(cur, LIT("]("))) sub_re(c.R("link_markup"), LIT("\\1")));
        PASS("title", strip_title());
        PASS("version", strip_re(c.R("version")));
        // downcase, then (moved ahead of lists/https, with which they commute: neither pattern
        // reads '&' or a quote character other than as lists' copied [^\n]) '&' -> 'and' and the
        // quote characters -> "'" (content_helper.rb:34-41), one pass
        PASS("downcase_amp_quote", {
            size_t amps = 0;
            downcase_quote_ascii(amps);
            for (size_t i = ascii_done_; i < cur.size(); ++i) downcase_one(cur[i], amps);
            if (amps) {
                S out;
                out.reserve(cur.size() + 2 * amps);
                const C* p = cur.data();
                const size_t n = cur.size();
                for (size_t i = 0;;) {
                    const size_t e = scan::find_char(p, i, n, U'&');
                    out.append(p + i, e - i);
                    if (e == n) break;
                    out += LIT("and");
                    i = e + 1;
                }
                cur.swap(out);
            }
            clean = false;
        });
        PASS("lists", sub_re(c.R("lists"), LIT("- \\1")));
        // the literal 'http:' (content_helper.rb:35) without the regex engine
        PASS("https", {
            size_t at = find_lit(cur, LIT("http:"));
            if (at != S::npos) {
                S out;
                size_t i = 0;
                for (; at != S::npos; at = find_lit(cur, LIT("http:"), i)) {
                    out.append(cur, i, at - i);
                    out += LIT("https:");
                    i = at + 5;
                }
                out.append(cur, i, S::npos);
                cur.swap(out);
                clean = false;
            }
        });
        // (?<!^)([\u2014\u2013-]+)(?!$) -> '-' changes nothing unless a run holds an em/en dash or
        // two hyphens: skip the regex when the text has neither
        PASS("dashes", {
            static const char32_t kDash[2] = {0x2014, 0x2013};
            if (scan::find_any(cur.data(), 0, cur.size(), kDash, 2) < cur.size() || contains(cur, LIT("--")))
                sub_re(c.R("dashes"), LIT("-"));
        });
        PASS("hyphenated", if (has_hyphen_break(cur)) sub_re(c.R("hyphenated"), LIT("\\1-\\2")));
        PASS("spelling", spelling());
        PASS("span_markup", sub_re(c.R("span_markup"), LIT("\\1")));
        PASS("bullet", sub_re(c.R("bullet"), LIT("\n\n- ")));
        PASS("bullet_paren", sub_re(c.R("bullet_paren"), LIT(")(")));
        // STRIP_METHODS (content_helper.rb:89-105)
        PASS("bom", strip_re(c.R("bom")));
        // (cur is lower case here and re.I's non-ASCII folds to ASCII letters are outside the
        // native envelope, python_only: a match holds its literal words in lower case)
        PASS("cc_optional", if (contains(cur, LIT("creative commons"))) {
            PASS("=cc_dedication", if (contains(cur, LIT("dedication"))) strip_re(c.R("cc_dedication")));
            PASS("=cc_wiki", if (contains(cur, LIT("creativecommons"))) strip_re(c.R("cc_wiki")));
        });
        PASS("cc0_optional", if (contains(cur, LIT("associating cc0"))) {
            strip_re(c.R("cc_legal_code"));
            strip_re(c.R("cc0_info"));
            strip_re(c.R("cc0_disclaimer"));
        });
        PASS("unlicense_optional", if (contains(cur, LIT("unlicense"))) strip_re(c.R("unlicense_info")));
        PASS("borders", strip_borders());
        PASS("title2", strip_title());
        PASS("version2", strip_re(c.R("version")));
        PASS("url", strip_re(c.R("url")));
        PASS("copyright", strip_copyright());
        PASS("title3", strip_title());
        PASS("block_markup", strip_re(c.R("block_markup")));
        PASS("developed_by", strip_re(c.R("developed_by")));
        PASS("end_of_terms", {
            std::vector<long> caps;
            if (c.R("end_of_terms").search(cur, 0, caps)) {
                cur.resize((size_t)caps[0]);
                clean = false;
            }
        });
        PASS("whitespace", collapse_whitespace());
        PASS("mit_optional", strip_re(c.R("mit_optional")));
        return cur;
    }
};

#undef LIT

// wordset scan (content_helper.rb:109): (?:[\w/-](?:'s|(?<=s)')?)+ with ASCII \w
inline bool wchar(char32_t c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_' || c == '/' || c == '-';
}

// The regex's own loop from a token start: returns the token's end
template <class C>
inline size_t word_end(const C* s, size_t i, size_t n) {
    while (i < n && wchar(cp(s[i]))) {
        const C ch = s[i++];
        if (i < n && s[i] == '\'') {
            if (i + 1 < n && s[i + 1] == 's') i += 2;
            else if (ch == 's') i += 1;
        }
    }
    return i;
}

// Tokens are the runs of [\w/-] (64-character masks), except that a run followed by '\'' is
// re-scanned by the regex's loop ('s and s' continue a token; an apostrophe never starts one).
// Per 64-character block the run starts and the run ends (the non-word character after a run)
// come from the mask, and the k-th start pairs with the k-th end; a token whose run continues
// past the block stays open until the next block's first end. A re-scanned token that ends past
// its run consumed the starts and ends before its end (resume).
template <class C, class F>
void scan_words(const C* p, size_t n, F&& emit) {
    uint64_t prev = 0;
    size_t open = SIZE_MAX;   // start of a token whose run continues past the block
    size_t resume = 0;        // after a re-scan: tokens start at or after it
    uint64_t starts = 0, ends = 0;
    size_t b0 = 0;
    auto finish = [&](size_t a, size_t e) {
        if (__builtin_expect(e < n && p[e] == '\'', 0)) {
            const size_t e2 = word_end(p, a, n);
            if (e2 > e) {
                resume = e2;
                const size_t r = e2 - b0;
                starts = r >= 64 ? 0 : starts & (~0ULL << r);
                ends = r >= 63 ? 0 : ends & (~0ULL << (r + 1));   // a run end at e2 is the token's own
            }
            e = e2;
        }
        emit(a, e);
    };
    for (; b0 < n; b0 += 64) {
        uint64_t hi;
        const uint64_t w = scan::ascii_word_mask<true>(p + b0, std::min<size_t>(64, n - b0), &hi);
        const uint64_t wp = (w << 1) | prev;
        starts = w & ~wp;
        ends = ~w & wp;
        prev = w >> 63;
        if (__builtin_expect(resume >= b0, 0)) {
            const size_t r = resume - b0;
            if (r >= 64) continue;
            starts &= ~0ULL << r;
            ends &= r >= 63 ? 0 : ~0ULL << (r + 1);
        }
        if (open != SIZE_MAX) {
            if (!ends) continue;
            const size_t e = b0 + (size_t)__builtin_ctzll(ends);
            ends &= ends - 1;
            finish(open, e);
            open = SIZE_MAX;
        }
        while (starts) {
            const size_t a = b0 + (size_t)__builtin_ctzll(starts);
            starts &= starts - 1;
            if (!ends) {
                open = a;
                break;
            }
            const size_t e = b0 + (size_t)__builtin_ctzll(ends);
            ends &= ends - 1;
            finish(a, e);
        }
    }
    if (open != SIZE_MAX) emit(open, n);
}

bool extname_is_html(const char* fn) {
    if (!fn) return false;
    std::string base(fn);
    size_t sl = base.rfind('/');
    if (sl != std::string::npos) base = base.substr(sl + 1);
    size_t st = base.find_first_not_of('.');
    if (st == std::string::npos) return false;
    std::string rest = base.substr(st);
    size_t dot = rest.rfind('.');
    if (dot == std::string::npos) return false;
    std::string ext = rest.substr(dot);
    for (auto& ch : ext) ch = (char)tolower((unsigned char)ch);
    return ext.find(".htm") != std::string::npos;   // /\.html?/i.match?(extname)
}

struct FileOut {
    int status = 0;      // 0 ok, 1 needs the Python path, 2 error
    bool ascii = false;  // the byte path ran: the text is normalized8
    Str normalized;
    Str8 normalized8;
    bool cc = false, copyright = false;
};

void prep_one_impl(const Ctx& c, const char* data, int64_t len, const char* filename, bool is_file, FileOut& o);

thread_local WordSet tl_words;

// prep_one with the regex engine's depth abort mapped to "use the Python path"
void prep_one(const Ctx& c, const char* data, int64_t len, const char* filename, bool is_file, FileOut& o) {
    try {
        prep_one_impl(c, data, len, filename, is_file, o);
    } catch (const rx::TooDeep&) {
        o = FileOut();
        o.status = 1;
    }
}

// Batch workers run on threads with kWorkerStack bytes of stack (reserved virtual memory; only
// touched pages are committed) and a matching regex frame limit (~0.27 KiB per frame).
constexpr size_t kWorkerStack = size_t(256) << 20;
constexpr size_t kWorkerMatchDepth = 600000;
// files a worker takes at a time (a non-ASCII text costs ~4x an ASCII one: small grains keep the
// batch's tail short)
constexpr int64_t kGrain = 2;

template <class F>
void run_workers(int32_t nthreads, F& work) {
    struct Arg {
        F* fn;
    } arg{&work};
    auto entry = [](void* p) -> void* {
        rx::set_match_depth(kWorkerMatchDepth);
        (*static_cast<Arg*>(p)->fn)();
        return nullptr;
    };
    std::vector<pthread_t> th;
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, kWorkerStack);
    for (int32_t t = 0; t < nthreads; ++t) {
        pthread_t id;
        if (pthread_create(&id, &attr, entry, &arg) == 0) th.push_back(id);
    }
    pthread_attr_destroy(&attr);
    if (th.empty()) {   // no thread could be created: run here (default frame limit)
        work();
        return;
    }
    for (auto& id : th) pthread_join(id, nullptr);
}

// true when every byte of data[0, len) is ASCII
bool all_ascii(const char* data, size_t len) {
    size_t i = 0;
#if defined(__AVX2__)
    __m256i acc = _mm256_setzero_si256();
    for (; i + 32 <= len; i += 32) acc = _mm256_or_si256(acc, _mm256_loadu_si256((const __m256i*)(data + i)));
    if (_mm256_movemask_epi8(acc)) return false;
#endif
    for (; i < len; ++i)
        if ((unsigned char)data[i] >= 0x80) return false;
    return true;
}

// the byte path of prep_one_impl: an ASCII text (every character's Python semantics is the
// ASCII rule; decoding is the identity)
void prep_ascii(const Ctx& c, const char* data, int64_t len, bool is_file, FileOut& o) {
    Str8 content;
    const char* cr = is_file ? (const char*)memchr(data, '\r', (size_t)len) : nullptr;
    if (cr) {   // universal newline (project_file.rb:41); the bytes before the first CR as one copy
        content.resize((size_t)len);
        size_t w = (size_t)(cr - data);
        memcpy(&content[0], data, w);
        for (size_t i = w; i < (size_t)len; ++i) {
            if (data[i] == '\r') {
                content[w++] = '\n';
                if (i + 1 < (size_t)len && data[i + 1] == '\n') ++i;
            } else {
                content[w++] = data[i];
            }
        }
        content.resize(w);
    } else {
        content.assign(data, (size_t)len);
    }
    std::vector<long> caps;
    const Str8 stripped = ruby_strip(content);
    PASS("cc_flag", o.cc = c.R("cc_false_positive").search(stripped, 0, caps));
    PASS("copyright_matcher", o.copyright = c.R("copyright_match").search(stripped, 0, caps));
    Normalizer<Str8> nz{c, Str8()};
    PASS("=normalizer_run", o.normalized8 = nz.run(content));
    o.ascii = true;
}

void prep_one_impl(const Ctx& c, const char* data, int64_t len, const char* filename, bool is_file, FileOut& o) {
    if (extname_is_html(filename)) { o.status = 1; return; }
    if (c.ascii_path && all_ascii(data, (size_t)len)) {
        prep_ascii(c, data, len, is_file, o);
        return;
    }
    Str content;
    PASS("decode", content = rx::from_utf8(data, (size_t)len));
    if (is_file) {   // universal newline (project_file.rb:41), in place
        const size_t n = content.size();
        size_t w = 0;
        for (size_t i = 0; i < n; ++i) {
            if (content[i] == '\r') {
                content[w++] = '\n';
                if (i + 1 < n && content[i + 1] == '\n') ++i;
            } else {
                content[w++] = content[i];
            }
        }
        content.resize(w);
    }
    bool outside = false;
    PASS("=u_check", {
        if (c.unicode) {   // (no early exit: the loop vectorizes)
            uint32_t any = 0;
            for (char32_t ch : content) any |= (uint32_t)python_only(ch);
            outside = any != 0;
        } else {
            for (char32_t ch : content)
                if (ch >= 0x80 && !safe_nonascii(ch)) { outside = true; break; }
        }
    });
    if (outside) { o.status = 1; return; }
    std::vector<long> caps;
    Str stripped;
    PASS("=u_strip", stripped = ruby_strip(content));
    PASS("cc_flag", o.cc = c.R("cc_false_positive").search(stripped, 0, caps));
    PASS("copyright_matcher", o.copyright = c.R("copyright_match").search(stripped, 0, caps));
    Normalizer<Str> nz{c, Str()};
    PASS("=u_normalizer_run", o.normalized = nz.run(content));
}

}  // namespace

extern "C" {

typedef struct lh_ctx lh_ctx;

lh_ctx* lh_create(int32_t n_patterns, const char* const* names, const char* const* patterns, const int32_t* flags,
                  int32_t n_spell, const char* const* spell_from, const char* const* spell_to, int32_t n_vocab,
                  const char* const* vocab, char* err, int32_t errcap) {
    // every normalization pass allocates a text-sized buffer (~4 B/char, often near glibc's
    // 128 KiB mmap threshold): keep them in the per-thread arenas instead of mmap/munmap
    // churn, which serializes the batch threads on the kernel's mm lock.
    mallopt(M_MMAP_THRESHOLD, 64 << 20);
    mallopt(M_TRIM_THRESHOLD, 128 << 20);
    Ctx* c = new Ctx();
    try {
        for (int32_t i = 0; i < n_patterns; ++i) c->re.emplace(names[i], Regex(patterns[i], flags[i]));
        int nsym = 1;
        for (int32_t i = 0; i < n_spell; ++i) {
            c->spell.push_back({rx::from_utf8(spell_from[i]), rx::from_utf8(spell_to[i])});
            const Str& k = c->spell.back().first;
            if (k.empty() || k[0] >= 128 || !kAsciiWord[k[0]]) throw std::runtime_error("spelling keys: ASCII word start");
            for (char32_t ch : k) {
                if (ch >= 128) throw std::runtime_error("spelling keys: ASCII only");
                if (!c->spell_sym[ch]) c->spell_sym[ch] = (uint8_t)nsym++;
            }
        }
        if (nsym > kSpellSyms) throw std::runtime_error("spelling keys: alphabet too large");
        if (n_spell > 32767) throw std::runtime_error("spelling keys: too many");
        {   // the byte path's prefix fingerprint: distinct kTeddyBytes-byte prefixes, sorted, in 8 runs
            std::vector<Str> pre;
            for (const auto& kv : c->spell) {
                if (kv.first.size() < (size_t)kTeddyBytes) c->teddy_ok = false;
                else pre.push_back(kv.first.substr(0, kTeddyBytes));
            }
            std::sort(pre.begin(), pre.end());
            pre.erase(std::unique(pre.begin(), pre.end()), pre.end());
            for (size_t j = 0; j < pre.size(); ++j) {
                const uint8_t bit = (uint8_t)(1u << (j * 8 / pre.size()));
                for (int k = 0; k < kTeddyBytes; ++k) {
                    const uint32_t ch = (uint32_t)pre[j][(size_t)k];   // ASCII (checked above)
                    for (int lane = 0; lane < 32; lane += 16) {
                        c->teddy[k][0][lane + (ch & 15)] |= bit;
                        c->teddy[k][1][lane + (ch >> 4)] |= bit;
                    }
                }
            }
        }
        c->spell_trie.assign(kSpellSyms, 0);
        c->spell_key.assign(1, -1);
        for (int32_t i = 0; i < n_spell; ++i) {
            int node = 0;
            for (char32_t ch : c->spell[(size_t)i].first) {
                int32_t& next = c->spell_trie[(size_t)node * kSpellSyms + c->spell_sym[ch]];
                if (next == 0) {
                    next = (int32_t)c->spell_key.size();
                    c->spell_key.push_back(-1);
                    c->spell_trie.resize(c->spell_trie.size() + kSpellSyms, 0);
                }
                node = c->spell_trie[(size_t)node * kSpellSyms + c->spell_sym[ch]];
            }
            if (c->spell_key[(size_t)node] < 0) c->spell_key[(size_t)node] = i;   // first in union order
            const Str& k = c->spell[(size_t)i].first;
            size_t len = 0;
            while (len < k.size() && kAsciiWord[k[len]]) ++len;
            const uint32_t h = spell_tok_slot(k[0], k[len - 1], len);
            c->spell_tok[h >> 6] |= 1ull << (h & 63);
            c->spell_tok_next.push_back(-1);   // appended at the chain's end: union order
            int16_t* link = &c->spell_tok_first[h];
            while (*link >= 0) link = &c->spell_tok_next[(size_t)*link];
            *link = (int16_t)i;
            uint64_t pre = 0, mask = 0;
            for (size_t j = 0; j < k.size() && j < 8; ++j) {
                pre |= (uint64_t)(k[j] & 0x7F) << (8 * j);   // (ASCII, checked above)
                mask |= 0xFFull << (8 * j);
            }
            c->spell_pre8.push_back(pre);
            c->spell_pre8_mask.push_back(mask);
        }
        for (const auto& kv : c->spell) {
            Str8 to;
            for (char32_t ch : kv.second) {
                if (ch >= 128) c->ascii_path = false;   // a non-ASCII replacement: UTF-32 only
                to.push_back((char)ch);
            }
            c->spell_to8.push_back(to);
        }
        if (getenv("LH_NO_BYTE_PATH")) c->ascii_path = false;   // A/B and parity switch (tests)
        c->vocab.build(n_vocab, vocab);
        c->n_vocab = n_vocab;
        c->w64 = (n_vocab + 63) / 64;
        const char* need[] = {"hrs", "comment_markup", "markdown_headings", "link_markup", "title", "version",
                              "lists", "https", "dashes", "quote", "hyphenated", "spelling", "span_markup",
                              "bullet", "bullet_paren", "bom", "cc_dedication", "cc_wiki", "cc_legal_code",
                              "cc0_info", "cc0_disclaimer", "unlicense_info", "border_markup", "url",
                              "strip_copyright", "block_markup", "developed_by", "end_of_terms", "whitespace",
                              "mit_optional", "cc_false_positive", "copyright_match"};
        for (const char* nm : need)
            if (!c->re.count(nm)) throw std::runtime_error(std::string("missing pattern ") + nm);
    } catch (const std::exception& e) {
        if (err && errcap > 0) snprintf(err, (size_t)errcap, "%s", e.what());
        delete c;
        return nullptr;
    }
    return reinterpret_cast<lh_ctx*>(c);
}

void lh_destroy(lh_ctx* ctx) { delete reinterpret_cast<Ctx*>(ctx); }

// Exact matcher data: template Lf bitsets over the vocabulary, |wordset| and field words
// (Lf ∪ fields = wordset, content_helper.rb:323-335).
int lh_set_templates(lh_ctx* ctx, int32_t n_templates, const uint64_t* lf_bits, const uint32_t* wordset_size,
                     const int32_t* field_off, const char* const* field_words) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    c->n_templates = n_templates;
    c->lf_bits.assign(lf_bits, lf_bits + (size_t)n_templates * c->w64);
    c->full_size.assign(wordset_size, wordset_size + n_templates);
    c->fields.assign(n_templates, {});
    c->field_ids.assign(n_templates, {});
    c->nv_fields.clear();
    c->field_need.assign(n_templates, 0);
    for (int32_t t = 0; t < n_templates; ++t)
        for (int32_t k = field_off[t]; k < field_off[t + 1]; ++k) {
            c->fields[t].push_back(field_words[k]);
            // a field word can still be vocabulary (another template's word): then its presence is
            // the file's vocabulary bit, else the WordSet holds it
            const Str w = rx::from_utf8(field_words[k], strlen(field_words[k]));
            const int32_t id = c->vocab.find(word_key(w.data(), w.size(), w.size()), w.data());
            c->field_ids[t].push_back(id);
            if (id >= 0) continue;
            size_t j = 0;
            while (j < c->nv_fields.size() && c->nv_fields[j] != field_words[k]) ++j;
            if (j == c->nv_fields.size()) c->nv_fields.push_back(field_words[k]);
            if (j < 64) c->field_need[(size_t)t] |= 1ULL << j;
        }
    return 0;
}

int32_t lh_template_field_masks(lh_ctx* ctx, uint64_t* need) {
    const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
    if (!c || c->nv_fields.size() > 64) return -1;
    if (need) std::copy(c->field_need.begin(), c->field_need.end(), need);
    return (int32_t)c->nv_fields.size();
}

// Normalize one text. Returns UTF-8 byte count written to out (NUL-terminated when room),
// the needed size when cap is too small, -1 when the text needs the Python path.
int lh_set_unicode(lh_ctx* ctx, int32_t n_lower, const uint32_t* lower_from, const uint32_t* lower_to,
                   int32_t n_word, const uint32_t* word_lo, const uint32_t* word_hi) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || n_lower < 0 || n_word < 0 || (n_lower && (!lower_from || !lower_to)) || (n_word && (!word_lo || !word_hi)))
        return -1;
    for (int32_t i = 1; i < n_word; ++i)
        if (word_lo[i] <= word_hi[i - 1] || word_lo[i] > word_hi[i]) return -1;
    c->lower.clear();
    c->lower_bmp.assign(0x10000 / 64, 0);
    for (int32_t i = 0; i < n_lower; ++i) {
        c->lower.emplace(lower_from[i], lower_to[i]);
        if (lower_from[i] < 0x10000) c->lower_bmp[lower_from[i] >> 6] |= 1ull << (lower_from[i] & 63);
    }
    rx::set_unicode_word_ranges(word_lo, word_hi, n_word);
    c->unicode = true;
    return 0;
}

int64_t lh_normalize(lh_ctx* ctx, const char* data, int64_t len, const char* filename, int32_t is_file, char* out,
                     int64_t cap) {
    const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
    FileOut o;
    prep_one(*c, data, len, filename, is_file != 0, o);
    if (o.status) return -1;
    const std::string u = o.ascii ? o.normalized8 : rx::to_utf8(o.normalized);
    if (out && cap > (int64_t)u.size()) {
        memcpy(out, u.data(), u.size());
        out[u.size()] = 0;
    }
    return (int64_t)u.size();
}

// Batched content_normalized for the device wordset scan (liblicensee_dice dice_batch_upload_text):
// each file's normalized text as bytes, a non-ASCII character as the one byte 0x80 (the wordset's
// [\w/-] is ASCII, content_helper.rb:109, so any such byte only separates tokens), placed at a
// 16-byte aligned offset of `out` in completion order (a bump allocator over `cap` bytes).
int64_t lh_normalize_files(lh_ctx* ctx, int64_t n, const char* const* data, const int64_t* lens,
                           const char* const* filenames, int32_t nthreads, char* out, int64_t cap, int64_t* off,
                           int32_t* tlen, int32_t* length, uint8_t* cc, uint8_t* copyright, uint8_t* status) {
    const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
    if (n < 0 || cap < 0 || (n > 0 && (!data || !lens || !out || !off || !tlen || !length || !cc || !copyright || !status)))
        return -1;
    if (nthreads < 1) nthreads = 1;
    std::atomic<int64_t> next{0}, used{0};
    auto work = [&]() {
        for (;;) {
            const int64_t i = next.fetch_add(kGrain);
            if (i >= n) break;
            for (int64_t f = i; f < std::min<int64_t>(n, i + kGrain); ++f) {
                FileOut o;
                PASS("=prep_one", prep_one(*c, data[f], lens[f], filenames ? filenames[f] : nullptr, true, o));
                off[f] = -1;
                tlen[f] = 0;
                status[f] = (uint8_t)o.status;
                if (o.status) continue;
                const size_t sz = o.ascii ? o.normalized8.size() : o.normalized.size();
                length[f] = (int32_t)sz;   // characters (one byte per character in `out`)
                cc[f] = o.cc;
                copyright[f] = o.copyright;
                const int64_t need = (int64_t)((sz + 15) & ~(size_t)15);
                int64_t at = used.load(std::memory_order_relaxed);
                while (at + need <= cap && !used.compare_exchange_weak(at, at + need, std::memory_order_relaxed)) {
                }
                if (at + need > cap || sz > (size_t)INT32_MAX) {
                    status[f] = 3;   // no room: the caller retries the file with a larger buffer
                    continue;
                }
                char* dst = out + at;
                if (o.ascii) {
                    memcpy(dst, o.normalized8.data(), sz);
                } else {
                    for (size_t k = 0; k < sz; ++k) {
                        const char32_t ch = o.normalized[k];
                        dst[k] = ch < 0x80 ? (char)ch : (char)0x80;
                    }
                }
                off[f] = at;
                tlen[f] = (int32_t)sz;
            }
        }
#ifdef LH_PASS_TIMING
        pass_flush();
#endif
    };
    run_workers(nthreads, work);
    return used.load();
}

// Batched LicenseFile preparation: decode, normalize, wordset scan, intern to the vocabulary
// bitset, |W_F|, len_F, CC flag, Copyright and Exact matchers.
//   status[i]: 0 ok; 1 the caller must use the Python path for file i (its outputs unset).
//   exact[i]:  first template (key order) whose wordset equals the file's, or -1 (NULL: not
//              computed -- the device decides Exact from field_mask, dice_batch_exact);
//   field_mask[i] (NULL: not computed): bit k = the file's wordset holds the k-th field word
//              outside the vocabulary (lh_template_field_masks).
int lh_prep_files(lh_ctx* ctx, int64_t n, const char* const* data, const int64_t* lens, const char* const* filenames,
                  int32_t nthreads, uint64_t* bits, uint32_t* wf, int32_t* length, uint8_t* cc, uint8_t* copyright,
                  int32_t* exact, uint8_t* status, uint64_t* field_mask) {
    const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
    if (field_mask && c->nv_fields.size() > 64) return -1;
    if (nthreads < 1) nthreads = 1;
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        std::vector<uint64_t> row((size_t)c->w64);
        for (;;) {
            const int64_t i = next.fetch_add(kGrain);
            if (i >= n) break;
            for (int64_t f = i; f < std::min<int64_t>(n, i + kGrain); ++f) {
                FileOut o;
                prep_one(*c, data[f], lens[f], filenames ? filenames[f] : nullptr, true, o);
                status[f] = (uint8_t)o.status;
                if (o.status) continue;
                std::fill(row.begin(), row.end(), 0);
                // distinct words: vocabulary words are de-duplicated by their bit in `row`, the
                // others through the per-thread WordSet
                WordSet& words = tl_words;
                auto scan = [&](const auto* text, size_t len) {
                    words.reset(text);
                    scan_words(text, len, [&](size_t a, size_t b) {
                        const auto* p = text + a;
                        const WordKey k = word_key(p, b - a, len - a);
                        const int32_t id = c->vocab.find(k, p);
                        if (id >= 0) row[(size_t)id >> 6] |= 1ULL << (id & 63);
                        else words.insert(text, a, k);
                    });
                };
                PASS("wordset", {
                    if (o.ascii) scan(o.normalized8.data(), o.normalized8.size());
                    else scan(o.normalized.data(), o.normalized.size());
                });
                size_t n_vocab_words = 0;
                for (uint64_t wd : row) n_vocab_words += (size_t)__builtin_popcountll(wd);
                const size_t n_words = n_vocab_words + words.count;
                memcpy(bits + (size_t)f * c->w64, row.data(), sizeof(uint64_t) * (size_t)c->w64);
                wf[f] = (uint32_t)n_words;
                length[f] = (int32_t)(o.ascii ? o.normalized8.size() : o.normalized.size());
                cc[f] = o.cc;
                copyright[f] = o.copyright;
                if (field_mask) {
                    uint64_t m = 0;
                    for (size_t k = 0; k < c->nv_fields.size(); ++k)
                        if (words.contains(c->nv_fields[k])) m |= 1ULL << k;
                    field_mask[f] = m;
                }
                if (!exact) continue;
                int32_t ex = -1;
                PASS("exact", for (int32_t t = 0; t < c->n_templates && ex < 0; ++t) {
                    if (c->full_size[t] != n_words) continue;
                    const uint64_t* L = c->lf_bits.data() + (size_t)t * c->w64;
                    bool ok = true;
                    for (int32_t k = 0; k < c->w64 && ok; ++k) ok = (row[k] & L[k]) == L[k];
                    for (size_t k = 0; k < c->fields[t].size() && ok; ++k) {
                        const int32_t id = c->field_ids[t][k];
                        ok = id >= 0 ? (row[(size_t)id >> 6] >> (id & 63) & 1) != 0 : words.contains(c->fields[t][k]);
                    }
                    if (ok) ex = t;
                });
                exact[f] = ex;
            }
        }
#ifdef LH_PASS_TIMING
        pass_flush();
#endif
    };
    run_workers(nthreads, work);
    return 0;
}

#ifdef LH_PASS_TIMING
// Diagnostic builds: "name seconds\n" per pass, summed over every thread since the last call.
int64_t lh_pass_timing(char* buf, int64_t cap) {
    std::lock_guard<std::mutex> g(g_pass_mu);
    std::string out;
    for (auto& e : g_pass_total.t) out += std::string(e.first) + " " + std::to_string(e.second) + "\n";
    g_pass_total.t.clear();
    if (buf && cap > 0) snprintf(buf, (size_t)cap, "%s", out.c_str());
    return (int64_t)out.size();
}
#endif

}  // extern "C"
