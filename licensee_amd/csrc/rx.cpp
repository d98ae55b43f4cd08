// Backtracking regex engine for the Python `re` subset of licensee_amd/content_helper.py.
// See rx.h for the supported syntax. Semantics follow Python's sre: leftmost match,
// ordered alternation, greedy / lazy quantifiers with backtracking, fixed-width lookbehind.
#include "rx.h"

#include <algorithm>
#include <stdexcept>

#include "scan.h"

namespace rx {

// ---- UTF-8 ---------------------------------------------------------------------------
// UTF-8 -> code points with Python's errors='ignore' semantics: an invalid sequence's
// maximal valid prefix (at least one byte) is dropped (project_file.rb:38-40 replace: '').
Str from_utf8(const std::string& s) { return from_utf8(s.data(), s.size()); }

// UTF-8 -> code points; invalid sequences drop their maximal subpart (Ruby's
// String#scrub('') as project_file.rb:39 applies it). ASCII runs are widened without checks.
Str from_utf8(const char* data, size_t n) {
    Str out;
    out.resize(n);   // code points <= bytes
    char32_t* o = &out[0];
    size_t w = 0, i = 0;
    auto byte = [&](size_t k) { return (unsigned)(unsigned char)data[k]; };
    while (i < n) {
        const unsigned c = byte(i);
        if (c < 0x80) {
#if defined(__AVX2__)
            if (i + 16 <= n) {   // 16 ASCII bytes at once (w <= i, so w + 16 <= n)
                const __m128i b = _mm_loadu_si128((const __m128i*)(data + i));
                if (_mm_movemask_epi8(b) == 0) {
                    _mm256_storeu_si256((__m256i*)(o + w), _mm256_cvtepu8_epi32(b));
                    _mm256_storeu_si256((__m256i*)(o + w + 8), _mm256_cvtepu8_epi32(_mm_srli_si128(b, 8)));
                    w += 16;
                    i += 16;
                    continue;
                }
            }
#endif
            o[w++] = c;
            ++i;
            continue;
        }
        int need;
        unsigned lo = 0x80, hi = 0xBF;   // allowed range of the first continuation byte
        char32_t cp;
        if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
        else if (c == 0xE0) { need = 2; lo = 0xA0; cp = c & 0x0F; }
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) { need = 2; cp = c & 0x0F; }
        else if (c == 0xED) { need = 2; hi = 0x9F; cp = c & 0x0F; }
        else if (c == 0xF0) { need = 3; lo = 0x90; cp = c & 0x07; }
        else if (c >= 0xF1 && c <= 0xF3) { need = 3; cp = c & 0x07; }
        else if (c == 0xF4) { need = 3; hi = 0x8F; cp = c & 0x07; }
        else { ++i; continue; }
        size_t k = 1;
        bool ok = true;
        for (; k <= (size_t)need; ++k) {
            if (i + k >= n) { ok = false; break; }
            const unsigned bb = byte(i + k);
            const unsigned l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
            if (bb < l || bb > h) { ok = false; break; }
            cp = (cp << 6) | (bb & 0x3F);
        }
        if (!ok) { i += k; continue; }   // drop the maximal subpart
        o[w++] = cp;
        i += (size_t)need + 1;
    }
    out.resize(w);
    return out;
}

std::string to_utf8(const Str& s) {
    std::string out;
    out.reserve(s.size());
    for (char32_t c : s) {
        if (c < 0x80) out.push_back((char)c);
        else if (c < 0x800) { out.push_back((char)(0xC0 | (c >> 6))); out.push_back((char)(0x80 | (c & 0x3F))); }
        else if (c < 0x10000) {
            out.push_back((char)(0xE0 | (c >> 12)));
            out.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (c & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (c >> 18)));
            out.push_back((char)(0x80 | ((c >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (c & 0x3F)));
        }
    }
    return out;
}

static inline char32_t fold(char32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// Python's \w for \b: [A-Za-z0-9_] plus the non-ASCII code points with str.isalnum() True,
// installed as sorted inclusive ranges by set_unicode_word_ranges (none: ASCII only).
static std::vector<std::pair<char32_t, char32_t>> g_word_ranges;
static std::vector<uint64_t> g_word_bmp;   // the ranges over the BMP as a bitmap (8 KiB)

void set_unicode_word_ranges(const uint32_t* lo, const uint32_t* hi, int32_t n) {
    g_word_ranges.clear();
    g_word_bmp.assign(0x10000 / 64, 0);
    for (int32_t i = 0; i < n; ++i) {
        g_word_ranges.push_back({lo[i], hi[i]});
        for (uint32_t c = lo[i]; c <= hi[i] && c < 0x10000; ++c) g_word_bmp[c >> 6] |= 1ull << (c & 63);
    }
}

bool is_word_char(char32_t c) {
    if (c < 128) return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
    if (c < 0x10000 && !g_word_bmp.empty()) return (g_word_bmp[c >> 6] >> (c & 63)) & 1;
    size_t a = 0, b = g_word_ranges.size();   // first range with hi >= c
    while (a < b) {
        const size_t m = (a + b) / 2;
        if (g_word_ranges[m].second < c) a = m + 1;
        else b = m;
    }
    return a < g_word_ranges.size() && g_word_ranges[a].first <= c;
}

static inline bool is_word(char32_t c) { return is_word_char(c); }

// ---- parser ----------------------------------------------------------------------------
struct Parser {
    Str p;
    size_t i = 0;
    int ngroups = 0;

    [[noreturn]] void err(const char* m) { throw std::runtime_error(std::string("rx parse: ") + m); }
    bool eof() const { return i >= p.size(); }
    char32_t peek() const { return p[i]; }

    NodeP mk(Node::Kind k) { auto n = std::make_shared<Node>(); n->kind = k; return n; }

    char32_t hex(int n) {
        char32_t v = 0;
        for (int k = 0; k < n; ++k) {
            if (eof()) err("short hex escape");
            char32_t c = p[i++];
            v = v * 16 + (c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : (err("bad hex"), 0));
        }
        return v;
    }

    // an escaped literal character (inside or outside classes); -1 if it is a class/anchor
    long escape_char(char32_t c) {
        switch (c) {
            case 'n': return '\n';
            case 't': return '\t';
            case 'v': return '\v';
            case 'f': return '\f';
            case 'r': return '\r';
            case 'u': return (long)hex(4);
            case 'x': return (long)hex(2);
            default:
                if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9')) return -1;
                return (long)c;
        }
    }

    NodeP parse_alt(bool icase, bool dotall) {
        auto alt = mk(Node::ALT);
        alt->kids.push_back(parse_seq(icase, dotall));
        while (!eof() && peek() == '|') {
            ++i;
            alt->kids.push_back(parse_seq(icase, dotall));
        }
        return alt->kids.size() == 1 ? alt->kids[0] : alt;
    }

    NodeP parse_seq(bool icase, bool dotall) {
        auto seq = mk(Node::SEQ);
        while (!eof() && peek() != '|' && peek() != ')') {
            NodeP a = parse_atom(icase, dotall);
            if (!a) continue;
            seq->kids.push_back(parse_quant(a));
        }
        return seq;
    }

    NodeP parse_quant(NodeP a) {
        while (!eof()) {
            int mn, mx;
            char32_t c = peek();
            if (c == '*') { mn = 0; mx = -1; ++i; }
            else if (c == '+') { mn = 1; mx = -1; ++i; }
            else if (c == '?') { mn = 0; mx = 1; ++i; }
            else if (c == '{') {
                size_t save = i++;
                auto num = [&](int& out) { bool any = false; out = 0; while (!eof() && peek() >= '0' && peek() <= '9') { out = out * 10 + (int)(peek() - '0'); ++i; any = true; } return any; };
                int a1 = 0, a2 = 0;
                bool h1 = num(a1);
                if (!eof() && peek() == '}') { ++i; if (!h1) { i = save; return a; } mn = mx = a1; }
                else if (!eof() && peek() == ',') {
                    ++i;
                    bool h2 = num(a2);
                    if (eof() || peek() != '}') { i = save; return a; }
                    ++i;
                    mn = h1 ? a1 : 0;
                    mx = h2 ? a2 : -1;
                } else { i = save; return a; }
            } else break;
            auto r = mk(Node::REPEAT);
            r->min = mn; r->max = mx;
            if (!eof() && peek() == '?') { r->lazy = true; ++i; }
            r->kids.push_back(a);
            a = r;
        }
        return a;
    }

    NodeP parse_class(bool icase) {
        auto c = mk(Node::CLASS);
        c->icase = icase;
        if (!eof() && peek() == '^') { c->negate = true; ++i; }
        bool first = true;
        while (!eof() && (peek() != ']' || first)) {
            first = false;
            char32_t lo = p[i++];
            if (lo == '\\') {
                if (eof()) err("bad class escape");
                long e = escape_char(p[i++]);
                if (e < 0) err("unsupported class escape");
                lo = (char32_t)e;
            }
            char32_t hi = lo;
            if (i + 1 < p.size() && peek() == '-' && p[i + 1] != ']') {
                ++i;
                hi = p[i++];
                if (hi == '\\') {
                    long e = escape_char(p[i++]);
                    if (e < 0) err("unsupported class escape");
                    hi = (char32_t)e;
                }
            }
            c->ranges.push_back({lo, hi});
        }
        if (eof()) err("unterminated class");
        ++i;
        return c;
    }

    NodeP parse_atom(bool icase, bool dotall) {
        char32_t c = p[i++];
        switch (c) {
            case '.': { auto n = mk(Node::ANY); n->dotall = dotall; return n; }
            case '^': return mk(Node::BOL);
            case '$': return mk(Node::EOL);
            case '[': return parse_class(icase);
            case '(': {
                if (!eof() && peek() == '?') {
                    ++i;
                    if (eof()) err("bad group");
                    char32_t k = p[i];
                    if (k == ':') { ++i; auto g = mk(Node::GROUP); g->kids.push_back(parse_alt(icase, dotall)); close(); return g; }
                    if (k == '=' || k == '!') {
                        ++i;
                        auto l = mk(Node::LOOK); l->negate = k == '!';
                        l->kids.push_back(parse_alt(icase, dotall)); close(); return l;
                    }
                    if (k == '<' && i + 1 < p.size() && (p[i + 1] == '=' || p[i + 1] == '!')) {
                        auto l = mk(Node::LOOK); l->behind = true; l->negate = p[i + 1] == '!';
                        i += 2;
                        l->kids.push_back(parse_alt(icase, dotall)); close();
                        l->width = width(l->kids[0]);
                        if (l->width < 0) err("lookbehind requires fixed width");
                        return l;
                    }
                    // scoped flags (?i:...) (?-i:...) (?s:...)
                    bool on = true, ic = icase, da = dotall;
                    while (!eof() && peek() != ':') {
                        char32_t f = p[i++];
                        if (f == '-') on = false;
                        else if (f == 'i') ic = on;
                        else if (f == 's') da = on;
                        else if (f == 'm' || f == 'x' || f == 'u') {}
                        else err("unsupported flag");
                    }
                    if (eof()) err("bad flags group");
                    ++i;
                    auto g = mk(Node::GROUP); g->kids.push_back(parse_alt(ic, da)); close(); return g;
                }
                auto g = mk(Node::GROUP);
                g->group = ++ngroups;
                g->kids.push_back(parse_alt(icase, dotall));
                close();
                return g;
            }
            case '\\': {
                if (eof()) err("trailing backslash");
                char32_t e = p[i++];
                if (e == 'A') return mk(Node::BOS);
                if (e == 'Z') return mk(Node::EOS);
                if (e == 'b') return mk(Node::WORDB);
                long v = escape_char(e);
                if (v < 0) err("unsupported escape");
                auto n = mk(Node::LIT); n->ch = (char32_t)v; n->icase = icase; return n;
            }
            default: { auto n = mk(Node::LIT); n->ch = c; n->icase = icase; return n; }
        }
    }

    void close() { if (eof() || peek() != ')') err("missing )"); ++i; }

    static int width(const NodeP& n) {
        switch (n->kind) {
            case Node::LIT: case Node::ANY: case Node::CLASS: return 1;
            case Node::BOL: case Node::EOL: case Node::BOS: case Node::EOS: case Node::WORDB: case Node::LOOK: return 0;
            case Node::SEQ: { int w = 0; for (auto& k : n->kids) { int x = width(k); if (x < 0) return -1; w += x; } return w; }
            case Node::ALT: { int w = -2; for (auto& k : n->kids) { int x = width(k); if (x < 0 || (w != -2 && x != w)) return -1; w = x; } return w < 0 ? 0 : w; }
            case Node::GROUP: return width(n->kids[0]);
            case Node::REPEAT: { if (n->min != n->max) return -1; int x = width(n->kids[0]); return x < 0 ? -1 : x * n->min; }
        }
        return -1;
    }
};

// ---- matcher (continuation passing over the node tree) -------------------------------
struct Cont {
    virtual bool operator()(size_t pos) const = 0;
};

namespace {
// Node frames per match: measured ~0.27 KiB of stack per frame (gcc -O3) (m -> seq/rep -> continuation),
// so the default (main thread and other callers' threads, 8 MiB stacks) keeps well inside
// 8 MiB; normalize.cpp raises it on its large-stack worker threads.
constexpr size_t kDefaultMatchDepth = 12000;
thread_local size_t tl_match_depth = kDefaultMatchDepth;
}  // namespace

size_t max_match_depth() { return tl_match_depth; }
void set_match_depth(size_t frames) { tl_match_depth = frames ? frames : kDefaultMatchDepth; }

// text character i as a code point (a byte-path text is ASCII)
static inline char32_t at(const char32_t* p, size_t i) { return p[i]; }
static inline char32_t at(const char* p, size_t i) { return (unsigned char)p[i]; }

template <class Ch>
struct Matcher {
    const Ch* s;
    size_t len;
    std::vector<long>& caps;
    // Continuation-passing backtracking nests one set of frames per matched node: a repeated
    // group such as the copyright pattern's (MAIN_LINE OPT*)+ goes deeper with every line it
    // matches. Past max_match_depth() the match aborts with TooDeep (the caller sends the text
    // to the Python path) instead of overflowing the thread's stack.
    size_t depth = 0;
    const size_t limit = max_match_depth();
    struct Guard {
        size_t& d;
        explicit Guard(size_t& dd, size_t lim) : d(dd) {
            if (++d > lim) {
                --d;
                throw TooDeep();
            }
        }
        ~Guard() { --d; }
    };

    bool lit(const Node* n, size_t pos) const {
        if (pos >= len) return false;
        char32_t c = at(s, pos);
        return n->icase ? fold(c) == fold(n->ch) : c == n->ch;
    }
    bool cls(const Node* n, size_t pos) const {
        if (pos >= len) return false;
        char32_t c = at(s, pos);
        bool in = false;
        for (auto& r : n->ranges) {
            if (c >= r.first && c <= r.second) { in = true; break; }
            if (n->icase) {
                char32_t f = fold(c), u = (c >= 'a' && c <= 'z') ? c - 32 : c;
                if ((f >= r.first && f <= r.second) || (u >= r.first && u <= r.second)) { in = true; break; }
            }
        }
        return in != n->negate;
    }

    // match node n at pos, then continuation k
    bool m(const Node* n, size_t pos, const Cont& k) {
        const Guard g(depth, limit);
        switch (n->kind) {
            case Node::LIT: return lit(n, pos) && k(pos + 1);
            case Node::ANY: return pos < len && (n->dotall || at(s, pos) != '\n') && k(pos + 1);
            case Node::CLASS: return cls(n, pos) && k(pos + 1);
            case Node::BOL: return (pos == 0 || at(s, pos - 1) == '\n') && k(pos);
            case Node::EOL: return (pos == len || at(s, pos) == '\n') && k(pos);
            case Node::BOS: return pos == 0 && k(pos);
            case Node::EOS: return pos == len && k(pos);
            case Node::WORDB: {
                bool a = pos > 0 && is_word(at(s, pos - 1)), b = pos < len && is_word(at(s, pos));
                return a != b && k(pos);
            }
            case Node::SEQ: return seq(n, 0, pos, k);
            case Node::ALT: {
                // branches that cannot start with at(s, pos) are skipped (first-character masks)
                const char32_t c = pos < len ? at(s, pos) : 0;
                const bool end = pos >= len;
                for (size_t i = 0; i < n->kids.size(); ++i) {
                    if (!n->alt_nullable[i]) {
                        if (end) continue;
                        if (c < 128 ? !(n->alt_first[2 * i + (c >> 6)] >> (c & 63) & 1) : !n->alt_nonascii[i]) continue;
                    }
                    if (m(n->kids[i].get(), pos, k)) return true;
                }
                return false;
            }
            case Node::GROUP: {
                if (n->group < 0) return m(n->kids[0].get(), pos, k);
                const long o0 = caps[2 * n->group], o1 = caps[2 * n->group + 1];
                struct C : Cont {
                    Matcher* self; const Node* n; size_t start; const Cont* k;
                    bool operator()(size_t e) const override {
                        const long p0 = self->caps[2 * n->group], p1 = self->caps[2 * n->group + 1];
                        self->caps[2 * n->group] = (long)start;
                        self->caps[2 * n->group + 1] = (long)e;
                        if ((*k)(e)) return true;
                        self->caps[2 * n->group] = p0;
                        self->caps[2 * n->group + 1] = p1;
                        return false;
                    }
                } c;
                c.self = this; c.n = n; c.start = pos; c.k = &k;
                if (m(n->kids[0].get(), pos, c)) return true;
                caps[2 * n->group] = o0; caps[2 * n->group + 1] = o1;
                return false;
            }
            case Node::REPEAT: return rep(n, 0, pos, (size_t)-1, k);
            case Node::LOOK: {
                bool ok;
                struct Acc : Cont { size_t want; bool any; bool operator()(size_t e) const override { return any || e == want; } } acc;
                std::vector<long> save(caps);
                if (n->behind) {
                    if (pos < (size_t)n->width) ok = false;
                    else { acc.want = pos; acc.any = false; ok = m(n->kids[0].get(), pos - n->width, acc); }
                } else {
                    acc.any = true; ok = m(n->kids[0].get(), pos, acc);
                }
                if (n->negate) { caps = save; return !ok && k(pos); }
                if (!ok) { caps = save; return false; }
                return k(pos);
            }
        }
        return false;
    }

    bool seq(const Node* n, size_t idx, size_t pos, const Cont& k) {
        if (idx == n->kids.size()) return k(pos);
        struct C : Cont {
            Matcher* self; const Node* n; size_t idx; const Cont* k;
            bool operator()(size_t p) const override { return self->seq(n, idx + 1, p, *k); }
        } c;
        c.self = this; c.n = n; c.idx = idx; c.k = &k;
        return m(n->kids[idx].get(), pos, c);
    }

    bool single(const Node* n, size_t pos) const {
        switch (n->kind) {
            case Node::LIT: return lit(n, pos);
            case Node::ANY: return pos < len && (n->dotall || at(s, pos) != '\n');
            case Node::CLASS: return cls(n, pos);
            default: return false;
        }
    }

    bool rep(const Node* n, int count, size_t pos, size_t last, const Cont& k) {
        const Node* kid = n->kids[0].get();
        if (count == 0 && (kid->kind == Node::LIT || kid->kind == Node::ANY || kid->kind == Node::CLASS)) {
            // one character per iteration: iterate instead of recursing per character
            size_t run = 0;
            const size_t cap = n->max < 0 ? (size_t)-1 : (size_t)n->max;
            if (n->lazy) {
                while (run < (size_t)n->min) { if (!single(kid, pos + run)) return false; ++run; }
                for (;;) {
                    if (k(pos + run)) return true;
                    if (run >= cap || !single(kid, pos + run)) return false;
                    ++run;
                }
            }
            while (run < cap && single(kid, pos + run)) ++run;
            if (run < (size_t)n->min) return false;
            for (size_t r = run + 1; r-- > (size_t)n->min;)
                if (k(pos + r)) return true;
            return false;
        }
        const bool can_more = n->max < 0 || count < n->max;
        const bool can_stop = count >= n->min;
        struct C : Cont {
            Matcher* self; const Node* n; int count; size_t start; const Cont* k;
            bool operator()(size_t p) const override {
                if (p == start && count >= n->min) return false;   // empty iteration: stop looping
                return self->rep(n, count + 1, p, start, *k);
            }
        } c;
        c.self = this; c.n = n; c.count = count; c.start = pos; c.k = &k;
        (void)last;
        if (n->lazy) {
            if (can_stop && k(pos)) return true;
            return can_more && m(kid, pos, c);
        }
        if (can_more && m(kid, pos, c)) return true;
        return can_stop && k(pos);
    }
};

static void first_chars(const NodeP& n, std::vector<bool>& set, bool& nonascii, bool& nullable) {
    // conservative first-character set of n (ASCII bitmap); nullable = may match empty
    switch (n->kind) {
        case Node::LIT:
            if (n->ch < 128) { set[n->ch] = true; if (n->icase) { set[fold(n->ch)] = true; if (n->ch >= 'a' && n->ch <= 'z') set[n->ch - 32] = true; } }
            else nonascii = true;
            nullable = false; return;
        case Node::ANY: for (int c = 0; c < 128; ++c) set[c] = true; nonascii = true; nullable = false; return;
        case Node::CLASS:
            if (n->negate) { for (int c = 0; c < 128; ++c) set[c] = true; nonascii = true; nullable = false; return; }
            for (auto& r : n->ranges) {
                for (char32_t c = r.first; c <= r.second && c < 128; ++c) {
                    set[c] = true;
                    if (n->icase) { set[fold(c)] = true; if (c >= 'a' && c <= 'z') set[c - 32] = true; }
                }
                if (r.second >= 128) nonascii = true;
            }
            nullable = false; return;
        case Node::SEQ: {
            for (auto& k : n->kids) {
                bool nl = false;
                first_chars(k, set, nonascii, nl);
                if (!nl) { nullable = false; return; }
            }
            nullable = true; return;
        }
        case Node::ALT: {
            bool any = false;
            for (auto& k : n->kids) { bool nl = false; first_chars(k, set, nonascii, nl); any |= nl; }
            nullable = any; return;
        }
        case Node::GROUP: first_chars(n->kids[0], set, nonascii, nullable); return;
        case Node::REPEAT: { bool nl = false; first_chars(n->kids[0], set, nonascii, nl); nullable = nl || n->min == 0; return; }
        default: nullable = true; return;   // anchors / lookarounds are zero-width
    }
}

// Fill every ALT node's per-branch first-character masks (Node::alt_first).
static void index_alternations(const NodeP& n) {
    for (auto& k : n->kids) index_alternations(k);
    if (n->kind != Node::ALT) return;
    const size_t nb = n->kids.size();
    n->alt_first.assign(2 * nb, 0);
    n->alt_nonascii.assign(nb, 0);
    n->alt_nullable.assign(nb, 0);
    for (size_t i = 0; i < nb; ++i) {
        std::vector<bool> set(128, false);
        bool nonascii = false, nullable = false;
        first_chars(n->kids[i], set, nonascii, nullable);
        for (int c = 0; c < 128; ++c)
            if (set[c]) n->alt_first[2 * i + (c >> 6)] |= 1ull << (c & 63);
        n->alt_nonascii[i] = nonascii;
        n->alt_nullable[i] = nullable;
    }
}

// The exact set of code points a match of n can start with, when it has at most kMaxFirst
// members (false otherwise, or when n can match empty: nullable).
static constexpr size_t kMaxFirst = 8;
static bool first_list(const NodeP& n, std::vector<char32_t>& out, bool& nullable) {
    auto add = [&](char32_t c, bool icase) {
        out.push_back(c);
        if (icase && c < 128) {   // fold() is ASCII-only: a letter matches its two cases
            out.push_back(fold(c));
            if (c >= 'a' && c <= 'z') out.push_back(c - 32);
        }
    };
    switch (n->kind) {
        case Node::LIT: add(n->ch, n->icase); nullable = false; break;
        case Node::ANY: return false;
        case Node::CLASS:
            if (n->negate) return false;
            for (auto& r : n->ranges) {
                if (r.second - r.first >= kMaxFirst) return false;
                for (char32_t c = r.first; c <= r.second; ++c) add(c, n->icase);
            }
            nullable = false;
            break;
        case Node::SEQ:
            nullable = true;
            for (auto& k : n->kids) {
                bool nl = false;
                if (!first_list(k, out, nl)) return false;
                if (!nl) { nullable = false; break; }
            }
            break;
        case Node::ALT:
            nullable = false;
            for (auto& k : n->kids) {
                bool nl = false;
                if (!first_list(k, out, nl)) return false;
                nullable |= nl;
            }
            break;
        case Node::GROUP: return first_list(n->kids[0], out, nullable);
        case Node::REPEAT: {
            bool nl = false;
            if (!first_list(n->kids[0], out, nl)) return false;
            nullable = nl || n->min == 0;
            break;
        }
        default: nullable = true; break;   // anchors / lookarounds are zero-width
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out.size() <= kMaxFirst;
}

// The longest run of consecutive literals on n's mandatory path (a sequence whose items every
// match consumes in order: literals, groups of them, the first iteration of a repetition with
// min >= 1); alternations and lookarounds end a run. Every match contains such a run, so a
// search whose text lacks it from the start position on cannot match.
struct LitRun {
    Str s;
    bool icase = false;
};
static void required_runs(const Node* n, LitRun& cur, LitRun& best) {
    auto flush = [&]() {
        if (cur.s.size() > best.s.size()) best = cur;
        cur = LitRun();
    };
    switch (n->kind) {
        case Node::LIT:
            if (!cur.s.empty() && cur.icase != n->icase) flush();
            cur.icase = n->icase;
            cur.s.push_back(n->icase ? fold(n->ch) : n->ch);
            return;
        case Node::SEQ:
            for (auto& k : n->kids) required_runs(k.get(), cur, best);
            return;
        case Node::GROUP:
            required_runs(n->kids[0].get(), cur, best);
            return;
        case Node::REPEAT:
            if (n->min >= 1) {   // the first iteration is mandatory; what follows it is not contiguous
                flush();
                required_runs(n->kids[0].get(), cur, best);
            }
            flush();
            return;
        case Node::BOL: case Node::EOL: case Node::BOS: case Node::EOS: case Node::WORDB:
            return;   // zero-width: literals on both sides stay adjacent
        default:      // ANY, CLASS, ALT, LOOK: the run ends here
            flush();
            return;
    }
}

// The literal run every match of n begins with: its literals from the start of its mandatory
// path (zero-width anchors between them skipped) up to the first other node. False once the run
// has ended.
static bool leading_run(const Node* n, LitRun& run) {
    switch (n->kind) {
        case Node::LIT:
            if (!run.s.empty() && run.icase != n->icase) return false;
            run.icase = n->icase;
            run.s.push_back(n->icase ? fold(n->ch) : n->ch);
            return true;
        case Node::SEQ:
            for (auto& k : n->kids)
                if (!leading_run(k.get(), run)) return false;
            return true;
        case Node::GROUP:
            return leading_run(n->kids[0].get(), run);
        case Node::REPEAT:   // the first iteration is mandatory; what follows it may differ
            if (n->min >= 1) leading_run(n->kids[0].get(), run);
            return false;
        case Node::BOL: case Node::EOL: case Node::BOS: case Node::EOS: case Node::WORDB:
            return true;
        default:
            return false;
    }
}

// first position >= from where req occurs (ASCII case folded when icase), or npos: candidates
// by a vector scan for the literal's first and last characters (both cases when folded)
template <class C>
static size_t find_required(const C* p, size_t n, size_t from, const Str& req, bool icase) {
    const size_t m = req.size();
    if (m == 0) return from;
    if (n < m || from > n - m) return Str::npos;
    auto upper = [&](char32_t c) { return icase && c >= 'a' && c <= 'z' ? c - 32 : c; };
    const char32_t a = req[0], b = req[m - 1];
    const size_t last = n - m;
    for (size_t i = scan::find_pair(p, from, last, m - 1, a, upper(a), b, upper(b)); i <= last;
         i = scan::find_pair(p, i + 1, last, m - 1, a, upper(a), b, upper(b))) {
        size_t k = 1;
        while (k + 1 < m && (icase ? fold(at(p, i + k)) : at(p, i + k)) == req[k]) ++k;
        if (k + 1 >= m) return i;
    }
    return Str::npos;
}

// Zero-width anchor every match of n must begin with: Node::BOS (\A), Node::BOL (^) or -1.
static int lead_anchor(const Node* n) {
    while (n->kind == Node::GROUP) n = n->kids[0].get();
    switch (n->kind) {
        case Node::BOS: return Node::BOS;
        case Node::BOL: return Node::BOL;
        case Node::SEQ: return n->kids.empty() ? -1 : lead_anchor(n->kids[0].get());
        // a repetition with at least one iteration begins with its first iteration
        case Node::REPEAT: return n->min >= 1 ? lead_anchor(n->kids[0].get()) : -1;
        case Node::ALT: {
            int a = -2;
            for (auto& k : n->kids) {
                const int b = lead_anchor(k.get());
                if (b < 0) return -1;
                if (a == -2) a = b;
                else if (a != b) a = Node::BOL;   // \A implies a line start too
            }
            return a < 0 ? -1 : a;
        }
        default: return -1;
    }
}

Regex::Regex(const std::string& utf8, int flags) {
    Parser ps;
    ps.p = from_utf8(utf8);
    root_ = ps.parse_alt((flags & IGNORECASE) != 0, (flags & DOTALL) != 0);
    if (!ps.eof()) throw std::runtime_error("rx parse: unbalanced )");
    ngroups_ = ps.ngroups;
    index_alternations(root_);
    {
        LitRun cur, best;
        required_runs(root_.get(), cur, best);
        if (cur.s.size() > best.s.size()) best = cur;
        if (best.s.size() >= 3) {
            req_ = best.s;
            req_icase_ = best.icase;
        }
    }
    {
        LitRun run;
        leading_run(root_.get(), run);
        if (run.s.size() >= 2) {
            lead_ = run.s;
            lead_icase_ = run.icase;
        }
    }
    // Where a match can start: \A-led patterns only at position 0, ^-led patterns only at line
    // starts (every pattern here is re.M). An alternation qualifies when all its branches do.
    const int lead = lead_anchor(root_.get());
    anchored_ = lead == Node::BOS;
    line_anchored_ = lead == Node::BOL;
    std::vector<bool> set(128, false);
    bool nonascii = false, nullable = false;
    first_chars(root_, set, nonascii, nullable);
    if (!nullable) {
        has_first_ = true;
        for (int c = 0; c < 128; ++c) first_[c] = set[c] ? 1 : 0;
        first_nonascii_ = nonascii;
        std::vector<char32_t> list;
        bool nl = false;
        if (first_list(root_, list, nl) && !nl && !list.empty()) {
            n_first_list_ = (int)list.size();
            std::copy(list.begin(), list.end(), first_list_);
        }
    }
}

bool Regex::search(const Str& s, size_t start, std::vector<long>& caps) const {
    return search_impl(s.data(), s.size(), start, caps);
}

bool Regex::search(const Str8& s, size_t start, std::vector<long>& caps) const {
    return search_impl(s.data(), s.size(), start, caps);
}

template <class C>
bool Regex::search_impl(const C* p, size_t n, size_t start, std::vector<long>& caps) const {
    caps.assign(2 * (ngroups_ + 1), -1);
    struct End : Cont { size_t* out; bool operator()(size_t e) const override { *out = e; return true; } } end;
    size_t e = 0;
    end.out = &e;
    Matcher<C> mt{p, n, caps};
    // a match at or after `start` contains req_ at or after `start` (anchored patterns are cheaper
    // to try at their few start positions)
    if (!anchored_ && !line_anchored_ && !req_.empty() && find_required(p, n, start, req_, req_icase_) == Str::npos)
        return false;
    auto first_ok = [&](char32_t c) { return c < 128 ? first_[c] != 0 : first_nonascii_; };
    for (size_t pos = start; pos <= n; ++pos) {
        if (anchored_ && pos > 0) return false;
        if (line_anchored_) {
            if (pos > 0 && p[pos - 1] != '\n') {   // next line start: the character after the next '\n'
                const size_t j = scan::find_char(p, pos, n, U'\n');
                if (j >= n) return false;
                pos = j + 1;
            }
            // a match starts with one of the first characters: else try the next line
            if (has_first_ && (pos == n || !first_ok(at(p, pos)))) {
                if (pos == n) return false;
                continue;
            }
        } else if (!lead_.empty()) {
            // skip to the next occurrence of the literal every match begins with
            pos = find_required(p, n, pos, lead_, lead_icase_);
            if (pos == Str::npos) return false;
        } else if (has_first_) {
            // skip to the next character a match can start with
            if (n_first_list_) {
                pos = scan::find_any(p, pos, n, first_list_, n_first_list_);
            } else {
                while (pos < n && !first_ok(at(p, pos))) ++pos;
            }
            if (pos == n) return false;
        }
        if (mt.m(root_.get(), pos, end)) {
            caps[0] = (long)pos;
            caps[1] = (long)e;
            return true;
        }
    }
    return false;
}

bool Regex::sub_into(Str& s, const Str& repl) const {
    std::vector<long> caps;
    if (!search(s, 0, caps)) return false;
    s = sub(s, repl);
    return true;
}

bool Regex::sub_into(Str8& s, const Str8& repl) const {
    std::vector<long> caps;
    if (!search(s, 0, caps)) return false;
    s = sub(s, repl);
    return true;
}

Str Regex::sub(const Str& s, const Str& repl, bool* changed) const { return sub_impl(s, repl, changed); }
Str8 Regex::sub(const Str8& s, const Str8& repl, bool* changed) const { return sub_impl(s, repl, changed); }

template <class S>
S Regex::sub_impl(const S& s, const S& repl, bool* changed) const {
    bool any = false;
    S out = sub_fn(s, [&](const S& src, const std::vector<long>& caps) {
        any = true;
        S r;
        for (size_t i = 0; i < repl.size(); ++i) {
            if (repl[i] == '\\' && i + 1 < repl.size() && repl[i + 1] >= '0' && repl[i + 1] <= '9') {
                int g = (int)(repl[i + 1] - '0');
                ++i;
                if (g <= ngroups_ && caps[2 * g] >= 0) r.append(src, (size_t)caps[2 * g], (size_t)(caps[2 * g + 1] - caps[2 * g]));
            } else {
                r.push_back(repl[i]);
            }
        }
        return r;
    });
    if (changed) *changed = any;
    return out;
}

}  // namespace rx
