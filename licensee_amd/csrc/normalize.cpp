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
#include <malloc.h>
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

using rx::Regex;
using rx::Str;

namespace {

const char32_t kSpace = U' ';

bool is_strip_char(char32_t c) { return c == 0 || c == ' ' || (c >= '\t' && c <= '\r'); }

Str ruby_strip(const Str& s) {
    size_t a = 0, b = s.size();
    while (a < b && is_strip_char(s[a])) ++a;
    while (b > a && is_strip_char(s[b - 1])) --b;
    return s.substr(a, b - a);
}

bool contains(const Str& s, const char* lit) {
    Str l = rx::from_utf8(lit);
    return s.find(l) != Str::npos;
}

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
bool python_only(char32_t c) { return c == 0x130 || c == 0x131 || c == 0x17F || c == 0x212A || c == 0x3A3; }

struct Ctx {
    std::map<std::string, Regex> re;
    std::vector<std::pair<Str, Str>> spell;
    std::vector<int> spell_first2[128 * 128];   // spell indices by first two characters, union order kept
    // Unicode tables (lh_set_unicode): Python str.lower() of non-ASCII code points
    bool unicode = false;
    std::unordered_map<char32_t, char32_t> lower;
    std::unordered_map<std::string, int32_t> vocab;
    int32_t n_vocab = 0, w64 = 0;
    // templates (Exact)
    int32_t n_templates = 0;
    std::vector<uint64_t> lf_bits;                  // [T][w64]
    std::vector<uint32_t> full_size;                // |wordset|
    std::vector<std::vector<std::string>> fields;   // field words in the wordset
    std::string err;

    const Regex& R(const char* name) const { return re.at(name); }
};

struct Normalizer {
    const Ctx& c;
    Str cur;
    bool clean = false;   // cur is already squeezed and stripped (a strip op without a match is a no-op)

    // squeeze(' ').strip in place (String#squeeze / #strip: only ' ' runs, \0\t\n\v\f\r ends)
    void squeeze_strip() {
        size_t w = 0;
        for (size_t r = 0; r < cur.size(); ++r) {
            if (cur[r] == kSpace && w > 0 && cur[w - 1] == kSpace) continue;
            cur[w++] = cur[r];
        }
        cur.resize(w);
        size_t b = cur.size();
        while (b > 0 && is_strip_char(cur[b - 1])) --b;
        cur.resize(b);
        size_t a = 0;
        while (a < cur.size() && is_strip_char(cur[a])) ++a;
        if (a) cur.erase(0, a);
    }
    // strip(re): gsub(re, ' ').squeeze(' ').strip (content_helper.rb:223-236)
    void strip_re(const Regex& r) {
        if (!r.sub_into(cur, U" ") && clean) return;
        squeeze_strip();
        clean = true;
    }
    void sub_re(const Regex& r, const char32_t* repl) {
        if (r.sub_into(cur, Str(repl))) clean = false;
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
    void strip_comments() {
        // String#split("\n") drops trailing empty fields
        std::vector<Str> lines;
        size_t a = 0;
        for (size_t i = 0; i <= cur.size(); ++i) {
            if (i == cur.size() || cur[i] == '\n') { lines.push_back(cur.substr(a, i - a)); a = i + 1; }
        }
        while (!lines.empty() && lines.back().empty()) lines.pop_back();
        if (lines.size() == 1) return;
        std::vector<long> caps;
        const Regex& cm = c.R("comment_markup");
        for (auto& l : lines)
            if (!cm.search(l, 0, caps)) return;
        strip_re(cm);
    }

    // hyphenated (content_helper.rb:40) can only match a '-' followed by [ \t\v\f\r]* and '\n'
    static bool has_hyphen_break(const Str& s) {
        for (size_t i = 0; i < s.size(); ++i) {
            if (s[i] != '-') continue;
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
        auto word = [](char32_t ch) {   // Python \b's \w
            return ch < 128 ? ((ch | 32) >= 'a' && (ch | 32) <= 'z') || (ch >= '0' && ch <= '9') || ch == '_'
                            : rx::is_word_char(ch);
        };
        // next hit at or after i: only word starts are candidates (every key starts with a
        // letter, so \b(?:key) can only match there); skips whole words otherwise
        auto next_hit = [&](size_t i, size_t& at, size_t& klen) -> const Str* {
            while (i < n) {
                const char32_t ch = cur[i];
                if (!word(ch)) {
                    ++i;
                    continue;
                }
                if (ch < 128 && i + 1 < n && cur[i + 1] < 128)
                    for (int si : c.spell_first2[ch * 128 + cur[i + 1]]) {
                        const Str& k = c.spell[si].first;
                        if (k.size() <= n - i && cur.compare(i, k.size(), k) == 0 &&
                            (i + k.size() == n || !word(cur[i + k.size()]))) {
                            at = i;
                            klen = k.size();
                            return &c.spell[si].second;
                        }
                    }
                while (i < n && word(cur[i])) ++i;
            }
            return nullptr;
        };
        size_t at = 0, klen = 0;
        const Str* rep = next_hit(0, at, klen);
        if (!rep) return;   // no varietal word: nothing to rebuild
        Str out;
        out.reserve(n);
        size_t i = 0;
        while (rep) {
            out.append(cur, i, at - i);
            out += *rep;
            i = at + klen;
            rep = next_hit(i, at, klen);
        }
        out.append(cur, i, Str::npos);
        cur.swap(out);
        clean = false;
    }

    // strip(:whitespace): gsub(/\s+/, ' ').squeeze(' ').strip, in place
    void collapse_whitespace() {
        size_t w = 0;
        for (size_t r = 0; r < cur.size(); ++r) {
            const char32_t ch = cur[r];
            const bool ws = ch == ' ' || (ch >= '\t' && ch <= '\r');
            if (ws) {
                if (w == 0 || cur[w - 1] != ' ') cur[w++] = ' ';
            } else {
                cur[w++] = ch;
            }
        }
        cur.resize(w);
        // no ' ' runs are left, so squeeze(' ') is the identity: strip only
        size_t b = cur.size();
        while (b > 0 && is_strip_char(cur[b - 1])) --b;
        cur.resize(b);
        size_t a = 0;
        while (a < cur.size() && is_strip_char(cur[a])) ++a;
        if (a) cur.erase(0, a);
        clean = true;
    }

    // content_without_title_and_version + content_normalized (content_helper.rb:144-168)
    Str run(const Str& content) {
        cur = ruby_strip(content);
        strip_re(c.R("hrs"));
        strip_comments();
        strip_re(c.R("markdown_headings"));
        // \[(.+?)\]\(.+?\) needs a literal "](": without one the lazy scans from every '[' are wasted
        if (contains(cur, "](")) sub_re(c.R("link_markup"), U"\\1");
        strip_title();
        strip_re(c.R("version"));
        for (auto& ch : cur) {
            if (ch < 128) {
                if (ch >= 'A' && ch <= 'Z') ch += 32;
            } else if (c.unicode) {
                auto it = c.lower.find(ch);
                if (it != c.lower.end()) ch = it->second;
            }
        }
        sub_re(c.R("lists"), U"- \\1");
        sub_re(c.R("https"), U"https:");
        {   // '&' -> 'and'
            Str out;
            for (char32_t ch : cur) {
                if (ch == '&') out += U"and";
                else out.push_back(ch);
            }
            cur.swap(out);
        }
        sub_re(c.R("dashes"), U"-");
        sub_re(c.R("quote"), U"'");
        if (has_hyphen_break(cur)) sub_re(c.R("hyphenated"), U"\\1-\\2");
        spelling();
        sub_re(c.R("span_markup"), U"\\1");
        sub_re(c.R("bullet"), U"\n\n- ");
        sub_re(c.R("bullet_paren"), U")(");
        // STRIP_METHODS (content_helper.rb:89-105)
        strip_re(c.R("bom"));
        if (contains(cur, "creative commons")) { strip_re(c.R("cc_dedication")); strip_re(c.R("cc_wiki")); }
        if (contains(cur, "associating cc0")) {
            strip_re(c.R("cc_legal_code")); strip_re(c.R("cc0_info")); strip_re(c.R("cc0_disclaimer"));
        }
        if (contains(cur, "unlicense")) strip_re(c.R("unlicense_info"));
        sub_re(c.R("border_markup"), U"\\1");
        strip_title();
        strip_re(c.R("version"));
        strip_re(c.R("url"));
        strip_copyright();
        strip_title();
        strip_re(c.R("block_markup"));
        strip_re(c.R("developed_by"));
        {
            std::vector<long> caps;
            if (c.R("end_of_terms").search(cur, 0, caps)) {
                cur.resize((size_t)caps[0]);
                clean = false;
            }
        }
        collapse_whitespace();
        strip_re(c.R("mit_optional"));
        return cur;
    }
};

// wordset scan (content_helper.rb:109): (?:[\w/-](?:'s|(?<=s)')?)+ with ASCII \w
inline bool wchar(char32_t c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_' || c == '/' || c == '-';
}

template <class F>
void scan_words(const Str& s, F&& emit) {
    size_t i = 0;
    const size_t n = s.size();
    while (i < n) {
        if (!wchar(s[i])) { ++i; continue; }
        const size_t a = i;
        while (i < n && wchar(s[i])) {
            const char32_t ch = s[i++];
            if (i + 1 < n + 1 && i < n && s[i] == '\'') {
                if (i + 1 < n && s[i + 1] == 's') i += 2;
                else if (ch == 's') i += 1;
            }
        }
        emit(a, i);
    }
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
    Str normalized;
    bool cc = false, copyright = false;
};

void prep_one_impl(const Ctx& c, const char* data, int64_t len, const char* filename, bool is_file, FileOut& o);

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

void prep_one_impl(const Ctx& c, const char* data, int64_t len, const char* filename, bool is_file, FileOut& o) {
    Str content = rx::from_utf8(std::string(data, (size_t)len));
    if (is_file) {   // universal newline (project_file.rb:41)
        Str t;
        t.reserve(content.size());
        for (size_t i = 0; i < content.size(); ++i) {
            if (content[i] == '\r') {
                t.push_back('\n');
                if (i + 1 < content.size() && content[i + 1] == '\n') ++i;
            } else t.push_back(content[i]);
        }
        content.swap(t);
    }
    for (char32_t ch : content)
        if (ch >= 0x80 && (c.unicode ? python_only(ch) : !safe_nonascii(ch))) { o.status = 1; return; }
    if (extname_is_html(filename)) { o.status = 1; return; }
    std::vector<long> caps;
    const Str stripped = ruby_strip(content);
    o.cc = c.R("cc_false_positive").search(stripped, 0, caps);
    o.copyright = c.R("copyright_match").search(stripped, 0, caps);
    Normalizer nz{c, Str()};
    o.normalized = nz.run(content);
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
        for (int32_t i = 0; i < n_spell; ++i) {
            c->spell.push_back({rx::from_utf8(spell_from[i]), rx::from_utf8(spell_to[i])});
            const Str& k = c->spell.back().first;
            if (k.size() < 2 || k[0] >= 128 || k[1] >= 128)
                throw std::runtime_error("spelling keys: >= 2 characters, ASCII first two");
            c->spell_first2[k[0] * 128 + k[1]].push_back(i);
        }
        for (int32_t i = 0; i < n_vocab; ++i) c->vocab.emplace(vocab[i], i);
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
    for (int32_t t = 0; t < n_templates; ++t)
        for (int32_t k = field_off[t]; k < field_off[t + 1]; ++k) c->fields[t].push_back(field_words[k]);
    return 0;
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
    for (int32_t i = 0; i < n_lower; ++i) c->lower.emplace(lower_from[i], lower_to[i]);
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
    const std::string u = rx::to_utf8(o.normalized);
    if (out && cap > (int64_t)u.size()) {
        memcpy(out, u.data(), u.size());
        out[u.size()] = 0;
    }
    return (int64_t)u.size();
}

// Batched LicenseFile preparation: decode, normalize, wordset scan, intern to the vocabulary
// bitset, |W_F|, len_F, CC flag, Copyright and Exact matchers.
//   status[i]: 0 ok; 1 the caller must use the Python path for file i (its outputs unset).
//   exact[i]:  first template (key order) whose wordset equals the file's, or -1.
int lh_prep_files(lh_ctx* ctx, int64_t n, const char* const* data, const int64_t* lens, const char* const* filenames,
                  int32_t nthreads, uint64_t* bits, uint32_t* wf, int32_t* length, uint8_t* cc, uint8_t* copyright,
                  int32_t* exact, uint8_t* status) {
    const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
    if (nthreads < 1) nthreads = 1;
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        std::vector<uint64_t> row((size_t)c->w64);
        for (;;) {
            const int64_t i = next.fetch_add(16);
            if (i >= n) break;
            for (int64_t f = i; f < std::min<int64_t>(n, i + 16); ++f) {
                FileOut o;
                prep_one(*c, data[f], lens[f], filenames ? filenames[f] : nullptr, true, o);
                status[f] = (uint8_t)o.status;
                if (o.status) continue;
                std::fill(row.begin(), row.end(), 0);
                std::unordered_set<std::string> words;
                std::string w;
                scan_words(o.normalized, [&](size_t a, size_t b) {
                    w.clear();
                    for (size_t k = a; k < b; ++k) w.push_back((char)o.normalized[k]);   // ASCII only
                    if (words.insert(w).second) {
                        auto it = c->vocab.find(w);
                        if (it != c->vocab.end()) row[(size_t)it->second >> 6] |= 1ULL << (it->second & 63);
                    }
                });
                memcpy(bits + (size_t)f * c->w64, row.data(), sizeof(uint64_t) * (size_t)c->w64);
                wf[f] = (uint32_t)words.size();
                length[f] = (int32_t)o.normalized.size();
                cc[f] = o.cc;
                copyright[f] = o.copyright;
                int32_t ex = -1;
                for (int32_t t = 0; t < c->n_templates && ex < 0; ++t) {
                    if (c->full_size[t] != words.size()) continue;
                    const uint64_t* L = c->lf_bits.data() + (size_t)t * c->w64;
                    bool ok = true;
                    for (int32_t k = 0; k < c->w64 && ok; ++k) ok = (row[k] & L[k]) == L[k];
                    for (size_t k = 0; k < c->fields[t].size() && ok; ++k) ok = words.count(c->fields[t][k]) > 0;
                    if (ok) ex = t;
                }
                exact[f] = ex;
            }
        }
    };
    run_workers(nthreads, work);
    return 0;
}

}  // extern "C"
