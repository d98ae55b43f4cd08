// Minimal backtracking regex engine over UTF-32 code points, implementing exactly the
// Python `re` subset used by licensee_amd/content_helper.py (the host restatement of
// lib/licensee/content_helper.rb): literals and escapes (\A \Z \b \n \t \v \f \r \uXXXX and
// escaped punctuation), classes with ranges / negation, '.', groups (capturing, (?:),
// scoped flags (?i:) (?-i:)), lookbehind (?<!..) (?<=..) and lookahead (?=..) (?!..) of
// fixed width, alternation, greedy and lazy quantifiers (* + ? {m,n}), ^ and $ (always
// multiline here, as every pattern is compiled with re.M). Case-insensitive matching folds
// ASCII only: the few non-ASCII characters Python's re.I equates with ASCII letters
// (U+0130, U+0131, U+017F, U+212A) send their text to the Python path (normalize.cpp).
#pragma once

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace rx {

using Str = std::u32string;
// A text whose every character is ASCII, one byte per character (the byte path of
// normalize.cpp: the same patterns, matched over 4x fewer bytes)
using Str8 = std::string;

enum Flags : int { IGNORECASE = 2, MULTILINE = 8, DOTALL = 16 };  // Python re flag values

// Thrown by a match that would nest deeper than max_match_depth() node frames (see Matcher in
// rx.cpp); callers treat the text as one for the Python path.
struct TooDeep {};
// Node-frame limit of one match on this thread: sized for the worker threads' stacks
// (normalize.cpp runs batch preparation on threads with kWorkerStack bytes of stack) and
// smaller on other threads (default 8 MiB stacks). set_match_depth() changes it per thread.
size_t max_match_depth();
void set_match_depth(size_t frames);

struct Node;
using NodeP = std::shared_ptr<Node>;

struct Node {
    enum Kind { LIT, ANY, CLASS, SEQ, ALT, GROUP, REPEAT, BOL, EOL, BOS, EOS, WORDB, LOOK };
    Kind kind;
    char32_t ch = 0;                                // LIT
    bool icase = false;                             // LIT / CLASS
    bool dotall = false;                            // ANY
    bool negate = false;                            // CLASS, LOOK (negative)
    bool behind = false;                            // LOOK
    std::vector<std::pair<char32_t, char32_t>> ranges;  // CLASS
    std::vector<NodeP> kids;                        // SEQ / ALT / GROUP(1) / REPEAT(1) / LOOK(1)
    int group = -1;                                 // GROUP capture index (-1: none)
    int min = 0, max = -1;                          // REPEAT (-1: unbounded)
    bool lazy = false;                              // REPEAT
    int width = -1;                                 // LOOK (behind): fixed width
    // ALT: per branch, the ASCII characters it can start with (bit c of first[2 * i + c / 64]),
    // whether it can start with a non-ASCII one, whether it can match empty (then never skipped)
    std::vector<uint64_t> alt_first;
    std::vector<uint8_t> alt_nonascii, alt_nullable;
};

class Regex {
public:
    Regex() = default;
    Regex(const std::string& utf8_pattern, int flags);
    // search from `start`; on success fills caps ([2*i], [2*i+1]; -1 when unset) for i <= ngroups
    bool search(const Str& s, size_t start, std::vector<long>& caps) const;
    bool search(const Str8& s, size_t start, std::vector<long>& caps) const;
    int ngroups() const { return ngroups_; }
    bool anchored() const { return anchored_; }
    // re.sub with a template supporting \1..\9 (and literal text); count = 0 -> all
    Str sub(const Str& s, const Str& repl, bool* changed = nullptr) const;
    Str8 sub(const Str8& s, const Str8& repl, bool* changed = nullptr) const;
    // in-place re.sub: returns false (s untouched, no copy) when nothing matches
    bool sub_into(Str& s, const Str& repl) const;
    bool sub_into(Str8& s, const Str8& repl) const;
    template <class S, class F>
    S sub_fn(const S& s, F&& fn) const;  // replacement computed from the match
    bool valid() const { return (bool)root_; }

private:
    NodeP root_;
    int ngroups_ = 0;
    bool anchored_ = false;           // every match starts with \A
    bool line_anchored_ = false;      // every match starts with ^ (a line start)
    bool has_first_ = false;          // first-character filter active
    uint8_t first_[128] = {};         // ASCII characters a match can start with
    bool first_nonascii_ = true;      // ... and whether any non-ASCII one can
    char32_t first_list_[8] = {};     // the exact first-character set when it is this small
    int n_first_list_ = 0;            // (vector scan; 0: use first_)
    Str req_;                         // a literal every match contains (empty: none found)
    bool req_icase_ = false;          // ... compared with ASCII case folding
    Str lead_;                        // a literal every match begins with (used from 2 characters)
    bool lead_icase_ = false;
    template <class C>
    bool search_impl(const C* p, size_t n, size_t start, std::vector<long>& caps) const;
    template <class S>
    S sub_impl(const S& s, const S& repl, bool* changed) const;
    template <class C>
    friend struct Matcher;
};

Str from_utf8(const std::string& s);
Str from_utf8(const char* data, size_t n);
std::string to_utf8(const Str& s);

// \b / \w word characters: ASCII [A-Za-z0-9_] plus the installed non-ASCII ranges (Python's
// str.isalnum(), supplied by the caller). Process-wide; set once before matching.
void set_unicode_word_ranges(const uint32_t* lo, const uint32_t* hi, int32_t n);
bool is_word_char(char32_t c);

}  // namespace rx

// ---- template implementation ---------------------------------------------------------
namespace rx {
template <class S, class F>
S Regex::sub_fn(const S& s, F&& fn) const {
    S out;
    size_t pos = 0, last = 0;
    std::vector<long> caps;
    while (pos <= s.size() && search(s, pos, caps)) {
        const size_t ms = (size_t)caps[0], me = (size_t)caps[1];
        out.append(s, last, ms - last);
        out += fn(s, caps);
        last = me;
        pos = me > ms ? me : me + 1;
        if (me == ms && ms < s.size()) out.push_back(s[ms]), last = ms + 1;
        if (anchored_) break;
    }
    if (last < s.size()) out.append(s, last, S::npos);
    return out;
}
}  // namespace rx
