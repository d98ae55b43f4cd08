// Runs the native host library (csrc/rx.cpp, normalize.cpp, vocab_pack.cpp) under
// AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on the C++ CPU path).
// Input: one binary file written by tests/test_sanitizers.py -- length-prefixed strings and
// arrays in a fixed order. Any sanitizer finding aborts the process (non-zero exit).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "licensee_host.h"

namespace {

struct Reader {
    std::vector<char> buf;
    size_t pos = 0;
    uint32_t u32() {
        uint32_t v;
        memcpy(&v, buf.data() + pos, 4);
        pos += 4;
        return v;
    }
    std::string str() {
        const uint32_t n = u32();
        std::string s(buf.data() + pos, n);
        pos += n;
        return s;
    }
    std::vector<std::string> strs() {
        const uint32_t n = u32();
        std::vector<std::string> v;
        for (uint32_t i = 0; i < n; ++i) v.push_back(str());
        return v;
    }
    template <class T>
    std::vector<T> arr() {   // u32 element count, then raw elements
        const uint32_t n = u32();
        std::vector<T> v(n);
        if (n) memcpy(v.data(), buf.data() + pos, sizeof(T) * n);
        pos += sizeof(T) * n;
        return v;
    }
};

std::vector<const char*> cptrs(const std::vector<std::string>& v) {
    std::vector<const char*> p;
    for (auto& s : v) p.push_back(s.c_str());
    if (p.empty()) p.push_back(nullptr);
    return p;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    Reader r;
    {
        FILE* f = fopen(argv[1], "rb");
        if (!f) return 2;
        fseek(f, 0, SEEK_END);
        r.buf.resize((size_t)ftell(f));
        fseek(f, 0, SEEK_SET);
        if (fread(r.buf.data(), 1, r.buf.size(), f) != r.buf.size()) return 2;
        fclose(f);
    }
    const auto names = r.strs(), pats = r.strs();
    const auto flags = r.arr<int32_t>();
    const auto sfrom = r.strs(), sto = r.strs(), vocab = r.strs();
    const int32_t T = (int32_t)r.u32();
    const auto lf = r.arr<uint64_t>();
    const auto wsz = r.arr<uint32_t>();
    const auto foff = r.arr<int32_t>();
    const auto fwords = r.strs();
    const auto lfrom = r.arr<uint32_t>(), lto = r.arr<uint32_t>(), wlo = r.arr<uint32_t>(), whi = r.arr<uint32_t>();
    const auto texts = r.strs();
    const auto sig = r.arr<uint64_t>();
    const int32_t sig_words = (int32_t)r.u32();

    auto pn = cptrs(names), pp = cptrs(pats), pf = cptrs(sfrom), pt = cptrs(sto), pv = cptrs(vocab), pw = cptrs(fwords);
    char err[512] = {0};
    lh_ctx* ctx = lh_create((int32_t)names.size(), pn.data(), pp.data(), flags.data(), (int32_t)sfrom.size(), pf.data(),
                            pt.data(), (int32_t)vocab.size(), pv.data(), err, sizeof err);
    if (!ctx) {
        fprintf(stderr, "lh_create: %s\n", err);
        return 3;
    }
    if (lh_set_unicode(ctx, (int32_t)lfrom.size(), lfrom.data(), lto.data(), (int32_t)wlo.size(), wlo.data(), whi.data()))
        return 4;
    if (lh_set_templates(ctx, T, lf.data(), wsz.data(), foff.data(), pw.data())) return 5;

    const int64_t n = (int64_t)texts.size();
    const int32_t w64 = (int32_t)((vocab.size() + 63) / 64);
    std::vector<const char*> data;
    std::vector<int64_t> lens;
    for (auto& t : texts) {
        data.push_back(t.data());
        lens.push_back((int64_t)t.size());
    }
    std::vector<uint64_t> bits((size_t)n * w64);
    std::vector<uint32_t> wf(n);
    std::vector<int32_t> length(n), exact(n);
    std::vector<uint8_t> cc(n), cr(n), st(n);
    std::vector<uint64_t> fmask(n), need(T);
    if (lh_prep_files(ctx, n, data.data(), lens.data(), nullptr, 4, bits.data(), wf.data(), length.data(), cc.data(),
                      cr.data(), exact.data(), st.data(), nullptr))
        return 6;
    // the device-Exact variant: no host Exact, per-file field masks
    if (lh_template_field_masks(ctx, need.data()) < 0 ||
        lh_prep_files(ctx, n, data.data(), lens.data(), nullptr, 4, bits.data(), wf.data(), length.data(), cc.data(),
                      cr.data(), nullptr, st.data(), fmask.data()))
        return 6;
    // the device-wordset host stage: normalized texts into a caller buffer, once with room for all and
    // once with room for about half (the rest report "no room", status 3)
    {
        int64_t total = 0;
        for (int64_t l : lens) total += l;
        std::vector<int64_t> off(n);
        std::vector<int32_t> tl(n), ln(n);
        for (int64_t cap : {total + 16 * n + 65536, total / 2}) {
            std::vector<char> buf((size_t)std::max<int64_t>(cap, 1));
            const int64_t used = lh_normalize_files(ctx, n, data.data(), lens.data(), nullptr, 4, buf.data(), cap,
                                                    off.data(), tl.data(), ln.data(), cc.data(), cr.data(), st.data());
            if (used < 0 || used > cap) return 9;
            for (int64_t i = 0; i < n; ++i)
                if (st[i] == 0 && (off[i] < 0 || off[i] % 16 || off[i] + tl[i] > used)) return 9;
        }
    }
    int64_t native = 0, total_len = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t m = lh_normalize(ctx, data[i], lens[i], "LICENSE", 1, nullptr, 0);
        if (m >= 0) {
            std::vector<char> out((size_t)m + 1);
            if (lh_normalize(ctx, data[i], lens[i], "LICENSE", 1, out.data(), m + 1) != m) return 7;
            ++native;
            total_len += m;
        }
    }
    lh_destroy(ctx);

    // vocabulary packing on the corpus signatures, both bin widths
    const int32_t V = (int32_t)(sig.size() / (size_t)sig_words);
    std::vector<int32_t> init(V), out(V);
    for (int32_t i = 0; i < V; ++i) init[i] = V - 1 - i;
    for (int bin : {32, 64})
        if (lh_vocab_pack(sig.data(), V, sig_words, T, init.data(), bin, 200000, 7, out.data()) < 0) return 8;
    printf("ok texts=%lld native=%lld chars=%lld V=%d\n", (long long)n, (long long)native, (long long)total_len, V);
    return 0;
}
