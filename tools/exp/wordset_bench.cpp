// Experiment (not product code): the wordset stage of lh_prep_files in isolation -- tokenizer,
// key packing, vocabulary probe, per-file word set -- on normalized texts, one thread.
//   python tools/exp/wordset_bench_inputs.py /tmp/wsb   (normalized texts + vocabulary)
//   g++ -O3 -march=x86-64-v3 -std=c++17 -pthread -o /tmp/wsb/bench tools/exp/wordset_bench.cpp \
//       licensee_amd/csrc/rx.cpp && /tmp/wsb/bench /tmp/wsb
#include <chrono>
#include <fstream>
#include <iostream>
#include <sstream>

#include "../../licensee_amd/csrc/normalize.cpp"

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp/wsb";
    std::vector<std::string> vocab;
    {
        std::ifstream f(dir + "/vocab.txt");
        for (std::string l; std::getline(f, l);) vocab.push_back(l);
    }
    std::vector<Str> texts;
    {
        std::ifstream f(dir + "/texts.txt");
        for (std::string l; std::getline(f, l);) texts.push_back(rx::from_utf8(l));
    }
    std::vector<const char*> vp;
    for (auto& w : vocab) vp.push_back(w.c_str());
    VocabTable vt;
    vt.build((int32_t)vp.size(), vp.data());
    const int32_t w64 = ((int32_t)vocab.size() + 63) / 64;
    std::vector<uint64_t> row((size_t)w64);
    WordSet words;
    size_t tokens = 0, hits = 0, sink = 0;
    for (auto& t : texts) scan_words(t, [&](size_t, size_t) { ++tokens; });
    auto run = [&](int mode) {
        const auto t0 = std::chrono::steady_clock::now();
        size_t h = 0;
        for (int rep = 0; rep < 3; ++rep)
            for (auto& t : texts) {
                std::fill(row.begin(), row.end(), 0);
                words.reset(t);
                scan_words(t, [&](size_t a, size_t b) {
                    if (mode == 0) { sink += b - a; return; }
                    const char32_t* p = t.data() + a;
                    const WordKey k = word_key(p, b - a, t.size() - a);
                    if (mode == 1) { sink += k.h & 1; return; }
                    const int32_t id = vt.find(k, p);
                    if (mode == 2) { sink += (size_t)id; return; }
                    if (id >= 0) {
                        row[(size_t)id >> 6] |= 1ULL << (id & 63);
                        ++h;
                    } else {
                        words.insert(a, k);
                    }
                });
            }
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 3;
        if (mode == 3) hits = h / 3;
        return s;
    };
    const char* names[] = {"tokenize", "+ key", "+ vocab probe", "+ row / word set"};
    for (int m = 0; m < 4; ++m) {
        double best = 1e9;
        for (int r = 0; r < 5; ++r) best = std::min(best, run(m));
        std::cout << names[m] << ": " << best / texts.size() * 1e6 << " us/file, " << best / tokens * 1e9
                  << " ns/token\n";
    }
    std::cout << texts.size() << " texts, " << tokens / (double)texts.size() << " tokens/file, "
              << hits / (double)tokens * 100 << "% vocabulary hits (sink " << (sink & 1) << ")\n";
    return 0;
}
