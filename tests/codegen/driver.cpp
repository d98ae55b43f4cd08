// Runs the generated kernels lane by lane on the host. Inputs/outputs are raw binary files.
// Each wave runs twice per kernel (host_shim.h): a vote pass collecting __all over the wave's
// 64 lanes, then the real pass whose outputs are kept.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "host_shim.h"
#include "prog.inc"
#include <vector>
template <class T> std::vector<T> load(const char* p, size_t n) {
    std::vector<T> v(n); FILE* f = fopen(p, "rb"); fread(v.data(), sizeof(T), n, f); fclose(f); return v;
}
template <class T> void save(const char* p, const std::vector<T>& v) {
    FILE* f = fopen(p, "wb"); fwrite(v.data(), sizeof(T), v.size(), f); fclose(f);
}
template <class F> void run_wave(unsigned b, unsigned w, F&& lane_fn) {
    blockIdx.x = b;
    g_vote_all = true;
    for (int phase = 0; phase < 2; ++phase) {
        g_vote_phase = phase;
        for (unsigned l = 0; l < 64; ++l) {
            threadIdx.x = w * 64 + l;
            lane_fn();
        }
    }
    if (!g_vote_all) ++g_slow_waves;
}
int main(int argc, char** argv) {
    // argv: dir n k
    const char* d = argv[1]; long long n = atoll(argv[2]); int k = atoi(argv[3]);
    long long ntiles = (n + 63) / 64, npad = ntiles * 64;
    char p[4096];
    snprintf(p, sizeof p, "%s/tiles.bin", d); auto tiles = load<uint4>(p, (size_t)ntiles * WQ * 64);
    snprintf(p, sizeof p, "%s/wf.bin", d); auto wf = load<u32>(p, npad);
    snprintf(p, sizeof p, "%s/len.bin", d); auto len = load<i32>(p, npad);
    snprintf(p, sizeof p, "%s/cc.bin", d); auto cc = load<unsigned char>(p, npad);
    std::vector<i32> best(n); std::vector<u32> ov(n); std::vector<double> sc_(n);
    std::vector<u32> mov(n * NT); std::vector<double> msc(n * NT);
    std::vector<i32> tki(n * (k ? k : 1)); std::vector<double> tks(n * (k ? k : 1));
    long long slow_match = 0;
    for (long long b = 0; b < (ntiles + 3) / 4; ++b)
        for (unsigned w = 0; w < 4; ++w) {
            const long long before = g_slow_waves;
            run_wave((unsigned)b, w, [&] {
                dice_prog_match(tiles.data(), n, wf.data(), len.data(), cc.data(), 98.0, best.data(), ov.data(), sc_.data());
            });
            slow_match += g_slow_waves - before;
            run_wave((unsigned)b, w, [&] {
                (k <= 4 ? dice_prog_matrix4 : dice_prog_matrix16)(tiles.data(), n, wf.data(), len.data(), cc.data(), k,
                                                                 mov.data(), msc.data(), k ? tki.data() : nullptr, tks.data());
            });
        }
    snprintf(p, sizeof p, "%s/best.out", d); save(p, best);
    snprintf(p, sizeof p, "%s/ov.out", d); save(p, ov);
    snprintf(p, sizeof p, "%s/score.out", d); save(p, sc_);
    snprintf(p, sizeof p, "%s/mov.out", d); save(p, mov);
    snprintf(p, sizeof p, "%s/msc.out", d); save(p, msc);
    snprintf(p, sizeof p, "%s/tki.out", d); save(p, tki);
    snprintf(p, sizeof p, "%s/tks.out", d); save(p, tks);
    // waves that voted slow (match kernel; tiles past n return before the vote and count as fast)
    printf("slow_waves %lld\n", slow_match);
    return 0;
}
