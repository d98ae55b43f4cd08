// Template-specialized sparse scoring program for small corpora (T <= 64), gfx950.
//
// The corpus is known when dice_create() runs, so the overlap loop
//     ov_t = sum_d popcount(file[d] & Lf_t[d])          (content_helper.rb:129)
// is emitted as straight-line HIP over the NONZERO (template, dword) pairs only: every file
// dword lives in a VGPR with a compile-time index and every template mask is an instruction
// literal, so an entry costs v_and_b32 (literal) + v_bcnt_u32_b32 (accumulate) and no
// memory traffic beyond the file's own bitset. With the interner's signature vocabulary
// order the 47 vendored templates need ~1.5k entries instead of 47 x 112 dense dwords,
// which moves the kernel from VALU-bound to HBM-bound.
//
// Each template's epilogue follows its accumulation: denominator
// (content_helper.rb:130-132,337-347, per-template constants baked in), CC filter
// (dice.rb:23-31) and the running argmax (dice.rb:34-48). The compare is an exact
// rational cross-multiplication on the fast path; waves holding a file outside the fast
// envelope (|W_F| >= 2^20 or len_F >= 2^21, or a corpus outside the envelope) run the same
// program with IEEE-double compares (see dice_common.h for why both orders coincide).
//
// The source is compiled with hiprtc for gfx950 and cached by hash under the library
// directory (lib/cache/dice_prog_<hash>.co), so a corpus compiles once per machine image.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <sys/stat.h>
#include <unistd.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/licensee_dice.h"
#include "dice_program.h"

// dice_ctx / dice_batch internals shared with dice.hip
#include "dice_internal.h"

namespace dice {

namespace {

const char* kPrelude = R"HIP(
typedef unsigned int u32;
typedef int i32;
typedef unsigned long long u64;
typedef long long i64;

#ifdef __HIP_DEVICE_COMPILE__
// v_mul_u32_u24: full-rate 24x24 multiply (low 32 bits); v_sad_u32: |a - b| + c in one op.
__device__ __forceinline__ u32 mul24(u32 a, u32 b) { u32 r; asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ u32 absdiff(u32 a, u32 b) { u32 r; asm("v_sad_u32 %0, %1, %2, 0" : "=v"(r) : "s"(a), "v"(b)); return r; }
__device__ __forceinline__ u32 subsat(u32 a, u32 b) { return __builtin_elementwise_sub_sat(a, b); }   // v_sub_u32 clamp
#else
__device__ __forceinline__ u32 subsat(u32 a, u32 b) { return a > b ? a - b : 0u; }
__device__ __forceinline__ u32 mul24(u32 a, u32 b) { return (a & 0xffffffu) * (b & 0xffffffu); }
__device__ __forceinline__ u32 absdiff(u32 a, u32 b) { return a > b ? a - b : b - a; }
#endif
// acc += popcount(x & MASK): v_and_b32 (literal) + v_bcnt_u32_b32 accumulate. Written as asm
// (ACC_ASM) because the compiler otherwise rebalances the chains into v_bcnt(x, 0) + v_add3.
#if defined(__HIP_DEVICE_COMPILE__) && ACC_ASM
#define ACC_ASM_ONLY(...) __VA_ARGS__
#define ACC_C_ONLY(...)
#else
#define ACC_ASM_ONLY(...)
#define ACC_C_ONLY(...) __VA_ARGS__
#endif
#if defined(__HIP_DEVICE_COMPILE__) && ACC_ASM
#define ACCM(acc, x, MASK) { u32 t_; asm("v_and_b32 %1, " #MASK ", %2\n\tv_bcnt_u32_b32 %0, %1, %0" : "+v"(acc), "=&v"(t_) : "v"(x)); }
#define ACCF1(acc, x) asm("v_bcnt_u32_b32 %0, %1, %0" : "+v"(acc) : "v"(x))
#else
#define ACCM(acc, x, MASK) acc = __builtin_popcount((x) & (MASK)) + acc
#define ACCF1(acc, x) acc = __builtin_popcount(x) + acc
#endif
// File-tile quad load; FILE_NT streams it with the non-temporal cache policy (each quad is
// read exactly once per launch).
#if FILE_NT && defined(__HIP_DEVICE_COMPILE__)
typedef u32 u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldq(const uint4* p) {
    const u32x4v v = __builtin_nontemporal_load((const u32x4v*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
#else
__device__ __forceinline__ uint4 ldq(const uint4* p) { return *p; }
#endif
#if OUT_NT && defined(__HIP_DEVICE_COMPILE__)
#define MSTORE(p, v) __builtin_nontemporal_store((v), (p))
#else
#define MSTORE(p, v) (*(p) = (v))
#endif
// Denominator (content_helper.rb:130-132,337-347); lengths are non-negative (len_F < 2^31).
__device__ __forceinline__ i32 dn(i32 base, i32 slack, i32 tlen, u32 wf, i32 lf) {
    const u32 d = absdiff((u32)tlen, (u32)lf);
    const u32 adj = slack <= 0 ? d : subsat(d, (u32)slack);   // max(d - slack, 0)
    return base + (i32)wf + (i32)(adj >> 2);
}
__device__ __forceinline__ double sc(u32 o, i32 d) { return ((double)o * 200.0) / (double)d; }
// Overlaps may carry a template index in bits 24-31 (match kernel): only bits 0-23 count.
template <bool FAST>
__device__ __forceinline__ bool ge(u32 oa, i32 da, u32 ob, i32 db) {
    if (FAST) {
#if NARROW_MUL
        // ov < 2^11 and den < 2^21: both products < 2^32, full-rate 24-bit multiplies are exact
        return mul24(oa, (u32)db) >= mul24(ob, (u32)da);
#else
        return (u64)(oa & 0xFFFFFFu) * (u64)(u32)db >= (u64)(ob & 0xFFFFFFu) * (u64)(u32)da;
#endif
    }
    return sc(oa & 0xFFFFFFu, da) >= sc(ob & 0xFFFFFFu, db);
}
#define ACC(d, m) a = __builtin_popcount(f[d] & (m##u)) + a
#define ACCF(d) a = __builtin_popcount(f[d]) + a
)HIP";

const char* kMatchKernel = R"HIP(
extern "C" __global__ __launch_bounds__(64 * WPB MATCH_WAVES) void dice_prog_match(
    const uint4* __restrict__ files, i64 n, const u32* __restrict__ wfp, const i32* __restrict__ lenp,
    const unsigned char* __restrict__ ccp, double thr, i32* __restrict__ best_out,
    u32* __restrict__ ov_out, double* __restrict__ score_out) {
    const int lane = threadIdx.x & 63;
    const i64 tile = (i64)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (tile * 64 >= n) return;
    const i64 file = tile * 64 + lane;
    const uint4* fp = files + tile * (i64)(WQ * 64) + lane;
#if WAVE_TIMING
    const u64 t0_ = __builtin_amdgcn_s_memrealtime();
#endif
    const u32 wf = wfp[file];
    const i32 lf = lenp[file];
    const bool cc = ccp[file] != 0;
    FILE_PROLOGUE
    const bool fast = CORPUS_FAST && wf < (1u << 20) && lf >= 0 && lf < (1 << 21);
    // running best: bo = template index << 24 | overlap (0xFF: none yet), bd = its denominator
    u32 bo = 0xFF000000u; i32 bd = 1;
    if (__all(fast)) {
        MATCH_BODY(true)
    } else {
        MATCH_BODY(false)
    }
    if (file < n) {
        const i32 bi = (bo >> 24) == 0xFFu ? -1 : (i32)(bo >> 24);
        const u32 bov = bo & 0xFFFFFFu;
        const double s = bi >= 0 ? sc(bov, bd) : 0.0;
        MSTORE(best_out + file, (bi >= 0 && s >= thr) ? bi : -1);
        MSTORE(ov_out + file, bov);
        MSTORE(score_out + file, s);
    }
#if WAVE_TIMING
    // diagnostics (DICE_PROG_DIAG=timing, results wrong): per wave its start and end real-time (100 MHz)
    // clock and the raw HW_ID / XCC_ID registers, in the tile's first output slots
    const u64 t1_ = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        score_out[tile * 64] = (double)t0_;
        score_out[tile * 64 + 1] = (double)t1_;
        ov_out[tile * 64] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        ov_out[tile * 64 + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
#endif
}
)HIP";

// Matrix kernel template: KM is the compile-time top-k slot count (4 or 16).
const char* kMatrixKernel = R"HIP(
extern "C" __global__ __launch_bounds__(64 * WPB) void KNAME(
    const uint4* __restrict__ files, i64 n, const u32* __restrict__ wfp, const i32* __restrict__ lenp,
    const unsigned char* __restrict__ ccp, i32 k, u32* __restrict__ ov_out, double* __restrict__ score_out,
    i32* __restrict__ topk_idx, double* __restrict__ topk_score) {
    const int lane = threadIdx.x & 63;
    const i64 tile = (i64)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (tile * 64 >= n) return;
    const i64 file = tile * 64 + lane;
    const bool valid = file < n;
    const uint4* fp = files + tile * (i64)(WQ * 64) + lane;
    const u32 wf = wfp[file];
    const i32 lf = lenp[file];
    const bool cc = ccp[file] != 0;
    FILE_PROLOGUE
    const bool fast = CORPUS_FAST && wf < (1u << 20) && lf >= 0 && lf < (1 << 21);
    i32 ti[KM]; u32 to[KM]; i32 td[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) { ti[j] = -1; to[j] = 0; td[j] = 1; }
    // template-major [NT][n] outputs: for a fixed template the 64 lanes store contiguously
    u32* orow = ov_out ? ov_out + file : nullptr;
    double* srow = score_out ? score_out + file : nullptr;
    if (__all(fast)) {
        MATRIX_BODY(true)
    } else {
        MATRIX_BODY(false)
    }
    if (valid && topk_idx) {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            if (j < k) {
                MSTORE(topk_idx + (i64)j * n + file, ti[j]);
                MSTORE(topk_score + (i64)j * n + file, ti[j] >= 0 ? sc(to[j], td[j]) : -1.0);
            }
        }
    }
}
)HIP";

// Per-template matrix epilogue: store the row entry, then rank-and-shift insertion into the
// KM sorted slots (p = slots that strictly outrank the candidate; a later template goes
// before equal-scored earlier ones, dice.rb:39). Branch-free selects only.
const char* kMatrixOffer = R"HIP(
#define MOFFER(T, CCF)                                                                  \
    {                                                                                   \
        if (valid) { if (orow) MSTORE(orow + (i64)(T) * n, a); if (srow) MSTORE(srow + (i64)(T) * n, sc(a, d)); } \
        if (!((CCF) && cc)) {                                                           \
            int p = 0;                                                                  \
            _Pragma("unroll") for (int j = 0; j < KM; ++j)                              \
                p += (ti[j] >= 0 && !ge<FASTV>(a, d, to[j], td[j])) ? 1 : 0;           \
            _Pragma("unroll") for (int j = KM - 1; j > 0; --j) {                        \
                const bool mv = j > p;                                                  \
                ti[j] = mv ? ti[j - 1] : ti[j];                                         \
                to[j] = mv ? to[j - 1] : to[j];                                         \
                td[j] = mv ? td[j - 1] : td[j];                                         \
            }                                                                           \
            _Pragma("unroll") for (int j = 0; j < KM; ++j) {                            \
                const bool put = j == p;                                                \
                ti[j] = put ? (T) : ti[j];                                              \
                to[j] = put ? a : to[j];                                                \
                td[j] = put ? d : td[j];                                                \
            }                                                                           \
        }                                                                               \
    }
)HIP";

uint64_t fnv1a(const std::string& s) {
    uint64_t h = 1469598103934665603ULL;
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ULL;
    }
    return h;
}

std::string lib_dir() {
    Dl_info info;
    if (dladdr((void*)&fnv1a, &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        size_t s = p.rfind('/');
        if (s != std::string::npos) return p.substr(0, s);
    }
    return ".";
}

std::string cache_dir() {
    const char* env = getenv("DICE_CACHE_DIR");
    std::string d = env && *env ? std::string(env) : lib_dir() + "/cache";
    mkdir(d.c_str(), 0755);
    return d;
}

bool read_file(const std::string& path, std::vector<char>& out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    out.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    return !out.empty();
}

}  // namespace

// Build the entry list (template-major, dword ascending) from the template bitsets.
static void build_entries(const dice_templates* t, int32_t w64, Program& p) {
    p.prog.clear();
    const int32_t w32 = w64 * 2;
    for (int32_t i = 0; i < t->n_templates; ++i) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(t->lf_bits + (size_t)i * w64);
        for (int32_t d = 0; d < w32; ++d)
            if (row[d]) p.prog.push_back(Entry{i, d, row[d]});
    }
}

// One dword-major accumulation statement (plain C; ACC_C_ONLY of acc_block).
static std::string acc_stmt(const Entry& en) {
    std::ostringstream o;
    if (en.mask == 0xFFFFFFFFu)
        o << "ACCF1(acc[" << en.tpl << "], f[" << en.dword % 4 << "]);\n";
    else
        o << "ACCM(acc[" << en.tpl << "], f[" << en.dword % 4 << "], 0x" << std::hex << en.mask << std::dec << ");\n";
    return o.str();
}

// A block of dword-major accumulations (entries of one quad) as ONE asm statement: the hazard
// recognizer pads every inline-asm boundary with an s_nop, so per-entry asm would cost an
// s_nop per v_and/v_bcnt pair. ACC_C_ONLY carries the plain-C form (host tests, ACC_ASM=0).
static std::string acc_block(const std::vector<Entry>& dm, size_t b, size_t e) {
    std::vector<int32_t> tpls;
    std::vector<int> fk;
    for (size_t i = b; i < e; ++i) {
        if (std::find(tpls.begin(), tpls.end(), dm[i].tpl) == tpls.end()) tpls.push_back(dm[i].tpl);
        const int k = dm[i].dword % 4;
        if (std::find(fk.begin(), fk.end(), k) == fk.end()) fk.push_back(k);
    }
    auto acc_op = [&](int32_t tpl) { return (int)(std::find(tpls.begin(), tpls.end(), tpl) - tpls.begin()); };
    // 4 temporaries: the v_and of up to 4 entries issue back to back, then their v_bcnt, so
    // no v_bcnt waits on the v_and right before it
    constexpr int kTmp = 4;
    const int tmp0 = (int)tpls.size();
    auto f_op = [&](int k) { return tmp0 + kTmp + (int)(std::find(fk.begin(), fk.end(), k) - fk.begin()); };
    std::ostringstream a, c;
    a << "ACC_ASM_ONLY(asm(\"";
    bool first = true;
    auto emit = [&](const std::string& ins) {
        if (!first) a << "\\n\\t";
        a << ins;
        first = false;
    };
    for (size_t g = b; g < e; g += kTmp) {
        const size_t ge = std::min(e, g + kTmp);
        for (size_t i = g; i < ge; ++i) {
            const Entry& en = dm[i];
            if (en.mask == 0xFFFFFFFFu) continue;
            std::ostringstream ins;
            ins << "v_and_b32 %" << tmp0 + (int)(i - g) << ", 0x" << std::hex << en.mask << std::dec << ", %"
                << f_op(en.dword % 4);
            emit(ins.str());
        }
        for (size_t i = g; i < ge; ++i) {
            const Entry& en = dm[i];
            std::ostringstream ins;
            const int src = en.mask == 0xFFFFFFFFu ? f_op(en.dword % 4) : tmp0 + (int)(i - g);
            ins << "v_bcnt_u32_b32 %" << acc_op(en.tpl) << ", %" << src << ", %" << acc_op(en.tpl);
            emit(ins.str());
        }
        for (size_t i = g; i < ge; ++i) c << acc_stmt(dm[i]);
    }
    a << "\" : ";
    for (size_t i = 0; i < tpls.size(); ++i) a << "\"+v\"(acc[" << tpls[i] << "]), ";
    for (int k = 0; k < kTmp; ++k) a << "\"=&v\"(t_[" << k << "])" << (k + 1 < kTmp ? ", " : "");
    a << " : ";
    for (size_t i = 0; i < fk.size(); ++i) a << (i ? ", " : "") << "\"v\"(f[" << fk[i] << "])";
    a << ");)";
    std::string cs = c.str();
    std::replace(cs.begin(), cs.end(), '\n', ' ');
    return "{ u32 t_[4]; " + a.str() + " ACC_C_ONLY(" + cs + ") (void)t_; }\n";
}

// Accumulations of one quad, in blocks of at most kAccBlock entries.
static std::string acc_quad(const std::vector<Entry>& dm, size_t b0, size_t end, int32_t q) {
    constexpr size_t kAccBlock = 4;   // entries per asm block (2 and 8 measured slower)
    std::string out;
    const char* diag = diag_env("DICE_PROG_DIAG");   // diagnostics only: results are wrong
    if (diag && strcmp(diag, "noacc") == 0) return "acc[" + std::to_string(q) + " % NT] ^= f[0] ^ f[1] ^ f[2] ^ f[3];\n";
    for (size_t b = b0; b < end; b += kAccBlock) out += acc_block(dm, b, std::min(end, b + kAccBlock));
    return out;
}


// Emits `text` as the body of a one-line-per-statement macro.
static void emit_macro(std::ostringstream& s, const std::string& head, const std::string& text) {
    s << "#define " << head << " \\\n";
    std::istringstream lines(text);
    std::string line;
    while (std::getline(lines, line)) s << line << " \\\n";
    s << "\n";
}

// Program order: dword-major -- every template accumulator stays live (acc[NT]); file quads are
// loaded in bursts right before they are consumed, so a file dword's live range is a few
// instructions; the epilogue (denominator, compare) runs once per template after the last quad.
// (The template-major order, the whole bitset loaded up front and each template retired in turn,
// measured 2% slower and is retired: DESIGN.md Appendix B.)
std::string program_source(const dice_templates* t, Program& p, int32_t wq, bool corpus_fast) {
    std::ostringstream s;
    s << "#define WPB " << p.wpb << "\n";
    s << "// dice sparse program: T=" << t->n_templates << " V=" << t->n_vocab << " entries=" << p.prog.size()
      << " order=d\n";
    s << "#define MATCH_WAVES \n";
    uint32_t max_lf = 0;
    for (int32_t i = 0; i < t->n_templates; ++i) max_lf = std::max(max_lf, t->lf_size[i]);
    // v_and/v_bcnt as asm blocks (ACC_ASM; host tests compile the plain-C form), non-temporal file
    // loads (FILE_NT) and outputs (OUT_NT: written once, never re-read; config 5 -1.9%, 3 reps)
    s << "#define ACC_ASM 1\n";
    s << "#define FILE_NT 1\n";
    s << "#define OUT_NT 1\n";
    s << "#define WQ " << wq << "\n#define NT " << t->n_templates << "\n#define CORPUS_FAST "
      << (corpus_fast ? 1 : 0) << "\n#define NARROW_MUL " << (max_lf < (1u << 11) ? 1 : 0) << "\n" << kPrelude;

    std::vector<std::string> den(t->n_templates);
    for (int32_t i = 0; i < t->n_templates; ++i) {
        const int32_t base = (int32_t)t->lf_size[i] - (int32_t)t->fields_set_size[i];
        std::ostringstream d;
        d << "d = dn(" << base << ", " << t->length_slack[i] << ", " << t->length[i] << ", wf, lf); ";
        den[i] = d.str();
    }
    auto offer = [&](int32_t i) {
        std::ostringstream o;
        if (t->is_cc[i]) o << "if (!cc) ";
        // a carries the template index in its top byte (ACC_INIT): one select moves index and
        // overlap together; v_mul_u32_u24 reads only the low 24 bits (the overlap)
        o << "{ if ((!FASTV && (bo >> 24) == 0xFFu) || ge<FASTV>(a, d, bo, bd)) { bo = a; bd = d; } }";
        return o.str();
    };
    std::ostringstream match_body, matrix_body, prologue;
    {
        std::vector<Entry> dm(p.prog);
        std::stable_sort(dm.begin(), dm.end(), [](const Entry& x, const Entry& y) {
            return x.dword != y.dword ? x.dword < y.dword : x.tpl < y.tpl;
        });
        prologue << "u32 acc[NT];\n_Pragma(\"unroll\") for (int i = 0; i < NT; ++i) acc[i] = ACC_INIT(i);\n";
        // quads the program touches, their entry ranges in dm and their VALU cost
        std::vector<int32_t> quads;
        std::vector<std::pair<size_t, size_t>> range;   // [begin, end) in dm, per quads[] slot
        std::vector<int> cost;
        for (size_t i = 0; i < dm.size(); ++i) {
            if (quads.empty() || quads.back() != dm[i].dword / 4) {
                quads.push_back(dm[i].dword / 4);
                range.push_back({i, i});
                cost.push_back(0);
            }
            range.back().second = i + 1;
            cost.back() += dm[i].mask == 0xFFFFFFFFu ? 1 : 2;
        }
        {   // processing order: alternating costliest and cheapest quads, which spreads the VALU
            // work evenly over the stream (the packed vocabulary puts the widely shared words --
            // 120-250 VALU per quad -- at the end, the rare ones at 4-40 first): -5.5% config 2 vs
            // memory order (costliest-first -4.4%, equal VALU per burst +-0)
            std::vector<size_t> idx(quads.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
            std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return cost[a] > cost[b]; });
            {
                std::vector<size_t> z;
                for (size_t lo = 0, hi = idx.size(); lo < hi;) {
                    z.push_back(idx[lo++]);
                    if (lo < hi) z.push_back(idx[--hi]);
                }
                idx.swap(z);
            }
            std::vector<int32_t> q2;
            std::vector<std::pair<size_t, size_t>> r2;
            for (size_t i : idx) {
                q2.push_back(quads[i]);
                r2.push_back(range[i]);
            }
            quads.swap(q2);
            range.swap(r2);
        }
        // Tile layout in processing order: tile slot i holds the vocabulary quad processed i-th
        // (dice_pack_tiles applies p.qperm), so a wave's loads walk its 28 KiB tile front to back
        // while the VALU work stays zipped.
        {
            p.qperm.clear();
            std::vector<char> seen((size_t)wq, 0);
            for (int32_t q : quads) {
                p.qperm.push_back(q);
                seen[(size_t)q] = 1;
            }
            for (int32_t q = 0; q < wq; ++q)
                if (!seen[(size_t)q]) p.qperm.push_back(q);   // quads no template reads (never loaded)
            for (size_t i = 0; i < quads.size(); ++i) quads[i] = (int32_t)i;
            s << "// QPERM";
            for (int32_t q : p.qperm) s << " " << q;
            s << "\n";
        }
        {
            // bursts: quads in groups of `nb` = 5, double-buffered in register sets p0_* / p1_*;
            // group g+1 is requested (nb contiguous 1 KiB wave loads back to back) before group g
            // is consumed. With non-temporal loads, bursts of 3 measured ~1.5% ahead of an 8-deep
            // ring at 92 instead of 124 VGPRs, 4 another ~3.5%, 5 another 1.8% (6: -0.3%)
            const int nb = std::max(1, std::min<int>(5, (int)quads.size()));
            const size_t ng = (quads.size() + nb - 1) / nb;
            auto group_loads = [&](std::ostringstream& o, size_t g, int set) {
                for (size_t i = g * nb; i < std::min(quads.size(), (g + 1) * nb); ++i)
                    o << "p" << set << "_" << (i - g * nb) << " = ldq(fp + " << quads[i] * 64 << "); ";
                o << "\n";
            };
            auto stream = [&](std::ostringstream& o) {
                for (size_t g = 0; g < ng; ++g) {
                    const int cur = (int)(g % 2), nxt = 1 - cur;
                    o << "__builtin_amdgcn_sched_barrier(0);\n";
                    if (g + 1 < ng) group_loads(o, g + 1, nxt);
                    o << "__builtin_amdgcn_sched_barrier(0);\n";
                    for (size_t i = g * nb; i < std::min(quads.size(), (g + 1) * nb); ++i) {
                        o << "{ const uint4 v = p" << cur << "_" << (i - g * nb) << "; const u32 f[4] = {v.x, v.y, v.z, v.w};\n";
                        o << acc_quad(dm, range[i].first, range[i].second, quads[i]);
                        o << "}\n";
                    }
                }
            };
            std::ostringstream decl;
            for (int i = 0; i < nb; ++i) decl << "uint4 p0_" << i << ", p1_" << i << ";\n";
            prologue << decl.str();
            group_loads(prologue, 0, 0);
            stream(prologue);
        }
        for (int32_t i = 0; i < t->n_templates; ++i) {
            match_body << "{ const u32 a = acc[" << i << "]; i32 d; " << den[i] << offer(i) << " }\n";
            matrix_body << "{ const u32 a = acc[" << i << "]; i32 d; " << den[i] << "MOFFER(" << i << ", "
                        << (t->is_cc[i] ? 1 : 0) << ") }\n";
        }
    }
    emit_macro(s, "FILE_PROLOGUE", prologue.str());
    const char* diag = diag_env("DICE_PROG_DIAG");   // diagnostics only: results are wrong
    s << "#define WAVE_TIMING " << (diag && strcmp(diag, "timing") == 0 ? 1 : 0) << "\n";
    if (diag && strcmp(diag, "noepi") == 0) {
        std::ostringstream mb;
        mb << "bd = 1; bo = 0; _Pragma(\"unroll\") for (int i = 0; i < NT; ++i) bo += acc[i];\n";
        match_body.str(mb.str());
    }
    emit_macro(s, "MATCH_BODY(FASTV_) { constexpr bool FASTV = FASTV_;", match_body.str() + "}");
    s << "#define ACC_INIT(i) ((u32)(i) << 24)\n" << kMatchKernel
      << "#undef ACC_INIT\n#define ACC_INIT(i) 0u\n";
    s << kMatrixOffer;
    emit_macro(s, "MATRIX_BODY(FASTV_) { constexpr bool FASTV = FASTV_;", matrix_body.str() + "}");
    for (int km : {4, 16}) {
        s << "#define KM " << km << "\n#define KNAME dice_prog_matrix" << km << "\n" << kMatrixKernel
          << "#undef KM\n#undef KNAME\n";
    }
    return s.str();
}

// Compile (or find in the cache) the code object for `src`. No device needed.
static int compile_cached(const std::string& src, std::vector<char>& code, std::string* path_out) {
    const uint64_t h = fnv1a(src);
    char name[64];
    snprintf(name, sizeof(name), "dice_prog_%016llx.co", (unsigned long long)h);
    const std::string path = cache_dir() + "/" + name;
    if (!read_file(path, code)) {
        hiprtcProgram prog;
        if (hiprtcCreateProgram(&prog, src.c_str(), "dice_prog.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
            return fail(DICE_E_DEVICE, "hiprtcCreateProgram failed");
        const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
        hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
        if (r != HIPRTC_SUCCESS) {
            size_t ls = 0;
            hiprtcGetProgramLogSize(prog, &ls);
            std::string log(ls, '\0');
            if (ls) hiprtcGetProgramLog(prog, &log[0]);
            hiprtcDestroyProgram(&prog);
            return fail(DICE_E_DEVICE, "hiprtc compile failed: " + log.substr(0, 2000));
        }
        size_t cs = 0;
        hiprtcGetCodeSize(prog, &cs);
        code.resize(cs);
        hiprtcGetCode(prog, code.data());
        hiprtcDestroyProgram(&prog);
        // best-effort cache write (atomic rename)
        const std::string tmp = path + ".tmp." + std::to_string(getpid());
        {
            std::ofstream out(tmp, std::ios::binary);
            if (out) out.write(code.data(), (std::streamsize)code.size());
        }
        rename(tmp.c_str(), path.c_str());
    }
    if (path_out) *path_out = path;
    return DICE_OK;
}

static int compile_or_load(dice_ctx* c, const std::string& src) {
    std::vector<char> code;
    int rc = compile_cached(src, code, nullptr);
    if (rc != DICE_OK) return rc;
    if (hipModuleLoadData(&c->module, code.data()) != hipSuccess) return fail(DICE_E_DEVICE, "hipModuleLoadData failed");
    if (hipModuleGetFunction(&c->prog_match, c->module, "dice_prog_match") != hipSuccess ||
        hipModuleGetFunction(&c->prog_matrix, c->module, "dice_prog_matrix4") != hipSuccess ||
        hipModuleGetFunction(&c->prog_matrix16, c->module, "dice_prog_matrix16") != hipSuccess)
        return fail(DICE_E_DEVICE, "hipModuleGetFunction failed");
    return DICE_OK;
}

static bool corpus_in_fast_envelope(const dice_templates* t) {
    // static fast-path envelope (dice_common.h): base >= 1, base < 2^18, len < 2^20,
    // 200*|Lf| < 1024*base  =>  every fast-file denominator is in [1, 2^21), scores < 1024.
    for (int32_t i = 0; i < t->n_templates; ++i) {
        const int64_t base = (int64_t)t->lf_size[i] - (int64_t)t->fields_set_size[i];
        if (!(base >= 1 && base < (1 << 18) && t->length[i] >= 0 && t->length[i] < (1 << 20) &&
              200 * (int64_t)t->lf_size[i] < 1024 * base))
            return false;
    }
    return true;
}

static std::string source_for(const dice_templates* t, Program& prog) {
    const int32_t w64 = (t->n_vocab + 63) / 64;
    build_entries(t, w64, prog);
    prog.wpb = 4;   // waves per workgroup (1, 2 and 8 within +-1.5%)
    return program_source(t, prog, (w64 + 1) / 2, corpus_in_fast_envelope(t));
}

bool program_wanted(const dice_templates* t) {
    const char* force = getenv("DICE_FORCE_DENSE");
    return !(force && *force == '1') && t->n_templates <= kProgramMaxTemplates;
}

int program_setup(dice_ctx* c, const dice_templates* t) {
    c->kind = 0;
    if (!program_wanted(t)) return DICE_OK;
    const std::string src = source_for(t, c->prog);
    int rc = compile_or_load(c, src);
    if (rc != DICE_OK) return rc;
    if (!c->prog.qperm.empty()) {
        const size_t bytes = c->prog.qperm.size() * sizeof(int32_t);
        if (c->prog.qperm.size() != (size_t)c->wq) return fail(DICE_E_STATE, "program tile permutation size");
        if ((rc = dalloc_bytes(reinterpret_cast<void**>(&c->d_qperm), bytes)) != DICE_OK) return rc;
        if (hipMemcpy(c->d_qperm, c->prog.qperm.data(), bytes, hipMemcpyHostToDevice) != hipSuccess)
            return fail(DICE_E_DEVICE, "program tile permutation upload failed");
    }
    c->kind = 1;
    return DICE_OK;
}

int program_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s) {
    const int64_t n_tiles = (b->n + 63) / 64;
    const int32_t wpb = c->prog.wpb;
    const unsigned grid = (unsigned)((n_tiles + wpb - 1) / wpb);
    hipFunction_t fn = c->prog_match;
    int64_t n = b->n;
    void* args[] = {&b->d_tiles, &n, &b->d_wf, &b->d_len, &b->d_cc, &thr, &b->d_best, &b->d_ov, &b->d_score};
    if (hipModuleLaunchKernel(fn, grid, 1, 1, 64 * wpb, 1, 1, 0, s, args, nullptr) != hipSuccess)
        return fail(DICE_E_DEVICE, "launch dice_prog_match failed");
    return DICE_OK;
}

int program_launch_matrix(dice_ctx* c, dice_batch* b, int32_t k, hipStream_t s) {
    const int64_t n_tiles = (b->n + 63) / 64;
    const int32_t wpb = c->prog.wpb;
    const unsigned grid = (unsigned)((n_tiles + wpb - 1) / wpb);
    int64_t n = b->n;
    int32_t kk = k;
    int32_t* tki = k > 0 ? b->d_tki : nullptr;
    double* tks = k > 0 ? b->d_tks : nullptr;
    void* args[] = {&b->d_tiles, &n, &b->d_wf, &b->d_len, &b->d_cc, &kk, &b->d_mov, &b->d_mscore, &tki, &tks};
    hipFunction_t fn = k <= 4 ? c->prog_matrix : c->prog_matrix16;
    if (hipModuleLaunchKernel(fn, grid, 1, 1, 64 * wpb, 1, 1, 0, s, args, nullptr) != hipSuccess)
        return fail(DICE_E_DEVICE, "launch dice_prog_matrix failed");
    return DICE_OK;
}

}  // namespace dice

extern "C" int dice_precompile(const dice_templates* t, char* path, int32_t path_cap) {
    if (!t || t->n_templates < 1 || t->n_vocab < 1 || !t->lf_bits) return dice::fail(DICE_E_ARG, "invalid dice_templates");
    if (!dice::program_wanted(t)) return dice::fail(DICE_E_STATE, "corpus uses the dense kernel");
    dice::Program prog;
    const std::string src = dice::source_for(t, prog);
    std::vector<char> code;
    std::string p;
    int rc = dice::compile_cached(src, code, &p);
    if (rc == DICE_OK && path && path_cap > 0) snprintf(path, (size_t)path_cap, "%s", p.c_str());
    return rc;
}

extern "C" int64_t dice_program_source(const dice_templates* t, char* buf, int64_t cap) {
    if (!t || t->n_templates < 1 || t->n_vocab < 1 || !t->lf_bits) return -1;
    dice::Program prog;
    const std::string src = dice::source_for(t, prog);
    if (buf && cap > 0) {
        const size_t n = std::min<size_t>((size_t)cap - 1, src.size());
        memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return (int64_t)src.size();
}
