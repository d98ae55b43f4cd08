// MI355X (gfx950) Dice scorer: kernels + C-ABI (include/licensee_dice.h).
//
// Hot path replaced: lib/licensee/matchers/dice.rb:34-53 looping
// License#similarity (lib/licensee/content_helper.rb:128-133,337-347) over every template.
//
// Device layout (HBM):
//   files   : tile layout [n_tiles][Wq][64 lanes] of uint4 -- one wave owns a tile of 64 files,
//             lane l holds file (tile*64 + l); quad q carries vocab bits [128q, 128q+128).
//             Every wave-instruction loads 1 KiB contiguous (global_load_dwordx4, coalesced).
//   scalars : |W_F| (u32), len_F (i32), cc flag (u8), SoA, padded to n_tiles*64.
//   tpl     : [Wq][Tpad] uint4 template quads (uniform -> scalar loads into SGPRs) + TplConst.
//   results : best (i32), overlap (u32), score (f64) per file, SoA.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <link.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/licensee_dice.h"
#include "dice_common.h"
#include "dice_internal.h"

using namespace dice;

namespace dice {
std::string& last_error() {
    static thread_local std::string err;
    return err;
}
}  // namespace dice

// ---------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------

// Row-major uint64 bitsets [n][W64] -> tile layout [n_tiles][Wq][64] uint4 (zero padded).
__global__ __launch_bounds__(256) void dice_pack_tiles(const uint64_t* __restrict__ rows, int64_t n,
                                                       int32_t w64, int32_t wq, const int32_t* __restrict__ qperm,
                                                       uint4* __restrict__ tiles, int64_t n_tiles) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = n_tiles * wq * kWave;
    if (gid >= total) return;
    const int lane = (int)(gid & (kWave - 1));
    const int64_t tq = gid >> 6;
    const int slot = (int)(tq % wq);
    const int q = qperm ? qperm[slot] : slot;   // tile slot -> vocabulary quad (sparse program order)
    const int64_t tile = tq / wq;
    const int64_t file = tile * kWave + lane;
    uint64_t a = 0, b = 0;
    if (file < n) {
        const uint64_t* r = rows + file * w64;
        if (2 * q < w64) a = r[2 * q];
        if (2 * q + 1 < w64) b = r[2 * q + 1];
    }
    tiles[gid] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

// Word-id lists -> row-major bitsets: one wave per file builds its row in LDS (ds_or_b64 per
// id, ids >= V ignored), then writes the whole row (coalesced, every word, zeros included).
template <class Id>
__global__ __launch_bounds__(256) void dice_rows_from_ids(const int64_t* __restrict__ offs, const Id* __restrict__ ids,
                                                          int64_t n, int32_t w64, uint32_t V,
                                                          uint64_t* __restrict__ rows) {
    extern __shared__ uint64_t lrow[];   // [4 waves][w64]
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x >> 6;
    const int64_t file = (int64_t)blockIdx.x * 4 + wave;
    if (file >= n) return;   // wave-uniform; no block barrier below
    uint64_t* r = lrow + (size_t)wave * w64;
    for (int32_t j = lane; j < w64; j += kWave) r[j] = 0;
    const int64_t a = offs[file], b = offs[file + 1];
    for (int64_t e = a + lane; e < b; e += kWave) {
        const uint32_t id = (uint32_t)ids[e];
        if (id < V) atomicOr(reinterpret_cast<unsigned long long*>(&r[id >> 6]), 1ull << (id & 63));
    }
    uint64_t* out = rows + file * w64;
    for (int32_t j = lane; j < w64; j += kWave) out[j] = r[j];
}

// [rows][cols] -> [cols][rows] through a padded 64x64 LDS tile (element size 4 or 8 bytes).
// Used to hand the template-major device matrix back in the ABI's row-major [n][T] layout.
template <class E>
__global__ __launch_bounds__(256) void dice_transpose(const E* __restrict__ src, E* __restrict__ dst,
                                                     int64_t rows, int64_t cols) {
    __shared__ E tile[64][65];
    const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {
        const int64_t r = r0 + i, c = c0 + tx;
        if (r < rows && c < cols) tile[i][tx] = src[r * cols + c];
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        const int64_t c = c0 + i, r = r0 + tx;
        if (r < rows && c < cols) dst[c * rows + r] = tile[tx][i];
    }
}

// Diagnostic: pure streaming read of the resident tile layout (same addresses and widths as
// the scorers, trivial compute, 16 B written per file). Measures the read ceiling that the
// Dice kernels are judged against (DESIGN.md "roofline").
__global__ __launch_bounds__(256) void dice_stream_probe(const uint4* __restrict__ files, int64_t n, int32_t wq,
                                                         uint4* __restrict__ out) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (tile * kWave >= n) return;
    const uint4* fp = files + tile * (int64_t)wq * kWave + lane;
    uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll 8
    for (int q = 0; q < wq; ++q) {
        const uint4 v = fp[(int64_t)q * kWave];
        x.x ^= v.x; x.y ^= v.y; x.z ^= v.z; x.w ^= v.w;
    }
    const int64_t file = tile * kWave + lane;
    if (file < n) out[file] = x;
}

// acc += popcount(f & m) over a quad: v_and_b32 (template dword from an SGPR) + v_bcnt_u32_b32
// accumulate, 8 VALU per quad (the compiler's own form, v_bcnt(x, 0) + v_add3 trees, is 10).
__device__ __forceinline__ void acc_and4(uint32_t& acc, uint4 f, uint4 m) {
    uint32_t t0, t1, t2, t3;
    asm("v_and_b32 %1, %5, %9\n\tv_and_b32 %2, %6, %10\n\tv_and_b32 %3, %7, %11\n\tv_and_b32 %4, %8, %12\n\t"
        "v_bcnt_u32_b32 %0, %1, %0\n\tv_bcnt_u32_b32 %0, %2, %0\n\tv_bcnt_u32_b32 %0, %3, %0\n\t"
        "v_bcnt_u32_b32 %0, %4, %0"
        : "+v"(acc), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
        : "s"(m.x), "s"(m.y), "s"(m.z), "s"(m.w), "v"(f.x), "v"(f.y), "v"(f.z), "v"(f.w));
}

// Dense scorer: any T, any V. Templates are uniform across the wave, so the compiler keeps
// them on the scalar path (s_load -> SGPR operand of v_and_b32); file quads stream through
// VGPRs. TT templates are accumulated per pass (compile-time register array).
template <int TT>
__global__ __launch_bounds__(256) void dice_dense_match(
    const uint4* __restrict__ files, int64_t n, int32_t wq, const uint4* __restrict__ tq,
    const int4* __restrict__ tc, int32_t T, int32_t tpad, const uint32_t* __restrict__ wf,
    const int32_t* __restrict__ lenf, const uint8_t* __restrict__ ccfp, double thr,
    int32_t* __restrict__ best_out, uint32_t* __restrict__ ov_out, double* __restrict__ score_out) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (tile * kWave >= n) return;  // wave-uniform
    const int64_t file = tile * kWave + lane;
    const uint4* fp = files + tile * (int64_t)wq * kWave + lane;
    const uint32_t my_wf = wf[file];
    const int32_t my_len = lenf[file];
    const bool my_cc = ccfp[file] != 0;

    Best best;
    best.init();
    for (int t0 = 0; t0 < T; t0 += TT) {
        uint32_t acc[TT];
#pragma unroll
        for (int j = 0; j < TT; ++j) acc[j] = 0;
        const uint4* mrow = tq + t0;
        for (int q = 0; q < wq; ++q) {
            const uint4 f = fp[(int64_t)q * kWave];
#pragma unroll
            for (int j = 0; j < TT; ++j) acc_and4(acc[j], f, mrow[j]);
            mrow += tpad;
        }
#pragma unroll
        for (int j = 0; j < TT; ++j) {
            const int t = t0 + j;
            if (t < T) {
                const int4 c = tc[t];
                if (!(c.w && my_cc)) best.offer(t, acc[j], dice_den(c, my_wf, my_len));
            }
        }
    }
    if (file < n) {
        const double s = best.idx >= 0 ? dice_score(best.ov, best.den) : 0.0;
        best_out[file] = (best.idx >= 0 && s >= thr) ? best.idx : -1;
        ov_out[file] = best.ov;
        score_out[file] = s;
    }
}

template <int TT, int KM>
__global__ __launch_bounds__(256) void dice_dense_matrix(
    const uint4* __restrict__ files, int64_t n, int32_t wq, const uint4* __restrict__ tq,
    const int4* __restrict__ tc, int32_t T, int32_t tpad, const uint32_t* __restrict__ wf,
    const int32_t* __restrict__ lenf, const uint8_t* __restrict__ ccfp, int32_t k,
    uint32_t* __restrict__ ov_out, double* __restrict__ score_out, int32_t* __restrict__ topk_idx,
    double* __restrict__ topk_score) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (tile * kWave >= n) return;
    const int64_t file = tile * kWave + lane;
    const bool valid = file < n;
    const uint4* fp = files + tile * (int64_t)wq * kWave + lane;
    const uint32_t my_wf = wf[file];
    const int32_t my_len = lenf[file];
    const bool my_cc = ccfp[file] != 0;

    TopK<KM> top;
    top.init();
    for (int t0 = 0; t0 < T; t0 += TT) {
        uint32_t acc[TT];
#pragma unroll
        for (int j = 0; j < TT; ++j) acc[j] = 0;
        const uint4* mrow = tq + t0;
        for (int q = 0; q < wq; ++q) {
            const uint4 f = fp[(int64_t)q * kWave];
#pragma unroll
            for (int j = 0; j < TT; ++j) acc_and4(acc[j], f, mrow[j]);
            mrow += tpad;
        }
#pragma unroll
        for (int j = 0; j < TT; ++j) {
            const int t = t0 + j;
            if (t < T) {
                const int4 c = tc[t];
                const int32_t den = dice_den(c, my_wf, my_len);
                if (valid) {
                    if (ov_out) ov_out[(int64_t)t * n + file] = acc[j];   // template-major [T][n]
                    if (score_out) score_out[(int64_t)t * n + file] = dice_score(acc[j], den);
                }
                if (!(c.w && my_cc)) top.offer(t, acc[j], den);
            }
        }
    }
    if (valid && topk_idx) {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            if (j < k) {
                topk_idx[(int64_t)j * n + file] = top.idx[j];
                topk_score[(int64_t)j * n + file] = top.idx[j] >= 0 ? dice_score(top.ov[j], top.den[j]) : -1.0;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
namespace {

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(DICE_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

constexpr int kTT = 48;        // templates per dense pass
constexpr int kBlock = 256;    // 4 waves, one 64-file tile each

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <class T>
int dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) return fail(DICE_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return DICE_OK;
}

}  // namespace

static hipStream_t pick_stream(dice_ctx* ctx, void* s) { return s ? (hipStream_t)s : ctx->stream; }

// A/B switch read per call (e.g. DICE_NO_SMALL_CALL=1: the small calls take the general path)
static bool getenv_flag(const char* name) {
    const char* v = getenv(name);
    return v && *v && *v != '0';
}

template <class E>
static int transpose_to(dice_batch* b, const E* d_src, int64_t rows, int64_t cols, E* dst, hipStream_t s,
                        hipMemcpyKind kind) {
    // rows x cols (template-major) -> cols x rows on device, then a copy to `dst` (host memory,
    // or another device's memory for the sharded device gather)
    const size_t bytes = (size_t)rows * cols * sizeof(E);
    if (b->stage_bytes < bytes) {
        if (b->d_stage) (void)hipFree(b->d_stage);
        b->d_stage = nullptr;
        b->stage_bytes = 0;
        if (hipMalloc(&b->d_stage, bytes) != hipSuccess) return fail(DICE_E_NOMEM, "stage alloc");
        b->stage_bytes = bytes;
    }
    dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
    hipLaunchKernelGGL(dice_transpose<E>, grid, dim3(256), 0, s, d_src, (E*)b->d_stage, rows, cols);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(dst, b->d_stage, bytes, kind, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DICE_OK;
}


// The per-file scalars and, for the tile-layout kernels, the repack (the rows are in b->d_rows).
// wf == NULL: |W_F| is already on the device (dice_batch_upload_text) and b->n_long is set.
int dice::upload_tail(dice_batch* b, int64_t n, const uint32_t* wf, const int32_t* len, const uint8_t* cc,
                      hipStream_t s) {
    dice_ctx* c = b->ctx;
    const int64_t n_tiles = (n + kWave - 1) / kWave;
    const int64_t npad = n_tiles * kWave;
    b->fmask_device = wf == nullptr;
    if (wf) HIP_TRY(hipMemcpyAsync(b->d_wf, wf, (size_t)n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(b->d_len, len, (size_t)n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(b->d_cc, cc, (size_t)n, hipMemcpyHostToDevice, s));
    if (npad > n) {
        HIP_TRY(hipMemsetAsync(b->d_wf + n, 0, (size_t)(npad - n) * 4, s));
        HIP_TRY(hipMemsetAsync(b->d_len + n, 0, (size_t)(npad - n) * 4, s));
        HIP_TRY(hipMemsetAsync(b->d_cc + n, 0, (size_t)(npad - n), s));
    }
    if (c->kind == 3) {   // the postings kernel reads the row-major bitsets
        if (!wf) return DICE_OK;
        b->n_long = 0;
        if (c->prune)
            for (int64_t i = 0; i < n; ++i) b->n_long += wf[i] > c->prune_max_lf;
        return DICE_OK;
    }
    return dice::repack(b, s);
}

// The tile-layout kernels' repack of the batch's row-major bitsets (kinds 0-2).
int dice::repack(dice_batch* b, hipStream_t s) {
    dice_ctx* c = b->ctx;
    if (c->kind == 3 || b->n == 0) return DICE_OK;
    const int64_t n_tiles = (b->n + kWave - 1) / kWave;
    const int64_t total = n_tiles * c->wq * kWave;
    const unsigned grid = (unsigned)((total + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(dice_pack_tiles, dim3(grid), dim3(kBlock), 0, s, b->d_rows, b->n, c->w64, c->wq,
                       c->kind == 1 ? (const int32_t*)c->d_qperm : nullptr, b->d_tiles, n_tiles);
    HIP_TRY(hipGetLastError());
    return DICE_OK;
}

extern "C" {

int32_t dice_words64(int32_t n_vocab) { return n_vocab <= 0 ? 0 : (n_vocab + 63) / 64; }

const char* dice_last_error(void) { return dice::last_error().c_str(); }

static void ctx_free(dice_ctx* c) {
    if (!c) return;
    if (c->scratch) dice_batch_destroy(c->scratch);
    if (c->small) dice_batch_destroy(c->small);
    if (c->h_small_in) (void)hipHostFree(c->h_small_in);
    if (c->h_small_out) (void)hipHostFree(c->h_small_out);
    if (c->d_tq) (void)hipFree(c->d_tq);
    if (c->d_tc) (void)hipFree(c->d_tc);
    if (c->d_qperm) (void)hipFree(c->d_qperm);
    void* plan[] = {c->d_lrec, c->d_lep,  c->d_les,  c->d_lwt,   c->d_pdmt,  c->d_prow,  c->d_povf,
                    c->d_ptc,  c->d_p4q8, c->d_p4tc, c->d_p4cc,  c->d_p4off, c->d_p4rec, c->d_p4slot};
    for (void* p : plan)
        if (p) (void)hipFree(p);
    if (c->module) (void)hipModuleUnload(c->module);
    for (int i = 0; i < 2; ++i) {
        if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
        if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
    }
    dice::exact_free(c);
    dice::words_free(c);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// One HIP runtime per process. The library binds libamdhip64.so.7 by soname, so it shares the
// runtime of a host that loaded one first (torch ships its own copy under that soname). A host
// that maps a second copy after this library -- a different file, so a second HSA runtime with
// its own view of the devices -- can find no GPU. Refuse to create a context once two distinct
// runtime files are mapped, naming both, instead of failing later in the other runtime.
static int check_hip_runtime(std::string* ours) {
    Dl_info di;
    if (dladdr(reinterpret_cast<void*>(&hipGetDeviceCount), &di) && di.dli_fname) *ours = di.dli_fname;
    struct Seen {
        std::vector<std::pair<dev_t, ino_t>> ids;
        std::vector<std::string> paths;
    } seen;
    dl_iterate_phdr(
        [](dl_phdr_info* info, size_t, void* p) -> int {
            auto* s = static_cast<Seen*>(p);
            const char* name = info->dlpi_name;
            const char* base = name ? std::strrchr(name, '/') : nullptr;
            base = base ? base + 1 : name;
            struct stat st;
            if (!base || std::strncmp(base, "libamdhip64.so", 14) != 0 || stat(name, &st) != 0) return 0;
            for (auto& id : s->ids)
                if (id.first == st.st_dev && id.second == st.st_ino) return 0;
            s->ids.emplace_back(st.st_dev, st.st_ino);
            s->paths.emplace_back(name);
            return 0;
        },
        &seen);
    if (seen.paths.size() > 1) {
        std::string msg = "two HIP runtimes are mapped in this process (";
        for (size_t i = 0; i < seen.paths.size(); ++i) msg += (i ? ", " : "") + seen.paths[i];
        msg += "); liblicensee_dice.so uses " + *ours +
               ": load the host's HIP runtime (e.g. torch's) before liblicensee_dice.so";
        return fail(DICE_E_DEVICE, msg);
    }
    return DICE_OK;
}

int dice_create(const dice_templates* t, int32_t device, dice_ctx** out) {
    if (!out) return fail(DICE_E_ARG, "out is NULL");
    *out = nullptr;
    if (!t || t->n_templates < 1 || t->n_vocab < 1 || !t->lf_bits || !t->lf_size ||
        !t->fields_set_size || !t->length_slack || !t->length || !t->is_cc)
        return fail(DICE_E_ARG, "invalid dice_templates");
    std::string runtime = "libamdhip64";
    if (int rc = check_hip_runtime(&runtime)) return rc;
    int ndev = 0;
    const hipError_t ec = hipGetDeviceCount(&ndev);
    if (ec != hipSuccess || ndev < 1) {
        (void)hipGetLastError();
        return fail(DICE_E_DEVICE, "the HIP runtime " + runtime + " reports no device" +
                                       (ec != hipSuccess ? std::string(" (") + hipGetErrorString(ec) + ")" : ""));
    }
    if (device < 0 || device >= ndev) return fail(DICE_E_DEVICE, "device ordinal out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(DICE_E_DEVICE, std::string("requires gfx950, found ") + prop.gcnArchName);
    DeviceGuard g(device);
    if (!g.ok) return fail(DICE_E_DEVICE, "hipSetDevice failed");

    dice_ctx* c = new (std::nothrow) dice_ctx();
    if (!c) return fail(DICE_E_NOMEM, "ctx alloc");
    c->device = device;
    c->T = t->n_templates;
    c->V = t->n_vocab;
    c->w64 = dice_words64(t->n_vocab);
    c->wq = (c->w64 + 1) / 2;
    c->tpad = ((c->T + kTT - 1) / kTT) * kTT;
    c->h_lf.assign(t->lf_bits, t->lf_bits + (size_t)c->T * c->w64);   // Exact tables (dice_exact.hip)
    int rc;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        ctx_free(c);
        return fail(DICE_E_DEVICE, "hipStreamCreate failed");
    }
    std::vector<uint4> hq((size_t)c->wq * c->tpad, make_uint4(0, 0, 0, 0));
    std::vector<int4> hc((size_t)c->tpad, make_int4(0, 0, 0, 0));
    for (int32_t i = 0; i < c->T; ++i) {
        const uint64_t* r = t->lf_bits + (size_t)i * c->w64;
        for (int32_t q = 0; q < c->wq; ++q) {
            uint64_t a = r[2 * q], b = (2 * q + 1 < c->w64) ? r[2 * q + 1] : 0;
            hq[(size_t)q * c->tpad + i] =
                make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
        }
        hc[i] = make_int4((int32_t)t->lf_size[i] - (int32_t)t->fields_set_size[i], t->length_slack[i],
                          t->length[i], t->is_cc[i] ? 1 : 0);
    }
    if ((rc = dalloc(&c->d_tq, hq.size())) || (rc = dalloc(&c->d_tc, hc.size()))) {
        ctx_free(c);
        return rc;
    }
    if (hipMemcpy(c->d_tq, hq.data(), hq.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_tc, hc.data(), hc.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess) {
        ctx_free(c);
        return fail(DICE_E_DEVICE, "template upload failed");
    }
    // Sparse-program kernel for small corpora (see dice_program.h).
    rc = dice::program_setup(c, t);  // selects kind 1 when T <= kProgramMaxTemplates
    if (rc == DICE_OK && c->kind == 0 && c->T > kProgramMaxTemplates) {
        // Large corpora: the postings kernel (dice_post.hip) where its LDS budget allows, else
        // the LDS-tiled record kernel (dice_lds.hip). DICE_LARGE_KERNEL=lds|post|dense picks one
        // (A/B and tests); DICE_FORCE_DENSE=1 keeps the dense kernel.
        const char* force = getenv("DICE_FORCE_DENSE");
        const char* pick = getenv("DICE_LARGE_KERNEL");
        const std::string want = pick && *pick ? pick : "post";
        if (!(force && *force == '1') && want != "dense") {
            if (want == "post" && dice::post_feasible(t)) {
                rc = dice::post_setup(c, t);
                if (rc == DICE_OK) rc = dice::prune_setup(c, t);   // match mode (DICE_POST_PRUNE=0: off)
            }
            else rc = dice::lds_setup(c, t);
        }
    }
    if (rc != DICE_OK) {
        ctx_free(c);
        return rc;
    }
    *out = c;
    return DICE_OK;
}

void dice_destroy(dice_ctx* ctx) {
    if (!ctx) return;
    DeviceGuard g(ctx->device);
    ctx_free(ctx);
}

int dice_ctx_info(const dice_ctx* ctx, int32_t* T, int32_t* V, int32_t* kind, int32_t* entries) {
    if (!ctx) return fail(DICE_E_ARG, "ctx is NULL");
    if (T) *T = ctx->T;
    if (V) *V = ctx->V;
    if (kind) *kind = ctx->kind;
    if (entries)
        *entries = ctx->kind == 2 ? (int32_t)ctx->lds_entries
                 : ctx->kind == 3 ? (int32_t)ctx->post_rows : (int32_t)ctx->prog.entries();
    return DICE_OK;
}

int32_t dice_ctx_match_kernel(const dice_ctx* ctx) {
    if (!ctx) return -1;
    return ctx->kind == 3 && ctx->prune ? 4 : ctx->kind;
}

void dice_batch_destroy(dice_batch* b) {
    if (!b) return;
    DeviceGuard g(b->ctx->device);
    if (b->d_in) {   // carved small-call batch: the regions own these
        b->d_wf = nullptr; b->d_len = nullptr; b->d_cc = nullptr; b->d_rows = nullptr;
        (void)hipFree(b->d_in);
    }
    if (b->d_out) {
        b->d_best = nullptr; b->d_ov = nullptr; b->d_score = nullptr;
        b->d_mov = nullptr; b->d_mscore = nullptr; b->d_tki = nullptr; b->d_tks = nullptr;
        (void)hipFree(b->d_out);
    }
    void* ptrs[] = {b->d_rows, b->d_tiles, b->d_wf,  b->d_len,    b->d_cc,    b->d_best,  b->d_ov,   b->d_score,
                    b->d_mov,  b->d_mscore, b->d_tki, b->d_tks, b->d_stage, b->d_pdense, b->d_ids, b->d_offs,
                    b->d_defer, b->d_ndefer, b->d_nscored, b->d_exact, b->d_fmask, b->d_text, b->d_toff,
                    b->d_tlen, b->d_wstat, b->d_wcnt};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete b;
}

int dice_batch_create(dice_ctx* ctx, int64_t capacity, dice_batch** out) {
    if (!ctx || !out || capacity < 1) return fail(DICE_E_ARG, "invalid batch arguments");
    *out = nullptr;
    DeviceGuard g(ctx->device);
    dice_batch* b = new (std::nothrow) dice_batch();
    if (!b) return fail(DICE_E_NOMEM, "batch alloc");
    b->ctx = ctx;
    b->capacity = capacity;
    b->n_tiles_cap = (capacity + kWave - 1) / kWave;
    const int64_t npad = b->n_tiles_cap * kWave;
    int rc;
    if ((rc = dalloc(&b->d_rows, (size_t)capacity * ctx->w64)) ||
        (rc = dalloc(&b->d_tiles, (size_t)b->n_tiles_cap * ctx->wq * kWave)) ||
        (rc = dalloc(&b->d_wf, npad)) || (rc = dalloc(&b->d_len, npad)) || (rc = dalloc(&b->d_cc, npad)) ||
        (rc = dalloc(&b->d_best, npad)) || (rc = dalloc(&b->d_ov, npad)) || (rc = dalloc(&b->d_score, npad)) ||
        (ctx->prune && (rc = dice::prune_reserve(ctx, b)))) {
        dice_batch_destroy(b);
        return rc;
    }

    *out = b;
    return DICE_OK;
}

int64_t dice_batch_bytes_per_file(const dice_batch* b) {
    if (!b) return -1;
    return (int64_t)b->ctx->wq * 16;
}

int dice_batch_upload(dice_batch* b, const dice_files* f, void* stream) {
    if (!b || !f) return fail(DICE_E_ARG, "NULL batch/files");
    dice_ctx* c = b->ctx;
    if (f->n_files < 0 || f->n_files > b->capacity) return fail(DICE_E_ARG, "n_files exceeds batch capacity");
    if (f->n_files > 0 && (!f->bits || !f->wordset_size || !f->length || !f->cc_false_positive))
        return fail(DICE_E_ARG, "NULL file arrays");
    DeviceGuard g(c->device);
    hipStream_t s = pick_stream(c, stream);
    const int64_t n = f->n_files;
    b->n = n;
    b->n_long = 0;
    b->fmask_device = false;
    if (n == 0) return DICE_OK;
    HIP_TRY(hipMemcpyAsync(b->d_rows, f->bits, (size_t)n * c->w64 * 8, hipMemcpyHostToDevice, s));
    return dice::upload_tail(b, n, f->wordset_size, f->length, f->cc_false_positive, s);
}

}  // extern "C"

// dice_batch_upload for rows the caller already copied into b->d_rows on stream `s` (the
// sharded path's pinned staging): the scalars and the repack.
int dice::upload_rows_resident(dice_batch* b, const dice_files* f, hipStream_t s) {
    if (f->n_files < 0 || f->n_files > b->capacity) return fail(DICE_E_ARG, "n_files exceeds batch capacity");
    DeviceGuard g(b->ctx->device);
    b->n = f->n_files;
    b->n_long = 0;
    b->fmask_device = false;
    if (b->n == 0) return DICE_OK;
    return upload_tail(b, b->n, f->wordset_size, f->length, f->cc_false_positive, s);
}

extern "C" {

int dice_batch_upload_ids(dice_batch* b, int64_t n, const int64_t* offsets, const void* ids, int32_t id_bytes,
                          const uint32_t* wordset_size, const int32_t* length, const uint8_t* cc, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (n < 0 || n > b->capacity) return fail(DICE_E_ARG, "n_files exceeds batch capacity");
    if (id_bytes != 2 && id_bytes != 4) return fail(DICE_E_ARG, "id_bytes must be 2 or 4");
    if (n > 0 && (!offsets || !wordset_size || !length || !cc)) return fail(DICE_E_ARG, "NULL file arrays");
    if (n > 0) {
        if (offsets[0] != 0) return fail(DICE_E_ARG, "offsets[0] must be 0");
        for (int64_t i = 0; i < n; ++i)
            if (offsets[i + 1] < offsets[i]) return fail(DICE_E_ARG, "offsets must be non-decreasing");
        if (offsets[n] > 0 && !ids) return fail(DICE_E_ARG, "NULL ids");
    }
    if ((int64_t)c->w64 * 8 * 4 > 64 * 1024) return fail(DICE_E_ARG, "vocabulary too large for id upload");
    DeviceGuard g(c->device);
    hipStream_t s = pick_stream(c, stream);
    b->n = n;
    b->n_long = 0;
    b->fmask_device = false;
    if (n == 0) return DICE_OK;
    const size_t need = (size_t)std::max<int64_t>(offsets[n], 1) * (size_t)id_bytes;
    if (need > b->ids_bytes) {
        HIP_TRY(hipStreamSynchronize(s));   // the staging may still feed an earlier upload
        if (b->d_ids) (void)hipFree(b->d_ids);
        b->d_ids = nullptr;
        b->ids_bytes = 0;
        int rc = dalloc_bytes(&b->d_ids, need);
        if (rc) return rc;
        b->ids_bytes = need;
    }
    if (!b->d_offs) {
        int rc = dalloc_bytes(reinterpret_cast<void**>(&b->d_offs), (size_t)(b->capacity + 1) * 8);
        if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(b->d_offs, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, s));
    if (offsets[n] > 0)
        HIP_TRY(hipMemcpyAsync(b->d_ids, ids, (size_t)offsets[n] * (size_t)id_bytes, hipMemcpyHostToDevice, s));
    const unsigned grid = (unsigned)((n + 3) / 4);
    const size_t lds = (size_t)4 * c->w64 * 8;
    if (id_bytes == 2)
        hipLaunchKernelGGL(dice_rows_from_ids<uint16_t>, dim3(grid), dim3(256), lds, s, b->d_offs,
                           (const uint16_t*)b->d_ids, n, c->w64, (uint32_t)c->V, b->d_rows);
    else
        hipLaunchKernelGGL(dice_rows_from_ids<uint32_t>, dim3(grid), dim3(256), lds, s, b->d_offs,
                           (const uint32_t*)b->d_ids, n, c->w64, (uint32_t)c->V, b->d_rows);
    HIP_TRY(hipGetLastError());
    return dice::upload_tail(b, n, wordset_size, length, cc, s);
}

}  // extern "C"

// Dice#confidence for the files dice_batch_match left without a match: overlap 0 and score 0.0
// (dice.rb:52-54: confidence is 0 when match is nil).
__global__ __launch_bounds__(256) void dice_confidence_outputs(const int32_t* __restrict__ best, uint32_t* __restrict__ ov,
                                                               double* __restrict__ score, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && best[i] < 0) {
        ov[i] = 0;
        score[i] = 0.0;
    }
}

static int batch_match(dice_batch* b, double thr, void* stream, bool confidence) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (b->n == 0) {
        b->last_match = 1;   // every pair of the empty batch scored: n * T = 0, nothing deferred
        return DICE_OK;
    }
    DeviceGuard g(c->device);
    hipStream_t s = pick_stream(c, stream);
    const int64_t n_tiles = (b->n + kWave - 1) / kWave;
    const unsigned grid = (unsigned)((n_tiles + (kBlock / kWave) - 1) / (kBlock / kWave));
    if (c->kind == 1) {
        int rc = dice::program_launch_match(c, b, thr, s);
        if (rc != DICE_OK) return rc;
    } else if (c->kind == 2) {
        int rc = dice::lds_launch_match(c, b, thr, s);
        if (rc != DICE_OK) return rc;
    } else if (c->kind == 3) {
        // the T > 64 kernels write Dice#confidence outputs themselves
        // (dice_match on a batch of mostly long files: the postings kernels, see prune_setup)
        const bool prune = c->prune && (confidence || c->prune_long_route == 0 || b->n_long < 0 ||
                                        b->n_long * c->prune_long_route < b->n);
        int rc = prune ? dice::prune_launch_match(c, b, thr, s, confidence)
                       : dice::post_launch_match(c, b, thr, s, confidence);
        if (rc != DICE_OK) return rc;
        b->last_match = prune ? 2 : 1;
    } else {
        hipLaunchKernelGGL(dice_dense_match<kTT>, dim3(grid), dim3(kBlock), 0, s, b->d_tiles, b->n, c->wq,
                           c->d_tq, c->d_tc, c->T, c->tpad, b->d_wf, b->d_len, b->d_cc, thr, b->d_best,
                           b->d_ov, b->d_score);
    }
    HIP_TRY(hipGetLastError());
    if (c->kind != 3) b->last_match = 1;
    if (confidence && c->kind != 3) {
        hipLaunchKernelGGL(dice_confidence_outputs, dim3((unsigned)((b->n + 255) / 256)), dim3(256), 0, s, b->d_best,
                           b->d_ov, b->d_score, b->n);
        HIP_TRY(hipGetLastError());
    }
    return DICE_OK;
}

extern "C" {

int dice_batch_match(dice_batch* b, double thr, void* stream) { return batch_match(b, thr, stream, false); }

int dice_batch_match_confidence(dice_batch* b, double thr, void* stream) { return batch_match(b, thr, stream, true); }

static int ensure_matrix(dice_batch* b, int32_t k) {
    dice_ctx* c = b->ctx;
    // row stride: kind 3 writes [n][post_ld] rows of whole 128-byte lines, the others [T][n]
    b->mat_ld = c->kind == 3 ? c->post_ld : c->T;
    if (b->mat_cap >= b->capacity && b->mat_k >= k && b->d_mov) return DICE_OK;
    void* ptrs[] = {b->d_mov, b->d_mscore, b->d_tki, b->d_tks};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    b->d_mov = nullptr; b->d_mscore = nullptr; b->d_tki = nullptr; b->d_tks = nullptr;
    int rc;
    const int32_t kk = std::max<int32_t>(k, 1);
    if ((rc = dalloc(&b->d_mov, (size_t)b->capacity * b->mat_ld)) ||
        (rc = dalloc(&b->d_mscore, (size_t)b->capacity * b->mat_ld)) ||
        (rc = dalloc(&b->d_tki, (size_t)b->capacity * kk)) || (rc = dalloc(&b->d_tks, (size_t)b->capacity * kk)))
        return rc;
    b->mat_cap = b->capacity;
    b->mat_k = kk;
    return DICE_OK;
}

int dice_batch_matrix(dice_batch* b, int32_t k, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    if (k < 0 || k > DICE_TOPK_MAX) return fail(DICE_E_ARG, "k out of range");
    dice_ctx* c = b->ctx;
    b->k_used = k;   // also on an empty batch: a later download with this k must be accepted
    if (b->n == 0) return DICE_OK;
    DeviceGuard g(c->device);
    int rc = ensure_matrix(b, k);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    const int64_t n_tiles = (b->n + kWave - 1) / kWave;
    const unsigned grid = (unsigned)((n_tiles + (kBlock / kWave) - 1) / (kBlock / kWave));
    b->mat_rowmajor = c->kind == 3;
    if (c->kind == 1) {
        rc = dice::program_launch_matrix(c, b, k, s);
        if (rc != DICE_OK) return rc;
    } else if (c->kind == 3) {
        rc = dice::post_launch_matrix(c, b, k, s);
        if (rc != DICE_OK) return rc;
    } else {
        if (k <= 4)
            hipLaunchKernelGGL((dice_dense_matrix<kTT, 4>), dim3(grid), dim3(kBlock), 0, s, b->d_tiles, b->n,
                               c->wq, c->d_tq, c->d_tc, c->T, c->tpad, b->d_wf, b->d_len, b->d_cc, k, b->d_mov,
                               b->d_mscore, k > 0 ? b->d_tki : nullptr, b->d_tks);
        else
            hipLaunchKernelGGL((dice_dense_matrix<kTT, kTopKMax>), dim3(grid), dim3(kBlock), 0, s, b->d_tiles,
                               b->n, c->wq, c->d_tq, c->d_tc, c->T, c->tpad, b->d_wf, b->d_len, b->d_cc, k,
                               b->d_mov, b->d_mscore, k > 0 ? b->d_tki : nullptr, b->d_tks);
    }
    HIP_TRY(hipGetLastError());
    return DICE_OK;
}

}  // extern "C"

namespace dice {

int download_match_to(dice_batch* b, int32_t* best, uint32_t* ov, double* score, hipStream_t s,
                      hipMemcpyKind kind) {
    const size_t n = (size_t)b->n;
    if (n) {
        if (best) HIP_TRY(hipMemcpyAsync(best, b->d_best, n * 4, kind, s));
        if (ov) HIP_TRY(hipMemcpyAsync(ov, b->d_ov, n * 4, kind, s));
        if (score) HIP_TRY(hipMemcpyAsync(score, b->d_score, n * 8, kind, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return DICE_OK;
}

int download_matrix_to(dice_batch* b, uint32_t* ov, double* score, int32_t* tki, double* tks, hipStream_t s,
                       hipMemcpyKind kind) {
    dice_ctx* c = b->ctx;
    const int64_t n = b->n;
    if (n && !b->d_mov) return fail(DICE_E_STATE, "dice_batch_matrix was not run");
    if (!n) return DICE_OK;
    int rc;
    if (b->mat_rowmajor) {   // already [n][ld] / [n][k]: rows of T entries at stride ld
        const size_t T = (size_t)c->T, ld = (size_t)b->mat_ld;
        if (ov) HIP_TRY(hipMemcpy2DAsync(ov, T * 4, b->d_mov, ld * 4, T * 4, (size_t)n, kind, s));
        if (score) HIP_TRY(hipMemcpy2DAsync(score, T * 8, b->d_mscore, ld * 8, T * 8, (size_t)n, kind, s));
        if (tki && b->k_used) HIP_TRY(hipMemcpyAsync(tki, b->d_tki, (size_t)n * b->k_used * 4, kind, s));
        if (tks && b->k_used) HIP_TRY(hipMemcpyAsync(tks, b->d_tks, (size_t)n * b->k_used * 8, kind, s));
        HIP_TRY(hipStreamSynchronize(s));
        return DICE_OK;
    }
    if (ov && (rc = transpose_to<uint32_t>(b, b->d_mov, c->T, n, ov, s, kind))) return rc;
    if (score && (rc = transpose_to<double>(b, b->d_mscore, c->T, n, score, s, kind))) return rc;
    if (tki && b->k_used && (rc = transpose_to<int32_t>(b, b->d_tki, b->k_used, n, tki, s, kind))) return rc;
    if (tks && b->k_used && (rc = transpose_to<double>(b, b->d_tks, b->k_used, n, tks, s, kind))) return rc;
    return DICE_OK;
}

}  // namespace dice

extern "C" {

int dice_batch_download_match(dice_batch* b, int32_t* best, uint32_t* ov, double* score, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    DeviceGuard g(c->device);
    return dice::download_match_to(b, best, ov, score, pick_stream(c, stream), hipMemcpyDeviceToHost);
}

int dice_batch_download_matrix(dice_batch* b, uint32_t* ov, double* score, int32_t k, int32_t* tki, double* tks,
                               void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    if ((tki || tks) && k != b->k_used)
        return fail(DICE_E_ARG, "top-k buffers are [n][k]: k must equal the last dice_batch_matrix k (" +
                                    std::to_string(b->k_used) + ")");
    dice_ctx* c = b->ctx;
    DeviceGuard g(c->device);
    return dice::download_matrix_to(b, ov, score, tki, tks, pick_stream(c, stream), hipMemcpyDeviceToHost);
}

int dice_batch_stream_probe(dice_batch* b, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (b->n == 0) return DICE_OK;
    if (c->w64 < 2) return fail(DICE_E_STATE, "probe needs >= 2 words per file");
    DeviceGuard g(c->device);
    hipStream_t s = pick_stream(c, stream);
    const int64_t n_tiles = (b->n + kWave - 1) / kWave;
    const unsigned grid = (unsigned)((n_tiles + (kBlock / kWave) - 1) / (kBlock / kWave));
    // results land in the (16 B/file) score+best+overlap area: reuse d_score as scratch
    hipLaunchKernelGGL(dice_stream_probe, dim3(grid), dim3(kBlock), 0, s, b->d_tiles, b->n, c->wq,
                       reinterpret_cast<uint4*>(b->d_rows));
    HIP_TRY(hipGetLastError());
    return DICE_OK;
}

int dice_batch_deferred(dice_batch* b, int64_t* deferred, void* stream) {
    if (!b || !deferred) return fail(DICE_E_ARG, "NULL batch/output");
    *deferred = 0;
    // only the bound-pruned match defers files (dice_match may route a batch of long files to the
    // postings kernels instead: the count of an earlier pruned call is then stale)
    if (!b->d_ndefer || !b->ctx->prune || b->last_match != 2) return DICE_OK;
    DeviceGuard g(b->ctx->device);
    uint32_t m = 0;
    hipStream_t s = pick_stream(b->ctx, stream);
    HIP_TRY(hipMemcpyAsync(&m, b->d_ndefer, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *deferred = m;
    return DICE_OK;
}

int dice_batch_scored_pairs(dice_batch* b, int64_t* pairs, void* stream) {
    if (!b || !pairs) return fail(DICE_E_ARG, "NULL batch/output");
    *pairs = 0;
    dice_ctx* c = b->ctx;
    if (b->last_match == 1) {
        *pairs = b->n * (int64_t)c->T;   // every kernel but the bound-pruned one scores every pair
    } else if (b->last_match == 2) {
        // the pruned kernel's exact scores (per-wave counts) + every pair of each deferred file
        // (the postings kernels score them all)
        DeviceGuard g(c->device);
        hipStream_t s = pick_stream(c, stream);
        // (dice_prune4's per-wave counts, then the number of files the postings kernels scored)
        const int64_t nw = b->prune_waves;
        std::vector<uint32_t> h((size_t)nw + 1);
        HIP_TRY(hipMemcpyAsync(h.data(), b->d_nscored, (size_t)nw * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h.data() + nw, b->d_ndefer, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        int64_t sum = 0;
        for (int64_t i = 0; i < nw; ++i) sum += h[(size_t)i];
        *pairs = sum + (int64_t)h[(size_t)nw] * c->T;
    }
    return DICE_OK;
}

int dice_batch_result_ptrs(dice_batch* b, void** best, void** ov, void** score) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    if (best) *best = b->d_best;
    if (ov) *ov = b->d_ov;
    if (score) *score = b->d_score;
    return DICE_OK;
}

}  // extern "C"

int dice::scratch_for(dice_ctx* ctx, int64_t n, dice_batch** out) {
    if (ctx->scratch && ctx->scratch->capacity >= n) {
        *out = ctx->scratch;
        return DICE_OK;
    }
    if (ctx->scratch) {
        dice_batch_destroy(ctx->scratch);
        ctx->scratch = nullptr;
    }
    int rc = dice_batch_create(ctx, std::max<int64_t>(n, 64), &ctx->scratch);
    *out = ctx->scratch;
    return rc;
}

// ---- small host-buffer calls ---------------------------------------------------------------
// licensee scores one file at a time (license_file.rb:92-98 -> dice.rb:34-41), so a drop-in
// binding calls dice_match / dice_similarity_matrix with n = 1. For n <= kSmallFiles the call
// packs its inputs into one page-locked region, copies it with one H2D into the small batch's
// input region (scalars first, then the rows), runs the usual kernels, and brings every result
// back with one D2H: two copies per call instead of seven, no pageable staging, no memsets.
namespace {

constexpr int64_t kSmallFiles = 64;
constexpr size_t kAlign = 256;

size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct SmallLayout {
    size_t wf, len, cc, rows, in_bytes;                    // input region
    size_t best, ov, score, mov, mscore, tki, tks, out_bytes;   // output region
};

SmallLayout small_layout(const dice_ctx* c) {
    const size_t n = (size_t)kSmallFiles, T = (size_t)std::max(c->T, c->post_ld), K = (size_t)DICE_TOPK_MAX;
    SmallLayout L;
    L.wf = 0;
    L.len = L.wf + n * 4;
    L.cc = L.len + n * 4;
    L.rows = align_up(L.cc + n);
    L.in_bytes = L.rows + n * (size_t)c->w64 * 8;
    L.best = 0;
    L.ov = L.best + n * 4;
    L.score = L.ov + n * 4;
    L.mov = align_up(L.score + n * 8);
    L.mscore = align_up(L.mov + T * n * 4);
    L.tki = align_up(L.mscore + T * n * 8);
    L.tks = align_up(L.tki + K * n * 4);
    L.out_bytes = L.tks + K * n * 8;
    return L;
}

int small_batch(dice_ctx* c, dice_batch** out) {
    if (c->small) {
        *out = c->small;
        return DICE_OK;
    }
    const SmallLayout L = small_layout(c);
    dice_batch* b = nullptr;
    int rc = dice_batch_create(c, kSmallFiles, &b);
    if (rc) return rc;
    void* old[] = {b->d_rows, b->d_wf, b->d_len, b->d_cc, b->d_best, b->d_ov, b->d_score};
    for (void* p : old) (void)hipFree(p);
    b->d_rows = nullptr; b->d_wf = nullptr; b->d_len = nullptr; b->d_cc = nullptr;
    b->d_best = nullptr; b->d_ov = nullptr; b->d_score = nullptr;
    if ((rc = dice::dalloc_bytes(&b->d_in, L.in_bytes)) || (rc = dice::dalloc_bytes(&b->d_out, L.out_bytes)) ||
        (!c->h_small_in && hipHostMalloc(&c->h_small_in, L.in_bytes, hipHostMallocDefault) != hipSuccess) ||
        (!c->h_small_out && hipHostMalloc(&c->h_small_out, L.out_bytes, hipHostMallocDefault) != hipSuccess)) {
        dice_batch_destroy(b);
        return rc ? rc : fail(DICE_E_NOMEM, "hipHostMalloc failed");
    }
    char* in = (char*)b->d_in;
    char* o = (char*)b->d_out;
    b->d_wf = (uint32_t*)(in + L.wf);
    b->d_len = (int32_t*)(in + L.len);
    b->d_cc = (uint8_t*)(in + L.cc);
    b->d_rows = (uint64_t*)(in + L.rows);
    b->d_best = (int32_t*)(o + L.best);
    b->d_ov = (uint32_t*)(o + L.ov);
    b->d_score = (double*)(o + L.score);
    b->d_mov = (uint32_t*)(o + L.mov);
    b->d_mscore = (double*)(o + L.mscore);
    b->d_tki = (int32_t*)(o + L.tki);
    b->d_tks = (double*)(o + L.tks);
    b->mat_cap = kSmallFiles;
    b->mat_k = DICE_TOPK_MAX;
    c->small = b;
    *out = b;
    return DICE_OK;
}

// inputs -> the page-locked region -> one H2D; the tile repack for the tile-layout kernels
int small_upload(dice_ctx* c, dice_batch* b, const dice_files* f, const SmallLayout& L) {
    const int64_t n = f->n_files;
    const int64_t npad = (n + kWave - 1) / kWave * kWave;
    char* h = (char*)c->h_small_in;
    std::memcpy(h + L.wf, f->wordset_size, (size_t)n * 4);
    std::memset(h + L.wf + n * 4, 0, (size_t)(npad - n) * 4);
    std::memcpy(h + L.len, f->length, (size_t)n * 4);
    std::memset(h + L.len + n * 4, 0, (size_t)(npad - n) * 4);
    std::memcpy(h + L.cc, f->cc_false_positive, (size_t)n);
    std::memset(h + L.cc + n, 0, (size_t)(npad - n));
    std::memcpy(h + L.rows, f->bits, (size_t)n * c->w64 * 8);
    b->n = n;
    HIP_TRY(hipMemcpyAsync(b->d_in, h, L.rows + (size_t)n * c->w64 * 8, hipMemcpyHostToDevice, c->stream));
    if (c->kind == 3) {   // (dice_match's long-file routing, upload_tail)
        b->n_long = 0;
        if (c->prune)
            for (int64_t i = 0; i < n; ++i) b->n_long += f->wordset_size[i] > c->prune_max_lf;
        return DICE_OK;
    }
    const int64_t n_tiles = npad / kWave;
    const int64_t total = n_tiles * c->wq * kWave;
    hipLaunchKernelGGL(dice_pack_tiles, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                       b->d_rows, n, c->w64, c->wq, c->kind == 1 ? (const int32_t*)c->d_qperm : nullptr, b->d_tiles,
                       n_tiles);
    HIP_TRY(hipGetLastError());
    return DICE_OK;
}

int small_match(dice_ctx* c, const dice_files* f, double thr, int32_t* best, uint32_t* ov, double* score,
                bool confidence) {
    DeviceGuard g(c->device);
    dice_batch* b = nullptr;
    int rc;
    if ((rc = small_batch(c, &b))) return rc;
    const SmallLayout L = small_layout(c);
    if ((rc = small_upload(c, b, f, L)) || (rc = batch_match(b, thr, nullptr, confidence))) return rc;
    const size_t n = (size_t)f->n_files;
    HIP_TRY(hipMemcpyAsync(c->h_small_out, b->d_out, L.score + n * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const char* h = (const char*)c->h_small_out;
    if (best) std::memcpy(best, h + L.best, n * 4);
    if (ov) std::memcpy(ov, h + L.ov, n * 4);
    if (score) std::memcpy(score, h + L.score, n * 8);
    return DICE_OK;
}

int small_matrix(dice_ctx* c, const dice_files* f, uint32_t* ov, double* score, int32_t k, int32_t* tki,
                 double* tks) {
    DeviceGuard g(c->device);
    dice_batch* b = nullptr;
    int rc;
    if ((rc = small_batch(c, &b))) return rc;
    const SmallLayout L = small_layout(c);
    // the matrix areas packed for this n ([T][n] or [n][T], [k][n] or [n][k]: n * T and n * k
    // entries either way), so one D2H moves exactly the results
    const size_t n = (size_t)f->n_files, T = (size_t)c->T, kk = (size_t)k;
    const size_t ld = c->kind == 3 ? (size_t)c->post_ld : T;   // row-major rows at stride ld (kind 3)
    const size_t o_mov = L.mov, o_msc = align_up(o_mov + n * ld * 4), o_tki = align_up(o_msc + n * ld * 8),
                 o_tks = align_up(o_tki + n * kk * 4), o_end = o_tks + n * kk * 8;
    char* d = (char*)b->d_out;
    b->d_mov = (uint32_t*)(d + o_mov);
    b->d_mscore = (double*)(d + o_msc);
    b->d_tki = (int32_t*)(d + o_tki);
    b->d_tks = (double*)(d + o_tks);
    if ((rc = small_upload(c, b, f, L)) || (rc = dice_batch_matrix(b, k, nullptr))) return rc;
    HIP_TRY(hipMemcpyAsync((char*)c->h_small_out + o_mov, d + o_mov, o_end - o_mov, hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const char* h = (const char*)c->h_small_out;
    const uint32_t* hm = (const uint32_t*)(h + o_mov);
    const double* hs = (const double*)(h + o_msc);
    const int32_t* hi = (const int32_t*)(h + o_tki);
    const double* hk = (const double*)(h + o_tks);
    if (b->mat_rowmajor) {
        for (size_t i = 0; i < n; ++i) {
            if (ov) std::memcpy(ov + i * T, hm + i * ld, T * 4);
            if (score) std::memcpy(score + i * T, hs + i * ld, T * 8);
        }
        if (k > 0) {
            std::memcpy(tki, hi, n * kk * 4);
            std::memcpy(tks, hk, n * kk * 8);
        }
        return DICE_OK;
    }
    for (size_t i = 0; i < n; ++i) {   // template-major [T][n] / [k][n]
        for (size_t t = 0; t < T; ++t) {
            if (ov) ov[i * T + t] = hm[t * n + i];
            if (score) score[i * T + t] = hs[t * n + i];
        }
        for (size_t j = 0; j < kk; ++j) {
            tki[i * kk + j] = hi[j * n + i];
            tks[i * kk + j] = hk[j * n + i];
        }
    }
    return DICE_OK;
}

}  // namespace

extern "C" {

static int host_match(dice_ctx* ctx, const dice_files* f, double thr, int32_t* best, uint32_t* ov, double* score,
                      bool confidence) {
    if (!ctx || !f) return fail(DICE_E_ARG, "NULL ctx/files");
    if (f->n_files == 0) return DICE_OK;
    if (f->n_files < 0) return fail(DICE_E_ARG, "n_files < 0");
    if (!f->bits || !f->wordset_size || !f->length || !f->cc_false_positive)
        return fail(DICE_E_ARG, "NULL file arrays");
    if (f->n_files <= kSmallFiles && !getenv_flag("DICE_NO_SMALL_CALL"))
        return small_match(ctx, f, thr, best, ov, score, confidence);
    dice_batch* b = nullptr;
    int rc = dice::scratch_for(ctx, f->n_files, &b);
    if (rc) return rc;
    if ((rc = dice_batch_upload(b, f, nullptr))) return rc;
    if ((rc = batch_match(b, thr, nullptr, confidence))) return rc;
    return dice_batch_download_match(b, best, ov, score, nullptr);
}

int dice_match(dice_ctx* ctx, const dice_files* f, double thr, int32_t* best, uint32_t* ov, double* score) {
    return host_match(ctx, f, thr, best, ov, score, false);
}

int dice_match_confidence(dice_ctx* ctx, const dice_files* f, double thr, int32_t* best, uint32_t* ov, double* score) {
    return host_match(ctx, f, thr, best, ov, score, true);
}

int dice_similarity_matrix(dice_ctx* ctx, const dice_files* f, uint32_t* ov, double* score, int32_t k,
                           int32_t* tki, double* tks) {
    if (!ctx || !f) return fail(DICE_E_ARG, "NULL ctx/files");
    if (k < 0 || k > DICE_TOPK_MAX) return fail(DICE_E_ARG, "k out of range");
    if (k > 0 && (!tki || !tks)) return fail(DICE_E_ARG, "top-k outputs required when k > 0");
    if (f->n_files == 0) return DICE_OK;
    if (f->n_files < 0) return fail(DICE_E_ARG, "n_files < 0");
    if (!f->bits || !f->wordset_size || !f->length || !f->cc_false_positive)
        return fail(DICE_E_ARG, "NULL file arrays");
    if (f->n_files <= kSmallFiles && !getenv_flag("DICE_NO_SMALL_CALL")) return small_matrix(ctx, f, ov, score, k, tki, tks);
    dice_batch* b = nullptr;
    int rc = dice::scratch_for(ctx, f->n_files, &b);
    if (rc) return rc;
    if ((rc = dice_batch_upload(b, f, nullptr))) return rc;
    if ((rc = dice_batch_matrix(b, k, nullptr))) return rc;
    return dice_batch_download_matrix(b, ov, score, k, k > 0 ? tki : nullptr, k > 0 ? tks : nullptr, nullptr);
}

}  // extern "C"
