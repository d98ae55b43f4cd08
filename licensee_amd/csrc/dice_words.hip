// ContentHelper#wordset on the device (the host preparation's largest
// pass moved to the GPU).
//
// Reference: lib/licensee/content_helper.rb:108-110 --
//   @wordset ||= content_normalized&.scan(WORDSET_REGEX)&.to_set
// with WORDSET_REGEX = /(?:[\w\/-](?:'s|(?<=s)')?)+/ (ASCII \w) over content_normalized, and the
// interning of those words into the corpus vocabulary's bitset (what dice_files.bits holds:
// licensee_amd/corpus.py) with |W_F| counting every distinct word, vocabulary or not
// (content_helper.rb:128-133 divides by wordset.size). The texts arrive normalized
// (licensee_host.h lh_normalize_files: one byte per character, non-ASCII characters as 0x80).
//
// One wave per file, persistent over the batch. The file streams through a per-wave LDS window of
// two 1 KiB chunks (one 16-byte load per lane, the chunk after next in flight while this one is
// scanned). Most chunks are scanned at once: each lane classifies its 16 bytes and the 4 on either
// side with SWAR, the regex's tokens are the runs of [\w/-] joined by the apostrophes it consumes,
// and the k-th run end closes the k-th run start (the token open from the previous chunk first).
// A chunk where that joining rule is not exact ("'s'"), or that a serial re-scan reached into,
// takes the block loop: 64-byte blocks, one byte per lane, a ballot word mask (as in the host scan,
// normalize.cpp scan_words), and a block with a run ending at an apostrophe next to an 's' scanned
// serially in the regex's own order. A token's first 16 bytes, read from the window, are its key
// (with its length and, past 16 bytes, a hash of the tail); tokens are looked up 64 at a time
// (lanes = tokens) in the context's vocabulary table (L2-resident, dice_vocab_setup: buckets of 8
// tagged slots, the full key checked, long words' tails compared byte by byte): a vocabulary word
// sets its row bit (ds_or), one of the extra words (template field words outside the vocabulary)
// its field-mask bit, any other word goes to the wave's LDS set of distinct words (CAS-claimed
// slots, full keys, long tokens' bytes compared). |W_F| = row bits + field bits + set size. A
// file whose set would pass kSetMax distinct non-vocabulary words is flagged; the caller prepares
// it on the host. LDS ~10 KiB per wave at the vendored vocabulary: four 4-wave workgroups per CU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "dice_common.h"
#include "dice_internal.h"
#include "dice_wave.h"

namespace dice {

// Phase-skip diagnostics (tools/build_variant.sh -DWORDS_DIAG=n; results are wrong): 1 skips the
// lookups, 2 the token keys and queue, 4 the block scan
#ifndef WORDS_DIAG
#define WORDS_DIAG 0
#endif
constexpr int kWordsWaves = 4;          // waves (files in flight) per workgroup
constexpr int kChunk = 1024;            // bytes per staged chunk (16 per lane)
constexpr int kWin = 2 * kChunk;        // the LDS window: two chunks, indexed by position & (kWin - 1)
constexpr int kSetCap = 256;            // per-wave set of distinct non-vocabulary words (slots)
constexpr int kSetMax = 192;            // more distinct such words: the file is flagged (host path);
                                        // a lookup pass adds at most 64, so the set never overfills
constexpr uint32_t kQKeep = 63;         // queued tokens left after a flush (lookups run 64 at a time)
constexpr int kQCap = kQKeep + 33;      // + one block's tokens (32 runs + the open one)
constexpr uint64_t kLongMark = 1ull << 63;   // set key of a token longer than 16 bytes
constexpr uint32_t kFastPos = kQCap * 16 / 2;   // run starts + ends of a fast-path chunk (u16 each in
                                                // the queue's qlo + qhi area)
#ifndef WORDS_DYNAMIC
#define WORDS_DYNAMIC 1   // 0: files by a fixed stride of the grid (A/B)
#endif
#ifndef WORDS_BLOCKS_ONLY
#define WORDS_BLOCKS_ONLY 0   // 1: every chunk through the block loop (A/B: tools/build_variant.sh)
#endif

// the hash of a token key: (first 16 bytes, little-endian, zero past the token), length, tail hash
__host__ __device__ inline uint64_t words_mix(uint64_t lo, uint64_t hi, uint32_t len, uint32_t tail) {
    const uint64_t p = (lo ^ (hi * 0xC2B2AE3D27D4EB4FULL) ^ ((uint64_t)len << 56) ^ tail) * 0x9E3779B97F4A7C15ULL;
    return p ^ (p >> 32);
}
__host__ __device__ inline uint32_t fnv_step(uint32_t h, uint32_t byte) { return (h ^ byte) * 16777619u; }

// [\w/-] with ASCII \w (bytes >= 0x80 never match)
__device__ __forceinline__ bool word_byte(uint32_t c) {
    const uint32_t lc = c | 0x20u;
    return (lc - 'a' < 26u) || (c - '0' < 10u) || c == '_' || c == '/' || c == '-';
}

struct VocabDev {
    const uint32_t* slots;   // [nb][kSlots]: (tag << id_bits) | (id + 1), 0 = empty
    const uint4* keys;       // [n] {lo, hi} of the word's first 16 bytes
    const uint32_t* wmeta;   // [n] length | tail hash... (see dice_vocab_setup): length
    const uint32_t* woff;    // [n] offset of the word's bytes in wtxt
    const uint8_t* wtxt;
    uint32_t bmask, id_bits, V, n_extra;
};

// the 16 bytes at window position p (the window holds the chunk of p and the next one)
__device__ __forceinline__ void window_key(const uint8_t* win, uint32_t p, uint64_t& lo, uint64_t& hi) {
    const uint32_t a = p & ~3u, s = p & 3u;
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = *reinterpret_cast<const uint32_t*>(win + ((a + 4u * k) & (kWin - 1)));
    const uint32_t x0 = __builtin_amdgcn_alignbyte(w[1], w[0], s), x1 = __builtin_amdgcn_alignbyte(w[2], w[1], s);
    const uint32_t x2 = __builtin_amdgcn_alignbyte(w[3], w[2], s), x3 = __builtin_amdgcn_alignbyte(w[4], w[3], s);
    lo = (uint64_t)x0 | ((uint64_t)x1 << 32);
    hi = (uint64_t)x2 | ((uint64_t)x3 << 32);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}
// window_key at a wave-uniform position, as scalars
__device__ __forceinline__ void window_key_u(const uint8_t* win, uint32_t p, uint64_t& lo, uint64_t& hi) {
    window_key(win, p, lo, hi);
    lo = rfl64(lo);
    hi = rfl64(hi);
}
__device__ __forceinline__ void mask_key(uint32_t len, uint64_t& lo, uint64_t& hi) {
    if (len < 8) lo &= (1ull << (8 * len)) - 1;
    if (len <= 8) hi = 0;
    else if (len < 16) hi &= (1ull << (8 * (len - 8))) - 1;
}
// Bytes [a, a + 32) of memory at `base` as 8 little-endian u32, from 9 independent aligned loads
// (one round trip instead of 32 dependent byte loads; the buffers keep 64 bytes of slack).
__device__ __forceinline__ void load32(const uint8_t* base, uint64_t a, uint32_t (&x)[8]) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (a & ~3ull));
    uint32_t r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) r[k] = w[k];
    const uint32_t sh = (uint32_t)(a & 3u);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = __builtin_amdgcn_alignbyte(r[k + 1], r[k], sh);
}
// FNV-1a of bytes [16, len) of the token at t
__device__ inline uint32_t tail_hash(const uint8_t* base, uint64_t pos, uint32_t len) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 16; i < len; i += 32) {
        uint32_t x[8];
        load32(base, pos + i, x);
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (i + 4u * k + b < len) h = fnv_step(h, (x[k] >> (8 * b)) & 0xFFu);
    }
    return h;
}
// bytes [from, len) of the tokens at a (in `ba`) and b (in `bb`) are equal
__device__ inline bool bytes_equal(const uint8_t* ba, uint64_t a, const uint8_t* bb, uint64_t b, uint32_t from,
                                   uint32_t len) {
    for (uint32_t i = from; i < len; i += 32) {
        uint32_t x[8], y[8];
        load32(ba, a + i, x);
        load32(bb, b + i, y);
        uint32_t diff = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t at = i + 4u * k;
            const uint32_t m = at >= len ? 0u : len - at >= 4 ? 0xFFFFFFFFu : (1u << (8 * (len - at))) - 1u;
            diff |= (x[k] ^ y[k]) & m;
        }
        if (diff) return false;
    }
    return true;
}

#ifndef WORDS_SLOTS
#define WORDS_SLOTS 8   // tagged slots per vocabulary bucket (4: one 16-byte load, measured slower)
#endif
constexpr int kSlots = WORDS_SLOTS;

__device__ __forceinline__ uint32_t pick8(const uint4& a, const uint4& b, int j) {   // (no indexed array)
    const uint4 q = j < 4 ? a : b;
    const int k = j & 3;
    return k < 2 ? (k == 0 ? q.x : q.y) : (k == 2 ? q.z : q.w);
}

// vocabulary id of the token (lo, hi, len) at text[pos], or -1
__device__ inline int32_t vocab_find(const VocabDev& v, uint64_t h, uint64_t lo, uint64_t hi, uint32_t len,
                                     const uint8_t* text, uint64_t pos) {
    const uint32_t idmask = (1u << v.id_bits) - 1u;
    const uint32_t tag = ((uint32_t)(h >> 40)) << v.id_bits;
    for (uint32_t b = (uint32_t)h & v.bmask, probe = 0; probe <= v.bmask; b = (b + 1) & v.bmask, ++probe) {
        const uint4* bk = reinterpret_cast<const uint4*>(v.slots + (size_t)b * kSlots);
        const uint4 s0 = bk[0], s1 = kSlots == 8 ? bk[1] : make_uint4(0, 0, 0, 0);
        const uint32_t s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        uint32_t hits = 0, empty = 0;
#pragma unroll
        for (int j = 0; j < kSlots; ++j) {
            empty |= (uint32_t)(s[j] == 0) << j;
            hits |= (uint32_t)(s[j] != 0 && (s[j] & ~idmask) == tag) << j;
        }
        while (hits) {   // (almost always one candidate)
            const int j = __builtin_ctz(hits);
            hits &= hits - 1;
            const int32_t id = (int32_t)(pick8(s0, s1, j) & idmask) - 1;
            const uint4 k = v.keys[id];
            // (a key of < 16 bytes holds a zero byte where the word ends: equal keys, equal lengths;
            // the length is read only for 16 bytes and more)
            if (((uint64_t)k.x | ((uint64_t)k.y << 32)) == lo && ((uint64_t)k.z | ((uint64_t)k.w << 32)) == hi &&
                (len < 16 || v.wmeta[id] == len) && (len <= 16 || bytes_equal(v.wtxt, v.woff[id], text, pos, 16, len)))
                return id;
        }
        if (empty) return -1;
    }
    return -1;
}

// Insert the token into the wave's set; true if it was not there. Keys: a token of <= 16 bytes is
// (lo, hi) itself (its bytes are nonzero ASCII, so lo != 0 and lo's top bit is clear); a longer
// one is (kLongMark | len << 32 | tail hash, lo ^ hi * K), its position kept for a byte compare.
__device__ inline bool set_insert(uint64_t* sa, uint64_t* sb, uint32_t* so, uint64_t h, uint64_t lo, uint64_t hi,
                                  uint32_t len, uint32_t tail, uint32_t pos, const uint8_t* text) {
    const uint64_t a = len <= 16 ? lo : (kLongMark | ((uint64_t)len << 32) | tail);
    const uint64_t b = len <= 16 ? hi : (lo ^ (hi * 0x9E3779B97F4A7C15ULL));
    uint32_t slot = (uint32_t)h & (kSetCap - 1);
    for (int probe = 0; probe < kSetCap; ++probe, slot = (slot + 1) & (kSetCap - 1)) {
        const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(sa + slot), 0ull, (unsigned long long)a);
        const bool won = old == 0;
        if (won) {
            sb[slot] = b;
            so[slot] = pos;
        }
        // the claiming lanes' writes come before any lane's read of a claimed slot (one wave, LDS
        // operations in program order; the fence keeps the compiler from hoisting the read)
        asm volatile("" ::: "memory");
        if (won) return true;
        if (old != a || sb[slot] != b) continue;
        if (len <= 16 || bytes_equal(text, so[slot], text, pos, 0, len)) return false;
    }
    return false;   // a full set: reached only by a pass that ends above kSetMax (the file is flagged)
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
        v |= (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_incl_scan(v), kWave - 1);
}

// LDS bytes per wave (a multiple of 16)
__host__ __device__ constexpr size_t words_lds_per_wave(int32_t w64) {
    return ((size_t)kWin + kQCap * 24 + kSetCap * 20 + (size_t)w64 * 8 + 15) / 16 * 16;
}

struct WaveLds {
    uint8_t* win;      // [kWin]
    uint64_t* qlo;     // [kQCap]
    uint64_t* qhi;
    uint2* qmeta;      // {position, length}
    uint64_t* sa;      // [kSetCap]
    uint64_t* sb;
    uint32_t* so;
    uint32_t* row;     // [2 * w64]
};

// One lookup pass over up to 64 tokens (lane = token; `act` lanes hold one): the vocabulary bit,
// the field-mask bit or the set; returns the number of new set words (wave total).
__device__ inline uint32_t lookup_tokens(const WaveLds& L, bool act, uint64_t lo, uint64_t hi, uint32_t len,
                                         uint32_t pos, const VocabDev& v, const uint8_t* ftext, uint64_t& fm) {
    uint32_t fresh = 0;
    uint64_t h = 0;
    uint32_t tail = 0;
    int32_t id = -1;
    if (act) {
        tail = len > 16 ? tail_hash(ftext, pos, len) : 0u;
        h = words_mix(lo, hi, len, tail);
        id = vocab_find(v, h, lo, hi, len, ftext, pos);
        if (id >= 0 && (uint32_t)id < v.V) atomicOr(L.row + (id >> 5), 1u << (id & 31));
        else if (id >= 0) fm |= 1ull << (id - (int32_t)v.V);
    }
    asm volatile("" ::: "memory");
    if (act && id < 0) fresh = set_insert(L.sa, L.sb, L.so, h, lo, hi, len, tail, pos, ftext) ? 1u : 0u;
    return wave_sum(fresh);
}

// ... over the first min(nq, 64) queued tokens
__device__ inline uint32_t lookup_pass(const WaveLds& L, uint32_t nq, const VocabDev& v, const uint8_t* ftext,
                                       uint64_t& fm, int lane) {
    const bool act = (uint32_t)lane < nq;
    uint64_t lo = 0, hi = 0;
    uint32_t len = 0, pos = 0;
    if (act) {
        lo = L.qlo[lane];
        hi = L.qhi[lane];
        const uint2 m = L.qmeta[lane];
        pos = m.x;
        len = m.y;
    }
    return lookup_tokens(L, act, lo, hi, len, pos, v, ftext, fm);
}

// The classes of four bytes (little-endian in x) as 4-bit masks: [\w/-] (ASCII \w; bytes >= 0x80
// never match), '\'' and 's'. SWAR on the low seven bits (no carries between bytes), then the
// bytes with the high bit set are cleared.
__device__ __forceinline__ void classify4(uint32_t x, uint32_t& w, uint32_t& q, uint32_t& s) {
    const uint32_t hib = x & 0x80808080u, y = x & 0x7F7F7F7Fu, H = 0x80808080u;
    auto eq = [&](uint32_t z) { return ~(z + 0x7F7F7F7Fu) & H; };   // per byte: z == 0 (z < 0x80)
    const uint32_t t = y | 0x20202020u;
    const uint32_t alpha = (t + 0x1F1F1F1Fu) & ~(t + 0x05050505u) & H;   // 'a' <= t <= 'z'
    const uint32_t digit = (y + 0x50505050u) & ~(y + 0x46464646u) & H;   // '0' <= y <= '9'
    const uint32_t under = eq(y ^ 0x5F5F5F5Fu);                           // '_'
    const uint32_t slash = eq((y | 0x02020202u) ^ 0x2F2F2F2Fu);           // '/' or '-'
    auto pack = [](uint32_t m) { return ((m >> 7) * 0x10204080u) >> 28; };   // bits 7, 15, 23, 31 -> 0..3
    w = pack((alpha | digit | under | slash) & ~hib);
    q = pack(eq(y ^ 0x27272727u) & ~hib);
    s = pack(eq(y ^ 0x73737373u) & ~hib);
}

// (4 waves per SIMD asked for: the allocator then fits the kernel in 4 waves' registers with room to
// spare; 1 = no request, for A/B: profiles/raw/r6w8_waves_per_eu_ab.txt)
#ifndef WORDS_WAVES_PER_EU
#define WORDS_WAVES_PER_EU 4
#endif
__global__ __launch_bounds__(kWordsWaves * kWave) __attribute__((amdgpu_waves_per_eu(WORDS_WAVES_PER_EU))) void dice_words_kernel(
    const uint8_t* __restrict__ text, int64_t text_bytes, const int64_t* __restrict__ off,
    const int32_t* __restrict__ tlen, int64_t n, VocabDev v, int32_t w64, uint64_t* __restrict__ rows,
    uint32_t* __restrict__ wf_out, uint64_t* __restrict__ fmask_out, uint8_t* __restrict__ status,
    uint32_t* __restrict__ counters, uint32_t max_lf) {
    extern __shared__ uint64_t lds64[];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (int)rfl(threadIdx.x >> 6);
    // per wave: window (first: 16-byte stores), queue, set, row
    uint64_t* base = lds64 + (size_t)wave * (words_lds_per_wave(w64) / 8);
    WaveLds L;
    L.win = reinterpret_cast<uint8_t*>(base);
    L.qlo = base + kWin / 8;
    L.qhi = L.qlo + kQCap;
    L.sa = L.qhi + kQCap;
    L.sb = L.sa + kSetCap;
    L.qmeta = reinterpret_cast<uint2*>(L.sb + kSetCap);
    L.so = reinterpret_cast<uint32_t*>(L.qmeta + kQCap);
    L.row = L.so + kSetCap;

#if WORDS_DYNAMIC
    // files handed out one at a time from a counter (counters[2], zeroed per upload): a wave's share
    // is then not a fixed stride of files whose sizes vary several-fold (the slowest wave's sum
    // set the kernel's end): 1.83 vs 2.51 ms per 64k texts, profiles/raw/r6w9_dynamic_ab.txt
    for (;;) {
        // (every lane takes part -- lane 0 adds 1, the rest 0 -- so no lane's result comes from a
        // divergent branch; lane 0's old value is the file)
        const uint32_t got = atomicAdd(counters + 2, lane == 0 ? 1u : 0u);
        const int64_t f = (int64_t)(uint32_t)__shfl((int)got, 0);
        if (f >= n) break;
#else
    for (int64_t f = (int64_t)blockIdx.x * kWordsWaves + wave; f < n; f += (int64_t)gridDim.x * kWordsWaves) {
#endif
        // (uniform values read from memory go through readfirstlane: the state below that derives
        // from them -- masks, resume, the open token -- then stays scalar instead of being carried
        // per lane with exec-masked branches)
        const int64_t fo = (int64_t)(((uint64_t)rfl((uint32_t)((uint64_t)off[f] >> 32)) << 32) | rfl((uint32_t)off[f]));
        const uint32_t nb = rfl((uint32_t)tlen[f]);
        const uint8_t* ft = text + fo;
        for (int32_t j = lane; j < 2 * w64; j += kWave) L.row[j] = 0;
        for (int j = lane; j < kSetCap; j += kWave) L.sa[j] = 0;
        const uint32_t nchunks = (nb + kChunk - 1) / kChunk;
        auto chunk_load = [&](uint32_t c) -> uint4 {
            const int64_t a = fo + (int64_t)c * kChunk + 16 * lane;
            return a + 16 <= text_bytes ? *reinterpret_cast<const uint4*>(text + a) : make_uint4(0, 0, 0, 0);
        };
        auto chunk_store = [&](uint32_t c, uint4 x) {
            *reinterpret_cast<uint4*>(L.win + ((c * kChunk + 16u * lane) & (kWin - 1))) = x;
        };
        if (nchunks > 0) chunk_store(0, chunk_load(0));
        if (nchunks > 1) chunk_store(1, chunk_load(1));
        uint64_t fm = 0;             // field-mask bits (per lane, OR-reduced at the end)
        uint32_t words = 0;          // distinct set words (wave-uniform)
        uint32_t nq = 0;             // queued tokens (uniform)
        bool over = false;
        bool open = false;           // a token whose run continues past the block
        uint32_t ostart = 0;
        uint64_t olo = 0, ohi = 0;   // its first 16 bytes (from the window at its start)
        uint32_t resume = 0;         // after a serial block: tokens start at or after it
        uint64_t prevw = 0;
        uint32_t ptail = 0;          // the last 4 bytes of the previous chunk (fast path)
        auto push = [&](bool has, uint32_t p, uint32_t len, uint64_t lo, uint64_t hi) {
            const uint64_t bal = __ballot(has);
            if (has) {
                const uint32_t at = nq + lane_rank(bal);
                L.qlo[at] = lo;
                L.qhi[at] = hi;
                L.qmeta[at] = make_uint2(p, len);
            }
            nq = rfl(nq + (uint32_t)__builtin_popcountll(bal));
        };
        auto flush = [&](uint32_t keep) {   // look up queued tokens until at most `keep` remain
            while (nq > keep && !over) {
                asm volatile("" ::: "memory");
                if (!(WORDS_DIAG & 1)) words += lookup_pass(L, nq, v, ft, fm, lane);
                const uint32_t done = nq < 64 ? nq : 64;
                asm volatile("" ::: "memory");
                // move the rest to the front
                for (uint32_t j = done + lane; j < nq; j += kWave) {
                    const uint64_t a = L.qlo[j], b = L.qhi[j];
                    const uint2 m = L.qmeta[j];
                    asm volatile("" ::: "memory");
                    L.qlo[j - done] = a;
                    L.qhi[j - done] = b;
                    L.qmeta[j - done] = m;
                }
                nq -= done;
                if (words > (uint32_t)kSetMax) over = true;
            }
        };
        for (uint32_t c = 0; c < nchunks && !over; ++c) {
            uint4 nx = make_uint4(0, 0, 0, 0);
            if (c + 2 < nchunks) nx = chunk_load(c + 2);
            const uint32_t c0 = c * kChunk;
#if !WORDS_BLOCKS_ONLY
            // The chunk at once (most chunks): a lane classifies its 16 bytes and the 4 on either
            // side (SWAR), and the regex's tokens are the runs of [\w/-] joined by the apostrophes
            // it consumes -- after a word character, one followed by 's' (the 's' then continues
            // the token) or one preceded by 's'. That rule is exact unless an 's' consumed that
            // way is itself followed by an apostrophe ("'s'"): such a chunk, one whose last two
            // bytes hold a joining apostrophe (the block loop of a next chunk must not start inside
            // the suffix), one a serial re-scan reached into, or one with more than kFastPos run
            // starts and ends takes the block loop below. The k-th run end closes the k-th run
            // start (the open token first); tokens are looked up 64 at a time straight from the
            // window.
            // (resume == c0: a re-scan consumed the run that reaches the chunk -- its end at c0 is
            // not a token end: the block loop's resume mask handles it)
            bool fast = resume == 0 || resume < c0;
            uint32_t starts = 0, ends = 0, ns = 0, ne = 0, ex = 0, NS = 0, NE = 0, wlast = 0;
            uint4 x = make_uint4(0, 0, 0, 0);
            if (fast) {
                const uint32_t base = c0 + 16u * (uint32_t)lane;
                x = *reinterpret_cast<const uint4*>(L.win + (base & (kWin - 1)));
                const uint32_t before = lane == 0 ? ptail : *reinterpret_cast<const uint32_t*>(L.win + ((base - 4u) & (kWin - 1)));
                const uint32_t after = *reinterpret_cast<const uint32_t*>(L.win + ((base + 16u) & (kWin - 1)));
                // 24 bytes: [base - 4, base + 20), bit j = byte base - 4 + j
                uint32_t w24 = 0, q24 = 0, s24 = 0;
                const uint32_t xs[6] = {before, x.x, x.y, x.z, x.w, after};
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    uint32_t a, b, d;
                    classify4(xs[k], a, b, d);
                    w24 |= a << (4 * k);
                    q24 |= b << (4 * k);
                    s24 |= d << (4 * k);
                }
                // bytes outside [0, nb)
                const int64_t lo_pos = (int64_t)base - 4, hi_pos = (int64_t)base + 20;
                const uint32_t v_lo = lo_pos >= 0 ? 0u : (uint32_t)(-lo_pos);          // invalid low bytes
                const uint32_t v_hi = hi_pos <= (int64_t)nb ? 24u : (uint32_t)max<int64_t>((int64_t)nb - lo_pos, 0);
                const uint32_t vm = (v_hi >= 24 ? 0xFFFFFFu : (1u << v_hi) - 1u) & ~((1u << v_lo) - 1u);
                w24 &= vm;
                q24 &= vm;
                s24 &= vm;
                const uint32_t join = q24 & (w24 << 1) & ((s24 >> 1) | (s24 << 1));
                const uint32_t W = w24 | join;
                const uint32_t tri = q24 & (s24 >> 1) & (q24 >> 2);   // "'s'" starting at bit j
                const bool hazard = (tri & 0x000FFFFEu) != 0 || (lane == kWave - 1 && (join & (3u << 18)) != 0);
                const uint32_t wm = (W >> 4) & 0xFFFFu, prev = (W >> 3) & 1u;
                const uint32_t wp = ((wm << 1) | prev) & 0xFFFFu;
                starts = wm & ~wp;
                ends = ~wm & wp & 0xFFFFu;
                wlast = (uint32_t)__builtin_amdgcn_readlane((int)(wm >> 15), kWave - 1);
                ns = (uint32_t)__builtin_popcount(starts);
                ne = (uint32_t)__builtin_popcount(ends);
                const uint32_t inc = wave_incl_scan(ns | (ne << 16));
                ex = inc - (ns | (ne << 16));
                const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
                NS = tot & 0xFFFFu;
                NE = tot >> 16;
                const uint32_t o = open ? 1u : 0u;   // (ends pair with the open token, then the starts)
                fast = __ballot(hazard) == 0 && NS + NE <= kFastPos && NE <= NS + o && NS + o <= NE + 1;
            }
            if (fast) {
                // run starts then run ends, as chunk offsets, in the (empty) queue's key area
                uint16_t* S = reinterpret_cast<uint16_t*>(L.qlo);
                uint16_t* E = S + NS;
                for (uint32_t m = starts, k = ex & 0xFFFFu; m; m &= m - 1, ++k)
                    S[k] = (uint16_t)(16u * (uint32_t)lane + (uint32_t)__builtin_ctz(m));
                for (uint32_t m = ends, k = ex >> 16; m; m &= m - 1, ++k)
                    E[k] = (uint16_t)(16u * (uint32_t)lane + (uint32_t)__builtin_ctz(m));
                asm volatile("" ::: "memory");
                const uint32_t o = open ? 1u : 0u;
                auto token = [&](uint32_t k, uint64_t& lo, uint64_t& hi, uint32_t& a, uint32_t& len) {
                    const bool first = k < o;   // the open token: its bytes were read at its start
                    a = first ? ostart : c0 + S[k - o];
                    len = c0 + E[k] - a;
                    if (first) {
                        lo = olo;
                        hi = ohi;
                    } else {
                        window_key(L.win, a, lo, hi);
                    }
                    mask_key(len, lo, hi);
                };
                for (uint32_t t0 = 0; t0 < NE && !over; t0 += kWave) {
                    const uint32_t k = t0 + (uint32_t)lane;
                    const bool act = k < NE;
                    uint64_t lo = 0, hi = 0;
                    uint32_t a = 0, len = 0;
                    if (act) token(k, lo, hi, a, len);
                    // (never taken -- the pairing was checked above -- but a token outside the text
                    // must not reach the reads below: the file would go to the host instead)
                    if (__ballot(act && (len == 0 || a >= nb || len > nb - a))) {
                        over = true;
                        break;
                    }
                    if (!(WORDS_DIAG & 1)) words += lookup_tokens(L, act, lo, hi, len, a, v, ft, fm);
                    if (words > (uint32_t)kSetMax) over = true;
                }
                // the last start without an end stays open (its first 16 bytes read now, while
                // its chunk is in the window)
                if (NS + o == NE) {
                    open = false;
                } else if (NS > 0) {   // (NS == 0: the open token runs on through the chunk)
                    open = true;
                    ostart = rfl(c0 + (uint32_t)S[NS - 1]);
                    window_key_u(L.win, ostart, olo, ohi);
                }
                prevw = wlast;   // (the block loop's view: a joined apostrophe continues the run)
                ptail = (uint32_t)__builtin_amdgcn_readlane((int)x.w, kWave - 1);
                asm volatile("" ::: "memory");
                if (c + 2 < nchunks) chunk_store(c + 2, nx);   // into the slot of chunk c
                continue;
            }
#endif
            for (uint32_t b0 = c * kChunk; b0 < nb && b0 < (c + 1) * kChunk && !(WORDS_DIAG & 4); b0 += kWave) {
                const uint32_t p = b0 + (uint32_t)lane;
                const uint32_t ch = p < nb ? L.win[p & (kWin - 1)] : 0u;
                const uint64_t w = __ballot(p < nb && word_byte(ch));
                const uint64_t q = __ballot(p < nb && ch == '\'');
                const uint64_t wp = (w << 1) | prevw;
                uint64_t starts = w & ~wp, ends = ~w & wp;
                prevw = w >> 63;
                if (resume >= b0 && resume > 0) {
                    const uint32_t r = resume - b0;
                    if (r >= 64) continue;
                    starts &= ~0ull << r;
                    ends &= r >= 63 ? 0ull : ~0ull << (r + 1);
                }
                // A run ending at an apostrophe continues the token when an 's' precedes or follows
                // the apostrophe ('s, s'): such blocks take the regex's order serially (rare:
                // possessives); a run ending at any other apostrophe ends there, as in the fast path.
                const uint64_t sm = __ballot(p < nb && ch == 's');
                if (ends & q & ((sm >> 1) | (sm << 1) | 1ull | (1ull << 63))) {
                    // the byte at x: from the window for chunks c and c + 1, else from memory (an open
                    // token's earlier bytes; a re-scan running past the next chunk)
                    auto byte_at = [&](uint32_t x) -> uint32_t {
                        return rfl(x >= c * kChunk && x < (c + 2) * kChunk ? (uint32_t)L.win[x & (kWin - 1)] : (uint32_t)ft[x]);
                    };
                    auto finish = [&](uint32_t a, uint32_t e) {
                        if ((q >> (e - b0)) & 1u) {
                            // the regex's loop from the run end (the run itself holds no apostrophe)
                            uint32_t x = e, prev = byte_at(e - 1);
                            for (;;) {
                                if (x < nb && byte_at(x) == '\'') {
                                    if (x + 1 < nb && byte_at(x + 1) == 's') x += 2;
                                    else if (prev == 's') x += 1;
                                }
                                if (!(x < nb && word_byte(byte_at(x)))) break;
                                prev = byte_at(x++);
                            }
                            if (x > e) {
                                resume = x;
                                const uint32_t r = x - b0;
                                starts = r >= 64 ? 0ull : starts & (~0ull << r);
                                ends = r >= 63 ? 0ull : ends & (~0ull << (r + 1));
                            }
                            e = x;
                        }
                        uint64_t lo = olo, hi = ohi;   // the open token's bytes, read at its start
                        if (a >= b0) window_key_u(L.win, a, lo, hi);
                        mask_key(e - a, lo, hi);
                        push(lane == 0, a, e - a, lo, hi);
                        flush(kQKeep);
                    };
                    if (open) {
                        const uint32_t e = b0 + (uint32_t)__builtin_ctzll(ends);
                        ends &= ends - 1;
                        open = false;
                        finish(ostart, e);
                    }
                    while (starts) {
                        const uint32_t a = b0 + (uint32_t)__builtin_ctzll(starts);
                        starts &= starts - 1;
                        if (!ends) {
                            open = true;
                            ostart = a;
                            window_key_u(L.win, a, olo, ohi);
                            break;
                        }
                        const uint32_t e = b0 + (uint32_t)__builtin_ctzll(ends);
                        ends &= ends - 1;
                        finish(a, e);
                    }
                    continue;
                }
                // the open token ends at this block's first run end
                if (open && ends) {
                    const uint32_t e = b0 + (uint32_t)__builtin_ctzll(ends);
                    const uint32_t len = e - ostart;
                    uint64_t lo = olo, hi = ohi;   // (read from the window at its start)
                    mask_key(len, lo, hi);
                    push(lane == 0, ostart, len, lo, hi);
                    open = false;
                }
                // this block's tokens: a start lane's run ends in the block, except the last one's
                const bool st = (starts >> lane) & 1u;
                const uint64_t rest = ~w >> lane;
                const bool ends_here = st && (rest != 0);
                uint64_t lo = 0, hi = 0;
                uint32_t len = 0;
                if (st && !(WORDS_DIAG & 2)) window_key(L.win, p, lo, hi);
                if (ends_here) {
                    len = (uint32_t)__builtin_ctzll(rest);
                    mask_key(len, lo, hi);
                }
                const uint64_t stay = __ballot(st && !ends_here);   // at most one lane: the block's last run
                if (stay) {
                    const int sl = 63 - __builtin_clzll(stay);
                    open = true;
                    ostart = b0 + (uint32_t)sl;
                    olo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lo, sl)) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(lo >> 32), sl) << 32);
                    ohi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hi, sl)) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hi >> 32), sl) << 32);
                }
                if (!(WORDS_DIAG & 2)) push(ends_here, p, len, lo, hi);
                flush(kQKeep);   // room for the next block's tokens (at most 33)
            }
#if !WORDS_BLOCKS_ONLY
            flush(0);   // (the next chunk may take the fast path, which uses the queue's key area)
            ptail = rfl(*reinterpret_cast<const uint32_t*>(L.win + ((c0 + kChunk - 4u) & (kWin - 1))));
#endif
            if (c + 2 < nchunks) chunk_store(c + 2, nx);   // into the slot of chunk c
        }
        if (open && !over) {   // the last run reaches the end of the text
            const uint32_t len = nb - ostart;
            uint64_t lo = olo, hi = ohi;
            mask_key(len, lo, hi);
            push(lane == 0, ostart, len, lo, hi);
        }
        flush(0);
        const uint64_t fmw = wave_or64(fm);
        uint32_t bits = 0;
        for (int32_t j = lane; j < 2 * w64; j += kWave) bits += (uint32_t)__builtin_popcount(L.row[j]);
        const uint32_t wf = wave_sum(bits) + (uint32_t)__builtin_popcountll(fmw) + words;
        uint64_t* out = rows + f * (int64_t)w64;
        for (int32_t j = lane; j < w64; j += kWave)
            out[j] = over ? 0ull : ((uint64_t)L.row[2 * j] | ((uint64_t)L.row[2 * j + 1] << 32));
        if (lane == 0) {
            wf_out[f] = over ? 0u : wf;
            fmask_out[f] = over ? 0ull : fmw;
            status[f] = over ? 1 : 0;
            if (over) atomicAdd(counters, 1u);
            else if (wf > max_lf) atomicAdd(counters + 1, 1u);
        }
    }
}

}  // namespace dice

// ---- host side ---------------------------------------------------------------------------

namespace dice {

void words_free(dice_ctx* c) {
    void* p[] = {c->d_wslots, c->d_wkeys, c->d_wlen, c->d_woff, c->d_wtxt};
    for (void* x : p)
        if (x) (void)hipFree(x);
    c->d_wslots = c->d_wkeys = c->d_wlen = c->d_woff = c->d_wtxt = nullptr;
    c->words_ready = false;
}

namespace {

struct WGuard {
    int prev = -1;
    explicit WGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~WGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <class T>
int grow(T** p, size_t& cap, size_t need) {
    if (*p && cap >= need) return DICE_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    int rc = dalloc_bytes(reinterpret_cast<void**>(p), need);
    if (!rc) cap = need;
    return rc;
}

void host_key(const std::string& w, uint64_t& lo, uint64_t& hi, uint32_t& tail) {
    lo = hi = 0;
    for (size_t i = 0; i < w.size() && i < 16; ++i) {
        const uint64_t b = (unsigned char)w[i];
        if (i < 8) lo |= b << (8 * i);
        else hi |= b << (8 * (i - 8));
    }
    tail = 0;
    if (w.size() > 16) {
        tail = 2166136261u;
        for (size_t i = 16; i < w.size(); ++i) tail = fnv_step(tail, (unsigned char)w[i]);
    }
}

__global__ __launch_bounds__(256) void dice_words_set_rows(const int64_t* __restrict__ idx, int64_t k,
                                                           const uint64_t* __restrict__ bits,
                                                           const uint32_t* __restrict__ wf,
                                                           const uint64_t* __restrict__ fm, int32_t w64,
                                                           uint64_t* __restrict__ rows, uint32_t* __restrict__ d_wf,
                                                           uint64_t* __restrict__ d_fm) {
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & (kWave - 1);
    if (j >= k) return;
    const int64_t f = idx[j];
    for (int32_t q = lane; q < w64; q += kWave) rows[f * w64 + q] = bits[j * w64 + q];
    if (lane == 0) {
        d_wf[f] = wf[j];
        d_fm[f] = fm ? fm[j] : 0ull;
    }
}

}  // namespace
}  // namespace dice

using dice::fail;

extern "C" {

int dice_vocab_setup(dice_ctx* c, int32_t n_words, const char* const* words, int32_t n_extra,
                     const char* const* extra) {
    if (!c) return fail(DICE_E_ARG, "NULL ctx");
    if (n_words != c->V) return fail(DICE_E_ARG, "n_words must equal the context's vocabulary size");
    if (n_extra < 0 || n_extra > 64) return fail(DICE_E_ARG, "n_extra must be in [0, 64]");
    if ((n_words > 0 && !words) || (n_extra > 0 && !extra)) return fail(DICE_E_ARG, "NULL word list");
    if (dice::words_lds_per_wave(c->w64) * dice::kWordsWaves > 160 * 1024)
        return fail(DICE_E_ARG, "vocabulary too large for the device wordset scan");
    const int32_t n = n_words + n_extra;
    std::vector<std::string> w((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        const char* s = i < n_words ? words[i] : extra[i - n_words];
        if (!s || !*s) return fail(DICE_E_ARG, "empty or NULL word");
        w[(size_t)i] = s;
        for (unsigned char ch : w[(size_t)i])
            if (ch >= 0x80) return fail(DICE_E_ARG, "words are ASCII (the wordset scan's [\\w/-])");
    }
    size_t nb = 2;
    while (nb * dice::kSlots < 2 * (size_t)n + 1) nb <<= 1;
    uint32_t id_bits = 1;
    while (((uint64_t)1 << id_bits) <= (uint64_t)n + 1) ++id_bits;
    if (id_bits > 28) return fail(DICE_E_ARG, "too many words");
    std::vector<uint32_t> slots(nb * dice::kSlots, 0), wlen((size_t)n), woff((size_t)n);
    std::vector<uint4> keys((size_t)n);
    std::string txt;
    for (int32_t i = 0; i < n; ++i) {
        uint64_t lo, hi;
        uint32_t tail;
        dice::host_key(w[(size_t)i], lo, hi, tail);
        keys[(size_t)i] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        wlen[(size_t)i] = (uint32_t)w[(size_t)i].size();
        woff[(size_t)i] = (uint32_t)txt.size();
        txt += w[(size_t)i];
        const uint64_t h = dice::words_mix(lo, hi, wlen[(size_t)i], tail);
        const uint32_t tag = ((uint32_t)(h >> 40)) << id_bits;
        for (size_t b = h & (nb - 1);; b = (b + 1) & (nb - 1)) {
            uint32_t* r = slots.data() + b * dice::kSlots;
            int j = 0;
            while (j < dice::kSlots && r[j]) {
                const uint32_t id = (r[j] & ((1u << id_bits) - 1u)) - 1u;
                if (w[id] == w[(size_t)i]) return fail(DICE_E_ARG, "duplicate word: " + w[(size_t)i]);
                ++j;
            }
            if (j < dice::kSlots) {
                r[j] = tag | (uint32_t)(i + 1);
                break;
            }
        }
    }
    if (txt.empty()) txt.push_back(0);
    dice::WGuard g(c->device);
    dice::words_free(c);
    int rc;
    if ((rc = dice::dalloc_bytes(&c->d_wslots, slots.size() * 4)) || (rc = dice::dalloc_bytes(&c->d_wkeys, keys.size() * 16 + 16)) ||
        (rc = dice::dalloc_bytes(&c->d_wlen, wlen.size() * 4 + 4)) || (rc = dice::dalloc_bytes(&c->d_woff, woff.size() * 4 + 4)) ||
        (rc = dice::dalloc_bytes(&c->d_wtxt, txt.size() + 64)))
        return rc;
    if (hipMemcpy(c->d_wslots, slots.data(), slots.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (n && hipMemcpy(c->d_wkeys, keys.data(), keys.size() * 16, hipMemcpyHostToDevice) != hipSuccess) ||
        (n && hipMemcpy(c->d_wlen, wlen.data(), wlen.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        (n && hipMemcpy(c->d_woff, woff.data(), woff.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(c->d_wtxt, txt.data(), txt.size(), hipMemcpyHostToDevice) != hipSuccess)
        return fail(DICE_E_DEVICE, "vocabulary table upload failed");
    c->words_bmask = (uint32_t)(nb - 1);
    c->words_id_bits = id_bits;
    c->words_extra = (uint32_t)n_extra;
    c->words_ready = true;
    return DICE_OK;
}

int dice_batch_upload_text(dice_batch* b, int64_t n, const uint8_t* text, int64_t text_bytes, const int64_t* offsets,
                           const int32_t* text_len, const int32_t* length, const uint8_t* cc, uint8_t* status,
                           int64_t* n_overflow, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (!c->words_ready) return fail(DICE_E_STATE, "dice_vocab_setup was not called");
    if (n < 0 || n > b->capacity) return fail(DICE_E_ARG, "n_files exceeds batch capacity");
    if (n > 0 && (!text || !offsets || !text_len || !length || !cc || !status)) return fail(DICE_E_ARG, "NULL file arrays");
    if (text_bytes < 0) return fail(DICE_E_ARG, "negative text_bytes");
    for (int64_t i = 0; i < n; ++i) {
        if (offsets[i] < 0 || (offsets[i] & 15) || text_len[i] < 0 || offsets[i] + text_len[i] > text_bytes)
            return fail(DICE_E_ARG, "file " + std::to_string(i) + ": offsets must be 16-byte aligned and inside the text");
    }
    dice::WGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int rc;
    size_t cap8 = (size_t)b->capacity * 8, cap4 = (size_t)b->capacity * 4, cap1 = (size_t)b->capacity, capc = 16;
    size_t tneed = (size_t)text_bytes + 64;   // (load32's slack past the last token)
    if (tneed > b->text_cap) {
        if (hipStreamSynchronize(s) != hipSuccess) return fail(DICE_E_DEVICE, "hipStreamSynchronize failed");
        if ((rc = dice::grow(&b->d_text, b->text_cap, tneed))) return rc;
    }
    size_t dummy = 0;
    if (!b->d_toff && (rc = dice::grow(&b->d_toff, dummy, cap8))) return rc;
    if (!b->d_tlen && (rc = dice::grow(&b->d_tlen, dummy, cap4))) return rc;
    if (!b->d_wstat && (rc = dice::grow(&b->d_wstat, dummy, cap1))) return rc;
    if (!b->d_wcnt && (rc = dice::grow(&b->d_wcnt, dummy, capc))) return rc;
    if (!b->d_fmask && (rc = dice::grow(&b->d_fmask, dummy, cap8))) return rc;
    b->n = n;
    b->n_long = 0;
    if (n_overflow) *n_overflow = 0;
    if (n == 0) return DICE_OK;
    if (hipMemcpyAsync(b->d_text, text, (size_t)text_bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(b->d_toff, offsets, (size_t)n * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(b->d_tlen, text_len, (size_t)n * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(b->d_wcnt, 0, 16, s) != hipSuccess)   // (overflow, long, next file)
        return fail(DICE_E_DEVICE, "text upload failed");
    dice::VocabDev v;
    v.slots = (const uint32_t*)c->d_wslots;
    v.keys = (const uint4*)c->d_wkeys;
    v.wmeta = (const uint32_t*)c->d_wlen;
    v.woff = (const uint32_t*)c->d_woff;
    v.wtxt = (const uint8_t*)c->d_wtxt;
    v.bmask = c->words_bmask;
    v.id_bits = c->words_id_bits;
    v.V = (uint32_t)c->V;
    v.n_extra = c->words_extra;
    const size_t lds = dice::words_lds_per_wave(c->w64) * dice::kWordsWaves;
    const int64_t groups = std::min<int64_t>((n + dice::kWordsWaves - 1) / dice::kWordsWaves, (int64_t)c->n_cu * 4);
    hipLaunchKernelGGL(dice::dice_words_kernel, dim3((unsigned)groups), dim3(dice::kWordsWaves * dice::kWave), lds, s,
                       (const uint8_t*)b->d_text, text_bytes, (const int64_t*)b->d_toff, (const int32_t*)b->d_tlen, n, v,
                       c->w64, b->d_rows, b->d_wf, b->d_fmask, b->d_wstat, b->d_wcnt,
                       c->kind == 3 && c->prune ? c->prune_max_lf : 0xFFFFFFFFu);
    if (hipGetLastError() != hipSuccess) return fail(DICE_E_DEVICE, "dice_words_kernel launch failed");
    uint32_t cnt[2] = {0, 0};
    if (hipMemcpyAsync(status, b->d_wstat, (size_t)n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(cnt, b->d_wcnt, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return fail(DICE_E_DEVICE, "wordset status download failed");
    if (n_overflow) *n_overflow = cnt[0];
    b->n_long = cnt[1];
    return dice::upload_tail(b, n, nullptr, length, cc, s);
}

int dice_batch_set_rows(dice_batch* b, int64_t k, const int64_t* index, const uint64_t* bits, const uint32_t* wordset_size,
                        const uint64_t* field_mask, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (k < 0 || (k > 0 && (!index || !bits || !wordset_size))) return fail(DICE_E_ARG, "NULL row arrays");
    for (int64_t j = 0; j < k; ++j)
        if (index[j] < 0 || index[j] >= b->n) return fail(DICE_E_ARG, "row index outside the batch");
    if (k == 0) return DICE_OK;
    dice::WGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int rc;
    size_t dummy = 0;
    if (!b->d_fmask && (rc = dice::grow(&b->d_fmask, dummy, (size_t)b->capacity * 8))) return rc;
    // staging: [index | wf | field masks | rows]
    const size_t bytes = (size_t)k * (8 + 4 + 8 + (size_t)c->w64 * 8) + 64;
    void* d = nullptr;
    if ((rc = dice::dalloc_bytes(&d, bytes))) return rc;
    char* p = (char*)d;
    int64_t* d_idx = (int64_t*)p;
    uint64_t* d_fm = (uint64_t*)(p + (size_t)k * 8);
    uint64_t* d_bits = (uint64_t*)(p + (size_t)k * 16);
    uint32_t* d_w = (uint32_t*)(p + (size_t)k * 16 + (size_t)k * c->w64 * 8);
    bool ok = hipMemcpyAsync(d_idx, index, (size_t)k * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
              hipMemcpyAsync(d_bits, bits, (size_t)k * c->w64 * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
              hipMemcpyAsync(d_w, wordset_size, (size_t)k * 4, hipMemcpyHostToDevice, s) == hipSuccess &&
              (!field_mask || hipMemcpyAsync(d_fm, field_mask, (size_t)k * 8, hipMemcpyHostToDevice, s) == hipSuccess);
    if (ok) {
        hipLaunchKernelGGL(dice::dice_words_set_rows, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, s, d_idx, k, d_bits, d_w,
                           field_mask ? d_fm : nullptr, c->w64, b->d_rows, b->d_wf, b->d_fmask);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
    }
    (void)hipFree(d);
    if (!ok) return fail(DICE_E_DEVICE, "row patch failed");
    if (c->kind == 3) {
        if (c->prune)
            for (int64_t j = 0; j < k; ++j) b->n_long += wordset_size[j] > c->prune_max_lf;
        return DICE_OK;
    }
    // the tile-layout kernels: repack (lengths and CC flags are already resident)
    return dice::repack(b, s);
}

int dice_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes < 0) return fail(DICE_E_ARG, "invalid host allocation");
    *out = nullptr;
    if (hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return fail(DICE_E_NOMEM, "hipHostMalloc failed");
    }
    return DICE_OK;
}

void dice_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int dice_batch_download_rows(dice_batch* b, uint64_t* bits, uint32_t* wordset_size, uint64_t* field_mask, void* stream) {
    if (!b) return fail(DICE_E_ARG, "NULL batch");
    dice_ctx* c = b->ctx;
    if (field_mask && b->n && !b->d_fmask) return fail(DICE_E_STATE, "the batch holds no field masks");
    dice::WGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const size_t n = (size_t)b->n;
    if (n && ((bits && hipMemcpyAsync(bits, b->d_rows, n * c->w64 * 8, hipMemcpyDeviceToHost, s) != hipSuccess) ||
              (wordset_size && hipMemcpyAsync(wordset_size, b->d_wf, n * 4, hipMemcpyDeviceToHost, s) != hipSuccess) ||
              (field_mask && hipMemcpyAsync(field_mask, b->d_fmask, n * 8, hipMemcpyDeviceToHost, s) != hipSuccess)))
        return fail(DICE_E_DEVICE, "row download failed");
    return hipStreamSynchronize(s) == hipSuccess ? DICE_OK : fail(DICE_E_DEVICE, "hipStreamSynchronize failed");
}

}  // extern "C"
