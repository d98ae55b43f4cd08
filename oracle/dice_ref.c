/*
 * ORACLE -- test infrastructure only (CPU baseline "port" + large-scale parity checker).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library;
 * the product (licensee_amd) never does.
 *
 * A C restatement of licensee's Dice scoring over interned word ids, following the
 * reference algorithm step for step:
 *
 *   License#similarity  lib/licensee/content_helper.rb:128-133
 *       overlap = (wordset_fieldless & other.wordset).size  -- Ruby Set#& iterates the
 *                 smaller set and probes the larger one's hash (set.rb), restated here
 *                 with open-addressing hash sets of word ids;
 *       total   = wordset_fieldless.size + other.wordset.size - fields_normalized_set.size
 *       score   = (overlap * 200.0) / (total + variation_adjusted_length_delta / 4)
 *   variation_adjusted_length_delta  content_helper.rb:337-347 (Integer, floor division /4)
 *   Dice#potential_matches (CC filter) lib/licensee/matchers/dice.rb:23-31
 *   Dice#matches_by_similarity / #match / #confidence  dice.rb:8-14,34-53: sort descending,
 *       first with score >= threshold. The sort is restated as an argmax over IEEE doubles;
 *       exact ties (parity-unpinned: Ruby's sort is unstable) go to the later template,
 *       the documented rule shared with the HIP kernels.
 *
 * Also a bitset variant (AND + popcount) as a stronger CPU comparison.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t cap;      /* power of two */
    int32_t *slots;   /* word id or -1 */
} idset;

static uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

static int idset_init(idset *s, const int32_t *ids, int32_t n) {
    int32_t cap = 16;
    while (cap < 2 * n + 1) cap <<= 1;
    s->cap = cap;
    s->slots = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
    if (!s->slots) return -1;
    memset(s->slots, 0xff, sizeof(int32_t) * (size_t)cap);
    for (int32_t i = 0; i < n; ++i) {
        uint32_t h = mix32((uint32_t)ids[i]) & (uint32_t)(cap - 1);
        while (s->slots[h] >= 0 && s->slots[h] != ids[i]) h = (h + 1) & (uint32_t)(cap - 1);
        s->slots[h] = ids[i];
    }
    return 0;
}

static int idset_has(const idset *s, int32_t id) {
    uint32_t h = mix32((uint32_t)id) & (uint32_t)(s->cap - 1);
    for (;;) {
        int32_t v = s->slots[h];
        if (v == id) return 1;
        if (v < 0) return 0;
        h = (h + 1) & (uint32_t)(s->cap - 1);
    }
}

typedef struct {
    int32_t T, V, w64;
    int32_t *lf_off, *lf_ids;   /* CSR of template wordset_fieldless ids */
    idset *lf_set;
    uint64_t *lf_bits;          /* [T][w64] */
    int32_t *base, *slack, *len;
    uint8_t *cc;
} oracle_ctx;

void oracle_destroy(oracle_ctx *c) {
    if (!c) return;
    if (c->lf_set)
        for (int32_t t = 0; t < c->T; ++t) free(c->lf_set[t].slots);
    free(c->lf_set); free(c->lf_off); free(c->lf_ids); free(c->lf_bits);
    free(c->base); free(c->slack); free(c->len); free(c->cc);
    free(c);
}

/* Templates given as CSR word-id lists (ids < V). */
oracle_ctx *oracle_create(int32_t T, int32_t V, const int32_t *lf_off, const int32_t *lf_ids,
                          const uint32_t *fields_set_size, const int32_t *length_slack,
                          const int32_t *length, const uint8_t *is_cc) {
    oracle_ctx *c = (oracle_ctx *)calloc(1, sizeof(oracle_ctx));
    if (!c) return NULL;
    c->T = T; c->V = V; c->w64 = (V + 63) / 64;
    int32_t nnz = lf_off[T];
    c->lf_off = (int32_t *)malloc(sizeof(int32_t) * (size_t)(T + 1));
    c->lf_ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    c->lf_set = (idset *)calloc((size_t)T, sizeof(idset));
    c->lf_bits = (uint64_t *)calloc((size_t)T * (size_t)c->w64, sizeof(uint64_t));
    c->base = (int32_t *)malloc(sizeof(int32_t) * (size_t)T);
    c->slack = (int32_t *)malloc(sizeof(int32_t) * (size_t)T);
    c->len = (int32_t *)malloc(sizeof(int32_t) * (size_t)T);
    c->cc = (uint8_t *)malloc((size_t)T);
    if (!c->lf_off || !c->lf_ids || !c->lf_set || !c->lf_bits || !c->base || !c->slack || !c->len || !c->cc) {
        oracle_destroy(c);
        return NULL;
    }
    memcpy(c->lf_off, lf_off, sizeof(int32_t) * (size_t)(T + 1));
    memcpy(c->lf_ids, lf_ids, sizeof(int32_t) * (size_t)nnz);
    for (int32_t t = 0; t < T; ++t) {
        int32_t a = lf_off[t], n = lf_off[t + 1] - lf_off[t];
        if (idset_init(&c->lf_set[t], lf_ids + a, n)) { oracle_destroy(c); return NULL; }
        for (int32_t i = 0; i < n; ++i) {
            int32_t id = lf_ids[a + i];
            c->lf_bits[(size_t)t * c->w64 + (id >> 6)] |= 1ULL << (id & 63);
        }
        c->base[t] = n - (int32_t)fields_set_size[t];
        c->slack[t] = length_slack[t];
        c->len[t] = length[t];
        c->cc[t] = is_cc[t];
    }
    return c;
}

static int32_t den_of(const oracle_ctx *c, int32_t t, uint32_t wf, int32_t lenf) {
    int32_t d = c->len[t] - lenf;
    if (d < 0) d = -d;
    int32_t adj = c->slack[t] < 0 ? d : (d - c->slack[t] > 0 ? d - c->slack[t] : 0);
    return c->base[t] + (int32_t)wf + adj / 4;
}

typedef struct {
    const oracle_ctx *c;
    int64_t lo, hi;
    int mode;                      /* 0 hash (Set#&), 1 bitset */
    const int64_t *f_off;          /* CSR of file in-vocabulary word ids */
    const int32_t *f_ids;
    const uint64_t *f_bits;        /* [n][w64] for bitset mode */
    const uint32_t *wf;
    const int32_t *lenf;
    const uint8_t *ccfp;
    double thr;
    int32_t *best;
    uint32_t *ov_out;
    double *score_out;
    uint32_t *mat_ov;              /* optional [n][T] */
    double *mat_score;
} job;

static uint32_t overlap_hash(const oracle_ctx *c, int32_t t, const int32_t *ids, int32_t nids,
                             const idset *fset, uint32_t wf) {
    /* Set#&: iterate the smaller set, probe the larger (other.wordset.size counts OOV words). */
    int32_t a = c->lf_off[t], na = c->lf_off[t + 1] - a;
    uint32_t n = 0;
    if ((uint32_t)na <= wf) {
        for (int32_t i = 0; i < na; ++i) n += (uint32_t)idset_has(fset, c->lf_ids[a + i]);
    } else {
        for (int32_t i = 0; i < nids; ++i) n += (uint32_t)idset_has(&c->lf_set[t], ids[i]);
    }
    return n;
}

static void *run_job(void *arg) {
    job *j = (job *)arg;
    const oracle_ctx *c = j->c;
    for (int64_t f = j->lo; f < j->hi; ++f) {
        idset fset = {0, NULL};
        const int32_t *ids = NULL;
        int32_t nids = 0;
        if (j->mode == 0) {
            ids = j->f_ids + j->f_off[f];
            nids = (int32_t)(j->f_off[f + 1] - j->f_off[f]);
            if (idset_init(&fset, ids, nids)) return (void *)1;
        }
        int32_t best = -1;
        uint32_t bov = 0;
        double bs = 0.0;
        for (int32_t t = 0; t < c->T; ++t) {
            uint32_t ov;
            if (j->mode == 0) {
                ov = overlap_hash(c, t, ids, nids, &fset, j->wf[f]);
            } else {
                const uint64_t *fb = j->f_bits + (size_t)f * c->w64, *tb = c->lf_bits + (size_t)t * c->w64;
                ov = 0;
                for (int32_t w = 0; w < c->w64; ++w) ov += (uint32_t)__builtin_popcountll(fb[w] & tb[w]);
            }
            int32_t den = den_of(c, t, j->wf[f], j->lenf[f]);
            double s = ((double)ov * 200.0) / (double)den;
            if (j->mat_ov) j->mat_ov[f * c->T + t] = ov;
            if (j->mat_score) j->mat_score[f * c->T + t] = s;
            if (c->cc[t] && j->ccfp[f]) continue;
            if (best < 0 || s >= bs) { best = t; bov = ov; bs = s; }
        }
        free(fset.slots);
        if (j->best) j->best[f] = (best >= 0 && bs >= j->thr) ? best : -1;
        if (j->ov_out) j->ov_out[f] = bov;
        if (j->score_out) j->score_out[f] = best >= 0 ? bs : 0.0;
    }
    return NULL;
}

static int run_threads(job *proto, int64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job jobs[256];
    int64_t chunk = (n + nthreads - 1) / nthreads;
    int started = 0, rc = 0;
    for (int i = 0; i < nthreads; ++i) {
        jobs[i] = *proto;
        jobs[i].lo = (int64_t)i * chunk;
        jobs[i].hi = jobs[i].lo + chunk < n ? jobs[i].lo + chunk : n;
        if (jobs[i].lo >= jobs[i].hi) break;
        if (pthread_create(&th[i], NULL, run_job, &jobs[i])) { rc = -1; break; }
        ++started;
    }
    for (int i = 0; i < started; ++i) {
        void *r = NULL;
        pthread_join(th[i], &r);
        if (r) rc = -1;
    }
    return rc;
}

/* Dice#match for every file: hash-set intersection (mode 0) or bitset popcount (mode 1).
 * Outputs follow dice_match() in include/licensee_dice.h. Returns 0 or -1. */
int oracle_match(const oracle_ctx *c, int64_t n, int mode, const int64_t *f_off, const int32_t *f_ids,
                 const uint64_t *f_bits, const uint32_t *wf, const int32_t *lenf, const uint8_t *ccfp,
                 double thr, int nthreads, int32_t *best, uint32_t *ov, double *score) {
    job p;
    memset(&p, 0, sizeof(p));
    p.c = c; p.mode = mode; p.f_off = f_off; p.f_ids = f_ids; p.f_bits = f_bits; p.wf = wf; p.lenf = lenf;
    p.ccfp = ccfp; p.thr = thr; p.best = best; p.ov_out = ov; p.score_out = score;
    return run_threads(&p, n, nthreads);
}

/* Full N x T overlap / score matrix (CC filter not applied), hash mode. */
int oracle_matrix(const oracle_ctx *c, int64_t n, const int64_t *f_off, const int32_t *f_ids,
                  const uint32_t *wf, const int32_t *lenf, const uint8_t *ccfp, int nthreads,
                  uint32_t *mat_ov, double *mat_score) {
    job p;
    memset(&p, 0, sizeof(p));
    p.c = c; p.mode = 0; p.f_off = f_off; p.f_ids = f_ids; p.wf = wf; p.lenf = lenf; p.ccfp = ccfp;
    p.thr = INFINITY; p.mat_ov = mat_ov; p.mat_score = mat_score;
    return run_threads(&p, n, nthreads);
}
