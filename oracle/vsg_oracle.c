/*
 * vsg_oracle.c — CPU restatement of the usearch HNSW path (TEST INFRASTRUCTURE).
 *
 * Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg, as the checker / baseline — never by the product.  See vsg_oracle.h for
 * the parity status ("HNSW parity unpinned against upstream usearch"; exact
 * path pinned by golden vectors and the reference KATs).
 *
 * Reference call sites restated (paths relative to /root/reference):
 *   usearch::Index::new + reserve      src/index/usearch.rs:89-99
 *   capacity()/size()/reserve()        src/index/usearch.rs:201-206
 *   remove(key)                        src/index/usearch.rs:215, :245
 *   add(key, &[f32])                   src/index/usearch.rs:221
 *   search(&[f32], k)                  src/index/usearch.rs:275-277
 *   size()                             src/index/usearch.rs:309
 * Algorithm inside those calls: unum-cloud/usearch (unpinned), restated from its
 * published index.hpp (HNSW) and index_plugins.hpp (metric_*_gt).
 */
#define _GNU_SOURCE
#include "vsg_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------ RNG -- */

uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* usearch choose_random_level_: level = floor(-ln(U) * 1/ln(M)).  The uniform
 * comes from a counter-based splitmix64 stream so the GPU index's host code
 * draws the identical level for the identical slot. */
int orc_sample_level(uint64_t seed, uint64_t slot, uint32_t connectivity) {
    uint64_t r = orc_splitmix64(orc_splitmix64(seed ^ 0x4C6576656C5EEDull) + slot);
    double u = (double)((r >> 11) + 1) * (1.0 / 9007199254740992.0); /* (0,1] */
    double lv = -log(u) / log((double)connectivity);
    int l = (int)lv;
    return l > 30 ? 30 : l;
}

/* --------------------------------------------------------------- metrics -- */

/* CPU-baseline mode: SIMD multi-accumulator kernels with FMA, dispatched to the
 * host's widest ISA (the shape of usearch's SimSIMD back-end; vsg_fast.c).  Parity mode (default): serial f32 loops exactly as the
 * generic metric_*_gt.  The baseline switches to fast mode only for timing. */
static int g_fast_metric = 0;
void orc_set_fast_metric(int on) { g_fast_metric = on; }

/* host-ISA kernels (vsg_fast.c: AVX-512 + FMA when present, as SimSIMD dispatches) */
float orc_fast_distance(int metric, const float* a, const float* b, size_t dim);

/* usearch metric_l2sq_gt / metric_ip_gt / metric_cos_gt, f32 result type. */
float orc_distance(int metric, const float* a, const float* b, size_t dim) {
    if (g_fast_metric) return orc_fast_distance(metric, a, b, dim);
    if (metric == ORC_METRIC_L2SQ) {
        float s = 0.f;
        for (size_t i = 0; i < dim; ++i) {
            float d = a[i] - b[i];
            s += d * d;
        }
        return s;
    }
    if (metric == ORC_METRIC_IP) {
        float s = 0.f;
        for (size_t i = 0; i < dim; ++i) s += a[i] * b[i];
        return 1.f - s;
    }
    float ab = 0.f, a2 = 0.f, b2 = 0.f;
    for (size_t i = 0; i < dim; ++i) {
        ab += a[i] * b[i];
        a2 += a[i] * a[i];
        b2 += b[i] * b[i];
    }
    if (a2 == 0.f && b2 == 0.f) return 0.f;
    if (a2 == 0.f || b2 == 0.f) return 1.f;
    return 1.f - ab / (sqrtf(a2) * sqrtf(b2));
}

/* ------------------------------------------------------------ threading -- */

typedef struct {
    void (*fn)(void* ctx, size_t i, int tid);
    void* ctx;
    size_t n;
    atomic_size_t next;
} par_job;

typedef struct {
    par_job* job;
    int tid;
} par_arg;

static void* par_worker(void* p) {
    par_arg* a = (par_arg*)p;
    for (;;) {
        size_t i = atomic_fetch_add(&a->job->next, 1);
        if (i >= a->job->n) break;
        a->job->fn(a->job->ctx, i, a->tid);
    }
    return NULL;
}

static int resolve_threads(int threads) {
    if (threads > 0) return threads;
    const char* env = getenv("SCYLLA_USEARCH_BACKGROUND_THREADS"); /* README.md:14-15 */
    if (env && atoi(env) > 0) return atoi(env);
    long n = sysconf(_SC_NPROCESSORS_ONLN);
    return n > 0 ? (int)n : 1;
}

static void parallel_for(size_t n, int threads, void (*fn)(void*, size_t, int), void* ctx) {
    if (threads <= 1 || n <= 1) {
        for (size_t i = 0; i < n; ++i) fn(ctx, i, 0);
        return;
    }
    if ((size_t)threads > n) threads = (int)n;
    par_job job = {fn, ctx, n, 0};
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    par_arg* args = (par_arg*)malloc(sizeof(par_arg) * threads);
    for (int t = 0; t < threads; ++t) {
        args[t].job = &job;
        args[t].tid = t;
        pthread_create(&th[t], NULL, par_worker, &args[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
    free(args);
}

/* ------------------------------------------------------ candidate lists -- */

typedef struct {
    float d;
    uint32_t id;
} cand_t;

static inline int cand_less(float da, uint32_t ia, float db, uint32_t ib) {
    return da < db || (da == db && ia < ib);
}

/* ---------------------------------------------------------- exact search -- */

typedef struct {
    int metric;
    const float* base;
    const uint64_t* keys;
    const uint8_t* removed;
    size_t n, dim;
    const float* q;
    size_t k;
    uint64_t* ok;
    float* od;
    size_t* oc;
} exact_ctx;

static void exact_one(void* p, size_t qi, int tid) {
    (void)tid;
    exact_ctx* c = (exact_ctx*)p;
    const float* q = c->q + qi * c->dim;
    uint64_t* ok = c->ok + qi * c->k;
    float* od = c->od + qi * c->k;
    size_t cnt = 0;
    for (size_t i = 0; i < c->n; ++i) {
        if (c->removed && c->removed[i]) continue;
        float d = orc_distance(c->metric, q, c->base + i * c->dim, c->dim);
        uint64_t key = c->keys ? c->keys[i] : (uint64_t)i;
        if (cnt == c->k) {
            float wd = od[cnt - 1];
            uint64_t wk = ok[cnt - 1];
            if (!(d < wd || (d == wd && key < wk))) continue;
            --cnt;
        }
        size_t pos = cnt;
        while (pos > 0 && (d < od[pos - 1] || (d == od[pos - 1] && key < ok[pos - 1]))) {
            od[pos] = od[pos - 1];
            ok[pos] = ok[pos - 1];
            --pos;
        }
        od[pos] = d;
        ok[pos] = key;
        ++cnt;
    }
    if (c->oc) c->oc[qi] = cnt;
    for (size_t j = cnt; j < c->k; ++j) {
        ok[j] = UINT64_MAX;
        od[j] = INFINITY;
    }
}

int orc_exact_search(int metric, const float* base, const uint64_t* keys,
                     const uint8_t* removed, size_t n, size_t dim,
                     const float* queries, size_t nq, size_t k,
                     uint64_t* out_keys, float* out_dist, size_t* out_counts,
                     int threads) {
    if (k == 0 || dim == 0) return 1;
    exact_ctx c = {metric, base, keys, removed, n, dim, queries, k, out_keys, out_dist, out_counts};
    parallel_for(nq, resolve_threads(threads), exact_one, &c);
    return 0;
}

/* ------------------------------------------------------------ key table -- */

typedef struct {
    uint64_t* keys; /* UINT64_MAX = empty, UINT64_MAX-1 = deleted */
    uint32_t* vals;
    size_t cap, used, live;
} keymap;

#define KM_EMPTY UINT64_MAX
#define KM_DEAD (UINT64_MAX - 1)

static size_t km_hash(uint64_t k, size_t cap) { return (size_t)(orc_splitmix64(k) & (cap - 1)); }

static void km_init(keymap* m, size_t cap) {
    m->cap = cap;
    m->used = m->live = 0;
    m->keys = (uint64_t*)malloc(cap * sizeof(uint64_t));
    m->vals = (uint32_t*)malloc(cap * sizeof(uint32_t));
    for (size_t i = 0; i < cap; ++i) m->keys[i] = KM_EMPTY;
}

static void km_free(keymap* m) {
    free(m->keys);
    free(m->vals);
}

static long km_find(const keymap* m, uint64_t k) {
    size_t i = km_hash(k, m->cap);
    for (;;) {
        if (m->keys[i] == KM_EMPTY) return -1;
        if (m->keys[i] == k) return (long)m->vals[i];
        i = (i + 1) & (m->cap - 1);
    }
}

static void km_put(keymap* m, uint64_t k, uint32_t v);

static void km_grow(keymap* m) {
    keymap n;
    km_init(&n, m->cap * 2);
    for (size_t i = 0; i < m->cap; ++i)
        if (m->keys[i] != KM_EMPTY && m->keys[i] != KM_DEAD) km_put(&n, m->keys[i], m->vals[i]);
    km_free(m);
    *m = n;
}

static void km_put(keymap* m, uint64_t k, uint32_t v) {
    if ((m->used + 1) * 2 > m->cap) km_grow(m);
    size_t i = km_hash(k, m->cap);
    for (;;) {
        if (m->keys[i] == KM_EMPTY) {
            m->keys[i] = k;
            m->vals[i] = v;
            m->used++;
            m->live++;
            return;
        }
        if (m->keys[i] == k) {
            m->vals[i] = v;
            return;
        }
        i = (i + 1) & (m->cap - 1);
    }
}

static int km_del(keymap* m, uint64_t k, uint32_t* v) {
    size_t i = km_hash(k, m->cap);
    for (;;) {
        if (m->keys[i] == KM_EMPTY) return 0;
        if (m->keys[i] == k) {
            *v = m->vals[i];
            m->keys[i] = KM_DEAD;
            m->live--;
            return 1;
        }
        i = (i + 1) & (m->cap - 1);
    }
}

/* ------------------------------------------------------------------ HNSW -- */

struct orc_hnsw {
    size_t dim;
    int metric;
    size_t M, M0, efC, ef;
    uint64_t seed;
    size_t cap, slots, live;
    float* vecs;
    uint64_t* keys;
    uint8_t* removed;
    int8_t* levels;
    uint32_t* adj0;
    uint32_t* upper_off;
    uint32_t* upper;
    size_t upper_cap;
    atomic_size_t upper_used;
    uint32_t entry;
    int max_level;
    pthread_mutex_t* node_locks;
    pthread_mutex_t global_lock;
    keymap km;
    /* usearch index_dense free_keys_: removed slots, oldest removal first
     * (ring[0] is the next to reuse); exactly the removed slots */
    uint32_t* ring;
    size_t ring_n, ring_cap;
    int reuse; /* 0: append-only adds (orc_hnsw_set_slot_reuse) */
    void* sscr; /* cached search scratch (scratch_t[sscr_n]) */
    int sscr_n;
    size_t sscr_slots, sscr_ef;
};

static inline const float* VEC(const orc_hnsw* h, uint32_t s) { return h->vecs + (size_t)s * h->dim; }

static inline uint32_t* ROW(const orc_hnsw* h, uint32_t s, int l) {
    if (l == 0) return h->adj0 + (size_t)s * h->M0;
    return h->upper + ((size_t)h->upper_off[s] + (size_t)(l - 1)) * h->M;
}

static inline size_t ROWLEN(const orc_hnsw* h, int l) { return l == 0 ? h->M0 : h->M; }

orc_hnsw* orc_hnsw_new(size_t dim, int metric, size_t connectivity, size_t expansion_add,
                       size_t expansion_search, uint64_t seed) {
    if (dim == 0 || metric < 0 || metric > 2) return NULL;
    orc_hnsw* h = (orc_hnsw*)calloc(1, sizeof(orc_hnsw));
    h->dim = dim;
    h->metric = metric;
    /* usearch defaults: default_connectivity()=16, default_expansion_add()=128,
     * default_expansion_search()=64; 0 from src/db.rs:400-410 means "default". */
    h->M = connectivity ? connectivity : 16;
    if (h->M < 2) h->M = 2;
    h->M0 = 2 * h->M;
    h->efC = expansion_add ? expansion_add : 128;
    h->ef = expansion_search ? expansion_search : 64;
    h->seed = seed;
    h->entry = ORC_EMPTY;
    h->max_level = -1;
    h->reuse = 1;
    pthread_mutex_init(&h->global_lock, NULL);
    km_init(&h->km, 1024);
    return h;
}

static void free_search_scratch(orc_hnsw* h);

void orc_hnsw_free(orc_hnsw* h) {
    if (!h) return;
    free_search_scratch(h);
    if (h->node_locks)
        for (size_t i = 0; i < h->cap; ++i) pthread_mutex_destroy(&h->node_locks[i]);
    free(h->node_locks);
    free(h->vecs);
    free(h->keys);
    free(h->removed);
    free(h->levels);
    free(h->adj0);
    free(h->upper_off);
    free(h->upper);
    free(h->ring);
    km_free(&h->km);
    pthread_mutex_destroy(&h->global_lock);
    free(h);
}

int orc_hnsw_reserve(orc_hnsw* h, size_t capacity) {
    if (capacity <= h->cap) return 0;
    size_t old = h->cap;
    h->vecs = (float*)realloc(h->vecs, capacity * h->dim * sizeof(float));
    h->keys = (uint64_t*)realloc(h->keys, capacity * sizeof(uint64_t));
    h->removed = (uint8_t*)realloc(h->removed, capacity);
    h->levels = (int8_t*)realloc(h->levels, capacity);
    h->adj0 = (uint32_t*)realloc(h->adj0, capacity * h->M0 * sizeof(uint32_t));
    h->upper_off = (uint32_t*)realloc(h->upper_off, capacity * sizeof(uint32_t));
    h->node_locks = (pthread_mutex_t*)realloc(h->node_locks, capacity * sizeof(pthread_mutex_t));
    if (!h->vecs || !h->keys || !h->removed || !h->levels || !h->adj0 || !h->upper_off || !h->node_locks)
        return 2;
    for (size_t i = old; i < capacity; ++i) pthread_mutex_init(&h->node_locks[i], NULL);
    memset(h->adj0 + old * h->M0, 0xFF, (capacity - old) * h->M0 * sizeof(uint32_t));
    memset(h->removed + old, 0, capacity - old);
    h->cap = capacity;
    return 0;
}

size_t orc_hnsw_size(const orc_hnsw* h) { return h->live; }
size_t orc_hnsw_slots(const orc_hnsw* h) { return h->slots; }
size_t orc_hnsw_capacity(const orc_hnsw* h) { return h->cap; }
size_t orc_hnsw_upper_rows(const orc_hnsw* h) { return atomic_load(&h->upper_used); }

void orc_hnsw_params(const orc_hnsw* h, size_t* M, size_t* M0, size_t* efC, size_t* ef) {
    *M = h->M;
    *M0 = h->M0;
    *efC = h->efC;
    *ef = h->ef;
}

void orc_hnsw_entry(const orc_hnsw* h, uint32_t* entry, int* max_level) {
    *entry = h->entry;
    *max_level = h->max_level;
}

/* Per-thread scratch: visited stamps + candidate lists. */
typedef struct {
    uint32_t* stamp;
    size_t stamp_cap;
    uint32_t gen;
    cand_t* list;
    uint8_t* expanded;
    size_t list_cap;
    uint32_t* nbr;
    cand_t* tmp;
    size_t tmp_cap;
    cand_t* heap; /* filtered search: usearch's `next` min-heap (grows) */
    size_t heap_cap;
    uint64_t ndist;
} scratch_t;

static void scratch_init(scratch_t* s, size_t slots, size_t list_cap, size_t M0) {
    memset(s, 0, sizeof(*s));
    s->stamp_cap = slots;
    s->stamp = (uint32_t*)calloc(slots ? slots : 1, sizeof(uint32_t));
    s->list_cap = list_cap;
    s->list = (cand_t*)malloc((list_cap + 1) * sizeof(cand_t));
    s->expanded = (uint8_t*)malloc(list_cap + 1);
    s->nbr = (uint32_t*)malloc(M0 * sizeof(uint32_t));
    s->tmp_cap = M0 + 1;
    s->tmp = (cand_t*)malloc(s->tmp_cap * sizeof(cand_t));
}

static void scratch_free(scratch_t* s) {
    free(s->stamp);
    free(s->list);
    free(s->expanded);
    free(s->nbr);
    free(s->tmp);
    free(s->heap);
}

static void free_search_scratch(orc_hnsw* h) {
    scratch_t* scr = (scratch_t*)h->sscr;
    for (int t = 0; scr && t < h->sscr_n; ++t) scratch_free(&scr[t]);
    free(scr);
    h->sscr = NULL;
    h->sscr_n = 0;
}

static inline void scratch_newgen(scratch_t* s) {
    if (++s->gen == 0) {
        memset(s->stamp, 0, s->stamp_cap * sizeof(uint32_t));
        s->gen = 1;
    }
}

/* Copy a node's adjacency row at level l (under its lock when concurrent). */
static size_t read_row(const orc_hnsw* h, uint32_t s, int l, uint32_t* out, int locked) {
    size_t m = ROWLEN(h, l);
    if (locked) pthread_mutex_lock(&h->node_locks[s]);
    const uint32_t* r = ROW(h, s, l);
    size_t c = 0;
    for (; c < m && r[c] != ORC_EMPTY; ++c) out[c] = r[c];
    if (locked) pthread_mutex_unlock(&h->node_locks[s]);
    return c;
}

/* usearch search_for_one_ (upper levels): greedy move to the closest
 * neighbour until no neighbour improves; ties by slot. */
static uint32_t greedy(const orc_hnsw* h, const float* q, uint32_t ep, float* dep, int l,
                       scratch_t* s, int locked, uint32_t self) {
    uint32_t cur = ep;
    float dcur = *dep;
    for (;;) {
        size_t c = read_row(h, cur, l, s->nbr, locked);
        uint32_t best = cur;
        float dbest = dcur;
        for (size_t i = 0; i < c; ++i) {
            uint32_t n = s->nbr[i];
            if (n == self) continue; /* a node is never its own candidate */
            float d = orc_distance(h->metric, q, VEC(h, n), h->dim);
            s->ndist++;
            if (cand_less(d, n, dbest, best)) {
                best = n;
                dbest = d;
            }
        }
        if (best == cur) break;
        cur = best;
        dcur = dbest;
    }
    *dep = dcur;
    return cur;
}

/* usearch search_to_find_in_base_ restated as "expand the best unexpanded
 * entry of the (distance, slot)-sorted top-ef list until none remains" —
 * equivalent to the two-heap formulation (a candidate evicted from the top
 * list can never be closer than the list's worst again). Returns list size. */
static size_t beam(const orc_hnsw* h, const float* q, uint32_t ep, float dep, size_t ef, int l,
                   scratch_t* s, int locked, uint32_t self) {
    scratch_newgen(s);
    /* the node being (re)linked is never its own candidate: a reused slot is
     * reachable through other nodes' kept links into it */
    if (self != ORC_EMPTY) s->stamp[self] = s->gen;
    cand_t* L = s->list;
    uint8_t* X = s->expanded;
    size_t n = 1;
    L[0].d = dep;
    L[0].id = ep;
    X[0] = 0;
    s->stamp[ep] = s->gen;
    size_t first = 0; /* all entries before `first` are expanded */
    for (;;) {
        while (first < n && X[first]) ++first;
        if (first >= n) break;
        X[first] = 1;
        uint32_t node = L[first].id;
        size_t c = read_row(h, node, l, s->nbr, locked);
        for (size_t i = 0; i < c; ++i) {
            uint32_t nb = s->nbr[i];
            if (s->stamp[nb] == s->gen) continue;
            s->stamp[nb] = s->gen;
            float d = orc_distance(h->metric, q, VEC(h, nb), h->dim);
            s->ndist++;
            if (n == ef && !cand_less(d, nb, L[n - 1].d, L[n - 1].id)) continue;
            /* insert keeping (d, id) order */
            size_t lo = 0, hi = n;
            while (lo < hi) {
                size_t mid = (lo + hi) >> 1;
                if (cand_less(L[mid].d, L[mid].id, d, nb)) lo = mid + 1;
                else hi = mid;
            }
            if (n == ef) --n;
            memmove(L + lo + 1, L + lo, (n - lo) * sizeof(cand_t));
            memmove(X + lo + 1, X + lo, (n - lo));
            L[lo].d = d;
            L[lo].id = nb;
            X[lo] = 0;
            ++n;
            if (lo < first) first = lo;
        }
    }
    return n;
}

static void heap_push(scratch_t* s, size_t* n, float d, uint32_t id) {
    if (*n == s->heap_cap) {
        s->heap_cap = s->heap_cap ? 2 * s->heap_cap : 256;
        s->heap = (cand_t*)realloc(s->heap, s->heap_cap * sizeof(cand_t));
    }
    size_t i = (*n)++;
    while (i > 0) {
        size_t p = (i - 1) >> 1;
        if (!cand_less(d, id, s->heap[p].d, s->heap[p].id)) break;
        s->heap[i] = s->heap[p];
        i = p;
    }
    s->heap[i].d = d;
    s->heap[i].id = id;
}

static void heap_pop(scratch_t* s, size_t* n) {
    cand_t last = s->heap[--(*n)];
    size_t i = 0;
    for (;;) {
        size_t c = 2 * i + 1;
        if (c >= *n) break;
        if (c + 1 < *n && cand_less(s->heap[c + 1].d, s->heap[c + 1].id, s->heap[c].d, s->heap[c].id)) ++c;
        if (!cand_less(s->heap[c].d, s->heap[c].id, last.d, last.id)) break;
        s->heap[i] = s->heap[c];
        i = c;
    }
    if (*n) s->heap[i] = last;
}

/* usearch search_to_find_in_base_ with index_dense's `allow` predicate
 * (member.key != free_key_), the base-level search of an index that holds
 * removed entries (usearch v2 series: index_dense_gt::search_ passes `allow`
 * into index_gt::search; reference call sites src/index/usearch.rs:215, 245
 * remove, :276 search).  Two sets, as usearch keeps them:
 *   next -- every admitted candidate, removed or not (the min-heap that drives
 *           the traversal: removed nodes are still expanded);
 *   top  -- the best `ef` ADMITTED LIVE candidates (the result list).
 * radius = the worst key of `top` (the start's key while `top` is empty);
 * a candidate is admitted when |top| < ef or it beats the radius; the loop
 * pops the nearest of `next` and stops when that is beyond the radius.  The
 * start node joins `top` only when live (the predicate is checked on it too).
 * Keys compare as (distance, slot) -- the restatement's canonical tie order.
 * Without removed entries this is beam() (every node of `next` that is not in
 * `top` was evicted from it and lies beyond the radius), so search_one() uses
 * it only when the index holds tombstones.  Returns |top| (in s->list). */
static size_t beam_filtered(const orc_hnsw* h, const float* q, uint32_t ep, float dep, size_t ef,
                            scratch_t* s) {
    scratch_newgen(s);
    cand_t* L = s->list;
    size_t n = 0, nh = 0;
    s->stamp[ep] = s->gen;
    heap_push(s, &nh, dep, ep);
    float rd = dep; /* radius key */
    uint32_t ri = ep;
    if (!h->removed[ep]) {
        L[0].d = dep;
        L[0].id = ep;
        n = 1;
    }
    while (nh) {
        const cand_t c = s->heap[0];
        if (cand_less(rd, ri, c.d, c.id)) break; /* nearest of `next` beyond the radius */
        heap_pop(s, &nh);
        size_t cnt = read_row(h, c.id, 0, s->nbr, 0);
        for (size_t i = 0; i < cnt; ++i) {
            uint32_t nb = s->nbr[i];
            if (s->stamp[nb] == s->gen) continue;
            s->stamp[nb] = s->gen;
            float d = orc_distance(h->metric, q, VEC(h, nb), h->dim);
            s->ndist++;
            if (!(n < ef || cand_less(d, nb, rd, ri))) continue;
            heap_push(s, &nh, d, nb);
            if (h->removed[nb]) continue; /* traversed, never a result */
            size_t lo = 0, hi = n;
            while (lo < hi) {
                size_t mid = (lo + hi) >> 1;
                if (cand_less(L[mid].d, L[mid].id, d, nb)) lo = mid + 1;
                else hi = mid;
            }
            if (n == ef) --n;
            memmove(L + lo + 1, L + lo, (n - lo) * sizeof(cand_t));
            L[lo].d = d;
            L[lo].id = nb;
            ++n;
            rd = L[n - 1].d;
            ri = L[n - 1].id;
        }
    }
    return n;
}

/* usearch refine_ (heuristic neighbour selection): walk candidates in
 * ascending (distance, slot); keep c unless some already-kept r is closer to
 * c than the base is (dist(c, r) < dist(c, base)).  No back-fill.  Fewer
 * candidates than `needed` are returned unfiltered (refine_'s early return
 * `if (top_count < needed) return {top_data, top_count};`) -- on the forward
 * links of a new node while the level holds fewer than M reachable nodes; a
 * reverse-link prune always has M_l + 1 candidates. */
static size_t select_heuristic(const orc_hnsw* h, const cand_t* C, size_t nc, size_t m,
                               uint32_t* out, scratch_t* s) {
    if (nc < m) {
        for (size_t i = 0; i < nc; ++i) out[i] = C[i].id;
        return nc;
    }
    size_t kept = 0;
    for (size_t i = 0; i < nc && kept < m; ++i) {
        int good = 1;
        const float* vc = VEC(h, C[i].id);
        for (size_t j = 0; j < kept; ++j) {
            float d = orc_distance(h->metric, vc, VEC(h, out[j]), h->dim);
            s->ndist++;
            if (d < C[i].d) {
                good = 0;
                break;
            }
        }
        if (good) out[kept++] = C[i].id;
    }
    return kept;
}

static int cand_cmp(const void* a, const void* b) {
    const cand_t* x = (const cand_t*)a;
    const cand_t* y = (const cand_t*)b;
    if (cand_less(x->d, x->id, y->d, y->id)) return -1;
    if (cand_less(y->d, y->id, x->d, x->id)) return 1;
    return 0;
}

/* Reverse link q -> n at level l (usearch form_reverse_links_): append while
 * there is room, otherwise re-select over existing + q with the heuristic. */
static void add_reverse(orc_hnsw* h, uint32_t n, uint32_t q, int l, scratch_t* s, int locked) {
    size_t m = ROWLEN(h, l);
    if (locked) pthread_mutex_lock(&h->node_locks[n]);
    uint32_t* r = ROW(h, n, l);
    size_t c = 0;
    int present = 0;
    for (; c < m && r[c] != ORC_EMPTY; ++c) present = present || r[c] == q;
    if (present) {
        /* usearch reconnect_neighbor_nodes_: "If new_slot is already present in
         * the neighboring connections of close_slot then no need to modify any
         * connections or run the heuristics" -- a reused slot's kept in-link */
    } else if (c < m) {
        r[c] = q;
    } else {
        cand_t* C = s->tmp;
        const float* vn = VEC(h, n);
        for (size_t i = 0; i < c; ++i) {
            C[i].id = r[i];
            C[i].d = orc_distance(h->metric, vn, VEC(h, r[i]), h->dim);
        }
        C[c].id = q;
        C[c].d = orc_distance(h->metric, vn, VEC(h, q), h->dim);
        s->ndist += c + 1;
        qsort(C, c + 1, sizeof(cand_t), cand_cmp);
        uint32_t* out = s->nbr;
        size_t k = select_heuristic(h, C, c + 1, m, out, s);
        for (size_t i = 0; i < m; ++i) r[i] = i < k ? out[i] : ORC_EMPTY;
    }
    if (locked) pthread_mutex_unlock(&h->node_locks[n]);
}

static void insert_slot(orc_hnsw* h, uint32_t q, scratch_t* s, int locked) {
    int L = h->levels[q];
    const float* vq = VEC(h, q);
    int hold_global = 0;
    if (locked) pthread_mutex_lock(&h->global_lock);
    uint32_t ep = h->entry;
    int maxl = h->max_level;
    if (locked) {
        if (L > maxl) hold_global = 1; /* hnswlib: keep global lock while raising the top */
        else pthread_mutex_unlock(&h->global_lock);
    }
    if (ep == ORC_EMPTY) {
        h->entry = q;
        h->max_level = L;
        if (hold_global) pthread_mutex_unlock(&h->global_lock);
        return;
    }
    float dep = orc_distance(h->metric, vq, VEC(h, ep), h->dim);
    s->ndist++;
    for (int l = maxl; l > L; --l) ep = greedy(h, vq, ep, &dep, l, s, locked, q);
    uint32_t* sel = (uint32_t*)malloc(h->M0 * sizeof(uint32_t));
    for (int l = (L < maxl ? L : maxl); l >= 0; --l) {
        size_t n = beam(h, vq, ep, dep, h->efC, l, s, locked, q);
        /* usearch connect_new_node_: refine_(metric, config_.connectivity, ...)
         * on EVERY level -- a new node keeps at most M outgoing links, level 0
         * included; its level-0 row (M0 = 2M slots) fills up to M0 only through
         * other nodes' reverse links (reconnect_neighbor_nodes_, add_reverse). */
        size_t k = select_heuristic(h, s->list, n, h->M, sel, s);
        size_t m = ROWLEN(h, l);
        if (locked) pthread_mutex_lock(&h->node_locks[q]);
        uint32_t* r = ROW(h, q, l);
        for (size_t i = 0; i < m; ++i) r[i] = i < k ? sel[i] : ORC_EMPTY;
        if (locked) pthread_mutex_unlock(&h->node_locks[q]);
        for (size_t i = 0; i < k; ++i) add_reverse(h, sel[i], q, l, s, locked);
        ep = s->list[0].id;
        dep = s->list[0].d;
    }
    free(sel);
    if (L > maxl) {
        h->entry = q;
        h->max_level = L;
    }
    if (hold_global) pthread_mutex_unlock(&h->global_lock);
}

typedef struct {
    orc_hnsw* h;
    const uint32_t* list; /* slots in insertion order */
    scratch_t* scr;
} add_ctx;

static void add_one(void* p, size_t i, int tid) {
    add_ctx* c = (add_ctx*)p;
    insert_slot(c->h, c->list[i], &c->scr[tid], 1);
}

static void ring_push(orc_hnsw* h, uint32_t slot) {
    if (h->ring_n == h->ring_cap) {
        h->ring_cap = h->ring_cap ? 2 * h->ring_cap : 256;
        h->ring = (uint32_t*)realloc(h->ring, h->ring_cap * sizeof(uint32_t));
    }
    h->ring[h->ring_n++] = slot;
}

/* Clear every row of slot s (levels 0..levels[s]); the level is kept. */
static void clear_rows(orc_hnsw* h, uint32_t s) {
    for (int l = 0; l <= h->levels[s]; ++l) {
        uint32_t* r = ROW(h, s, l);
        for (size_t i = 0; i < ROWLEN(h, l); ++i) r[i] = ORC_EMPTY;
    }
}

/* s1: a caller-owned scratch for a single-threaded call (orc_hnsw_replace reuses
 * one across its keys instead of allocating a slot-sized stamp array per key) */
static int add_impl(orc_hnsw* h, const uint64_t* keys, const float* vecs, size_t n, int threads, scratch_t* s1);

int orc_hnsw_add(orc_hnsw* h, const uint64_t* keys, const float* vecs, size_t n, int threads) {
    return add_impl(h, keys, vecs, n, threads, NULL);
}

static int add_impl(orc_hnsw* h, const uint64_t* keys, const float* vecs, size_t n, int threads, scratch_t* s1) {
    if (n == 0) return 0;
    /* validate: no reserved key, no live duplicate, no duplicate inside batch */
    for (size_t i = 0; i < n; ++i) {
        if (keys[i] >= KM_DEAD) return 1;
        if (km_find(&h->km, keys[i]) >= 0) return 3;
    }
    {
        keymap tmp;
        size_t cap = 16;
        while (cap < 2 * n) cap <<= 1;
        km_init(&tmp, cap);
        for (size_t i = 0; i < n; ++i) {
            if (km_find(&tmp, keys[i]) >= 0) {
                km_free(&tmp);
                return 3;
            }
            km_put(&tmp, keys[i], 0);
        }
        km_free(&tmp);
    }
    /* free-slot reuse (index_dense_gt::add_ pops free_keys_): the oldest removed
     * slots first; the entry point's slot is skipped and keeps its place */
    uint32_t* list = (uint32_t*)malloc(n * sizeof(uint32_t));
    size_t r = 0;
    if (h->reuse) {
        size_t kept = 0;
        for (size_t i = 0; i < h->ring_n; ++i) {
            const uint32_t sl = h->ring[i];
            if (r < n && sl != h->entry) list[r++] = sl;
            else h->ring[kept++] = sl;
        }
        h->ring_n = kept;
    }
    const size_t na = n - r;
    if (h->slots + na > h->cap) {
        size_t want = h->cap ? h->cap : 1024;
        while (want < h->slots + na) want *= 2;
        if (orc_hnsw_reserve(h, want)) {
            free(list);
            return 2;
        }
    }
    /* the reused slots' keys are mapped now (the call is accepted); each slot is
     * staged right before its own re-link below */
    for (size_t i = 0; i < r; ++i) km_put(&h->km, keys[i], list[i]);
    size_t base = h->slots;
    size_t need_upper = 0;
    for (size_t i = 0; i < na; ++i) {
        uint32_t s = (uint32_t)(base + i);
        int L = orc_sample_level(h->seed, s, (uint32_t)h->M);
        h->levels[s] = (int8_t)L;
        need_upper += (size_t)L;
    }
    size_t used = atomic_load(&h->upper_used);
    if (used + need_upper > h->upper_cap) {
        size_t want = h->upper_cap ? h->upper_cap : 256;
        while (want < used + need_upper) want *= 2;
        h->upper = (uint32_t*)realloc(h->upper, want * h->M * sizeof(uint32_t));
        memset(h->upper + h->upper_cap * h->M, 0xFF, (want - h->upper_cap) * h->M * sizeof(uint32_t));
        h->upper_cap = want;
    }
    for (size_t i = 0; i < na; ++i) {
        uint32_t s = (uint32_t)(base + i);
        int L = h->levels[s];
        h->upper_off[s] = L > 0 ? (uint32_t)used : ORC_EMPTY;
        used += (size_t)L;
        memcpy(h->vecs + (size_t)s * h->dim, vecs + (r + i) * h->dim, h->dim * sizeof(float));
        h->keys[s] = keys[r + i];
        h->removed[s] = 0;
        km_put(&h->km, keys[r + i], s);
        list[r + i] = s;
    }
    atomic_store(&h->upper_used, used);
    h->slots += na;
    h->live += n;

    /* insertion order: the reused slots (call order), then the appended ones */
    threads = s1 ? 1 : resolve_threads(threads);
    if ((size_t)threads > na) threads = (int)na;
    if (threads < 1) threads = 1;
    scratch_t* scr = s1;
    if (s1) {
        if (s1->stamp_cap < h->cap) { /* the index grew: a larger stamp array */
            free(s1->stamp);
            s1->stamp = (uint32_t*)calloc(h->cap, sizeof(uint32_t));
            s1->stamp_cap = h->cap;
            s1->gen = 0;
        }
    } else {
        scr = (scratch_t*)malloc(sizeof(scratch_t) * threads);
        for (int t = 0; t < threads; ++t) scratch_init(&scr[t], h->cap, h->efC > h->ef ? h->efC : h->ef, h->M0);
    }
    /* Reused slots one key at a time, as a sequence of single adds (index_dense
     * add_ pops ONE free slot per call and runs index_gt::update on it): the slot
     * gets its new key and vector, its rows (every level) are cleared, it is live
     * again -- and it is re-linked before the next key's slot is touched, so the
     * slots later in the call still hold their old vectors and links.  Always
     * sequential (their order is the call's). */
    for (size_t i = 0; i < r; ++i) {
        const uint32_t sl = list[i];
        memcpy(h->vecs + (size_t)sl * h->dim, vecs + i * h->dim, h->dim * sizeof(float));
        h->keys[sl] = keys[i];
        h->removed[sl] = 0;
        clear_rows(h, sl);
        insert_slot(h, sl, &scr[0], 0);
    }
    if (threads == 1) {
        for (size_t i = r; i < n; ++i) insert_slot(h, list[i], &scr[0], 0);
    } else if (na) {
        /* the very first node must exist before concurrent inserts start */
        size_t start = r;
        if (h->entry == ORC_EMPTY) {
            insert_slot(h, list[start], &scr[0], 0);
            ++start;
        }
        add_ctx c = {h, list + start, scr};
        parallel_for(n - start, threads, add_one, &c);
    }
    if (!s1) {
        for (int t = 0; t < threads; ++t) scratch_free(&scr[t]);
        free(scr);
    }
    free(list);
    return 0;
}

size_t orc_hnsw_remove(orc_hnsw* h, const uint64_t* keys, size_t n) {
    size_t r = 0;
    for (size_t i = 0; i < n; ++i) {
        uint32_t s;
        if (km_del(&h->km, keys[i], &s)) {
            h->removed[s] = 1;
            h->live--;
            ring_push(h, s); /* usearch index_dense_gt::remove: free_keys_.push(slot) */
            ++r;
        }
    }
    return r;
}

/* The reference's AddOrReplace stream, one message at a time
 * (src/index/usearch.rs:214-221: `if remove { idx.remove(key) }` then
 * `idx.add(key, &embedding)`, each message before the next).  status[i]
 * (optional) = the add's code for message i; a failed add fails only its own
 * vector (usearch.rs:221-232). */
int orc_hnsw_replace(orc_hnsw* h, const uint64_t* keys, const float* vecs, size_t n, int* status) {
    int first = 0;
    scratch_t scr;
    scratch_init(&scr, h->cap, h->efC > h->ef ? h->efC : h->ef, h->M0);
    for (size_t i = 0; i < n; ++i) {
        (void)orc_hnsw_remove(h, keys + i, 1);
        const int rc = add_impl(h, keys + i, vecs + i * h->dim, 1, 1, &scr);
        if (status) status[i] = rc;
        if (rc && !first) first = rc;
    }
    scratch_free(&scr);
    return first;
}

size_t orc_hnsw_free_list(const orc_hnsw* h, uint32_t* out, size_t cap) {
    for (size_t i = 0; out && i < h->ring_n && i < cap; ++i) out[i] = h->ring[i];
    return h->ring_n;
}

void orc_hnsw_set_slot_reuse(orc_hnsw* h, int on) { h->reuse = on ? 1 : 0; }

typedef struct {
    const orc_hnsw* h;
    const float* q;
    size_t k, ef;
    uint64_t* ok;
    float* od;
    size_t* oc;
    scratch_t* scr;
} search_ctx;

static void search_one(void* p, size_t qi, int tid) {
    search_ctx* c = (search_ctx*)p;
    const orc_hnsw* h = c->h;
    scratch_t* s = &c->scr[tid];
    const float* q = c->q + qi * h->dim;
    uint64_t* ok = c->ok + qi * c->k;
    float* od = c->od + qi * c->k;
    size_t cnt = 0;
    if (h->entry != ORC_EMPTY) {
        uint32_t ep = h->entry;
        float dep = orc_distance(h->metric, q, VEC(h, ep), h->dim);
        s->ndist++;
        for (int l = h->max_level; l >= 1; --l) ep = greedy(h, q, ep, &dep, l, s, 0, ORC_EMPTY);
        /* removed entries: traversed, never admitted into the result list */
        size_t n = h->live < h->slots ? beam_filtered(h, q, ep, dep, c->ef, s)
                                      : beam(h, q, ep, dep, c->ef, 0, s, 0, ORC_EMPTY);
        for (size_t i = 0; i < n && cnt < c->k; ++i) {
            uint32_t id = s->list[i].id;
            ok[cnt] = h->keys[id];
            od[cnt] = s->list[i].d;
            ++cnt;
        }
    }
    if (c->oc) c->oc[qi] = cnt;
    for (size_t j = cnt; j < c->k; ++j) {
        ok[j] = UINT64_MAX;
        od[j] = INFINITY;
    }
}

int orc_hnsw_search(const orc_hnsw* h, const float* queries, size_t nq, size_t k,
                    size_t ef_override, uint64_t* out_keys, float* out_dist,
                    size_t* out_counts, int threads, uint64_t* out_ndist) {
    if (k == 0) return 1;
    size_t ef = ef_override ? ef_override : h->ef;
    if (ef < k) ef = k; /* usearch: expansion = max(expansion_search, wanted) */
    threads = resolve_threads(threads);
    if ((size_t)threads > nq) threads = nq ? (int)nq : 1;
    /* per-thread scratch is cached on the index so repeated searches (the CPU
     * baseline's timed calls) do not pay the visited-array allocation */
    orc_hnsw* hm = (orc_hnsw*)h;
    scratch_t* scr = (scratch_t*)hm->sscr;
    if (!scr || hm->sscr_n < threads || hm->sscr_slots < h->slots || hm->sscr_ef < ef) {
        for (int t = 0; scr && t < hm->sscr_n; ++t) scratch_free(&scr[t]);
        free(scr);
        scr = (scratch_t*)malloc(sizeof(scratch_t) * threads);
        for (int t = 0; t < threads; ++t) scratch_init(&scr[t], h->slots, ef, h->M0);
        hm->sscr = scr;
        hm->sscr_n = threads;
        hm->sscr_slots = h->slots;
        hm->sscr_ef = ef;
    }
    for (int t = 0; t < threads; ++t) scr[t].ndist = 0;
    search_ctx c = {h, queries, k, ef, out_keys, out_dist, out_counts, scr};
    parallel_for(nq, threads, search_one, &c);
    uint64_t nd = 0;
    for (int t = 0; t < threads; ++t) nd += scr[t].ndist;
    if (out_ndist) *out_ndist = nd;
    return 0;
}

int orc_hnsw_export(const orc_hnsw* h, float* vecs, uint64_t* keys, uint8_t* removed,
                    int8_t* levels, uint32_t* adj0, uint32_t* upper_off, uint32_t* upper) {
    size_t s = h->slots;
    if (vecs) memcpy(vecs, h->vecs, s * h->dim * sizeof(float));
    if (keys) memcpy(keys, h->keys, s * sizeof(uint64_t));
    if (removed) memcpy(removed, h->removed, s);
    if (levels) memcpy(levels, h->levels, s);
    if (adj0) memcpy(adj0, h->adj0, s * h->M0 * sizeof(uint32_t));
    if (upper_off) memcpy(upper_off, h->upper_off, s * sizeof(uint32_t));
    if (upper) memcpy(upper, h->upper, atomic_load(&h->upper_used) * h->M * sizeof(uint32_t));
    return 0;
}

int orc_hnsw_import(orc_hnsw* h, size_t slots, const float* vecs, const uint64_t* keys,
                    const uint8_t* removed, const int8_t* levels, const uint32_t* adj0,
                    const uint32_t* upper_off, const uint32_t* upper, size_t n_upper_rows,
                    uint32_t entry, int max_level) {
    if (h->slots) return 5;
    if (orc_hnsw_reserve(h, slots > 0 ? slots : 1)) return 2;
    memcpy(h->vecs, vecs, slots * h->dim * sizeof(float));
    memcpy(h->keys, keys, slots * sizeof(uint64_t));
    memcpy(h->removed, removed, slots);
    memcpy(h->levels, levels, slots);
    memcpy(h->adj0, adj0, slots * h->M0 * sizeof(uint32_t));
    memcpy(h->upper_off, upper_off, slots * sizeof(uint32_t));
    h->upper = (uint32_t*)realloc(h->upper, (n_upper_rows ? n_upper_rows : 1) * h->M * sizeof(uint32_t));
    memcpy(h->upper, upper, n_upper_rows * h->M * sizeof(uint32_t));
    h->upper_cap = n_upper_rows ? n_upper_rows : 1;
    atomic_store(&h->upper_used, n_upper_rows);
    h->slots = slots;
    h->live = 0;
    h->ring_n = 0;
    for (size_t i = 0; i < slots; ++i) {
        if (!removed[i]) {
            km_put(&h->km, keys[i], (uint32_t)i);
            h->live++;
        } else {
            ring_push(h, (uint32_t)i); /* no removal order in the interchange: ascending */
        }
    }
    h->entry = entry;
    h->max_level = max_level;
    return 0;
}
