// vsg_sharded.cpp — one logical index row-sharded over the GPUs of a node
// (include/vsg.h "Sharded index"; SURVEY §8b create(opts{..., n_gpus}), §8e).
//
// Built on the single-shard ABI: shard g is a vsg_index_t on devices[g] with its
// own HNSW graph.  This file routes keys to shards, runs the shards' builds and
// searches concurrently (one host thread / one stream per shard) and merges the
// per-shard top-k rows on the answering device:
//
//   queries (answer dev) --peer DMA--> each other shard device
//   shard g: HNSW (or exact) top-k on its own stream
//   top-k rows --peer DMA over xGMI--> gather[g] on the answer device
//   merge_topk64_kernel: parts x nq x k -> nq x k, (distance, key) order
//
// Per step at nq = 10,000, k = 10 a shard ships 1.2 MB of results: the gather is
// latency-bound, not link-bound, so a point-to-point copy per shard (one DMA on
// the shard's own xGMI link) is the whole exchange.  An all-gather would land
// every shard's rows on every device, of which only the answering one merges.
// The reference's one-device index this replaces: src/index/usearch.rs:89-99.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/vsg.h"
#include "roctx_range.hpp"

namespace vsg {
void set_last_error(const std::string& msg);  // vsg_index.cpp
size_t index_first_live(const vsg_index_t* h, const uint64_t* keys, size_t n);
// vsg_index.cpp: the per-device memory pool (stream-ordered frees, no device-wide
// wait), the process-wide pinned and stream caches
hipError_t pool_malloc(void** p, size_t bytes, hipStream_t s);
void pool_free(void* p, hipStream_t s);
hipError_t pinned_take(uint8_t** p, size_t* cap, size_t want, bool coherent);
void pinned_return(uint8_t* p, size_t cap, bool coherent);
hipError_t stream_get(hipStream_t* s);
void stream_put(hipStream_t s);
}  // namespace vsg

namespace {

int sfail(int code, const std::string& msg) {
    vsg::set_last_error(msg);
    return code;
}

#define SH_TRY(expr)                                                                         \
    do {                                                                                     \
        hipError_t e__ = (expr);                                                             \
        if (e__ != hipSuccess)                                                               \
            return sfail(VSG_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e__));  \
    } while (0)

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        hipGetDevice(&prev);
        if (prev != dev) hipSetDevice(dev);
    }
    ~DevGuard() {
        int cur = -1;
        hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) hipSetDevice(prev);
    }
};

uint64_t route_hash(uint64_t x) {  // splitmix64 finaliser
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// f(g) for every shard on its own host thread; a thread that cannot be started
// runs its shard on the caller (nothing may throw across the C ABI)
template <typename F>
void per_shard(size_t n, F&& f) {
    if (n == 1) {
        f((size_t)0);
        return;
    }
    std::vector<std::thread> th;
    size_t g = 0;
    try {
        for (; g < n; ++g) th.emplace_back([&f, g] { f(g); });
    } catch (const std::system_error&) {
    }
    for (; g < n; ++g) f(g);
    for (auto& t : th) t.join();
}

// grow a device buffer on stream s (the old block returns to the pool after s's
// earlier work; callers have waited for other streams' readers)
template <typename X>
hipError_t grow(X** p, size_t& cap, size_t bytes, hipStream_t s) {
    if (bytes <= cap) return hipSuccess;
    const size_t want = std::max(bytes, cap * 2);
    vsg::pool_free(*p, s);
    *p = nullptr;
    cap = 0;
    const hipError_t e = vsg::pool_malloc((void**)p, want, s);
    if (e == hipSuccess) cap = want;
    return e;
}

}  // namespace

// One in-flight sharded search: streams, events and buffers that only grow.
// Pooled per index; a context is reused only after its previous search's merge
// completed (`done`, waited on by every shard stream before it writes again).
struct ShardCtx {
    std::vector<hipStream_t> s;   // per shard, on its device
    std::vector<hipEvent_t> ev;   // per shard: its rows are in the gather buffer
    std::vector<uint8_t*> out;    // per shard not on the answer device: keys | dists
    std::vector<size_t> out_cap;
    std::vector<uint8_t*> q;      // per distinct device (index into devs): broadcast queries
    std::vector<size_t> q_cap;
    std::vector<hipEvent_t> q_ev;  // per distinct device: queries present
    hipStream_t sa = nullptr;      // answer device stream (host API)
    hipEvent_t start = nullptr;    // queries ready on the answer device
    hipEvent_t done = nullptr;     // merge of the last search finished
    bool pending = false;
    uint8_t* gather = nullptr;     // answer device: parts x nq x k keys, then dists
    size_t gather_cap = 0;
    uint8_t* res = nullptr;        // answer device (host API): queries | keys | dists
    size_t res_cap = 0;
    uint8_t* pin = nullptr;
    size_t pin_cap = 0;
};

struct vsg_sharded {
    vsg_index_options_t opt{};
    uint32_t n = 0;
    int ans = 0;                       // answering device
    std::vector<int> dev;              // per shard
    std::vector<int> devs;             // distinct devices
    std::vector<int> dev_slot;         // per shard: index into devs
    std::vector<int> first_on;         // per distinct device: its first shard
    std::vector<vsg_index_t*> shard;
    std::mutex wmu;                    // writers
    std::mutex ctx_mu;
    std::vector<ShardCtx*> ctx_free;

    uint32_t route(uint64_t key) const { return n == 1 ? 0u : (uint32_t)(route_hash(key) % n); }
};

static void ctx_destroy(vsg_sharded* h, ShardCtx* c) {
    for (size_t g = 0; g < c->s.size(); ++g) {
        DevGuard dg(h->dev[g]);
        if (c->s[g]) (void)hipStreamSynchronize(c->s[g]);
        if (c->ev[g]) (void)hipEventDestroy(c->ev[g]);
    }
    DevGuard dga(h->ans);
    if (c->sa) (void)hipStreamSynchronize(c->sa);
    if (c->pending) (void)hipEventSynchronize(c->done);
    // every stream of the context is idle: buffers back to their device's pool
    // (ordered on an idle stream of that device), streams back to the cache
    for (size_t g = 0; g < c->s.size(); ++g) {
        DevGuard dg(h->dev[g]);
        vsg::pool_free(c->out[g], c->s[g]);
    }
    for (size_t d = 0; d < c->q.size(); ++d) {
        DevGuard dg(h->devs[d]);
        vsg::pool_free(c->q[d], c->s[h->first_on[d]]);
        if (c->q_ev[d]) (void)hipEventDestroy(c->q_ev[d]);
    }
    vsg::pool_free(c->gather, c->sa);
    vsg::pool_free(c->res, c->sa);
    for (size_t g = 0; g < c->s.size(); ++g) {
        DevGuard dg(h->dev[g]);
        if (c->s[g]) (void)hipStreamSynchronize(c->s[g]);
        vsg::stream_put(c->s[g]);
    }
    if (c->sa) (void)hipStreamSynchronize(c->sa);
    vsg::stream_put(c->sa);
    if (c->start) (void)hipEventDestroy(c->start);
    if (c->done) (void)hipEventDestroy(c->done);
    vsg::pinned_return(c->pin, c->pin_cap, true);
    delete c;
}

static int ctx_acquire(vsg_sharded* h, ShardCtx** out) {
    {
        std::lock_guard<std::mutex> lk(h->ctx_mu);
        if (!h->ctx_free.empty()) {
            *out = h->ctx_free.back();
            h->ctx_free.pop_back();
            return VSG_OK;
        }
    }
    auto* c = new ShardCtx;
    c->s.assign(h->n, nullptr);
    c->ev.assign(h->n, nullptr);
    c->out.assign(h->n, nullptr);
    c->out_cap.assign(h->n, 0);
    c->q.assign(h->devs.size(), nullptr);
    c->q_cap.assign(h->devs.size(), 0);
    c->q_ev.assign(h->devs.size(), nullptr);
    hipError_t e = hipSuccess;
    for (uint32_t g = 0; g < h->n && e == hipSuccess; ++g) {
        DevGuard dg(h->dev[g]);
        e = vsg::stream_get(&c->s[g]);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev[g], hipEventDisableTiming);
    }
    for (size_t d = 0; d < h->devs.size() && e == hipSuccess; ++d) {
        DevGuard dg(h->devs[d]);
        e = hipEventCreateWithFlags(&c->q_ev[d], hipEventDisableTiming);
    }
    if (e == hipSuccess) {
        DevGuard dg(h->ans);
        e = vsg::stream_get(&c->sa);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->start, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        ctx_destroy(h, c);
        return sfail(VSG_EDEVICE, std::string("sharded search context: ") + hipGetErrorString(e));
    }
    *out = c;
    return VSG_OK;
}

static void ctx_release(vsg_sharded* h, ShardCtx* c) {
    std::lock_guard<std::mutex> lk(h->ctx_mu);
    h->ctx_free.push_back(c);
}

// broadcast -> per-shard search -> gather -> merge, all enqueued (stream `sa` on
// the answer device is the caller's); q / ok / od live on the answer device
static int search_enqueue(vsg_sharded* h, ShardCtx* c, const float* q, size_t nq, size_t k, size_t ef, bool exact,
                          uint64_t* ok, float* od, hipStream_t sa) {
    const size_t dim = h->opt.dimensions, n = h->n;
    const size_t kb = nq * k * 8, db = nq * k * 4;
    if (c->pending) {  // a buffer about to grow may still be read by the last search
        bool grows = n * (kb + db) > c->gather_cap;
        for (size_t d = 0; d < h->devs.size(); ++d) grows |= h->devs[d] != h->ans && nq * dim * 4 > c->q_cap[d];
        for (size_t g = 0; g < n; ++g) grows |= h->dev[g] != h->ans && kb + db > c->out_cap[g];
        if (grows) {
            SH_TRY(hipEventSynchronize(c->done));
            c->pending = false;
        }
    }
    {
        DevGuard dg(h->ans);
        SH_TRY(grow(&c->gather, c->gather_cap, n * (kb + db), sa));
        SH_TRY(hipEventRecord(c->start, sa));
    }
    uint8_t* gk = c->gather;
    uint8_t* gd = c->gather + n * kb;
    // queries to every other device, on the stream of its first shard
    for (size_t d = 0; d < h->devs.size(); ++d) {
        const int dv = h->devs[d];
        if (dv == h->ans) continue;
        const int g0 = h->first_on[d];
        DevGuard dg(dv);
        SH_TRY(grow(&c->q[d], c->q_cap[d], nq * dim * 4, c->s[g0]));
        if (c->pending) SH_TRY(hipStreamWaitEvent(c->s[g0], c->done, 0));
        SH_TRY(hipStreamWaitEvent(c->s[g0], c->start, 0));
        SH_TRY(hipMemcpyPeerAsync(c->q[d], dv, q, h->ans, nq * dim * 4, c->s[g0]));
        SH_TRY(hipEventRecord(c->q_ev[d], c->s[g0]));
    }
    for (size_t g = 0; g < n; ++g) {
        const int dv = h->dev[g];
        const int d = h->dev_slot[g];
        DevGuard dg(dv);
        hipStream_t st = c->s[g];
        const float* qg = q;
        uint64_t* K = reinterpret_cast<uint64_t*>(gk + g * kb);
        float* D = reinterpret_cast<float*>(gd + g * db);
        if (dv == h->ans) {
            if (c->pending) SH_TRY(hipStreamWaitEvent(st, c->done, 0));
            SH_TRY(hipStreamWaitEvent(st, c->start, 0));
        } else {
            if (h->first_on[d] != (int)g) {
                if (c->pending) SH_TRY(hipStreamWaitEvent(st, c->done, 0));
                SH_TRY(hipStreamWaitEvent(st, c->q_ev[d], 0));
            }
            qg = reinterpret_cast<const float*>(c->q[d]);
            SH_TRY(grow(&c->out[g], c->out_cap[g], kb + db, st));
            K = reinterpret_cast<uint64_t*>(c->out[g]);
            D = reinterpret_cast<float*>(c->out[g] + kb);
        }
        const int rc = exact ? vsg_index_exact_search_device(h->shard[g], qg, nq, k, K, D, nullptr, st)
                             : vsg_index_search_device(h->shard[g], qg, nq, k, ef, K, D, nullptr, st);
        if (rc) return rc;
        if (dv != h->ans) {  // the shard's top-k rows over its xGMI link
            SH_TRY(hipMemcpyPeerAsync(gk + g * kb, h->ans, K, dv, kb, st));
            SH_TRY(hipMemcpyPeerAsync(gd + g * db, h->ans, D, dv, db, st));
        }
        SH_TRY(hipEventRecord(c->ev[g], st));
    }
    DevGuard dg(h->ans);
    for (size_t g = 0; g < n; ++g) SH_TRY(hipStreamWaitEvent(sa, c->ev[g], 0));
    const int rc = vsg_merge_topk_device(reinterpret_cast<const uint64_t*>(gk), reinterpret_cast<const float*>(gd), n,
                                         nq, k, k, ok, od, sa);
    if (rc) return rc;
    SH_TRY(hipEventRecord(c->done, sa));
    c->pending = true;
    return VSG_OK;
}

// Host<->device copies in <= 16 MiB pieces (see vsg_index.cpp copy_chunked)
static hipError_t copy_pieces(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
    const size_t CH = (size_t)16 << 20;
    for (size_t off = 0; off < bytes; off += CH) {
        const hipError_t e = hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, static_cast<const uint8_t*>(src) + off,
                                            std::min(CH, bytes - off), kind, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

static int search_host(vsg_sharded* h, const float* queries, size_t nq, size_t k, size_t ef, bool exact,
                       uint64_t* out_keys, float* out_dist, size_t* out_counts) {
    if (!h || (nq && (!queries || !out_keys || !out_dist))) return sfail(VSG_EINVAL, "null argument");
    if (k == 0) return sfail(VSG_EINVAL, "k must be >= 1 (Limit is NonZeroUsize)");
    if (nq == 0) return VSG_OK;
    ShardCtx* c = nullptr;
    int rc = ctx_acquire(h, &c);
    if (rc) return rc;
    const size_t qb = (nq * h->opt.dimensions * 4 + 255) & ~(size_t)255, kb = (nq * k * 8 + 255) & ~(size_t)255,
                 db = nq * k * 4;
    hipError_t e = hipSuccess;
    {
        DevGuard dg(h->ans);
        e = grow(&c->res, c->res_cap, qb + kb + db, c->sa);
        if (e == hipSuccess && std::max(qb, kb + db) > c->pin_cap) {
            vsg::pinned_return(c->pin, c->pin_cap, true);
            c->pin = nullptr;
            c->pin_cap = 0;
            e = vsg::pinned_take(&c->pin, &c->pin_cap, std::max(qb, kb + db), true);
        }
        if (e == hipSuccess) {
            std::memcpy(c->pin, queries, nq * h->opt.dimensions * 4);
            e = copy_pieces(c->res, c->pin, nq * h->opt.dimensions * 4, hipMemcpyHostToDevice, c->sa);
        }
    }
    if (e != hipSuccess) rc = sfail(VSG_EDEVICE, std::string("sharded search staging: ") + hipGetErrorString(e));
    uint64_t* dk = reinterpret_cast<uint64_t*>(c->res + qb);
    float* dd = reinterpret_cast<float*>(c->res + qb + kb);
    if (rc == VSG_OK) rc = search_enqueue(h, c, reinterpret_cast<const float*>(c->res), nq, k, ef, exact, dk, dd, c->sa);
    {
        DevGuard dg(h->ans);
        if (rc == VSG_OK && copy_pieces(c->pin, dk, kb + db, hipMemcpyDeviceToHost, c->sa) != hipSuccess)
            rc = sfail(VSG_EDEVICE, "sharded search: D2H results");
        // drain every stream this call used (also after an error: the context is reused)
        e = hipStreamSynchronize(c->sa);
        for (size_t g = 0; g < h->n; ++g) {
            DevGuard dgs(h->dev[g]);
            const hipError_t e2 = hipStreamSynchronize(c->s[g]);
            if (e == hipSuccess) e = e2;
        }
        c->pending = false;
    }
    if (rc == VSG_OK && e != hipSuccess) rc = sfail(VSG_EDEVICE, std::string("sharded search: ") + hipGetErrorString(e));
    if (rc == VSG_OK) {
        std::memcpy(out_keys, c->pin, nq * k * 8);
        std::memcpy(out_dist, c->pin + kb, nq * k * 4);
        if (out_counts)
            for (size_t i = 0; i < nq; ++i) {
                size_t m = 0;
                while (m < k && out_keys[i * k + m] != VSG_NO_KEY) ++m;
                out_counts[i] = m;
            }
    }
    ctx_release(h, c);
    return rc;
}

extern "C" {

int vsg_sharded_new(const vsg_sharded_options_t* o, vsg_sharded_t** out) {
    VSG_RANGE();
    if (!o || !out) return sfail(VSG_EINVAL, "null argument");
    *out = nullptr;
    if (o->n_shards == 0 || o->n_shards > VSG_MAX_SHARDS)
        return sfail(VSG_EINVAL, "n_shards must be in [1, " + std::to_string(VSG_MAX_SHARDS) + "]");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return sfail(VSG_EDEVICE, "no HIP device visible");
    auto h = std::make_unique<vsg_sharded>();
    h->opt = o->index;
    h->n = o->n_shards;
    for (uint32_t g = 0; g < h->n; ++g) {
        const int d = o->devices ? o->devices[g] : (int)(g % (uint32_t)ndev);
        if (d < 0 || d >= ndev) return sfail(VSG_EINVAL, "shard device ordinal out of range");
        h->dev.push_back(d);
        auto it = std::find(h->devs.begin(), h->devs.end(), d);
        if (it == h->devs.end()) {
            h->dev_slot.push_back((int)h->devs.size());
            h->first_on.push_back((int)g);
            h->devs.push_back(d);
        } else {
            h->dev_slot.push_back((int)(it - h->devs.begin()));
        }
    }
    h->ans = o->answer_device >= 0 ? o->answer_device : h->dev[0];
    if (h->ans >= ndev) return sfail(VSG_EINVAL, "answer device ordinal out of range");
    // peer access answer <-> shard devices (xGMI DMA; hipMemcpyPeerAsync stages
    // through the host where it is unavailable)
    for (int d : h->devs) {
        if (d == h->ans) continue;
        int can = 0;
        for (auto [a, b] : {std::pair<int, int>{h->ans, d}, std::pair<int, int>{d, h->ans}}) {
            if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
                DevGuard dg(a);
                const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return sfail(VSG_EDEVICE, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();
            }
        }
    }
    for (uint32_t g = 0; g < h->n; ++g) {
        vsg_index_options_t so = o->index;
        so.device = h->dev[g];
        so.seed = o->index.seed + g;
        vsg_index_t* s = nullptr;
        const int rc = vsg_index_new(&so, &s);
        if (rc) {
            for (vsg_index_t* x : h->shard) vsg_index_free(x);
            return rc;
        }
        h->shard.push_back(s);
    }
    *out = h.release();
    return VSG_OK;
}

void vsg_sharded_free(vsg_sharded_t* h) {
    VSG_RANGE();
    if (!h) return;
    for (ShardCtx* c : h->ctx_free) ctx_destroy(h, c);
    for (vsg_index_t* s : h->shard) vsg_index_free(s);
    delete h;
}

int vsg_sharded_reserve(vsg_sharded_t* h, size_t capacity) {
    VSG_RANGE();
    if (!h) return sfail(VSG_EINVAL, "null index");
    std::lock_guard<std::mutex> wl(h->wmu);
    const size_t per = (capacity + h->n - 1) / h->n;
    for (vsg_index_t* s : h->shard) {
        const int rc = vsg_index_reserve(s, per);
        if (rc) return rc;
    }
    return VSG_OK;
}

size_t vsg_sharded_capacity(const vsg_sharded_t* h) {
    size_t c = 0;
    if (h)
        for (vsg_index_t* s : h->shard) c += vsg_index_capacity(s);
    return c;
}

size_t vsg_sharded_size(const vsg_sharded_t* h) {
    size_t c = 0;
    if (h)
        for (vsg_index_t* s : h->shard) c += vsg_index_size(s);
    return c;
}

size_t vsg_sharded_dimensions(const vsg_sharded_t* h) { return h ? h->opt.dimensions : 0; }
size_t vsg_sharded_shard_count(const vsg_sharded_t* h) { return h ? h->n : 0; }
uint32_t vsg_sharded_route(const vsg_sharded_t* h, uint64_t key) { return h ? h->route(key) : 0; }
vsg_index_t* vsg_sharded_shard(vsg_sharded_t* h, size_t g) { return h && g < h->n ? h->shard[g] : nullptr; }

int vsg_sharded_contains(const vsg_sharded_t* h, uint64_t key) {
    return h ? vsg_index_contains(h->shard[h->route(key)], key) : 0;
}

int vsg_sharded_add(vsg_sharded_t* h, const uint64_t* keys, const float* vectors, size_t n) {
    VSG_RANGE();
    if (!h || (n && (!keys || !vectors))) return sfail(VSG_EINVAL, "null argument");
    if (n == 0) return VSG_OK;
    std::lock_guard<std::mutex> wl(h->wmu);
    const size_t dim = h->opt.dimensions;
    std::vector<std::vector<uint32_t>> rows(h->n);  // batch rows per shard, in batch order
    for (size_t i = 0; i < n; ++i) {
        if (keys[i] >= UINT64_MAX - 1) return sfail(VSG_EINVAL, "keys UINT64_MAX and UINT64_MAX-1 are reserved");
        rows[h->route(keys[i])].push_back((uint32_t)i);
    }
    if (n > (size_t)UINT32_MAX) return sfail(VSG_EINVAL, "batch too large");
    std::vector<std::vector<uint64_t>> skeys(h->n);
    std::vector<int> rc(h->n, VSG_OK);
    std::vector<std::string> msg(h->n);
    // 1. every shard checks its keys (duplicates inside the batch, live keys)
    //    before any shard inserts: a duplicate anywhere inserts nothing
    per_shard(h->n, [&](size_t g) {
        std::vector<uint64_t>& k = skeys[g];
        k.resize(rows[g].size());
        for (size_t j = 0; j < k.size(); ++j) k[j] = keys[rows[g][j]];
        std::vector<uint64_t> sorted(k);
        std::sort(sorted.begin(), sorted.end());
        const auto dup = std::adjacent_find(sorted.begin(), sorted.end());
        if (dup != sorted.end()) {
            rc[g] = VSG_EDUPKEY;
            msg[g] = "Duplicate keys not allowed: " + std::to_string(*dup);
            return;
        }
        const size_t live = vsg::index_first_live(h->shard[g], k.data(), k.size());
        if (live < k.size()) {
            rc[g] = VSG_EDUPKEY;
            msg[g] = "Duplicate keys not allowed: " + std::to_string(k[live]);
        }
    });
    for (size_t g = 0; g < h->n; ++g)
        if (rc[g]) return sfail(rc[g], msg[g]);
    // 2. every shard builds its rows concurrently: rows gathered through a pinned
    //    piece buffer into one device block, then one batched add on the device
    per_shard(h->n, [&](size_t g) {
        const size_t ng = rows[g].size();
        if (ng == 0) return;
        DevGuard dg(h->dev[g]);
        float* dv = nullptr;
        float* pin = nullptr;
        hipStream_t st = nullptr;
        const size_t piece = std::min<size_t>(ng, std::max<size_t>(1, ((size_t)16 << 20) / (dim * 4)));
        size_t pin_cap = 0;
        hipError_t e = vsg::stream_get(&st);
        if (e == hipSuccess) e = vsg::pool_malloc((void**)&dv, ng * dim * 4, st);
        if (e == hipSuccess) e = vsg::pinned_take(reinterpret_cast<uint8_t**>(&pin), &pin_cap, piece * dim * 4, false);
        for (size_t off = 0; off < ng && e == hipSuccess; off += piece) {
            const size_t c = std::min(piece, ng - off);
            for (size_t j = 0; j < c; ++j)
                std::memcpy(pin + j * dim, vectors + (size_t)rows[g][off + j] * dim, dim * 4);
            e = hipMemcpyAsync(dv + off * dim, pin, c * dim * 4, hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
        }
        if (e != hipSuccess) {
            rc[g] = VSG_EDEVICE;
            msg[g] = std::string("sharded add staging: ") + hipGetErrorString(e);
        } else {
            rc[g] = vsg_index_add_device(h->shard[g], skeys[g].data(), dv, ng, st);
            if (rc[g]) msg[g] = vsg_last_error();  // thread-local: read on this thread
        }
        if (st) (void)hipStreamSynchronize(st);
        vsg::pinned_return(reinterpret_cast<uint8_t*>(pin), pin_cap, false);
        if (st) {
            vsg::pool_free(dv, st);
            (void)hipStreamSynchronize(st);
            vsg::stream_put(st);
        }
    });
    size_t bad = h->n;
    for (size_t g = 0; g < h->n; ++g)
        if (rc[g] && bad == h->n) bad = g;
    if (bad == h->n) return VSG_OK;
    // a shard failed (device error): the other shards' keys leave again
    for (size_t g = 0; g < h->n; ++g)
        if (rc[g] == VSG_OK && !skeys[g].empty())
            (void)vsg_index_remove(h->shard[g], skeys[g].data(), skeys[g].size(), nullptr);
    return sfail(rc[bad], "shard " + std::to_string(bad) + ": " + msg[bad]);
}

// vsg_index_replace per shard: a key and all its messages meet on one shard
// (route), so each shard applies its sub-stream in call order, all concurrently.
int vsg_sharded_replace(vsg_sharded_t* h, const uint64_t* keys, const float* vectors, size_t n, size_t batch,
                        uint32_t flags, int* status, size_t* n_applied) {
    VSG_RANGE();
    if (n_applied) *n_applied = 0;
    if (!h || (n && (!keys || !vectors))) return sfail(VSG_EINVAL, "null argument");
    for (size_t i = 0; status && i < n; ++i) status[i] = VSG_OK;
    if (n == 0) return VSG_OK;
    std::lock_guard<std::mutex> wl(h->wmu);
    const size_t dim = h->opt.dimensions;
    std::vector<std::vector<uint32_t>> rows(h->n);
    for (size_t i = 0; i < n; ++i) rows[h->route(keys[i])].push_back((uint32_t)i);
    std::vector<int> rc(h->n, VSG_OK);
    std::vector<std::string> msg(h->n);
    std::vector<size_t> applied(h->n, 0);
    per_shard(h->n, [&](size_t g) {
        const size_t ng = rows[g].size();
        if (ng == 0) return;
        std::vector<uint64_t> k(ng);
        std::vector<float> v(ng * dim);
        std::vector<int> st(ng, VSG_OK);
        for (size_t j = 0; j < ng; ++j) {
            k[j] = keys[rows[g][j]];
            std::memcpy(&v[j * dim], vectors + (size_t)rows[g][j] * dim, dim * 4);
        }
        rc[g] = vsg_index_replace(h->shard[g], k.data(), v.data(), ng, batch, flags, st.data(), &applied[g]);
        if (rc[g]) msg[g] = vsg_last_error();  // thread-local: read on this thread
        for (size_t j = 0; status && j < ng; ++j) status[rows[g][j]] = st[j];
    });
    for (size_t g = 0; n_applied && g < h->n; ++g) *n_applied += applied[g];
    for (size_t g = 0; g < h->n; ++g)
        if (rc[g]) return sfail(rc[g], "shard " + std::to_string(g) + ": " + msg[g]);
    return VSG_OK;
}

int vsg_sharded_remove(vsg_sharded_t* h, const uint64_t* keys, size_t n, size_t* n_removed) {
    VSG_RANGE();
    if (!h || (n && !keys)) return sfail(VSG_EINVAL, "null argument");
    std::lock_guard<std::mutex> wl(h->wmu);
    std::vector<std::vector<uint64_t>> sk(h->n);
    for (size_t i = 0; i < n; ++i) sk[h->route(keys[i])].push_back(keys[i]);
    size_t total = 0;
    for (size_t g = 0; g < h->n; ++g) {
        if (sk[g].empty()) continue;
        size_t r = 0;
        const int rc = vsg_index_remove(h->shard[g], sk[g].data(), sk[g].size(), &r);
        if (rc) return rc;
        total += r;
    }
    if (n_removed) *n_removed = total;
    return VSG_OK;
}

int vsg_sharded_search(vsg_sharded_t* h, const float* queries, size_t nq, size_t k, size_t ef, uint64_t* out_keys,
                       float* out_distances, size_t* out_counts) {
    VSG_RANGE();
    return search_host(h, queries, nq, k, ef, false, out_keys, out_distances, out_counts);
}

int vsg_sharded_exact_search(vsg_sharded_t* h, const float* queries, size_t nq, size_t k, uint64_t* out_keys,
                             float* out_distances, size_t* out_counts) {
    VSG_RANGE();
    return search_host(h, queries, nq, k, 0, true, out_keys, out_distances, out_counts);
}

int vsg_sharded_search_device(vsg_sharded_t* h, const float* q, size_t nq, size_t k, size_t ef, int exact,
                              uint64_t* ok, float* od, void* stream) {
    VSG_RANGE();
    if (!h || (nq && (!q || !ok || !od))) return sfail(VSG_EINVAL, "null argument");
    if (k == 0) return sfail(VSG_EINVAL, "k must be >= 1 (Limit is NonZeroUsize)");
    if (nq == 0) return VSG_OK;
    ShardCtx* c = nullptr;
    int rc = ctx_acquire(h, &c);
    if (rc) return rc;
    rc = search_enqueue(h, c, q, nq, k, ef, exact != 0, ok, od, (hipStream_t)stream);
    if (rc) {  // drain what was enqueued before the context is reused
        for (size_t g = 0; g < h->n; ++g) {
            DevGuard dg(h->dev[g]);
            (void)hipStreamSynchronize(c->s[g]);
        }
        c->pending = false;
    }
    ctx_release(h, c);
    return rc;
}

int vsg_sharded_compact(vsg_sharded_t* h, size_t* n_dropped) {
    VSG_RANGE();
    if (!h) return sfail(VSG_EINVAL, "null index");
    std::lock_guard<std::mutex> wl(h->wmu);
    std::vector<int> rc(h->n, VSG_OK);
    std::vector<size_t> dropped(h->n, 0);
    std::vector<std::string> msg(h->n);
    per_shard(h->n, [&](size_t g) {
        rc[g] = vsg_index_compact(h->shard[g], &dropped[g]);
        if (rc[g]) msg[g] = vsg_last_error();
    });
    size_t total = 0;
    for (size_t g = 0; g < h->n; ++g) {
        if (rc[g]) return sfail(rc[g], "shard " + std::to_string(g) + ": " + msg[g]);
        total += dropped[g];
    }
    if (n_dropped) *n_dropped = total;
    return VSG_OK;
}

int vsg_sharded_stats(const vsg_sharded_t* h, vsg_stats_t* out) {
    if (!h || !out) return sfail(VSG_EINVAL, "null argument");
    std::memset(out, 0, sizeof(*out));
    // counters add up over the shards; the build device times do not -- the
    // shards build concurrently (one stream per shard), so the sharded index's
    // build took as long as its slowest shard: the maximum of each
    for (vsg_index_t* s : h->shard) {
        vsg_stats_t t;
        const int rc = vsg_index_stats(s, &t);
        if (rc) return rc;
        const uint64_t* a = reinterpret_cast<const uint64_t*>(&t);
        uint64_t* b = reinterpret_cast<uint64_t*>(out);
        for (size_t i = 0; i < sizeof(vsg_stats_t) / 8; ++i) b[i] += a[i];
        out->build_insert_ns -= t.build_insert_ns;
        out->build_sort_ns -= t.build_sort_ns;
        out->build_reverse_ns -= t.build_reverse_ns;
        out->build_select_ns -= t.build_select_ns;
        out->build_insert_ns = std::max(out->build_insert_ns, t.build_insert_ns);
        out->build_sort_ns = std::max(out->build_sort_ns, t.build_sort_ns);
        out->build_reverse_ns = std::max(out->build_reverse_ns, t.build_reverse_ns);
        out->build_select_ns = std::max(out->build_select_ns, t.build_select_ns);
    }
    return VSG_OK;
}

int vsg_sharded_reset_stats(vsg_sharded_t* h) {
    if (!h) return sfail(VSG_EINVAL, "null index");
    for (vsg_index_t* s : h->shard) {
        const int rc = vsg_index_reset_stats(s);
        if (rc) return rc;
    }
    return VSG_OK;
}

}  // extern "C"
