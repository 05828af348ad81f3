// Host logic of the coalescing index actor (csrc/actor.hpp) against a mock
// backend: FIFO semantics of add/replace/remove, batching of concurrent anns,
// ef grouping, capacity growth (src/index/usearch.rs:200-212), error counting.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <map>
#include <mutex>
#include <random>
#include <shared_mutex>
#include <thread>

#include "../../vector-store-text_amd/csrc/actor.hpp"

#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                             \
        }                                                             \
    } while (0)

struct Call {
    char op;
    size_t n, k, ef;
};

// exact l2sq over a std::map, ties by key; records every call
struct Mock final : vsg::ActorBackend {
    size_t dim, ef0, cap = 0;
    std::map<uint64_t, std::vector<float>> rows;
    std::vector<Call>* log;
    std::vector<size_t>* reserves;
    int search_sleep_us;
    bool fail_add = false;
    Mock(size_t d, size_t ef, std::vector<Call>* l, std::vector<size_t>* r, int sleep_us)
        : dim(d), ef0(ef), log(l), reserves(r), search_sleep_us(sleep_us) {}
    size_t dimensions() const override { return dim; }
    size_t size() const override { return rows.size(); }
    size_t capacity() const override { return cap; }
    size_t expansion_search() const override { return ef0; }
    bool contains(uint64_t k) const override { return rows.count(k) != 0; }
    int reserve(size_t c) override {
        reserves->push_back(c);
        if (c > cap) cap = c;
        return 0;
    }
    int add(const uint64_t* k, const float* v, size_t n) override {
        log->push_back({'a', n, 0, 0});
        if (fail_add) return 4;
        for (size_t i = 0; i < n; ++i)
            if (rows.count(k[i])) return 3;  // duplicate: nothing inserted
        if (rows.size() + n > cap) return 2;
        for (size_t i = 0; i < n; ++i) rows[k[i]] = std::vector<float>(v + i * dim, v + (i + 1) * dim);
        return 0;
    }
    int remove(const uint64_t* k, size_t n, size_t* r) override {
        log->push_back({'r', n, 0, 0});
        size_t c = 0;
        for (size_t i = 0; i < n; ++i) c += rows.erase(k[i]);
        if (r) *r = c;
        return 0;
    }
    int search(const float* q, size_t nq, size_t k, size_t ef, uint64_t* keys, float* dist,
               size_t* counts) override {
        log->push_back({'s', nq, k, ef});
        if (search_sleep_us) std::this_thread::sleep_for(std::chrono::microseconds(search_sleep_us));
        for (size_t i = 0; i < nq; ++i) {
            std::vector<std::pair<float, uint64_t>> all;
            for (auto& kv : rows) {
                float s = 0;
                for (size_t t = 0; t < dim; ++t) {
                    const float df = kv.second[t] - q[i * dim + t];
                    s += df * df;
                }
                all.push_back({s, kv.first});
            }
            std::sort(all.begin(), all.end());
            const size_t c = std::min(k, all.size());
            for (size_t j = 0; j < k; ++j) {
                keys[i * k + j] = j < c ? all[j].second : ~0ull;
                dist[i * k + j] = j < c ? all[j].first : INFINITY;
            }
            counts[i] = c;
        }
        return 0;
    }
};

static std::vector<float> vec_of(uint64_t seed, size_t dim) {
    std::mt19937_64 r(seed);
    std::vector<float> v(dim);
    for (auto& x : v) x = (float)(r() % 1000) / 10.f;
    return v;
}

// 1) FIFO semantics: a random single-threaded add/replace/remove stream ends in
//    the state a sequential map reaches, however the worker batches it.
static void test_fifo_semantics() {
    std::vector<Call> log;
    std::vector<size_t> res;
    auto* m = new Mock(4, 16, &log, &res, 0);
    Mock* mp = m;
    vsg::ActorConfig cfg;
    cfg.reserve_increment = 64;
    cfg.reserve_threshold = 21;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
    CHECK(a.init() == 0);
    std::map<uint64_t, std::vector<float>> ref;
    std::mt19937_64 rng(3);
    for (int it = 0; it < 20000; ++it) {
        const uint64_t k = rng() % 300;
        if (rng() % 4 == 0) {
            a.remove(k);
            ref.erase(k);
        } else {
            auto v = vec_of(rng(), 4);
            a.add_or_replace(k, v.data());
            ref[k] = v;
        }
        if (it % 5000 == 4999) {
            size_t n = 0;
            CHECK(a.count(&n) == 0);
            CHECK(n == ref.size());
        }
    }
    CHECK(a.flush() == 0);
    CHECK(mp->rows == ref);
    const auto c = a.counters();
    CHECK(c.add_errors == 0 && c.remove_errors == 0);
    CHECK(c.writes == 20000);
    CHECK(c.add_calls < 20000);  // coalesced
    // capacity rule: every reserve adds one increment, only when free < threshold
    for (size_t i = 1; i < res.size(); ++i) CHECK(res[i] == res[i - 1] + 64);
    CHECK(mp->cap - mp->rows.size() >= 21 - 1);
}

// 2) concurrent anns are batched, and each answer equals the backend's own
//    answer for that query alone.
static void test_concurrent_anns() {
    std::vector<Call> log;
    std::vector<size_t> res;
    auto* m = new Mock(8, 16, &log, &res, 2000);
    vsg::ActorConfig cfg;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
    CHECK(a.init() == 0);
    for (uint64_t k = 0; k < 500; ++k) {
        auto v = vec_of(k + 100, 8);
        a.add_or_replace(k, v.data());
    }
    CHECK(a.flush() == 0);
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    const int T = 32, Q = 40;
    for (int t = 0; t < T; ++t) {
        th.emplace_back([&, t] {
            for (int i = 0; i < Q; ++i) {
                auto q = vec_of(7000 + t * 1000 + i, 8);
                const size_t k = 1 + (size_t)((t + i) % 12);
                std::vector<uint64_t> keys(k);
                std::vector<float> dist(k);
                size_t cnt = 0;
                if (a.ann(q.data(), 8, k, keys.data(), dist.data(), &cnt) != 0) { bad++; continue; }
                // direct answer (mock is exact => top-k is a prefix of top-kmax)
                std::vector<std::pair<float, uint64_t>> all;
                for (uint64_t r = 0; r < 500; ++r) {
                    auto v = vec_of(r + 100, 8);
                    float s = 0;
                    for (int d = 0; d < 8; ++d) s += (v[d] - q[d]) * (v[d] - q[d]);
                    all.push_back({s, r});
                }
                std::sort(all.begin(), all.end());
                if (cnt != k) bad++;
                for (size_t j = 0; j < k; ++j)
                    if (keys[j] != all[j].second || dist[j] != all[j].first) bad++;
            }
        });
    }
    for (auto& x : th) x.join();
    CHECK(bad == 0);
    const auto c = a.counters();
    CHECK(c.anns == (uint64_t)(T * Q));
    CHECK(c.search_calls < c.anns);  // batched
    CHECK(c.max_search_batch > 1);
}

// 2b) anns with completions (ann_cb, the oneshot form): a closed loop of 64 clients
//     driven only from the callbacks answers like the exact scan, batched, with every
//     completion run once; a rejected query gets no completion.
struct CbCtx {
    vsg::Actor* a;
    int client, i;
    std::vector<uint64_t> keys;
    std::vector<float> dist;
    std::atomic<int>* bad;
    std::atomic<int>* finished;
};
static std::vector<float> cb_query(int client, int i) { return vec_of(9000 + client * 100 + i, 8); }
static void cb_done(void* p, int status, size_t cnt) {
    auto* c = static_cast<CbCtx*>(p);
    auto q = cb_query(c->client, c->i);
    std::vector<std::pair<float, uint64_t>> all;
    for (uint64_t r = 0; r < 500; ++r) {
        auto v = vec_of(r + 100, 8);
        float s = 0;
        for (int d = 0; d < 8; ++d) s += (v[d] - q[d]) * (v[d] - q[d]);
        all.push_back({s, r});
    }
    std::sort(all.begin(), all.end());
    if (status != 0 || cnt != c->keys.size()) (*c->bad)++;
    for (size_t j = 0; j < c->keys.size(); ++j)
        if (c->keys[j] != all[j].second || c->dist[j] != all[j].first) (*c->bad)++;
    if (++c->i < 20) {
        auto nq = cb_query(c->client, c->i);
        if (c->a->ann_cb(nq.data(), 8, c->keys.size(), c->keys.data(), c->dist.data(), cb_done, c) != 0) (*c->bad)++;
        return;
    }
    (*c->finished)++;
}
static void test_ann_completions() {
    std::vector<Call> log;
    std::vector<size_t> res;
    auto* m = new Mock(8, 16, &log, &res, 2000);
    vsg::ActorConfig cfg;
    cfg.concurrent_reads = 2;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
    CHECK(a.init() == 0);
    for (uint64_t k = 0; k < 500; ++k) {
        auto v = vec_of(k + 100, 8);
        a.add_or_replace(k, v.data());
    }
    CHECK(a.flush() == 0);
    std::atomic<int> bad{0}, finished{0};
    const int C = 64;
    std::vector<CbCtx> cl(C);
    for (int t = 0; t < C; ++t) {
        cl[t] = CbCtx{&a, t, 0, std::vector<uint64_t>(1 + t % 10), std::vector<float>(1 + t % 10), &bad, &finished};
        auto q = cb_query(t, 0);
        CHECK(a.ann_cb(q.data(), 8, cl[t].keys.size(), cl[t].keys.data(), cl[t].dist.data(), cb_done, &cl[t]) == 0);
    }
    for (int w = 0; w < 2000 && finished.load() < C; ++w) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    CHECK(finished.load() == C);
    CHECK(bad == 0);
    const auto c = a.counters();
    CHECK(c.anns == (uint64_t)(C * 20));
    CHECK(c.search_calls < c.anns);  // batched
    uint64_t kk[1];
    float dd[1];
    auto q = cb_query(0, 0);
    CHECK(a.ann_cb(q.data(), 3, 1, kk, dd, cb_done, nullptr) == 1);  // wrong dims: rejected, no completion
}

// 3) effective-ef grouping: one drained run with k below and above ef0 makes
//    two searches, each at ef = max(ef0, k); wrong dims are rejected up front.
static void test_ef_groups_and_errors() {
    std::vector<Call> log;
    std::vector<size_t> res;
    auto* m = new Mock(2, 4, &log, &res, 20000);
    vsg::ActorConfig cfg;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
    CHECK(a.init() == 0);
    for (uint64_t k = 0; k < 50; ++k) {
        float v[2] = {(float)k, 0.f};
        a.add_or_replace(k, v);
    }
    CHECK(a.flush() == 0);
    // occupy the worker with one slow search, queue a mixed run behind it
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int t = 0; t < 7; ++t) {
        th.emplace_back([&, t] {
            if (t) std::this_thread::sleep_for(std::chrono::milliseconds(5));
            float q[2] = {(float)t, 0.f};
            const size_t k = t % 2 ? 2 : 9;  // ef = 4 or 9
            std::vector<uint64_t> keys(k);
            std::vector<float> dist(k);
            size_t cnt = 0;
            if (a.ann(q, 2, k, keys.data(), dist.data(), &cnt) != 0 || cnt != k || keys[0] != (uint64_t)t) bad++;
        });
    }
    for (auto& x : th) x.join();
    CHECK(bad == 0);
    bool saw4 = false, saw9 = false;
    for (auto& c : log)
        if (c.op == 's') {
            CHECK(c.ef == std::max<size_t>(4, c.k));
            saw4 |= c.ef == 4;
            saw9 |= c.ef == 9;
        }
    CHECK(saw4 && saw9);
    float q[3] = {0, 0, 0};
    uint64_t kk[1];
    float dd[1];
    CHECK(a.ann(q, 3, 1, kk, dd, nullptr) == 1);
    CHECK(a.ann(q, 2, 0, kk, dd, nullptr) == 1);
}

// 4) add failures are counted and swallowed, later messages still apply
static void test_add_errors_swallowed() {
    std::vector<Call> log;
    std::vector<size_t> res;
    auto* m = new Mock(2, 4, &log, &res, 0);
    Mock* mp = m;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), vsg::ActorConfig{});
    CHECK(a.init() == 0);
    mp->fail_add = true;
    float v[2] = {1, 2};
    a.add_or_replace(1, v);
    CHECK(a.flush() == 0);
    mp->fail_add = false;
    a.add_or_replace(2, v);
    size_t n = 0;
    CHECK(a.count(&n) == 0 && n == 1);
    CHECK(a.counters().add_errors == 1);
}

// 4b) add completions (vsg_actor_add_or_replace_cb): every add reports the status
//     of the batched add that carried it, on the worker, once -- the host shim's
//     BiMap rollback of a failed add (src/index/usearch.rs:230-232)
struct DoneLog {
    std::mutex m;
    std::map<uint64_t, int> status;
    int calls = 0;
};
static void on_done(void* ctx, uint64_t key, int st) {
    auto* d = static_cast<DoneLog*>(ctx);
    std::lock_guard<std::mutex> lk(d->m);
    d->status[key] = st;
    d->calls++;
}

static void test_add_completions() {
    std::vector<Call> log;
    std::vector<size_t> res;
    auto* m = new Mock(2, 4, &log, &res, 0);
    Mock* mp = m;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), vsg::ActorConfig{});
    CHECK(a.init() == 0);
    DoneLog d;
    float v[2] = {1, 2};
    for (uint64_t k = 0; k < 5; ++k) a.add_or_replace(k, v, on_done, &d);
    CHECK(a.flush() == 0);
    mp->fail_add = true;
    a.add_or_replace(7, v, on_done, &d);
    a.add_or_replace(3, v, on_done, &d);  // a replace whose add fails
    CHECK(a.flush() == 0);
    mp->fail_add = false;
    a.add_or_replace(9, v);  // no completion requested
    CHECK(a.flush() == 0);
    CHECK(d.calls == 7);
    for (uint64_t k = 0; k < 5; ++k) CHECK(d.status[k] == (k == 3 ? 4 : 0));
    CHECK(d.status[7] == 4);
    CHECK(a.size_now() == 5);  // 0,1,2,4 and 9; 3's old row was removed by the replace
}

// 5) tombstones (removes, and the old row of every replace) trigger a
//    compaction once they reach compact_percent of the stored rows
struct TombMock final : vsg::ActorBackend {
    std::map<uint64_t, int> live;
    size_t stored = 0, cap = 0, compactions = 0;
    size_t dimensions() const override { return 1; }
    size_t size() const override { return live.size(); }
    size_t capacity() const override { return cap; }
    size_t expansion_search() const override { return 4; }
    bool contains(uint64_t k) const override { return live.count(k) != 0; }
    int reserve(size_t c) override {
        cap = std::max(cap, c);
        return 0;
    }
    int add(const uint64_t* k, const float*, size_t n) override {
        for (size_t i = 0; i < n; ++i) live[k[i]] = 1;
        stored += n;
        return 0;
    }
    int remove(const uint64_t* k, size_t n, size_t* r) override {
        size_t c = 0;
        for (size_t i = 0; i < n; ++i) c += live.erase(k[i]);
        if (r) *r = c;
        return 0;
    }
    int search(const float*, size_t, size_t, size_t, uint64_t*, float*, size_t*) override { return 0; }
    size_t slots() const override { return stored; }
    int compact(size_t* dropped) override {
        *dropped = stored - live.size();
        stored = live.size();
        ++compactions;
        return 0;
    }
};

static void test_auto_compaction() {
    auto* m = new TombMock;
    TombMock* mp = m;
    vsg::ActorConfig cfg;
    cfg.compact_percent = 50;
    cfg.compact_min_dead = 100;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
    CHECK(a.init() == 0);
    float v = 1.f;
    for (uint64_t k = 0; k < 200; ++k) a.add_or_replace(k, &v);
    CHECK(a.flush() == 0 && mp->compactions == 0);
    for (uint64_t k = 0; k < 150; ++k) a.add_or_replace(k, &v);  // 150 replaces: 150 dead of 350
    CHECK(a.flush() == 0 && mp->compactions == 0);
    // 60 more: the ratio crosses 50 % after the 25th (200 dead of 400) or, with
    // coarser batching, later; exactly one compaction either way
    for (uint64_t k = 0; k < 60; ++k) a.add_or_replace(k, &v);
    CHECK(a.flush() == 0 && mp->compactions == 1);
    const size_t dropped = a.counters().compacted_rows;
    CHECK(dropped >= 200 && dropped <= 210 && mp->stored == 200 + (210 - dropped));
    for (uint64_t k = 0; k < 80; ++k) a.remove(k);  // <= 90 dead: under compact_min_dead
    CHECK(a.flush() == 0 && mp->compactions == 1);
    size_t n = 0;
    CHECK(a.count(&n) == 0 && n == 120);
    cfg.compact_percent = 100;  // disabled
    auto* m2 = new TombMock;
    vsg::Actor b(std::unique_ptr<vsg::ActorBackend>(m2), cfg);
    CHECK(b.init() == 0);
    for (int r = 0; r < 5; ++r)
        for (uint64_t k = 0; k < 200; ++k) b.add_or_replace(k, &v);
    CHECK(b.flush() == 0 && m2->compactions == 0 && m2->stored == 1000);
}

// 6) concurrent_reads: a backend shaped like vsg_index (an add builds for a long
//    time with no lock held, then publishes its rows under the exclusive lock;
//    searches take the shared side).  An Ann issued during a 300 ms add answers
//    long before the add ends, from a prefix of the writes; in the default mode
//    the same Ann waits for the add (submission order).
struct ConcMock final : vsg::ActorBackend {
    mutable std::shared_mutex mu;
    std::map<uint64_t, float> rows;  // key -> 1-d value
    size_t cap = 0;
    std::atomic<int> adds_in_flight{0};
    size_t dimensions() const override { return 1; }
    size_t size() const override {
        std::shared_lock<std::shared_mutex> lk(mu);
        return rows.size();
    }
    size_t capacity() const override { return cap; }
    size_t expansion_search() const override { return 16; }
    bool contains(uint64_t k) const override {
        std::shared_lock<std::shared_mutex> lk(mu);
        return rows.count(k) != 0;
    }
    int reserve(size_t c) override {
        cap = std::max(cap, c);
        return 0;
    }
    int add(const uint64_t* k, const float* v, size_t n) override {
        adds_in_flight++;
        std::this_thread::sleep_for(std::chrono::milliseconds(300));  // the batched build
        std::unique_lock<std::shared_mutex> lk(mu);                    // publish
        for (size_t i = 0; i < n; ++i) rows[k[i]] = v[i];
        adds_in_flight--;
        return 0;
    }
    int remove(const uint64_t* k, size_t n, size_t* r) override {
        std::unique_lock<std::shared_mutex> lk(mu);
        size_t c = 0;
        for (size_t i = 0; i < n; ++i) c += rows.erase(k[i]);
        if (r) *r = c;
        return 0;
    }
    int search(const float* q, size_t nq, size_t k, size_t, uint64_t* keys, float* dist,
               size_t* counts) override {
        std::shared_lock<std::shared_mutex> lk(mu);
        for (size_t i = 0; i < nq; ++i) {
            std::vector<std::pair<float, uint64_t>> all;
            for (auto& kv : rows) all.push_back({(kv.second - q[i]) * (kv.second - q[i]), kv.first});
            std::sort(all.begin(), all.end());
            const size_t c = std::min(k, all.size());
            for (size_t j = 0; j < k; ++j) {
                keys[i * k + j] = j < c ? all[j].second : ~0ull;
                dist[i * k + j] = j < c ? all[j].first : INFINITY;
            }
            counts[i] = c;
        }
        return 0;
    }
};

static void test_concurrent_reads_beside_writes() {
    for (int concurrent = 1; concurrent >= 0; --concurrent) {
        auto* m = new ConcMock;
        ConcMock* mp = m;
        vsg::ActorConfig cfg;
        cfg.reserve_increment = 1000;
        cfg.concurrent_reads = concurrent != 0;
        vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
        CHECK(a.init() == 0);
        const float v1 = 1.f, v2 = 2.f;
        a.add_or_replace(1, &v1);
        CHECK(a.flush() == 0);
        a.add_or_replace(2, &v2);  // a 300 ms "build"
        while (mp->adds_in_flight.load() == 0) std::this_thread::sleep_for(std::chrono::microseconds(100));
        uint64_t keys[2];
        float dist[2];
        size_t cnt = 0;
        const auto t0 = std::chrono::steady_clock::now();
        CHECK(a.ann(&v2, 1, 2, keys, dist, &cnt) == 0);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (concurrent) {
            CHECK(ms < 150.0);                              // answered during the build
            CHECK(cnt == 1 && keys[0] == 1);                // the prefix before the add
            CHECK(mp->adds_in_flight.load() == 1);
        } else {
            CHECK(ms > 150.0);                              // waited for the add (FIFO)
            CHECK(cnt == 2 && keys[0] == 2 && keys[1] == 1);
        }
        CHECK(a.flush() == 0);
        CHECK(a.ann(&v2, 1, 2, keys, dist, &cnt) == 0 && cnt == 2 && keys[0] == 2);
    }
}

// 7) concurrent_reads = 2: two Anns from two clients are searched at the same time
//    (a backend whose search takes 100 ms answers both in ~100 ms, not ~200 ms),
//    with the results one reader gives.
struct SlowSearch final : vsg::ActorBackend {
    std::atomic<int> in_flight{0}, max_in_flight{0};
    size_t dimensions() const override { return 1; }
    size_t size() const override { return 3; }
    size_t capacity() const override { return 1000; }
    size_t expansion_search() const override { return 16; }
    bool contains(uint64_t) const override { return false; }
    int reserve(size_t) override { return 0; }
    int add(const uint64_t*, const float*, size_t) override { return 0; }
    int remove(const uint64_t*, size_t, size_t* r) override {
        if (r) *r = 0;
        return 0;
    }
    int search(const float* q, size_t nq, size_t k, size_t, uint64_t* keys, float* dist, size_t* counts) override {
        const int now = ++in_flight;
        int m = max_in_flight.load();
        while (now > m && !max_in_flight.compare_exchange_weak(m, now)) {
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        for (size_t i = 0; i < nq; ++i) {
            for (size_t j = 0; j < k; ++j) {
                keys[i * k + j] = (uint64_t)(q[i] * 10) + j;
                dist[i * k + j] = (float)j;
            }
            counts[i] = k;
        }
        --in_flight;
        return 0;
    }
};

static void test_read_workers_overlap() {
    for (uint32_t readers : {2u, 1u}) {
        auto* m = new SlowSearch;
        SlowSearch* mp = m;
        vsg::ActorConfig cfg;
        cfg.concurrent_reads = readers;
        vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
        CHECK(a.init() == 0);
        uint64_t ka[2], kb[2];
        float da[2], db[2];
        size_t ca = 0, cb = 0;
        int ra = -1, rb = -1;
        const float qa = 1.f, qb = 2.f;
        const auto t0 = std::chrono::steady_clock::now();
        std::thread ta([&] { ra = a.ann(&qa, 1, 2, ka, da, &ca); });
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
        std::thread tb([&] { rb = a.ann(&qb, 1, 2, kb, db, &cb); });
        ta.join();
        tb.join();
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        CHECK(ra == 0 && rb == 0 && ca == 2 && cb == 2);
        CHECK(ka[0] == 10 && ka[1] == 11 && kb[0] == 20 && kb[1] == 21);
        if (readers == 2) {
            CHECK(mp->max_in_flight.load() == 2);
            CHECK(ms < 180.0);
        } else {
            CHECK(mp->max_in_flight.load() == 1);
            CHECK(ms > 190.0);
        }
    }
}

// 8) replace runs: every run of AddOrReplace messages reaches the backend as one
//    replace call in submission order (keys may repeat; vsg_index_replace applies
//    them as the reference's one-message-at-a-time remove + add), every run of
//    removes as one remove call; the final state is the sequential one
struct ReplMock final : vsg::ActorBackend {
    std::map<uint64_t, float> rows;
    std::vector<Call> log;
    size_t cap = 0;
    size_t dimensions() const override { return 1; }
    size_t size() const override { return rows.size(); }
    size_t capacity() const override { return cap; }
    size_t expansion_search() const override { return 4; }
    bool contains(uint64_t k) const override { return rows.count(k) != 0; }
    int reserve(size_t c) override {
        cap = std::max(cap, c);
        return 0;
    }
    int add(const uint64_t*, const float*, size_t n) override {
        log.push_back({'a', n, 0, 0});
        return 4;
    }
    int remove(const uint64_t* k, size_t n, size_t* r) override {
        log.push_back({'r', n, 0, 0});
        size_t c = 0;
        for (size_t i = 0; i < n; ++i) c += rows.erase(k[i]);
        if (r) *r = c;
        return 0;
    }
    int replace(const uint64_t* k, const float* v, size_t n, size_t, bool, int* status) override {
        log.push_back({'p', n, 0, 0});
        for (size_t i = 0; i < n; ++i) {
            rows[k[i]] = v[i];
            status[i] = 0;
        }
        return 0;
    }
    int search(const float*, size_t, size_t, size_t, uint64_t*, float*, size_t*) override { return 0; }
};

static void test_replace_runs() {
    auto* m = new ReplMock;
    ReplMock* mp = m;
    vsg::ActorConfig cfg;
    cfg.reserve_increment = 4096;
    vsg::Actor a(std::unique_ptr<vsg::ActorBackend>(m), cfg);
    CHECK(a.init() == 0);
    for (uint64_t k = 0; k < 640; ++k) {
        const float v = 1.f;
        a.add_or_replace(k, &v);
    }
    CHECK(a.flush() == 0);
    mp->log.clear();
    for (uint64_t k = 0; k < 100; ++k) {
        const float w = 3.f;
        a.add_or_replace(k, &w);
    }
    const float x = 5.f, y = 7.f, z = 9.f;
    a.remove(5);
    a.add_or_replace(5, &x);
    a.add_or_replace(7, &y);
    a.add_or_replace(7, &z);  // repeated inside one run: the later message wins
    CHECK(a.flush() == 0);
    size_t replaced = 0, removed = 0;
    for (const Call& c : mp->log) {
        CHECK(c.op != 'a');  // adds only through replace
        if (c.op == 'p') replaced += c.n;
        if (c.op == 'r') removed += c.n;
    }
    CHECK(replaced == 103 && removed == 1);
    CHECK(mp->rows.size() == 640 && mp->rows[5] == 5.f && mp->rows[7] == 9.f && mp->rows[50] == 3.f &&
          mp->rows[300] == 1.f);
}

int main() {
    test_concurrent_reads_beside_writes();
    test_read_workers_overlap();
    test_fifo_semantics();
    test_concurrent_anns();
    test_ann_completions();
    test_ef_groups_and_errors();
    test_add_errors_swallowed();
    test_add_completions();
    test_auto_compaction();
    test_replace_runs();
    std::printf("ok\n");
    return 0;
}
