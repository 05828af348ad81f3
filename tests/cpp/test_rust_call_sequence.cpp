// The exact libvsg.so symbol sequence of rust/src/index/gpu.rs (the Rust shim that
// replaces /root/reference/src/index/usearch.rs:36-311), driven from C++ because
// cargo/rustc are not in the image.  Two parts:
//
//  1. the direct usearch::Index replacement (usearch.rs:98-99, 215, 221, 276, 309):
//     vsg_index_new -> vsg_index_reserve(1M) -> vsg_index_add -> replace
//     (vsg_index_remove + vsg_index_add of the same key) -> vsg_index_search ->
//     vsg_index_size -> vsg_index_free;
//  2. the actor path gpu.rs uses (vsg_actor_*, concurrent_reads = 1): the reference's own
//     unit KAT (usearch.rs:322-425, D = 3, keys 1/2/3, replace, remove, count) with its
//     polling (anns may run before earlier writes land, as the reference's fire-and-forget
//     adds allow; it polls for 10 s, usearch.rs:352-358).  Adds go through
//     vsg_actor_add_or_replace_cb (gpu.rs rolls the BiMap back from the completion,
//     usearch.rs:230-232), anns through vsg_actor_ann_cb (gpu.rs sends the oneshot reply
//     from the completion, round 5), counts through vsg_actor_size (usearch.rs:308-311).  Run once
//     on a one-device actor (new_gpu) and once on a two-shard actor on device 0
//     (new_gpu_sharded(&[0, 0]), vsg_actor_new_sharded).
// Metric l2sq: the KAT is an f32 rounding tie under cosine.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/vsg.h"

#define CHECK(c)                                                                        \
    do {                                                                                \
        if (!(c)) {                                                                     \
            std::printf("FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, vsg_last_error()); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

static void direct_index() {
    vsg_index_options_t o{};
    o.dimensions = 3;
    o.metric = VSG_METRIC_L2SQ;
    o.quantization = VSG_SCALAR_F32;
    vsg_index_t* h = nullptr;
    CHECK(vsg_index_new(&o, &h) == VSG_OK);
    CHECK(vsg_index_reserve(h, 1000000) == VSG_OK);  // usearch.rs:99
    CHECK(vsg_index_capacity(h) >= 1000000);
    const uint64_t keys[3] = {0, 1, 2};
    const float rows[9] = {1, 1, 1, 2, -2, 2, 3, 3, 3};
    CHECK(vsg_index_add(h, keys, rows, 3) == VSG_OK);
    CHECK(vsg_index_add(h, keys + 1, rows + 3, 1) == VSG_EDUPKEY);  // usearch: duplicates rejected
    CHECK(vsg_index_size(h) == 3);
    // replace key 2 (usearch.rs:214-221: remove first, then add)
    size_t removed = 0;
    CHECK(vsg_index_remove(h, keys + 2, 1, &removed) == VSG_OK && removed == 1);
    const float repl[3] = {2.1f, -2.1f, 2.1f};
    CHECK(vsg_index_add(h, keys + 2, repl, 1) == VSG_OK);
    const float q[3] = {2.2f, -2.2f, 2.2f};
    uint64_t k[2];
    float d[2];
    size_t cnt[1];
    CHECK(vsg_index_search(h, q, 1, 2, 0, k, d, cnt) == VSG_OK);
    CHECK(cnt[0] == 2 && k[0] == 2 && k[1] == 1 && d[0] <= d[1]);
    CHECK(vsg_index_size(h) == 3);
    vsg_index_free(h);
}

// gpu.rs ann: vsg_actor_ann_cb, the reply arrives in the completion (a oneshot here)
struct AnnReply {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    int status = -1;
    size_t count = 0;
};
static void ann_done(void* ctx, int status, size_t count) {
    auto* r = static_cast<AnnReply*>(ctx);
    std::lock_guard<std::mutex> lk(r->m);
    r->status = status;
    r->count = count;
    r->done = true;
    r->cv.notify_all();
}
static int ann_cb(vsg_actor_t* a, const float* q, size_t dims, size_t limit, uint64_t* k, float* d, size_t* n) {
    AnnReply r;
    const int rc = vsg_actor_ann_cb(a, q, dims, limit, k, d, ann_done, &r);
    if (rc != VSG_OK) return rc;  // rejected: no completion
    std::unique_lock<std::mutex> lk(r.m);
    r.cv.wait(lk, [&] { return r.done; });
    *n = r.count;
    return r.status;
}

// poll an ann until it returns `want` (or 10 s), as the reference test does
static bool ann_becomes(vsg_actor_t* a, const float* q, uint64_t want) {
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10)) {
        uint64_t k = 0;
        float d = 0;
        size_t n = 0;
        if (ann_cb(a, q, 3, 1, &k, &d, &n) != VSG_OK) return false;
        if (n == 1 && k == want) return true;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return false;
}

// count as gpu.rs answers Index::Count (vsg_actor_size), polled like the reference test
static bool count_becomes(vsg_actor_t* a, size_t want) {
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10)) {
        if (vsg_actor_size(a) == want) return true;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return false;
}

// gpu.rs add_done: counts completions; a failure would drop the BiMap entry
static std::atomic<int> g_done{0}, g_failed{0};
static void add_done(void*, uint64_t, int status) {
    g_done++;
    if (status != VSG_OK) g_failed++;
}

static void actor_kat(bool sharded) {
    vsg_actor_options_t o{};
    o.index.dimensions = 3;
    o.index.metric = VSG_METRIC_L2SQ;
    o.reserve_increment = 1000000;  // RESERVE_INCREMENT, usearch.rs:62
    o.reserve_threshold = 1000000 / 3;
    o.concurrent_reads = 1;  // as rust/src/index/gpu.rs
    vsg_actor_t* a = nullptr;
    const int32_t devs[2] = {0, 0};
    if (sharded) {
        CHECK(vsg_actor_new_sharded(&o, 2, devs, &a) == VSG_OK);
        CHECK(vsg_actor_sharded(a) != nullptr && vsg_sharded_shard_count(vsg_actor_sharded(a)) == 2);
    } else {
        CHECK(vsg_actor_new(&o, &a) == VSG_OK);
        CHECK(vsg_actor_sharded(a) == nullptr);
    }
    g_done = 0;
    g_failed = 0;
    // PrimaryKey -> u64 as gpu.rs allocates them: 1 -> 0, 2 -> 1, 3 -> 2
    const float r1[3] = {1, 1, 1}, r2[3] = {2, -2, 2}, r3[3] = {3, 3, 3};
    CHECK(vsg_actor_add_or_replace_cb(a, 0, r1, 3, add_done, nullptr) == VSG_OK);
    CHECK(vsg_actor_add_or_replace_cb(a, 1, r2, 3, add_done, nullptr) == VSG_OK);
    CHECK(vsg_actor_add_or_replace_cb(a, 2, r3, 3, add_done, nullptr) == VSG_OK);
    CHECK(count_becomes(a, 3));
    const float q[3] = {2.2f, -2.2f, 2.2f};
    CHECK(ann_becomes(a, q, 1));  // PK 2
    const float r3b[3] = {2.1f, -2.1f, 2.1f};
    CHECK(vsg_actor_add_or_replace_cb(a, 2, r3b, 3, add_done, nullptr) == VSG_OK);  // replace PK 3: same key
    CHECK(ann_becomes(a, q, 2));  // PK 3
    CHECK(vsg_actor_remove(a, 2) == VSG_OK);
    CHECK(count_becomes(a, 2));
    CHECK(ann_becomes(a, q, 1));  // PK 2 again
    // dimension checks before any search (usearch.rs:259-272)
    uint64_t k;
    float d;
    size_t n;
    CHECK(ann_cb(a, q, 2, 1, &k, &d, &n) == VSG_EINVAL);
    CHECK(ann_cb(a, q, 3, 0, &k, &d, &n) == VSG_EINVAL);
    CHECK(vsg_actor_ann(a, q, 2, 1, &k, &d, &n) == VSG_EINVAL);  // the blocking form checks the same
    CHECK(vsg_actor_flush(a) == VSG_OK);
    vsg_actor_counters_t c{};
    CHECK(vsg_actor_counters(a, &c) == VSG_OK && c.add_errors == 0);
    CHECK(g_done == 4 && g_failed == 0);
    if (sharded) {
        CHECK(vsg_sharded_size(vsg_actor_sharded(a)) == 2);
    } else {
        CHECK(vsg_actor_index(a) != nullptr && vsg_index_size(vsg_actor_index(a)) == 2);
    }
    // a rejected message: wrong dimensions (gpu.rs drops the new mapping at once)
    CHECK(vsg_actor_add_or_replace_cb(a, 7, r1, 2, add_done, nullptr) == VSG_EINVAL);
    vsg_actor_free(a);
}

int main() {
    direct_index();
    actor_kat(false);
    actor_kat(true);
    std::printf("ok\n");
    return 0;
}
