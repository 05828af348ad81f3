// vsg_actor.cpp — C ABI of the index actor (include/vsg.h, "Actor" section):
// the GPU index behind the reference's message API (src/index/usearch.rs
// :82-311), with request coalescing (csrc/actor.hpp).
#include <cstdlib>
#include <string>

#include "../../include/vsg.h"
#include "actor.hpp"
#include "roctx_range.hpp"

namespace vsg {
void set_last_error(const std::string& msg);  // vsg_index.cpp
int index_search_gather(vsg_index_t* h, const float* const* q, size_t nq, size_t k, size_t ef, uint64_t* out_keys,
                        float* out_distances, size_t* out_counts);
}

namespace {

int actor_fail(int code, const std::string& msg) {
    vsg::set_last_error(msg);
    return code;
}

struct IndexBackend final : vsg::ActorBackend {
    vsg_index_t* h;
    size_t ef;
    explicit IndexBackend(vsg_index_t* idx, size_t ef_) : h(idx), ef(ef_) {}
    ~IndexBackend() override { vsg_index_free(h); }
    size_t dimensions() const override { return vsg_index_dimensions(h); }
    size_t size() const override { return vsg_index_size(h); }
    size_t capacity() const override { return vsg_index_capacity(h); }
    size_t expansion_search() const override { return ef; }
    bool contains(uint64_t key) const override { return vsg_index_contains(h, key) == 1; }
    int reserve(size_t c) override { return vsg_index_reserve(h, c); }
    int add(const uint64_t* k, const float* v, size_t n) override { return vsg_index_add(h, k, v, n); }
    int remove(const uint64_t* k, size_t n, size_t* r) override { return vsg_index_remove(h, k, n, r); }
    int replace(const uint64_t* k, const float* v, size_t n, size_t batch, bool hold, int* status) override {
        return vsg_index_replace(h, k, v, n, batch, hold ? VSG_REPLACE_HOLD_TAIL : 0u, status, nullptr);
    }
    void set_error(const std::string& msg) override { vsg::set_last_error(msg); }
    int search(const float* q, size_t nq, size_t k, size_t e, uint64_t* keys, float* dist,
               size_t* counts) override {
        return vsg_index_search(h, q, nq, k, e, keys, dist, counts);
    }
    int search_gather(const float* const* q, size_t nq, size_t k, size_t e, uint64_t* keys, float* dist,
                      size_t* counts) override {
        return vsg::index_search_gather(h, q, nq, k, e, keys, dist, counts);
    }
    size_t slots() const override {
        size_t s = 0;
        return vsg_index_graph_info(h, &s, nullptr, nullptr, nullptr, nullptr) == VSG_OK ? s : size();
    }
    int compact(size_t* dropped) override { return vsg_index_compact(h, dropped); }
    // called on the worker thread, right after the failing call
    const char* last_error() const override { return vsg_last_error(); }
};

// the same actor over a row-sharded index (include/vsg.h "Sharded index")
struct ShardedBackend final : vsg::ActorBackend {
    vsg_sharded_t* h;
    size_t ef;
    explicit ShardedBackend(vsg_sharded_t* idx, size_t ef_) : h(idx), ef(ef_) {}
    ~ShardedBackend() override { vsg_sharded_free(h); }
    size_t dimensions() const override { return vsg_sharded_dimensions(h); }
    size_t size() const override { return vsg_sharded_size(h); }
    size_t capacity() const override { return vsg_sharded_capacity(h); }
    size_t expansion_search() const override { return ef; }
    bool contains(uint64_t key) const override { return vsg_sharded_contains(h, key) == 1; }
    int reserve(size_t c) override { return vsg_sharded_reserve(h, c); }
    int add(const uint64_t* k, const float* v, size_t n) override { return vsg_sharded_add(h, k, v, n); }
    int remove(const uint64_t* k, size_t n, size_t* r) override { return vsg_sharded_remove(h, k, n, r); }
    int replace(const uint64_t* k, const float* v, size_t n, size_t batch, bool hold, int* status) override {
        return vsg_sharded_replace(h, k, v, n, batch, hold ? VSG_REPLACE_HOLD_TAIL : 0u, status, nullptr);
    }
    void set_error(const std::string& msg) override { vsg::set_last_error(msg); }
    int search(const float* q, size_t nq, size_t k, size_t e, uint64_t* keys, float* dist,
               size_t* counts) override {
        return vsg_sharded_search(h, q, nq, k, e, keys, dist, counts);
    }
    size_t slots() const override {
        size_t total = 0;
        for (size_t g = 0; g < vsg_sharded_shard_count(h); ++g) {
            size_t s = 0;
            if (vsg_index_graph_info(vsg_sharded_shard(h, g), &s, nullptr, nullptr, nullptr, nullptr) != VSG_OK)
                return size();
            total += s;
        }
        return total;
    }
    int compact(size_t* dropped) override { return vsg_sharded_compact(h, dropped); }
    const char* last_error() const override { return vsg_last_error(); }
};

vsg::ActorConfig actor_config(const vsg_actor_options_t* o) {
    vsg::ActorConfig cfg;
    if (o->reserve_increment) cfg.reserve_increment = o->reserve_increment;
    cfg.reserve_threshold = o->reserve_threshold ? o->reserve_threshold : cfg.reserve_increment / 3;
    if (o->max_batch) cfg.max_batch = o->max_batch;
    cfg.max_wait_us = o->max_wait_us;
    if (o->compact_percent) cfg.compact_percent = o->compact_percent;  // 0 => never (vsg.h)
    if (o->compact_min_dead) cfg.compact_min_dead = o->compact_min_dead;
    cfg.concurrent_reads = o->concurrent_reads;  // 0, 1, or n read workers (capped at 8)
    // keys per re-link chunk of a replace run (probes; 0 = the index default)
    if (const char* e = std::getenv("VSG_ACTOR_REPLACE_BATCH")) cfg.replace_batch = std::strtoull(e, nullptr, 10);
    // how long a held chunk tail waits for more writes (tests, probes)
    if (const char* e = std::getenv("VSG_ACTOR_HOLD_US")) cfg.hold_us = (uint32_t)std::strtoul(e, nullptr, 10);
    return cfg;
}

}  // namespace

struct vsg_actor {
    vsg_index_t* index = nullptr;      // borrowed view; owned by the backend
    vsg_sharded_t* sharded = nullptr;  // borrowed view (sharded actor)
    vsg::Actor* actor = nullptr;
};

extern "C" {

int vsg_actor_new(const vsg_actor_options_t* o, vsg_actor_t** out) {
    VSG_RANGE();
    if (!o || !out) return actor_fail(VSG_EINVAL, "null argument");
    *out = nullptr;
    vsg_index_t* h = nullptr;
    int rc = vsg_index_new(&o->index, &h);
    if (rc) return actor_fail(rc, vsg_last_error());
    const vsg::ActorConfig cfg = actor_config(o);
    const size_t ef = o->index.expansion_search ? o->index.expansion_search : 64;
    auto* a = new vsg_actor;
    a->index = h;
    a->actor = new vsg::Actor(std::make_unique<IndexBackend>(h, ef), cfg);
    rc = a->actor->init();
    if (rc) {
        std::string msg = vsg_last_error();
        delete a->actor;
        delete a;
        return actor_fail(rc, "reserve: " + msg);
    }
    *out = a;
    return VSG_OK;
}

int vsg_actor_new_sharded(const vsg_actor_options_t* o, uint32_t n_shards, const int32_t* devices,
                          vsg_actor_t** out) {
    VSG_RANGE();
    if (!o || !out) return actor_fail(VSG_EINVAL, "null argument");
    *out = nullptr;
    vsg_sharded_options_t so{};
    so.index = o->index;
    so.n_shards = n_shards;
    so.answer_device = -1;
    so.devices = devices;
    vsg_sharded_t* h = nullptr;
    int rc = vsg_sharded_new(&so, &h);
    if (rc) return actor_fail(rc, vsg_last_error());
    const size_t ef = o->index.expansion_search ? o->index.expansion_search : 64;
    auto* a = new vsg_actor;
    a->sharded = h;
    a->index = vsg_sharded_shard(h, 0);
    a->actor = new vsg::Actor(std::make_unique<ShardedBackend>(h, ef), actor_config(o));
    rc = a->actor->init();
    if (rc) {
        std::string msg = vsg_last_error();
        delete a->actor;
        delete a;
        return actor_fail(rc, "reserve: " + msg);
    }
    *out = a;
    return VSG_OK;
}

vsg_sharded_t* vsg_actor_sharded(vsg_actor_t* a) { return a ? a->sharded : nullptr; }

void vsg_actor_free(vsg_actor_t* a) {
    VSG_RANGE();
    if (!a) return;
    delete a->actor;  // drains the queue, joins the worker, frees the index
    delete a;
}

int vsg_actor_add_or_replace(vsg_actor_t* a, uint64_t key, const float* embedding, size_t dims) {
    if (!a || !embedding) return actor_fail(VSG_EINVAL, "null argument");
    if (dims != a->actor->dimensions())
        return actor_fail(VSG_EINVAL, "add_or_replace: wrong embedding dimensions: " + std::to_string(dims) +
                                          " != " + std::to_string(a->actor->dimensions()));
    if (key >= UINT64_MAX - 1) return actor_fail(VSG_EINVAL, "add_or_replace: reserved key");
    a->actor->add_or_replace(key, embedding);
    return VSG_OK;
}

int vsg_actor_add_or_replace_cb(vsg_actor_t* a, uint64_t key, const float* embedding, size_t dims,
                                vsg_add_done_fn done, void* ctx) {
    if (!a || !embedding) return actor_fail(VSG_EINVAL, "null argument");
    if (dims != a->actor->dimensions())
        return actor_fail(VSG_EINVAL, "add_or_replace: wrong embedding dimensions: " + std::to_string(dims) +
                                          " != " + std::to_string(a->actor->dimensions()));
    if (key >= UINT64_MAX - 1) return actor_fail(VSG_EINVAL, "add_or_replace: reserved key");
    a->actor->add_or_replace(key, embedding, done, ctx);
    return VSG_OK;
}

size_t vsg_actor_size(const vsg_actor_t* a) { return a ? a->actor->size_now() : 0; }

int vsg_actor_remove(vsg_actor_t* a, uint64_t key) {
    if (!a) return actor_fail(VSG_EINVAL, "null argument");
    a->actor->remove(key);
    return VSG_OK;
}

int vsg_actor_ann(vsg_actor_t* a, const float* embedding, size_t dims, size_t limit, uint64_t* out_keys,
                  float* out_distances, size_t* out_count) {
    VSG_RANGE();
    if (!a || (!embedding && dims) || !out_keys || !out_distances) return actor_fail(VSG_EINVAL, "null argument");
    // usearch.rs:259-272
    if (dims == 0) return actor_fail(VSG_EINVAL, "ann: embedding dimensions == 0");
    if (dims != a->actor->dimensions())
        return actor_fail(VSG_EINVAL, "ann: wrong embedding dimensions: " + std::to_string(dims) +
                                          " != " + std::to_string(a->actor->dimensions()));
    if (limit == 0) return actor_fail(VSG_EINVAL, "ann: limit must be >= 1");
    std::string err;
    const int rc = a->actor->ann(embedding, dims, limit, out_keys, out_distances, out_count, &err);
    if (rc) return actor_fail(rc, "ann: search failed: " + err);
    return VSG_OK;
}

int vsg_actor_ann_cb(vsg_actor_t* a, const float* embedding, size_t dims, size_t limit, uint64_t* out_keys,
                     float* out_distances, vsg_ann_done_fn done, void* ctx) {
    VSG_RANGE();
    if (!a || (!embedding && dims) || !out_keys || !out_distances || !done)
        return actor_fail(VSG_EINVAL, "null argument");
    // usearch.rs:259-272, checked before the message is queued
    if (dims == 0) return actor_fail(VSG_EINVAL, "ann: embedding dimensions == 0");
    if (dims != a->actor->dimensions())
        return actor_fail(VSG_EINVAL, "ann: wrong embedding dimensions: " + std::to_string(dims) +
                                          " != " + std::to_string(a->actor->dimensions()));
    if (limit == 0) return actor_fail(VSG_EINVAL, "ann: limit must be >= 1");
    return a->actor->ann_cb(embedding, dims, limit, out_keys, out_distances, done, ctx) ? VSG_EINVAL : VSG_OK;
}

int vsg_actor_count(vsg_actor_t* a, size_t* out) {
    VSG_RANGE();
    if (!a || !out) return actor_fail(VSG_EINVAL, "null argument");
    return a->actor->count(out);
}

int vsg_actor_flush(vsg_actor_t* a) {
    VSG_RANGE();
    if (!a) return actor_fail(VSG_EINVAL, "null argument");
    return a->actor->flush();
}

int vsg_actor_counters(const vsg_actor_t* a, vsg_actor_counters_t* out) {
    if (!a || !out) return actor_fail(VSG_EINVAL, "null argument");
    const vsg::ActorCounters c = a->actor->counters();
    out->messages = c.messages;
    out->writes = c.writes;
    out->anns = c.anns;
    out->counts = c.counts;
    out->add_calls = c.add_calls;
    out->remove_calls = c.remove_calls;
    out->search_calls = c.search_calls;
    out->reserve_calls = c.reserve_calls;
    out->add_errors = c.add_errors;
    out->remove_errors = c.remove_errors;
    out->search_errors = c.search_errors;
    out->max_search_batch = c.max_search_batch;
    out->max_add_batch = c.max_add_batch;
    out->compactions = c.compactions;
    out->compacted_rows = c.compacted_rows;
    out->compact_errors = c.compact_errors;
    out->ann_queue_ns = c.ann_queue_ns;
    out->ann_wake_ns = c.ann_wake_ns;
    out->batch_search_ns = c.batch_search_ns;
    out->batch_notify_ns = c.batch_notify_ns;
    return VSG_OK;
}

vsg_index_t* vsg_actor_index(vsg_actor_t* a) { return a ? a->index : nullptr; }

}  // extern "C"
