// actor.hpp — the index actor of src/index/usearch.rs restated for a GPU
// backend: one worker thread per index drains a FIFO of messages and turns
// runs of single-vector / single-query messages into batched GPU calls
// (SURVEY §8f row 1).  Header-only and HIP-free so the host logic is tested
// with g++ against a mock backend (tests/cpp/test_actor.cpp).
//
// Reference behaviour mirrored (src/index/usearch.rs):
//   * Index::{AddOrReplace, Remove, Ann, Count} messages          :141-172
//   * capacity growth: free < RESERVE_THRESHOLD => reserve(capacity +
//     RESERVE_INCREMENT), 1M / 333,333 by default                 :61-66, :200-212
//   * replace = remove the live key, then add                      :214-221
//   * add/remove failures are swallowed (counted here, logged there) :207-224, :246
//   * ann dimension checks before any search                       :259-272
//   * count = live size                                            :308-311
// Ordering, default: stronger than the reference's (which spawns every message
// as its own task): messages are applied in submission order, so an Ann sees
// every write submitted before it.  With concurrent_reads = n, Anns go to n read
// workers that search while the writer builds (the reference's behaviour:
// add is fire-and-forget on rayon, search runs beside it under the shared lock,
// usearch.rs:200-221, :274-277): an Ann then sees a prefix of the writes, and a
// burst of inserts no longer delays queries by the whole batched build.  n >= 2
// keeps n search batches in flight, so one batch's GPU tail overlaps the next.
// Batching never changes a result: an Ann run is split by effective ef =
// max(ef, k) and a query's top-k is the prefix of its group's top-kmax (the
// search returns the first k live entries of its list).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace vsg {

// What the actor needs from an index shard (implemented over vsg_index_t in
// vsg_actor.cpp, and by a mock in the tests).  Return codes follow vsg.h.
struct ActorBackend {
    virtual ~ActorBackend() = default;
    virtual size_t dimensions() const = 0;
    virtual size_t size() const = 0;
    virtual size_t capacity() const = 0;
    virtual size_t expansion_search() const = 0;
    virtual bool contains(uint64_t key) const = 0;
    virtual int reserve(size_t capacity) = 0;
    virtual int add(const uint64_t* keys, const float* vecs, size_t n) = 0;
    virtual int remove(const uint64_t* keys, size_t n, size_t* removed) = 0;
    // AddOrReplace messages in order (usearch.rs:214-221: per key, remove the live
    // copy, then add; vsg_index_replace): status[i] per key, kHeld for a key left
    // unapplied when hold_tail is set (an incomplete last chunk, re-submitted by the
    // actor ahead of the next messages).  This default applies them one at a time
    // and never holds (the mocks of tests/cpp); the GPU backends batch them.
    static constexpr int kHeld = 6;  // VSG_HELD
    virtual int replace(const uint64_t* keys, const float* vecs, size_t n, size_t batch, bool hold_tail,
                        int* status) {
        (void)batch;
        (void)hold_tail;
        int first = 0;
        const size_t d = dimensions();
        for (size_t i = 0; i < n; ++i) {
            int rc = 0;
            if (contains(keys[i])) rc = remove(keys + i, 1, nullptr);
            if (rc == 0) rc = add(keys + i, vecs + i * d, 1);
            status[i] = rc;
            if (rc && !first) first = rc;
        }
        return first;
    }
    // the worker restores a captured error message before each failed ann_cb
    // completion (a completion may run other calls that overwrite the thread's error)
    virtual void set_error(const std::string& msg) { (void)msg; }
    virtual int search(const float* q, size_t nq, size_t k, size_t ef, uint64_t* keys, float* dist,
                       size_t* counts) = 0;
    // the batched search of an Ann run, one pointer per query (the messages' own
    // vectors): a backend that stages queries itself copies each straight to its
    // staging buffer; this default gathers them and calls search()
    virtual int search_gather(const float* const* q, size_t nq, size_t k, size_t ef, uint64_t* keys, float* dist,
                              size_t* counts) {
        const size_t d = dimensions();
        std::vector<float> qs(nq * d);
        for (size_t i = 0; i < nq; ++i) std::memcpy(&qs[i * d], q[i], d * 4);
        return search(qs.data(), nq, k, ef, keys, dist, counts);
    }
    virtual const char* last_error() const { return ""; }
    // stored rows including tombstones, and dropping the tombstones
    virtual size_t slots() const { return size(); }
    virtual int compact(size_t* dropped) {
        if (dropped) *dropped = 0;
        return 0;
    }
};

struct ActorConfig {
    size_t reserve_increment = 1000000;  // RESERVE_INCREMENT, usearch.rs:63
    size_t reserve_threshold = 333333;   // RESERVE_THRESHOLD = increment / 3, :67
    size_t max_batch = 65536;            // messages drained per worker wake-up
    uint32_t max_wait_us = 0;            // optional coalescing window (0: natural batching)
    // compact once tombstones reach this percentage of the stored rows (and at
    // least compact_min_dead rows); >= 100 disables (the default since round 5:
    // a replace's remove frees its slot and the next add re-links it in place,
    // usearch index_dense's free-slot reuse, so an upsert stream no longer grows
    // the index; compaction only returns the slots of net deletes)
    uint32_t compact_percent = 100;
    size_t compact_min_dead = 4096;
    // Anns on their own workers, beside the writes (needs a backend whose search
    // may run concurrently with add/remove, as vsg_index's does): 0 = submission
    // order on the one worker; n >= 1 = n read workers, so up to n search batches
    // are in flight at once (the GPU overlaps one batch's tail with the next,
    // DESIGN.md §3.2); at most 8
    uint32_t concurrent_reads = 0;
    // AddOrReplace runs go to the backend's replace in submission order (the
    // reference's per-message remove + add, usearch.rs:214-221); `replace_batch` =
    // keys per chunk (0: the index defaults, vsg_index_replace).  The chunks follow
    // the keys and the index state, never the drain timing: an incomplete last
    // chunk of a drained run is held back and re-submitted ahead of the next
    // messages, applied at once when a barrier follows it (a Remove, or an Ann /
    // Count / Flush in submission-order mode) and after hold_us without new writes
    // (liveness; the only timing-dependent cut).  Round 5 cut a run into
    // remove-all-then-add-all segments bounded to live / 64 removes at drain
    // boundaries: self-recall 0.983-0.995 against 0.999 for the one-at-a-time
    // sequence.
    size_t replace_batch = 0;
    uint32_t hold_us = 2000;
};

struct ActorCounters {
    uint64_t messages = 0, writes = 0, anns = 0, counts = 0;
    uint64_t add_calls = 0, remove_calls = 0, search_calls = 0, reserve_calls = 0;
    uint64_t add_errors = 0, remove_errors = 0, search_errors = 0;
    uint64_t max_search_batch = 0, max_add_batch = 0;
    uint64_t compactions = 0, compacted_rows = 0, compact_errors = 0;
    // serving-path time breakdown (steady clock, ns), summed: per ann, enqueue ->
    // its batch starts and the waiter's wake-up (finish -> caller running); per
    // search batch, the batched search call and the result copies + wake calls
    uint64_t ann_queue_ns = 0, ann_wake_ns = 0, batch_search_ns = 0, batch_notify_ns = 0;
};

inline uint64_t steady_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

class Actor {
  public:
    enum Kind { ADD, REMOVE, ANN, COUNT, FLUSH };

    // completion of a blocking message (Ann / Count / Flush)
    struct Waiter {
        std::mutex m;
        std::condition_variable cv;
        bool done = false;
        int rc = 0;
        uint64_t* keys = nullptr;
        float* dist = nullptr;
        size_t count = 0;  // Ann: results written; Count: live size
        std::string err;   // backend message when rc != 0
        uint64_t t_fin = 0;  // steady_ns() at finish (wake-up latency)
        void finish(int r) {
            std::lock_guard<std::mutex> lk(m);
            rc = r;
            done = true;
            t_fin = steady_ns();
            cv.notify_all();
        }
        int wait() {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return done; });
            return rc;
        }
    };

    // completion of one AddOrReplace (optional): status of the add that carried it,
    // called on the worker thread (the reference awaits each add, usearch.rs:230-232)
    using AddDone = void (*)(void* ctx, uint64_t key, int status);

    struct Msg {
        Kind kind;
        uint64_t key = 0;
        size_t k = 0;
        uint64_t t_enq = 0;  // steady_ns() at submission
        // ann_cb: outputs and completion (w == nullptr)
        uint64_t* out_keys = nullptr;
        float* out_dist = nullptr;
        void (*ann_done)(void* ctx, int status, size_t count) = nullptr;
        std::vector<float> vec;
        Waiter* w = nullptr;
        AddDone done = nullptr;
        void* done_ctx = nullptr;
    };

    Actor(std::unique_ptr<ActorBackend> be, const ActorConfig& cfg) : be_(std::move(be)), cfg_(cfg) {
        if (cfg_.max_batch == 0) cfg_.max_batch = 1;
        if (cfg_.concurrent_reads > 8) cfg_.concurrent_reads = 8;
        worker_ = std::thread([this] { run(q_, qcv_); });
        for (uint32_t i = 0; i < cfg_.concurrent_reads; ++i) readers_.emplace_back([this] { run(rq_, rcv_); });
    }

    ~Actor() {
        {
            std::lock_guard<std::mutex> lk(qm_);
            stop_ = true;
        }
        qcv_.notify_all();
        rcv_.notify_all();
        worker_.join();
        for (std::thread& t : readers_) t.join();
    }

    // initial reservation, usearch.rs:99
    int init() { return be_->reserve(std::max(be_->capacity(), cfg_.reserve_increment)); }

    size_t dimensions() const { return be_->dimensions(); }

    // Index::AddOrReplace — fire and forget, like the reference's channel send
    void add_or_replace(uint64_t key, const float* vec, AddDone done = nullptr, void* done_ctx = nullptr) {
        Msg m;
        m.kind = ADD;
        m.key = key;
        m.done = done;
        m.done_ctx = done_ctx;
        m.vec.assign(vec, vec + be_->dimensions());
        push(std::move(m));
    }

    // Index::Remove
    void remove(uint64_t key) {
        Msg m;
        m.kind = REMOVE;
        m.key = key;
        push(std::move(m));
    }

    // Index::Ann — blocks until the batched search that contains it finishes.
    // Dimension check first (usearch.rs:259-272); k >= 1 (Limit is NonZero).
    int ann(const float* q, size_t dims, size_t k, uint64_t* keys, float* dist, size_t* count,
            std::string* err = nullptr) {
        if (k == 0 || dims != be_->dimensions()) return 1;  // VSG_EINVAL
        Waiter w;
        w.keys = keys;
        w.dist = dist;
        Msg m;
        m.kind = ANN;
        m.k = k;
        m.vec.assign(q, q + dims);
        m.w = &w;
        push(std::move(m));
        const int rc = w.wait();
        wake_ns_.fetch_add(steady_ns() - w.t_fin, std::memory_order_relaxed);
        if (count) *count = w.count;
        if (err) *err = w.err;
        return rc;
    }

    // Index::Ann with a completion instead of a blocked thread: the C form of the
    // reference's oneshot reply (usearch.rs:251-306: the caller awaits a
    // oneshot::Receiver).  done(ctx, status, count) runs on the worker thread once
    // the batched search carrying this query finished, after keys / dist (limit
    // entries, ascending, padded) were written -- no thread wake-up per query.
    using AnnDone = void (*)(void* ctx, int status, size_t count);
    int ann_cb(const float* q, size_t dims, size_t k, uint64_t* keys, float* dist, AnnDone done, void* ctx) {
        if (k == 0 || dims != be_->dimensions() || !done) return 1;  // VSG_EINVAL
        Msg m;
        m.kind = ANN;
        m.k = k;
        m.vec.assign(q, q + dims);
        m.out_keys = keys;
        m.out_dist = dist;
        m.ann_done = done;
        m.done_ctx = ctx;
        push(std::move(m));
        return 0;
    }

    // Index::Count
    int count(size_t* out) {
        Waiter w;
        Msg m;
        m.kind = COUNT;
        m.w = &w;
        push(std::move(m));
        const int rc = w.wait();
        if (out) *out = w.count;
        return rc;
    }

    // live size now, without waiting for queued writes: the reference's count is a
    // read-lock size() beside its fire-and-forget adds (usearch.rs:308-311)
    size_t size_now() const { return be_->size(); }

    // wait until every message submitted before this call has been applied
    int flush() {
        Waiter w;
        Msg m;
        m.kind = FLUSH;
        m.w = &w;
        push(std::move(m));
        return w.wait();
    }

    ActorCounters counters() const {
        std::lock_guard<std::mutex> lk(cm_);
        ActorCounters c = ctr_;
        c.ann_wake_ns = wake_ns_.load(std::memory_order_relaxed);
        return c;
    }

  private:
    void push(Msg&& m) {
        m.t_enq = steady_ns();
        const bool read = cfg_.concurrent_reads > 0 && m.kind == ANN;
        if (read) inflight_.fetch_add(1, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(qm_);
            (read ? rq_ : q_).push_back(std::move(m));
        }
        (read ? rcv_ : qcv_).notify_one();
    }

    // one worker: the FIFO of writes (and, by default, everything else), or the
    // Ann queue of concurrent_reads; both share qm_
    void run(std::deque<Msg>& q, std::condition_variable& cv) {
        const bool writer = &q == &q_;
        std::vector<Msg> batch;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(qm_);
                if (writer && !held_.empty()) {
                    // a held chunk tail: apply it once the writes pause (liveness)
                    if (!cv.wait_for(lk, std::chrono::microseconds(cfg_.hold_us),
                                     [&] { return stop_ || !q.empty(); })) {
                        lk.unlock();
                        flush_held();
                        continue;
                    }
                } else {
                    cv.wait(lk, [&] { return stop_ || !q.empty(); });
                }
                if (q.empty() && stop_) {
                    lk.unlock();
                    if (writer) flush_held();
                    return;
                }
                size_t cap = cfg_.max_batch;
                if (!writer && cfg_.concurrent_reads >= 2) {
                    // Two or more read workers split the anns in flight evenly, so that as
                    // many search batches overlap on the device: a worker takes its share
                    // -- ceil(anns in flight / workers), in flight = queued or being searched
                    // -- waiting up to the coalescing window (max_wait_us, else 300 us) for
                    // it to be queued.  Closed-loop clients then form one group per worker,
                    // each group's next batch filling while the other groups' run (round 5:
                    // one batch of all the clients at a time, the device idle between them).
                    const size_t readers = cfg_.concurrent_reads;
                    const size_t share = std::max<size_t>(
                        1, (inflight_.load(std::memory_order_relaxed) + readers - 1) / readers);
                    cap = std::min(cap, share);
                    const uint32_t win = cfg_.max_wait_us ? cfg_.max_wait_us : 300;
                    if (q.size() < cap && !stop_)
                        cv.wait_for(lk, std::chrono::microseconds(win), [&] { return stop_ || q.size() >= cap; });
                } else if (cfg_.max_wait_us && q.size() < cfg_.max_batch && !stop_) {
                    cv.wait_for(lk, std::chrono::microseconds(cfg_.max_wait_us),
                                [&] { return stop_ || q.size() >= cfg_.max_batch; });
                }
                const size_t n = std::min(q.size(), cap);
                batch.clear();
                batch.reserve(n);
                for (size_t i = 0; i < n; ++i) {
                    batch.push_back(std::move(q.front()));
                    q.pop_front();
                }
                if (!writer && !q.empty()) cv.notify_one();  // the rest: another read worker
            }
            process(batch, writer);
        }
    }

    void process(std::vector<Msg>& b, bool writer) {
        {
            std::lock_guard<std::mutex> lk(cm_);
            ctr_.messages += b.size();
        }
        size_t i = 0;
        while (i < b.size()) {
            size_t j = i;
            if (b[i].kind == ADD || b[i].kind == REMOVE) {
                while (j < b.size() && (b[j].kind == ADD || b[j].kind == REMOVE)) ++j;
                writes(b, i, j, j == b.size());
                maybe_compact();
            } else if (writer && !held_.empty()) {
                flush_held();  // a barrier: every earlier write applies first
                continue;
            } else if (b[i].kind == ANN) {
                while (j < b.size() && b[j].kind == ANN) ++j;
                anns(b, i, j);
            } else {
                if (b[i].kind == COUNT) {
                    std::lock_guard<std::mutex> lk(cm_);
                    ctr_.counts++;
                }
                b[i].w->count = be_->size();
                b[i].w->finish(0);
                j = i + 1;
            }
            i = j;
        }
    }

    // ---------------------------------------------------------------- writes --
    // A run of AddOrReplace / Remove messages in FIFO order: each maximal run of
    // AddOrReplace messages is one backend replace call (keys may repeat: the
    // backend applies them in order), each run of Removes one remove call.  A held
    // tail (held_) leads the next AddOrReplace run; may_hold: the run ends the
    // drained batch (no barrier after it), so its incomplete last chunk may wait.
    void writes(std::vector<Msg>& b, size_t i0, size_t i1, bool may_hold) {
        {
            std::lock_guard<std::mutex> lk(cm_);
            ctr_.writes += i1 - i0;
        }
        size_t i = i0;
        while (i < i1) {
            size_t j = i;
            if (b[i].kind == REMOVE) {
                flush_held();
                std::vector<uint64_t> keys;
                while (j < i1 && b[j].kind == REMOVE) keys.push_back(b[j++].key);
                size_t removed = 0;
                const int rc = be_->remove(keys.data(), keys.size(), &removed);
                std::lock_guard<std::mutex> lk(cm_);
                ctr_.remove_calls++;
                if (rc) ctr_.remove_errors += keys.size();
            } else {
                while (j < i1 && b[j].kind == ADD) held_.push_back(std::move(b[j++]));
                apply_held(may_hold && j == i1);
            }
            i = j;
        }
    }

    void flush_held() {
        if (!held_.empty()) apply_held(false);
    }

    // one replace call over the held AddOrReplace messages; with hold, the ones the
    // backend left unapplied (status kHeld) stay held, in order
    void apply_held(bool hold) {
        const size_t n = held_.size();
        if (n == 0) return;
        const size_t d = be_->dimensions();
        std::vector<uint64_t> keys(n);
        std::vector<float> vecs(n * d);
        for (size_t t = 0; t < n; ++t) {
            keys[t] = held_[t].key;
            std::memcpy(&vecs[t * d], held_[t].vec.data(), d * 4);
        }
        // usearch.rs:200-212 as if the run's vectors arrived one by one: the last one
        // still finds free >= threshold before its add
        int rc = 0;
        while (rc == 0 && be_->capacity() - be_->size() < cfg_.reserve_threshold + n - 1) {
            rc = be_->reserve(be_->capacity() + cfg_.reserve_increment);
            std::lock_guard<std::mutex> lk(cm_);
            ctr_.reserve_calls++;
        }
        std::vector<int> status(n, rc);
        if (rc == 0) be_->replace(keys.data(), vecs.data(), n, cfg_.replace_batch, hold, status.data());
        size_t bad = 0, applied = 0;
        for (int st : status) {
            bad += st != 0 && st != ActorBackend::kHeld;
            applied += st != ActorBackend::kHeld;
        }
        {
            std::lock_guard<std::mutex> lk(cm_);
            if (applied) ctr_.add_calls++;
            ctr_.max_add_batch = std::max<uint64_t>(ctr_.max_add_batch, applied);
            ctr_.add_errors += bad;
        }
        std::vector<Msg> keep;
        for (size_t t = 0; t < n; ++t) {
            if (status[t] == ActorBackend::kHeld) {
                keep.push_back(std::move(held_[t]));
            } else if (held_[t].done) {
                held_[t].done(held_[t].done_ctx, keys[t], status[t]);
            }
        }
        held_.swap(keep);
    }

    void maybe_compact() {
        if (cfg_.compact_percent >= 100) return;
        const size_t slots = be_->slots(), live = be_->size();
        const size_t dead = slots > live ? slots - live : 0;
        if (dead < cfg_.compact_min_dead || dead * 100 < (size_t)cfg_.compact_percent * slots) return;
        size_t dropped = 0;
        const int rc = be_->compact(&dropped);
        std::lock_guard<std::mutex> lk(cm_);
        ctr_.compactions++;
        ctr_.compacted_rows += dropped;
        if (rc) ctr_.compact_errors++;
    }

    // ------------------------------------------------------------------ anns --
    void anns(std::vector<Msg>& b, size_t i0, size_t i1) {
        const size_t ef0 = be_->expansion_search();
        const uint64_t t0 = steady_ns();
        {
            uint64_t qw = 0;
            for (size_t i = i0; i < i1; ++i) qw += t0 - std::min(t0, b[i].t_enq);
            std::lock_guard<std::mutex> lk(cm_);
            ctr_.anns += i1 - i0;
            ctr_.ann_queue_ns += qw;
        }
        // group by effective ef so batching cannot change any result
        std::unordered_map<size_t, std::vector<size_t>> groups;
        std::vector<size_t> order;
        for (size_t i = i0; i < i1; ++i) {
            const size_t e = std::max(ef0, b[i].k);
            auto it = groups.find(e);
            if (it == groups.end()) {
                order.push_back(e);
                groups[e].push_back(i);
            } else {
                it->second.push_back(i);
            }
        }
        std::vector<const float*> qs;
        std::vector<uint64_t> keys;
        std::vector<float> dist;
        std::vector<size_t> counts;
        for (size_t e : order) {
            const std::vector<size_t>& g = groups[e];
            size_t kmax = 0;
            for (size_t i : g) kmax = std::max(kmax, b[i].k);
            qs.resize(g.size());
            for (size_t r = 0; r < g.size(); ++r) qs[r] = b[g[r]].vec.data();
            keys.resize(g.size() * kmax);
            dist.resize(g.size() * kmax);
            counts.resize(g.size());
            const uint64_t ts = steady_ns();
            const int rc = be_->search_gather(qs.data(), g.size(), kmax, e, keys.data(), dist.data(), counts.data());
            const uint64_t tn = steady_ns();
            {
                std::lock_guard<std::mutex> lk(cm_);
                ctr_.search_calls++;
                ctr_.max_search_batch = std::max<uint64_t>(ctr_.max_search_batch, g.size());
                if (rc) ctr_.search_errors += g.size();
                ctr_.batch_search_ns += tn - ts;
            }
            const std::string err = rc ? be_->last_error() : std::string();
            for (size_t r = 0; r < g.size(); ++r) {
                Msg& m = b[g[r]];
                uint64_t* ok = m.w ? m.w->keys : m.out_keys;
                float* od = m.w ? m.w->dist : m.out_dist;
                size_t c = 0;
                if (rc == 0) {
                    c = std::min(counts[r], m.k);
                    std::memcpy(ok, &keys[r * kmax], c * 8);
                    std::memcpy(od, &dist[r * kmax], c * 4);
                    for (size_t t = c; t < m.k; ++t) {
                        ok[t] = ~0ull;
                        od[t] = __builtin_inff();
                    }
                }
                if (m.w) {  // a blocked caller (ann): wake it
                    if (rc == 0) m.w->count = c;
                    else m.w->err = err;
                    m.w->finish(rc);
                } else {  // ann_cb: the completion runs here, like a oneshot send
                    if (rc) be_->set_error(err);  // an earlier completion may have overwritten it
                    m.ann_done(m.done_ctx, rc, c);
                }
                if (cfg_.concurrent_reads > 0) inflight_.fetch_sub(1, std::memory_order_relaxed);
            }
            const uint64_t dn = steady_ns() - tn;
            std::lock_guard<std::mutex> lk(cm_);
            ctr_.batch_notify_ns += dn;
        }
    }

    std::unique_ptr<ActorBackend> be_;
    ActorConfig cfg_;
    std::mutex qm_;
    std::condition_variable qcv_, rcv_;
    std::deque<Msg> q_, rq_;
    bool stop_ = false;
    mutable std::mutex cm_;
    ActorCounters ctr_;
    std::atomic<uint64_t> wake_ns_{0};  // ann wake-up latency, summed (lock-free: every caller adds)
    std::atomic<size_t> inflight_{0};   // anns on the read queue or in a search (concurrent_reads)
    std::vector<Msg> held_;  // AddOrReplace messages of an incomplete chunk (writer only)
    std::thread worker_;
    std::vector<std::thread> readers_;
};

}  // namespace vsg
