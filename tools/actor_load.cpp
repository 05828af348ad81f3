// actor_load — serving-path load generator for the coalescing actor
// (include/vsg.h "Actor").  C clients (std::thread) issue blocking
// single-query vsg_actor_ann calls, like the reference's per-request
// Index::Ann messages (src/index/usearch.rs:251-306); reports QPS, latency
// percentiles, how the worker batched them, and the same queries as one
// batched vsg_index_search for comparison.
//
// build: make -C tools actor_load   (links ../vector-store-text_amd/lib/libvsg.so)
// usage: actor_load rows dim metric(0 l2sq,1 ip,2 cos) clients queries_per_client k ef [max_wait_us]
//        [read_workers: 0 = anns on the one FIFO worker; n = concurrent_reads n]
//        [mode: 0 = one OS thread per client blocked in vsg_actor_ann; 1 = clients as
//         completions (vsg_actor_ann_cb, the reference's oneshot reply): each finished
//         query submits that client's next one from its callback -- no thread per client]
//        [seed: the index's level seed (bench.py passes its own, so the graph is the
//         headline index's)] [max_batch: anns per worker drain, 0 = the actor default]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../include/vsg.h"

#define TRY(x)                                                                    \
    do {                                                                          \
        int rc__ = (x);                                                           \
        if (rc__) {                                                               \
            std::fprintf(stderr, "%s failed: %d %s\n", #x, rc__, vsg_last_error()); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
    if (argc < 8) {
        std::fprintf(stderr, "usage: %s rows dim metric clients qpc k ef [max_wait_us] [read_workers]\n", argv[0]);
        return 2;
    }
    const size_t rows = std::strtoull(argv[1], nullptr, 10), dim = std::strtoull(argv[2], nullptr, 10);
    const unsigned metric = (unsigned)std::atoi(argv[3]);
    const int clients = std::atoi(argv[4]), qpc = std::atoi(argv[5]);
    const size_t k = std::strtoull(argv[6], nullptr, 10), ef = std::strtoull(argv[7], nullptr, 10);
    const unsigned wait_us = argc > 8 ? (unsigned)std::atoi(argv[8]) : 0;
    const unsigned readers = argc > 9 ? (unsigned)std::atoi(argv[9]) : 0;
    const int mode = argc > 10 ? std::atoi(argv[10]) : 0;
    const uint64_t index_seed = argc > 11 ? std::strtoull(argv[11], nullptr, 0) : 1;
    const unsigned max_batch = argc > 12 ? (unsigned)std::atoi(argv[12]) : 0;
    const uint64_t cfg = 2, base_seed = 0x5EED0000 + cfg, q_seed = 0x5EED1000 + cfg, m_seed = 0x5EED2000 + cfg;

    vsg_actor_options_t o{};
    o.index.dimensions = (uint32_t)dim;
    o.index.metric = metric;
    o.index.connectivity = 16;
    o.index.expansion_add = 128;
    o.index.expansion_search = (uint32_t)ef;
    o.index.seed = index_seed;
    o.max_wait_us = wait_us;
    o.max_batch = max_batch;
    o.concurrent_reads = readers;
    vsg_actor_t* a = nullptr;
    TRY(vsg_actor_new(&o, &a));
    vsg_index_t* h = vsg_actor_index(a);

    // base rows straight into the actor's index (setup, not the measured path)
    float* d_x = nullptr;
    if (hipMalloc(&d_x, rows * dim * 4) != hipSuccess) return 1;
    TRY(vsg_datagen_device(0, rows, dim, base_seed, m_seed, 0, d_x, nullptr));
    std::vector<uint64_t> keys(rows);
    for (size_t i = 0; i < rows; ++i) keys[i] = i;
    TRY(vsg_index_add_device(h, keys.data(), d_x, rows, nullptr));
    (void)hipDeviceSynchronize();
    (void)hipFree(d_x);

    const size_t nq = (size_t)clients * qpc;
    float* d_q = nullptr;
    if (hipMalloc(&d_q, nq * dim * 4) != hipSuccess) return 1;
    TRY(vsg_datagen_device(0, nq, dim, q_seed, m_seed, 0, d_q, nullptr));
    std::vector<float> q(nq * dim);
    (void)hipMemcpy(q.data(), d_q, nq * dim * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_q);

    // batched reference: all queries in one call
    std::vector<uint64_t> bk(nq * k);
    std::vector<float> bd(nq * k);
    std::vector<size_t> bc(nq);
    TRY(vsg_index_search(h, q.data(), nq, k, ef, bk.data(), bd.data(), bc.data()));  // warm
    std::vector<uint64_t> bk1 = bk;
    auto t0 = clk::now();
    TRY(vsg_index_search(h, q.data(), nq, k, ef, bk.data(), bd.data(), bc.data()));
    const double batched_s = std::chrono::duration<double>(clk::now() - t0).count();

    vsg_actor_counters_t c0{};
    vsg_actor_counters(a, &c0);
    vsg_stats_t s0{};
    vsg_index_stats(h, &s0);
    std::vector<double> lat(nq);
    std::vector<uint64_t> ak(nq * k);
    std::atomic<int> mismatch{0}, errors{0};
    auto client = [&](int t) {
        std::vector<uint64_t> ok(k);
        std::vector<float> od(k);
        for (int i = 0; i < qpc; ++i) {
            const size_t qi = (size_t)i * clients + t;
            size_t cnt = 0;
            auto s = clk::now();
            if (vsg_actor_ann(a, &q[qi * dim], dim, k, ok.data(), od.data(), &cnt)) {
                errors++;
                continue;
            }
            lat[qi] = std::chrono::duration<double, std::micro>(clk::now() - s).count();
            std::copy(ok.begin(), ok.end(), ak.begin() + qi * k);
            for (size_t j = 0; j < k; ++j)
                if (ok[j] != bk[qi * k + j] || od[j] != bd[qi * k + j]) {
                    if (mismatch++ < 3)
                        std::fprintf(stderr, "mismatch q%zu j%zu cnt %zu: %llu %.9g vs batched %llu %.9g\n", qi, j,
                                     cnt, (unsigned long long)ok[j], od[j], (unsigned long long)bk[qi * k + j],
                                     bd[qi * k + j]);
                    break;
                }
        }
    };
    // callback clients: client t's i-th query is qi = i * clients + t, submitted from the
    // completion of its (i-1)-th; outputs per client, checked in the completion
    struct CbClient {
        void* owner = nullptr;  // the CbRun
        int t = 0, i = 0;
        clk::time_point s;
        std::vector<uint64_t> ok;
        std::vector<float> od;
    };
    struct CbRun {
        vsg_actor_t* a;
        const float* q;
        size_t dim, k;
        int clients, qpc;
        std::vector<CbClient> cl;
        std::vector<double>* lat;
        std::vector<uint64_t>* ak;
        const std::vector<uint64_t>* bk;
        const std::vector<float>* bd;
        std::atomic<int>* mismatch;
        std::atomic<int>* errors;
        std::atomic<size_t> finished{0};
        std::mutex m;
        std::condition_variable cv;
    } run{a, q.data(), dim, k, clients, qpc, {}, &lat, &ak, &bk, &bd, &mismatch, &errors};
    struct Cb {
        static int submit(CbRun* r, CbClient* c) {
            const size_t qi = (size_t)c->i * r->clients + c->t;
            c->s = clk::now();
            return vsg_actor_ann_cb(r->a, r->q + qi * r->dim, r->dim, r->k, c->ok.data(), c->od.data(), done,
                                    (void*)c);
        }
        static void done(void* ctx, int status, size_t) {
            CbClient* c = static_cast<CbClient*>(ctx);
            CbRun* r = static_cast<CbRun*>(c->owner);
            const size_t qi = (size_t)c->i * r->clients + c->t;
            if (status) {
                (*r->errors)++;
            } else {
                (*r->lat)[qi] = std::chrono::duration<double, std::micro>(clk::now() - c->s).count();
                std::copy(c->ok.begin(), c->ok.end(), r->ak->begin() + qi * r->k);
                for (size_t j = 0; j < r->k; ++j)
                    if (c->ok[j] != (*r->bk)[qi * r->k + j] || c->od[j] != (*r->bd)[qi * r->k + j]) {
                        (*r->mismatch)++;
                        break;
                    }
            }
            if (++c->i < r->qpc && submit(r, c) == VSG_OK) return;
            if (c->i < r->qpc) (*r->errors)++;
            if (++r->finished == (size_t)r->clients) {
                std::lock_guard<std::mutex> lk(r->m);
                r->cv.notify_all();
            }
        }
    };
    std::vector<std::thread> th;
    t0 = clk::now();
    if (mode == 1) {
        run.cl.resize(clients);
        for (int t = 0; t < clients; ++t) {
            run.cl[t].owner = &run;
            run.cl[t].t = t;
            run.cl[t].ok.assign(k, 0);
            run.cl[t].od.assign(k, 0.f);
        }
        for (int t = 0; t < clients; ++t) TRY(Cb::submit(&run, &run.cl[t]));
        std::unique_lock<std::mutex> lk(run.m);
        run.cv.wait(lk, [&] { return run.finished.load() == (size_t)clients; });
    } else {
        for (int t = 0; t < clients; ++t) th.emplace_back(client, t);
        for (auto& x : th) x.join();
    }
    const double served_s = std::chrono::duration<double>(clk::now() - t0).count();
    vsg_actor_counters_t c1{};
    vsg_actor_counters(a, &c1);
    vsg_stats_t s1{};
    vsg_index_stats(h, &s1);
    // diagnostics: does the batched answer itself drift after the load?
    {
        std::vector<uint64_t> bk2(nq * k);
        std::vector<float> bd2(nq * k);
        TRY(vsg_index_search(h, q.data(), nq, k, ef, bk2.data(), bd2.data(), bc.data()));
        size_t d1 = 0, d2 = 0, first = nq;
        for (size_t i = 0; i < nq; ++i) {
            bool x = false, y = false;
            for (size_t j = 0; j < k; ++j) {
                x |= bk2[i * k + j] != bk[i * k + j];
                y |= bk2[i * k + j] != ak[i * k + j];
            }
            d1 += x;
            d2 += y;
            if (x && first == nq) first = i;
        }
        size_t d0 = 0, f0 = nq;
        for (size_t i = 0; i < nq; ++i)
            for (size_t j = 0; j < k; ++j)
                if (bk2[i * k + j] != bk1[i * k + j]) {
                    d0++;
                    if (f0 == nq) f0 = i;
                    break;
                }
        std::fprintf(stderr, "batched-before vs batched-after: %zu rows differ (first %zu); warm call: %zu (first %zu); actor vs after: %zu\n", d1,
                     first, d0, f0, d2);
    }
    std::sort(lat.begin(), lat.end());
    const uint64_t calls = c1.search_calls - c0.search_calls;
    double lat_mean = 0;
    for (double x : lat) lat_mean += x;
    lat_mean /= (double)nq;
    // where an ann's time goes (us): per ann, queueing before its batch starts and the
    // wake-up after its completion; per batch, the search call (host staging + H2D +
    // kernels + D2H + sync; VSG_PROFILE_HOST_SEARCH=1 splits the device part) and the
    // copies + completion signals of its anns
    const double na = (double)(c1.anns - c0.anns), nb = (double)std::max<uint64_t>(1, calls);
    const double hs = (double)std::max<uint64_t>(1, s1.host_searches - s0.host_searches);
    std::fprintf(stderr,
                 "{\"breakdown_us\": {\"ann_latency_mean\": %.1f, \"ann_queue_mean\": %.1f, \"ann_wake_mean\": %.1f, "
                 "\"batch_search_mean\": %.1f, \"batch_notify_mean\": %.1f, \"host_search_wall_mean\": %.1f, "
                 "\"h2d_mean\": %.1f, \"device_mean\": %.1f, \"d2h_mean\": %.1f}}\n",
                 lat_mean, (c1.ann_queue_ns - c0.ann_queue_ns) / 1e3 / na, (c1.ann_wake_ns - c0.ann_wake_ns) / 1e3 / na,
                 (c1.batch_search_ns - c0.batch_search_ns) / 1e3 / nb, (c1.batch_notify_ns - c0.batch_notify_ns) / 1e3 / nb,
                 (s1.host_search_ns - s0.host_search_ns) / 1e3 / hs, (s1.host_h2d_ns - s0.host_h2d_ns) / 1e3 / hs,
                 (s1.host_device_ns - s0.host_device_ns) / 1e3 / hs, (s1.host_d2h_ns - s0.host_d2h_ns) / 1e3 / hs);
    std::printf(
        "{\"rows\": %zu, \"dim\": %zu, \"clients\": %d, \"queries\": %zu, \"k\": %zu, \"ef\": %zu, "
        "\"max_wait_us\": %u, \"max_batch\": %u, \"read_workers\": %u, \"clients_as\": \"%s\", \"actor_qps\": %.1f, \"batched_qps\": %.1f, \"lat_us_p50\": %.1f, "
        "\"lat_us_p99\": %.1f, \"search_calls\": %llu, \"mean_batch\": %.1f, \"max_batch\": %llu, "
        "\"mismatch_vs_batched\": %d, \"errors\": %d}\n",
        rows, dim, clients, nq, k, ef, wait_us, max_batch, readers, mode == 1 ? "completions" : "threads", nq / served_s, nq / batched_s, lat[nq / 2], lat[nq * 99 / 100],
        (unsigned long long)calls, calls ? (double)nq / calls : 0.0, (unsigned long long)c1.max_search_batch,
        mismatch.load(), errors.load());
    vsg_actor_free(a);
    return mismatch || errors ? 1 : 0;
}
