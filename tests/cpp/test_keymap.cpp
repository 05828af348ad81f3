// Randomised differential test of vsg::KeyMap against std::unordered_map: the
// serial insert/erase/find path and the multi-threaded bulk insert_all().
#include <cstdio>
#include <functional>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../vector-store-text_amd/csrc/keymap.hpp"

// pfor(n, f(lo, hi)) on 8 threads, as vsg_index.cpp's host_parallel
static void pfor8(size_t n, const std::function<void(size_t, size_t)>& f) {
    std::vector<std::thread> th;
    const size_t step = (n + 7) / 8;
    for (size_t lo = 0; lo < n; lo += step) th.emplace_back([&f, lo, n, step] { f(lo, std::min(n, lo + step)); });
    for (auto& t : th) t.join();
}

// insert_all (the bulk-add path): all or nothing against the serial semantics
static int bulk() {
    std::mt19937_64 rng(11);
    for (int round = 0; round < 40; ++round) {
        vsg::KeyMap m;
        std::unordered_map<uint64_t, uint32_t> ref;
        uint32_t slot = 0;
        for (int call = 0; call < 30; ++call) {
            // erase some live keys first (tombstones on the probe paths)
            for (int e = 0; e < 200 && !ref.empty(); ++e) {
                const uint64_t k = rng() % 400000;
                uint32_t v;
                const bool a = m.erase(k, &v);
                auto f = ref.find(k);
                if (a != (f != ref.end())) { std::printf("bulk erase mismatch\n"); return 1; }
                if (a) ref.erase(f);
            }
            const size_t n = 1 + rng() % 20000;
            std::vector<uint64_t> keys(n);
            for (auto& k : keys) k = rng() % 400000;
            const int kind = (int)(rng() % 4);  // 0: may collide; 1: fresh keys; 2: in-batch dup; 3: reserved
            if (kind >= 1) {
                for (size_t i = 0; i < n; ++i) keys[i] = (1ull << 32) + (uint64_t)call * 100000 + i + round * 10000000ull;
                if (kind == 2) keys[n - 1] = keys[rng() % n];
                if (kind == 3) keys[rng() % n] = vsg::KeyMap::DEAD + rng() % 2;
            }
            bool expect = true;
            {
                std::unordered_map<uint64_t, int> seen;
                for (auto k : keys)
                    if (k >= vsg::KeyMap::DEAD || ref.count(k) || seen[k]++) expect = false;
            }
            const size_t before = m.size();
            const bool got = m.insert_all(keys.data(), n, slot, pfor8);
            if (got != expect || (!got && m.size() != before)) {
                std::printf("insert_all mismatch round %d call %d: got %d expect %d\n", round, call, got, expect);
                return 1;
            }
            if (got) {
                for (size_t i = 0; i < n; ++i) ref.emplace(keys[i], slot + (uint32_t)i);
                slot += (uint32_t)n;
            }
            for (auto& kv : ref) {
                uint32_t v;
                if (!m.find(kv.first, &v) || v != kv.second) { std::printf("bulk find mismatch\n"); return 1; }
            }
            if (m.size() != ref.size()) { std::printf("bulk size mismatch\n"); return 1; }
        }
    }
    return 0;
}

int main() {
    if (bulk()) return 1;
    vsg::KeyMap m;
    std::unordered_map<uint64_t, uint32_t> ref;
    std::mt19937_64 rng(7);
    for (int it = 0; it < 2000000; ++it) {
        const uint64_t k = rng() % 50000 + (it % 3 == 0 ? 0 : (1ull << 40));
        const int op = (int)(rng() % 10);
        if (op < 5) {
            const bool a = m.insert(k, (uint32_t)it);
            const bool b = ref.emplace(k, (uint32_t)it).second;
            if (a != b) { std::printf("insert mismatch %llu\n", (unsigned long long)k); return 1; }
        } else if (op < 8) {
            uint32_t v = 0;
            const bool a = m.erase(k, &v);
            auto f = ref.find(k);
            const bool b = f != ref.end();
            if (a != b || (a && v != f->second)) { std::printf("erase mismatch\n"); return 1; }
            if (b) ref.erase(f);
        } else {
            uint32_t v = 0;
            const bool a = m.find(k, &v);
            auto f = ref.find(k);
            if (a != (f != ref.end()) || (a && v != f->second)) { std::printf("find mismatch\n"); return 1; }
        }
        if (m.size() != ref.size()) { std::printf("size mismatch\n"); return 1; }
    }
    // reserved keys: after ordinary erasures left tombstones on
    // the probe paths, UINT64_MAX-1 / UINT64_MAX are never found, erased or inserted
    for (uint64_t rk : {vsg::KeyMap::DEAD, vsg::KeyMap::EMPTY}) {
        const size_t before = m.size();
        uint32_t v = 0;
        if (m.find(rk, &v) || m.erase(rk, &v) || m.insert(rk, 1) || m.size() != before) {
            std::printf("reserved key %llx accepted\n", (unsigned long long)rk);
            return 1;
        }
    }
    std::printf("ok %zu\n", m.size());
    return 0;
}
