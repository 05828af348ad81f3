// Randomised differential test of vsg::KeyMap against std::unordered_map.
#include <cstdio>
#include <random>
#include <unordered_map>

#include "../../vector-store-text_amd/csrc/keymap.hpp"

int main() {
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
