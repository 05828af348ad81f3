// keymap.hpp — host-side key -> slot map of one shard (the u64 side of the
// reference's BiMap<PrimaryKey, Key>, src/index/usearch.rs:109-113).
// Open addressing, linear probing, 12 B per bucket, load <= 1/2, tombstones on
// erase (rebuilt on growth).  ~10x faster and ~3x smaller than std::unordered_map
// at 10^8 keys, which is what bulk loads of C4 (100M rows) need.
#pragma once
#include <stdint.h>

#include <vector>

namespace vsg {

class KeyMap {
  public:
    static constexpr uint64_t EMPTY = ~0ull;        // VSG_NO_KEY is never a valid key
    static constexpr uint64_t DEAD = ~0ull - 1;     // tombstone (key UINT64_MAX-1 rejected too)

    size_t size() const { return live_; }

    // reserved keys (EMPTY, DEAD) are never present: without this check a
    // probe for DEAD would match the first tombstone on its path
    bool find(uint64_t k, uint32_t* v) const {
        if (cap_ == 0 || k >= DEAD) return false;
        for (size_t i = hash(k) & (cap_ - 1);; i = (i + 1) & (cap_ - 1)) {
            if (keys_[i] == EMPTY) return false;
            if (keys_[i] == k) {
                if (v) *v = vals_[i];
                return true;
            }
        }
    }

    // false if k is already present or reserved (nothing changed)
    bool insert(uint64_t k, uint32_t v) {
        if (k >= DEAD) return false;
        if ((used_ + 1) * 2 > cap_) grow();
        size_t tomb = SIZE_MAX;
        for (size_t i = hash(k) & (cap_ - 1);; i = (i + 1) & (cap_ - 1)) {
            if (keys_[i] == k) return false;
            if (keys_[i] == DEAD && tomb == SIZE_MAX) tomb = i;
            if (keys_[i] == EMPTY) {
                const size_t at = tomb != SIZE_MAX ? tomb : i;
                if (at == i) ++used_;
                keys_[at] = k;
                vals_[at] = v;
                ++live_;
                return true;
            }
        }
    }

    bool erase(uint64_t k, uint32_t* v) {
        if (cap_ == 0 || k >= DEAD) return false;
        for (size_t i = hash(k) & (cap_ - 1);; i = (i + 1) & (cap_ - 1)) {
            if (keys_[i] == EMPTY) return false;
            if (keys_[i] == k) {
                if (v) *v = vals_[i];
                keys_[i] = DEAD;
                --live_;
                return true;
            }
        }
    }

    void reserve(size_t n) {
        size_t want = 16;
        while (want < 2 * n + 2) want <<= 1;
        if (want > cap_) rehash(want);
    }

  private:
    static size_t hash(uint64_t x) {
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 33;
        x *= 0xc4ceb9fe1a85ec53ull;
        x ^= x >> 33;
        return (size_t)x;
    }

    void grow() { rehash(cap_ ? (live_ * 2 + 2 > cap_ / 2 ? cap_ * 2 : cap_) : 1024); }

    void rehash(size_t ncap) {
        std::vector<uint64_t> ok(std::move(keys_));
        std::vector<uint32_t> ov(std::move(vals_));
        keys_.assign(ncap, EMPTY);
        vals_.assign(ncap, 0);
        cap_ = ncap;
        used_ = live_ = 0;
        for (size_t i = 0; i < ok.size(); ++i)
            if (ok[i] != EMPTY && ok[i] != DEAD) insert(ok[i], ov[i]);
    }

    std::vector<uint64_t> keys_;
    std::vector<uint32_t> vals_;
    size_t cap_ = 0, used_ = 0, live_ = 0;
};

}  // namespace vsg
