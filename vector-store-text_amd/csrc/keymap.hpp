// keymap.hpp — host-side key -> slot map of one shard (the u64 side of the
// reference's BiMap<PrimaryKey, Key>, src/index/usearch.rs:109-113).
// Open addressing, linear probing, 12 B per bucket, load <= 1/2, tombstones on
// erase (rebuilt on growth).  ~10x faster and ~3x smaller than std::unordered_map
// at 10^8 keys, which is what bulk loads of C4 (100M rows) need.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
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

    // Bulk insert keys[i] -> s0 + i (i < n) with pfor(n, f(lo, hi)) workers:
    // the table is sized first (no resize while they run), then each bucket is
    // claimed with a CAS on EMPTY -- lock-free linear probing; tombstones are not
    // reused here.  All or nothing: on a reserved key, a live duplicate or a
    // duplicate inside the batch every key this call inserted is erased again and
    // false is returned (the caller re-runs insert() serially for its error).
    template <class PF>
    bool insert_all(const uint64_t* keys, size_t n, uint32_t s0, PF&& pfor) {
        if (n == 0) return true;
        if ((used_ + n) * 2 > cap_) {
            size_t want = cap_ ? cap_ : 16;
            while (want < 2 * (live_ + n) + 2) want <<= 1;
            rehash(want);
        }
        uint64_t* kk = keys_.data();
        uint32_t* vv = vals_.data();
        const size_t mask = cap_ - 1;
        std::atomic<bool> ok{true};
        std::atomic<size_t> added{0};
        pfor(n, [&](size_t lo, size_t hi) {
            size_t mine = 0;
            for (size_t i = lo; i < hi && ok.load(std::memory_order_relaxed); ++i) {
                const uint64_t k = keys[i];
                if (k >= DEAD) {
                    ok = false;
                    break;
                }
                for (size_t b = hash(k) & mask;; b = (b + 1) & mask) {
                    uint64_t cur = __atomic_load_n(&kk[b], __ATOMIC_ACQUIRE);
                    if (cur == EMPTY &&
                        __atomic_compare_exchange_n(&kk[b], &cur, k, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                        vv[b] = s0 + (uint32_t)i;
                        ++mine;
                        break;
                    }
                    if (cur == k) {  // live key, or a duplicate claimed by another worker
                        ok = false;
                        break;
                    }
                }
                if (!ok.load(std::memory_order_relaxed)) break;
            }
            added += mine;
        });
        used_ += added;
        live_ += added;
        if (ok) return true;
        for (size_t i = 0; i < n; ++i) {
            uint32_t v;
            if (find(keys[i], &v) && v >= s0 && v - s0 < n) erase(keys[i], nullptr);
        }
        return false;
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
