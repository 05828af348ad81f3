// hnsw_regset.hpp — the HNSW beam with its candidate set in VGPRs (used by
// hnsw_search_reg_kernel and by the insert kernel); see hnsw_search_reg.hip
// for the argument that it expands the same nodes as the sorted-list beam.
#pragma once
#include "hnsw_common.hpp"

namespace vsg {

#define VSG_KEY_EMPTY (~0ull)

// compaction may stop at a prefix range instead of the exact keep-th key (probes)
#ifndef VSG_COMPACT_EARLY
#define VSG_COMPACT_EARLY 0
#endif

// (distance, slot) -> key whose unsigned order is cand_less order (-0 == +0).
__device__ __forceinline__ uint64_t cand_key(float d, uint32_t id) {
    uint32_t b = __float_as_uint(d);
    if (b == 0x80000000u) b = 0u;
    const uint32_t u = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return ((uint64_t)u << 32) | (id & VSG_ID_MASK);
}
__device__ __forceinline__ float key_dist(uint64_t k) {
    const uint32_t u = (uint32_t)(k >> 32);
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int o) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
template <int CTRL> __device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}
// Wave minimum, result in every lane.  A minimum is exact in any order, so the
// 16-lane rows reduce with DPP moves (quad xor 1 / 2, half-row and row mirrors:
// every lane of a row then holds the row's minimum) and the four rows meet in
// scalar registers -- no ds_bpermute round trips (12 of them in the xor
// butterfly of two 32-bit halves).
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#if VSG_DPP_REDUCE
    uint64_t w;
    w = dpp64<0xB1>(v);
    v = w < v ? w : v;
    w = dpp64<0x4E>(v);
    v = w < v ? w : v;
    w = dpp64<0x141>(v);
    v = w < v ? w : v;
    w = dpp64<0x140>(v);
    v = w < v ? w : v;
    const uint64_t r0 = readlane64(v, 0), r1 = readlane64(v, 16), r2 = readlane64(v, 32), r3 = readlane64(v, 48);
    const uint64_t a = r0 < r1 ? r0 : r1, b = r2 < r3 ? r2 : r3;
    return a < b ? a : b;
#else
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = shfl_xor64(v, o);
        v = w < v ? w : v;
    }
    return v;
#endif
}

template <int R> struct RegSet {
    uint64_t k[R];   // slot r of this lane; VSG_KEY_EMPTY = free
    uint32_t expm;   // bit r: slot r expanded
    int size;        // occupied slots (wave-uniform)
    uint64_t tkey;   // admission bound (wave-uniform)

    __device__ __forceinline__ void init(uint64_t first) {
#pragma unroll
        for (int r = 0; r < R; ++r) k[r] = VSG_KEY_EMPTY;
        if (lane_id() == 0) k[0] = first;
        expm = 0;
        size = 1;
        tkey = VSG_KEY_EMPTY;
    }

    // smallest unexpanded key (VSG_KEY_EMPTY if none)
    __device__ __forceinline__ uint64_t min_unexpanded() const {
        uint64_t b = VSG_KEY_EMPTY;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (!((expm >> r) & 1u) && k[r] < b) b = k[r];
        return wave_min64(b);
    }

    // #keys below x (wave-uniform)
    __device__ __forceinline__ int count_below(uint64_t x) const {
        int c = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) c += popc64(__ballot(k[r] < x));
        return c;
    }

    __device__ __forceinline__ void mark_expanded(uint64_t x) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (k[r] == x) expm |= 1u << r;
    }

    __device__ __forceinline__ bool contains(uint64_t x) const {
        bool h = false;
#pragma unroll
        for (int r = 0; r < R; ++r) h = h || k[r] == x;
        return __ballot(h) != 0;
    }

    // keep the `keep` smallest keys (size > keep); tkey = the largest kept.
    // MSB-first radix select on the distance word: bit b of the answer is 0
    // iff at least `need` keys share its higher bits and have 0 there.  The
    // slot word is only selected on when several kept candidates tie on the
    // cut distance (then `need` < their count).
    // excl (filtered search): slots whose keys are not counted -- removed nodes;
    // the cut is then the keep-th smallest counted key, every key above it (of
    // either kind) is dropped, and the size is recounted.
    __device__ __forceinline__ void compact(int keep, uint32_t excl = 0) {
        uint32_t ph = 0;
        int need = keep;
#if VSG_COMPACT_EARLY
        // Any cut at or above the keep-th key keeps B a superset of the top
        // `keep` (the traversal only needs that), so the select may stop at the
        // first prefix range whose keys, with every key below it, fit in half
        // the slack between `keep` and 64 (R - 1) (room for one more expansion):
        // fewer ballot passes, and the next compaction is not much earlier.
        int rsize = size;  // keys in the current prefix range (bits above b fixed)
        const int cap = keep + (64 * (R - 1) - keep) / 2;
#endif
#pragma unroll 1
        for (int b = 31; b >= 0; --b) {
            const uint32_t hm = b == 31 ? 0u : (~0u << (b + 1));
            int c = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t hi = (uint32_t)(k[r] >> 32);
                c += popc64(__ballot(k[r] != VSG_KEY_EMPTY && !((excl >> r) & 1u) && (hi & hm) == ph && !((hi >> b) & 1u)));
            }
            if (c < need) {
                need -= c;
                ph |= 1u << b;
#if VSG_COMPACT_EARLY
                rsize -= c;
#endif
            }
#if VSG_COMPACT_EARLY
            else {
                rsize = c;
            }
            const int kept = keep - need + rsize;  // keys below the range + the range
            if (b > 0 && kept <= cap) {
                const uint64_t cut = ((uint64_t)(ph | ((1u << b) - 1u)) << 32) | 0xFFFFFFFFull;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (k[r] > cut) {
                        k[r] = VSG_KEY_EMPTY;
                        expm &= ~(1u << r);
                    }
                size = kept;
                tkey = cut;
                return;
            }
#endif
        }
        int ceq = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            ceq += popc64(__ballot(k[r] != VSG_KEY_EMPTY && !((excl >> r) & 1u) && (uint32_t)(k[r] >> 32) == ph));
        uint64_t cut;
        if (need == ceq) {
            // every key on the cut distance stays: the cut is the largest of them
            uint64_t mx = 0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (k[r] != VSG_KEY_EMPTY && !((excl >> r) & 1u) && (uint32_t)(k[r] >> 32) == ph && k[r] > mx) mx = k[r];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const uint64_t w = shfl_xor64(mx, o);
                mx = w > mx ? w : mx;
            }
            cut = mx;
        } else {
            uint32_t pl = 0;
#pragma unroll 1
            for (int b = 31; b >= 0; --b) {
                const uint32_t hm = b == 31 ? 0u : (~0u << (b + 1));
                int c = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t lo = (uint32_t)k[r];
                    c += popc64(__ballot(k[r] != VSG_KEY_EMPTY && !((excl >> r) & 1u) && (uint32_t)(k[r] >> 32) == ph &&
                                         (lo & hm) == pl && !((lo >> b) & 1u)));
                }
                if (c < need) {
                    need -= c;
                    pl |= 1u << b;
                }
            }
            cut = ((uint64_t)ph << 32) | pl;
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (k[r] > cut) {
                k[r] = VSG_KEY_EMPTY;
                expm &= ~(1u << r);
            }
        if (excl) {
            int c = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) c += popc64(__ballot(k[r] != VSG_KEY_EMPTY));
            size = c;
        } else {
            size = keep;
        }
        tkey = cut;
    }

    // place the nc staged keys sk[0..nc) into free slots
    __device__ __forceinline__ void fill(const uint64_t* sk, int nc) {
        int acc = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (acc < nc) {
                const bool fr = k[r] == VSG_KEY_EMPTY;
                const uint64_t em = __ballot(fr);
                const int idx = acc + lanes_below(em);
                if (fr && idx < nc) {
                    k[r] = sk[idx];
                    expm &= ~(1u << r);
                }
                acc += popc64(em);
            }
        }
        size += nc;
    }
};

// Admit this lane's candidate key `ck` if `mine` (one expansion's batch).
// pf: compaction cycles (the make prof build only).
template <int R>
__device__ __forceinline__ void admit(RegSet<R>& B, bool mine, uint64_t ck, bool lossy, int ef, uint64_t* sk,
                                      BeamProf* pf = nullptr) {
    (void)pf;
    const int lane = lane_id();
    bool valid = mine && ck < B.tkey;
    uint64_t vm = __ballot(valid);
    if (lossy && vm) {
        // a forgotten id evaluated again: drop it if B still holds it
        for (uint64_t mm = vm; mm; mm &= mm - 1) {
            const int j = __builtin_ctzll(mm);
            if (B.contains(readlane64(ck, j))) vm &= ~(1ull << j);
        }
        valid = (vm >> lane) & 1ull;
    }
    int nc = popc64(vm);
    if (nc && B.size + nc > 64 * R) {
#ifdef VSG_SEARCH_PROFILE
        const uint64_t tc = VSG_CYC();
#endif
        B.compact(ef);
        valid = valid && ck < B.tkey;
        vm = __ballot(valid);
        nc = popc64(vm);
#ifdef VSG_SEARCH_PROFILE
        if (pf) {
            pf->c_comp += VSG_CYC() - tc;
            pf->ncomp++;
        }
#endif
    }
    if (nc) {
        if (valid) sk[lanes_below(vm)] = ck;
        wave_sync();
        B.fill(sk, nc);
        wave_sync();
    }
}

// Beam on level l (oracle beam()).  Preparing the runner-up expansion
// alongside (its adjacency row and distances in the same round trips,
// committed only when it is the sequential next step) was measured 0-15%
// slower: the runner-up is rarely still next (profiles/r01_search_phases.jsonl).
// Prefetching only the runner-up's adjacency row: C4 shard search -8 %, C2
// search +2 %, C2 build -5 % (profiles/r02_search_probes.jsonl) -- not kept.
// Round 6 loaded the row of the exact next expansion (the smallest of B's
// unexpanded keys and this batch's candidates below tkey, known before the
// admit) under the admit and compaction: bit-exact, but no faster at 512 or 10k
// queries (C2 0.523 -> 0.526 ms, 2.954 -> 2.978 ms; C4 shard ef 192 3.08 -> 3.27 ms
// with 12 more VGPRs, profiles/r06_prefetch_ab.jsonl).  The SQ counters of the C4
// shard search say why: waves issue 34 % of their cycles, stall on issue 21 %,
// wait on memory 45 %, and the SIMDs' issue slots are nearly all taken
// (profiles/r06_c4_sq.json) -- latency is hidden by the other resident waves, so a
// shorter chain per wave does not shorten the launch.  Not kept.
// self: the node an insert (re)links, never admitted (VSG_EMPTY in searches).
template <int G, int VM, int U, typename T, int MET, int R>
__device__ __forceinline__ void beam_reg(const GraphDev& g, const QReg<G, VM, T>& q, int l, uint32_t ep, float dep, int ef, WaveLds& w,
                         RegSet<R>& B, uint64_t& ndist, uint64_t& nadj, BeamProf& pf, uint32_t self = VSG_EMPTY) {
    const int lane = lane_id();
    // select on values (readfirstlane), not on field addresses: a
    // select-of-loads folded into a load-of-select pinned the graph
    // descriptor in scratch inside the insert kernel
    const int m0r = __builtin_amdgcn_readfirstlane(g.M0), mr = __builtin_amdgcn_readfirstlane(g.M);
    const int m = l == 0 ? m0r : mr;
    auto rfl_ptr = [](const uint32_t* p) {
        const uint64_t v = (uint64_t)p;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
        return (const uint32_t*)(((uint64_t)hi << 32) | lo);
    };
    const uint32_t* adj0 = rfl_ptr(g.adj0);
    const uint32_t* upper = rfl_ptr(g.upper);
    const uint32_t* upper_off = rfl_ptr(g.upper_off);
    w.vis.clear();
    if (ep != VSG_EMPTY) {
        if (lane == 0) {
            bool unrec;
            w.vis.insert(ep, unrec);
        }
        B.init(cand_key(dep, ep));
    } else {
        // seeded (beam_reg_seeded): B already holds the start set; mark it
        // visited and unexpanded, admission bound open
        wave_sync();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (B.k[r] != VSG_KEY_EMPTY) {
                bool unrec;
                w.vis.insert((uint32_t)B.k[r] & VSG_ID_MASK, unrec);
            }
        B.expm = 0;
        B.tkey = VSG_KEY_EMPTY;
    }
    bool lossy = false;
    uint64_t* sk = reinterpret_cast<uint64_t*>(w.sd);  // sd + si: 64 x 8 B
    wave_sync();
    auto row_of = [&](uint32_t n) {
        return l == 0 ? adj0 + (size_t)n * m0r : upper + ((size_t)upper_off[n] + (size_t)(l - 1)) * mr;
    };
    for (;;) {
        const uint64_t t0 = VSG_CLK();
        [[maybe_unused]] uint64_t c0c = VSG_CYC();
        const uint64_t a = B.min_unexpanded();
        if (a == VSG_KEY_EMPTY) break;
        if (B.size > ef && B.count_below(a) >= ef) break;
        B.mark_expanded(a);
        const uint32_t na = (uint32_t)a & VSG_ID_MASK;
        const uint32_t* row = row_of(na);
        ++nadj;
#ifdef VSG_SEARCH_PROFILE
        {
            const uint64_t c = VSG_CYC();
            pf.c_sel += c - c0c;
            pf.nexp++;
            c0c = c;
        }
#endif
        // one 64-entry piece of the row per pass (M0 = 2M <= 128); the expansion's
        // pieces are admitted one after another, which leaves the same set as one
        // batch (B only ever keeps the best ef of everything evaluated)
        for (int c0 = 0; c0 < m; c0 += 64) {
            const uint32_t nb = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
            const bool full = __ballot(nb != VSG_EMPTY) == ~0ull;
#ifdef VSG_SEARCH_PROFILE
            {
                const uint64_t c = VSG_CYC();
                pf.c_adj += c - c0c;
                c0c = c;
            }
#endif
            bool fresh = false, evicted = false;
            if (nb != VSG_EMPTY && nb != self) fresh = w.vis.insert(nb, evicted);
            const uint64_t mask = __ballot(fresh);
            lossy = lossy || __ballot(evicted) != 0;
            const int cnt = popc64(mask);
            if (fresh) w.todo[lanes_below(mask)] = nb;
            wave_sync();
            const uint64_t t1 = VSG_CLK();
            pf.adj += t1 - t0;
#ifdef VSG_SEARCH_PROFILE
            {
                const uint64_t c = VSG_CYC();
                pf.c_vis += c - c0c;
                c0c = c;
            }
#endif
            if (cnt) {
#ifdef VSG_SEARCH_PROFILE
                rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist, &pf.rows);
#else
                rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
#endif
                wave_sync();
                ndist += (uint64_t)cnt;
                const uint64_t ck = lane < cnt ? cand_key(w.tdist[lane], w.todo[lane]) : VSG_KEY_EMPTY;
                const uint64_t t2 = VSG_CLK();
                pf.dist += t2 - t1;
#ifdef VSG_SEARCH_PROFILE
                const uint64_t ca = VSG_CYC();
                admit<R>(B, lane < cnt, ck, lossy, ef, sk, &pf);
                c0c = VSG_CYC();
                pf.c_admit += c0c - ca;
#else
                admit<R>(B, lane < cnt, ck, lossy, ef, sk);
#endif
                pf.merge += VSG_CLK() - t2;
            }
            if (!full) break;  // compact prefix: the row ended inside this piece
        }
    }
}


// ------------------------------------------------ filtered base-level search --
// usearch's base-level search of an index holding removed entries
// (search_to_find_in_base_ with index_dense's `allow` predicate, restated in
// oracle beam_filtered()): every admitted candidate joins `next` and is
// expanded in key order, removed or not; only live ones join `top`, the best ef
// admitted live keys; radius = worst key of `top` (the start's key while `top`
// is empty); a candidate is admitted when |top| < ef or below the radius; the
// traversal stops when the nearest unexpanded candidate is beyond the radius.
//
// In the register set: B holds live and removed keys (remm marks the removed
// slots).  live_below(a) >= ef <=> a lies beyond the ef-th smallest live key,
// the radius of a full `top` (B's ef smallest live keys are exactly `top`: an
// over-admitted live key exceeds the radius of its admission, and the radius
// only falls once `top` is full); while fewer than ef live keys are in B no live
// key has left it, so the radius is the largest one (maxlive).  Unexpanded keys
// of B at or below the radius are exactly usearch's unexpanded `next` entries at
// or below it -- an over-admitted removed key lies beyond the radius forever --
// so both expand the same node or both stop.  Compaction keeps the ef smallest
// live keys and every key at or below the ef-th, expanded or not: an expanded
// removed key stays in B so that a forgotten id evaluated again is recognised
// (B.contains) and never expanded twice -- which also bounds the traversal.
// A key dropped by compaction lies above tkey and is never admitted again.
//
// Room: B must hold the ef live keys and the removed ones at or below the
// radius; the row class is sized from the index's removed fraction for that.
// If it still runs out, the query degrades (counted in F.overflow): every
// removed key leaves B and no removed candidate is admitted any more -- the
// classic live-only traversal, which terminates; its results are well-formed
// but no longer usearch's exactly.
struct FiltState {
    uint32_t remm;     // bit r: slot r of this lane holds a removed node
    int nlive;         // live keys in B (wave-uniform)
    uint64_t maxlive;  // largest live key in B while nlive < ef
    uint64_t rad0;     // the start's key: the radius while no live key is admitted
    uint32_t overflow; // keys / candidates dropped for want of room (0 in the tests)
    bool degraded;     // out of room once: removed nodes are no longer admitted
};

__device__ __forceinline__ uint64_t wave_max64(uint64_t v) { return ~wave_min64(~v); }

// #live keys of B below x (wave-uniform)
template <int R> __device__ __forceinline__ int live_below(const RegSet<R>& B, const FiltState& F, uint64_t x) {
    int c = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) c += popc64(__ballot(B.k[r] < x && !((F.remm >> r) & 1u)));
    return c;
}

template <int R> __device__ __forceinline__ void recount(RegSet<R>& B, FiltState& F) {
    int c = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool e = B.k[r] == VSG_KEY_EMPTY;
        if (e) {
            F.remm &= ~(1u << r);
            B.expm &= ~(1u << r);
        }
        c += popc64(__ballot(!e));
    }
    B.size = c;
}

// Make room in B: with >= ef live keys, every key beyond the ef-th live key
// goes (tkey = that key, the radius).
template <int R> __device__ __forceinline__ void compact_filt(RegSet<R>& B, FiltState& F, int ef) {
    if (F.nlive >= ef) {
        B.compact(ef, F.remm);  // drops keys above the cut; recounts the size
        F.nlive = ef;
        recount(B, F);
    }
}

// place the nc staged keys sk[0..nc) (removed flags sf[]) into free slots
template <int R>
__device__ __forceinline__ void fill_filt(RegSet<R>& B, FiltState& F, const uint64_t* sk, const uint32_t* sf, int nc) {
    int acc = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (acc < nc) {
            const bool fr = B.k[r] == VSG_KEY_EMPTY;
            const uint64_t em = __ballot(fr);
            const int idx = acc + lanes_below(em);
            if (fr && idx < nc) {
                B.k[r] = sk[idx];
                B.expm &= ~(1u << r);
                if (sf[idx]) F.remm |= 1u << r;
                else F.remm &= ~(1u << r);
            }
            acc += popc64(em);
        }
    }
    B.size += nc;
}

// Admit this lane's candidate (key ck, removed flag rem) if `mine`.
template <int R>
__device__ __forceinline__ void admit_filt(RegSet<R>& B, FiltState& F, bool mine, uint64_t ck, bool rem, bool lossy,
                                           int ef, uint64_t* sk, uint32_t* sf) {
    const int lane = lane_id();
    // |top| < ef admits everything (tkey is open until a compaction with >= ef
    // live keys sets it to the radius; it only over-admits)
    bool valid = mine && ck < B.tkey && !(F.degraded && rem);
    uint64_t vm = __ballot(valid);
    if (lossy && vm) {
        for (uint64_t mm = vm; mm; mm &= mm - 1) {
            const int j = __builtin_ctzll(mm);
            if (B.contains(readlane64(ck, j))) vm &= ~(1ull << j);
        }
        valid = (vm >> lane) & 1ull;
    }
    int nc = popc64(vm);
    if (nc && B.size + nc > 64 * R) {
        compact_filt(B, F, ef);
        valid = valid && ck < B.tkey;
        vm = __ballot(valid);
        nc = popc64(vm);
        if (B.size + nc > 64 * R) {
            // No room even so: degrade (see FiltState).  Every removed key leaves
            // B and removed candidates are refused from now on; the live keys
            // (< ef, or ef after the compaction) and this batch's live candidates
            // fit in 64 R >= ef + 64 slots.
            const uint64_t before = (uint64_t)B.size;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if ((F.remm >> r) & 1u) B.k[r] = VSG_KEY_EMPTY;
            recount(B, F);
            F.overflow += (uint32_t)(before - (uint64_t)B.size) + (uint32_t)popc64(__ballot(valid && rem));
            F.degraded = true;
            valid = valid && !rem;
            vm = __ballot(valid);
            nc = popc64(vm);
        }
    }
    if (nc) {
        if (valid) {
            sk[lanes_below(vm)] = ck;
            sf[lanes_below(vm)] = rem ? 1u : 0u;
        }
        wave_sync();
        fill_filt(B, F, sk, sf, nc);
        wave_sync();
        const bool lv = valid && !rem;
        const int nl = popc64(__ballot(lv));
        if (nl && F.nlive < ef) F.maxlive = max(F.maxlive, wave_max64(lv ? ck : 0ull));
        F.nlive += nl;
    }
}

// Filtered beam on level 0 (oracle beam_filtered()).  flags: slot -> bit 0 =
// removed.  ep == VSG_EMPTY: B already holds a seed set (opt-in multi-entry
// descent); its removed flags are read here and the radius while no seed is
// live is the largest seed key.
// stop: end the traversal at the first overflow (the caller re-runs the query
// on a list that cannot overflow) instead of degrading.
template <int G, int VM, int U, typename T, int MET, int R>
__device__ __forceinline__ void beam_reg_filt(const GraphDev& g, const QReg<G, VM, T>& q, const uint8_t* flags,
                                              uint32_t ep, float dep, int ef, WaveLds& w, RegSet<R>& B, FiltState& F,
                                              uint64_t& ndist, uint64_t& nadj, BeamProf& pf, bool stop = false) {
    const int lane = lane_id();
    const int m0r = __builtin_amdgcn_readfirstlane(g.M0);
    const uint32_t* adj0 = g.adj0;
    w.vis.clear();
    F.remm = 0;
    F.overflow = 0;
    F.degraded = false;
    if (ep != VSG_EMPTY) {
        if (lane == 0) {
            bool unrec;
            w.vis.insert(ep, unrec);
        }
        const uint64_t k0 = cand_key(dep, ep);
        B.init(k0);
        const bool r0 = flags[ep] & 1;
        if (r0 && lane == 0) F.remm = 1u;
        F.nlive = r0 ? 0 : 1;
        F.maxlive = r0 ? 0ull : k0;
        F.rad0 = k0;
    } else {
        wave_sync();
        uint64_t mx = 0, ml = 0;
        int nl = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool has = B.k[r] != VSG_KEY_EMPTY;
            bool rm = false;
            if (has) {
                const uint32_t s = (uint32_t)B.k[r] & VSG_ID_MASK;
                bool unrec;
                w.vis.insert(s, unrec);
                rm = flags[s] & 1;
                mx = B.k[r] > mx ? B.k[r] : mx;
                if (!rm) ml = B.k[r] > ml ? B.k[r] : ml;
            }
            if (rm) F.remm |= 1u << r;
            nl += popc64(__ballot(has && !rm));
        }
        B.expm = 0;
        B.tkey = VSG_KEY_EMPTY;
        F.nlive = nl;
        F.maxlive = wave_max64(ml);
        F.rad0 = wave_max64(mx);
    }
    bool lossy = false;
    uint64_t* sk = reinterpret_cast<uint64_t*>(w.sd);  // sd + si: 64 x 8 B
    uint32_t* sf = reinterpret_cast<uint32_t*>(w.tdist);
    wave_sync();
    for (;;) {
        const uint64_t t0 = VSG_CLK();
        const uint64_t a = B.min_unexpanded();
        if (a == VSG_KEY_EMPTY) break;
        if (F.nlive >= ef) {
            if (live_below(B, F, a) >= ef) break;  // beyond the ef-th live key
        } else if (a > (F.nlive ? F.maxlive : F.rad0)) {
            break;
        }
        B.mark_expanded(a);
        const uint32_t na = (uint32_t)a & VSG_ID_MASK;
        const uint32_t* row = adj0 + (size_t)na * m0r;
        ++nadj;
        for (int c0 = 0; c0 < m0r; c0 += 64) {
            const uint32_t nb = c0 + lane < m0r ? row[c0 + lane] : VSG_EMPTY;
            const bool full = __ballot(nb != VSG_EMPTY) == ~0ull;
            bool fresh = false, evicted = false;
            if (nb != VSG_EMPTY) fresh = w.vis.insert(nb, evicted);
            const uint64_t mask = __ballot(fresh);
            lossy = lossy || __ballot(evicted) != 0;
            const int cnt = popc64(mask);
            if (fresh) w.todo[lanes_below(mask)] = nb;
            wave_sync();
            const uint64_t t1 = VSG_CLK();
            pf.adj += t1 - t0;
            if (cnt) {
                // the removed flag of this lane's candidate, loaded under the rows
                const uint32_t cid = lane < cnt ? w.todo[lane] : 0u;
                const uint8_t cfl = lane < cnt ? flags[cid] : (uint8_t)0;
                rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
                wave_sync();
                ndist += (uint64_t)cnt;
                const uint64_t ck = lane < cnt ? cand_key(w.tdist[lane], cid) : VSG_KEY_EMPTY;
                const bool crm = lane < cnt && (cfl & 1);
                wave_sync();
                const uint64_t t2 = VSG_CLK();
                pf.dist += t2 - t1;
                admit_filt<R>(B, F, lane < cnt, ck, crm, lossy, ef, sk, sf);
                pf.merge += VSG_CLK() - t2;
            }
            if (!full || (stop && F.degraded)) break;
        }
        if (stop && F.degraded) break;
    }
}

// The top min(ef, |B|) keys of B in ascending order into w.list (buffer 0),
// as the LDS-list beam leaves them (the heuristic selection walks it).  B is
// consumed.
template <int R>
__device__ __forceinline__ void regset_to_list(RegSet<R>& B, int ef, WaveLds& w) {
    const int lane = lane_id();
    List& L = w.list;
    const int lim = min(ef, B.size);
    int x = 0;
    for (; x < lim; ++x) {
        uint64_t b = VSG_KEY_EMPTY;
#pragma unroll
        for (int r = 0; r < R; ++r) b = B.k[r] < b ? B.k[r] : b;
        b = wave_min64(b);
        if (b == VSG_KEY_EMPTY) break;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (B.k[r] == b) B.k[r] = VSG_KEY_EMPTY;
        if (lane == 0) {
            L.d0[x] = key_dist(b);
            L.i0[x] = (uint32_t)b & VSG_ID_MASK;
        }
    }
    L.cur = 0;
    L.size = x;
    wave_sync();
}


}  // namespace vsg
