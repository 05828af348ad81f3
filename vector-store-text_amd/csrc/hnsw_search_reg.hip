// hnsw_search_reg.hip — HNSW kNN search with the level-0 candidate set held in
// VGPRs instead of a sorted list in LDS.
//
// Same traversal as hnsw_search_kernel (oracle beam(), usearch
// search_to_find_in_base_ restated; reference call site
// src/index/usearch.rs:275-277), hence the same results, bit for bit.  What
// changes is the data structure of the beam level:
//
// The sorted top-ef list L_t of the reference equals top_ef(S_t), S_t = every
// node whose distance has been evaluated so far (an entry only leaves L when
// ef better ones exist, and S only grows, so it never returns).  This kernel
// keeps a superset B of top_ef(S) as an unordered set of 64-bit keys
// (ordered-float distance << 32 | slot) in R registers per lane (64 R slots):
//   * next node to expand = the smallest unexpanded key in B, provided fewer
//     than ef keys of B are below it (otherwise every top-ef entry is expanded
//     and the search ends) -- a register min + a wave butterfly, no LDS;
//   * a candidate enters B if its key is below `tkey`, the ef-th smallest key
//     at the last compaction (the reference's "better than the worst of a full
//     list"; tkey only over-admits, as the true threshold only falls);
//   * when B would overflow, it is cut back to its ef smallest keys (radix
//     select with ballots, distance word then slot word on ties) and tkey
//     updated;
//   * a forgetful visited table (Visited::insert) may re-evaluate a node: a
//     candidate already in B is dropped (register compare), one that left B is
//     above tkey.
// LDS then holds only the visited table and 1 KB of staging, so more queries
// are resident per CU at large ef, and the per-expansion list work is a few
// dozen VALU instructions instead of dependent LDS searches.
#include <hip/hip_runtime.h>

#include "hnsw_common.hpp"
#include "vsg_dispatch.hpp"

namespace vsg {

#define VSG_KEY_EMPTY (~0ull)

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
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = shfl_xor64(v, o);
        v = w < v ? w : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
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
    __device__ void compact(int keep) {
        uint32_t ph = 0;
        int need = keep;
#pragma unroll 1
        for (int b = 31; b >= 0; --b) {
            const uint32_t hm = b == 31 ? 0u : (~0u << (b + 1));
            int c = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t hi = (uint32_t)(k[r] >> 32);
                c += popc64(__ballot(k[r] != VSG_KEY_EMPTY && (hi & hm) == ph && !((hi >> b) & 1u)));
            }
            if (c < need) {
                need -= c;
                ph |= 1u << b;
            }
        }
        int ceq = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) ceq += popc64(__ballot(k[r] != VSG_KEY_EMPTY && (uint32_t)(k[r] >> 32) == ph));
        uint64_t cut;
        if (need == ceq) {
            // every key on the cut distance stays: the cut is the largest of them
            uint64_t mx = 0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (k[r] != VSG_KEY_EMPTY && (uint32_t)(k[r] >> 32) == ph && k[r] > mx) mx = k[r];
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
                    c += popc64(__ballot(k[r] != VSG_KEY_EMPTY && (uint32_t)(k[r] >> 32) == ph && (lo & hm) == pl &&
                                         !((lo >> b) & 1u)));
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
        size = keep;
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
template <int R>
__device__ __forceinline__ void admit(RegSet<R>& B, bool mine, uint64_t ck, bool lossy, int ef, uint64_t* sk) {
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
        B.compact(ef);
        valid = valid && ck < B.tkey;
        vm = __ballot(valid);
        nc = popc64(vm);
    }
    if (nc) {
        if (valid) sk[lanes_below(vm)] = ck;
        wave_sync();
        B.fill(sk, nc);
        wave_sync();
    }
}

// Level-0 beam (oracle beam() on level 0).  Preparing the runner-up expansion
// alongside (its adjacency row and distances in the same round trips,
// committed only when it is the sequential next step) was measured 0-15%
// slower: the runner-up is rarely still next (profiles/r01_search_phases.jsonl).
template <int G, int VM, int U, typename T, int MET, int R>
__device__ void beam0_reg(const GraphDev& g, const QReg<G, VM, T>& q, uint32_t ep, float dep, int ef, WaveLds& w,
                          RegSet<R>& B, uint64_t& ndist, uint64_t& nadj, BeamProf& pf) {
    const int lane = lane_id();
    const int m = g.M0;
    w.vis.clear();
    bool lossy = false;
    if (lane == 0) {
        bool unrec;
        w.vis.insert(ep, unrec);
    }
    B.init(cand_key(dep, ep));
    uint64_t* sk = reinterpret_cast<uint64_t*>(w.sd);  // sd + si: 64 x 8 B
    wave_sync();
    for (;;) {
        const uint64_t t0 = VSG_CLK();
        const uint64_t a = B.min_unexpanded();
        if (a == VSG_KEY_EMPTY) break;
        if (B.size > ef && B.count_below(a) >= ef) break;
        B.mark_expanded(a);
        const uint32_t* row = g.row((uint32_t)a & VSG_ID_MASK, 0);
        const uint32_t nb = lane < m ? row[lane] : VSG_EMPTY;
        ++nadj;
        bool fresh = false, evicted = false;
        if (nb != VSG_EMPTY) fresh = w.vis.insert(nb, evicted);
        const uint64_t mask = __ballot(fresh);
        lossy = lossy || __ballot(evicted) != 0;
        const int cnt = popc64(mask);
        if (fresh) w.todo[lanes_below(mask)] = nb;
        wave_sync();
        const uint64_t t1 = VSG_CLK();
        pf.adj += t1 - t0;
        if (cnt == 0) continue;
        rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
        wave_sync();
        ndist += (uint64_t)cnt;
        const uint64_t ck = lane < cnt ? cand_key(w.tdist[lane], w.todo[lane]) : VSG_KEY_EMPTY;
        const uint64_t t2 = VSG_CLK();
        pf.dist += t2 - t1;
        admit<R>(B, lane < cnt, ck, lossy, ef, sk);
        pf.merge += VSG_CLK() - t2;
    }
}

template <int G, int VM, int U, typename T, int MET, int R>
__global__ __launch_bounds__(64) void hnsw_search_reg_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int qi = blockIdx.x;
    if (p.xcd_map) {
        const int nq = p.nq, qd = nq >> 3, rm = nq & 7;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        qi = x * qd + min(x, rm) + j;
    }
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, 0, p.hash_size, false);
    uint64_t ndist = 0, nadj = 0;
    BeamProf pf;
    int count = 0;
    uint64_t* ok = p.out_keys + (size_t)qi * p.k;
    float* od = p.out_dist + (size_t)qi * p.k;
    if (p.entry != VSG_EMPTY) {
        QReg<G, VM, T> q;
        q.load(p.queries + (size_t)qi * g.row_bytes, g.nchunks);
        uint32_t cur = p.entry;
        float dcur = dist_one<G, VM, U, T, MET>(g, q, cur, w);
        ++ndist;
        for (int l = p.max_level; l >= 1; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
        RegSet<R> B;
        beam0_reg<G, VM, U, T, MET, R>(g, q, cur, dcur, p.ef, w, B, ndist, nadj, pf);
        // tombstones: skipped in the output, still traversed
        uint32_t alive = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (B.k[r] != VSG_KEY_EMPTY && !(p.flags[(uint32_t)B.k[r] & VSG_ID_MASK] & 1)) alive |= 1u << r;
        // ascending extraction of the top-ef keys; slots of the alive ones
        // staged in the (finished) visited table, keys gathered after
        uint32_t* sel = w.vis.tab;
        const int lim = min(p.ef, B.size);
        for (int x = 0; x < lim && count < p.k; ++x) {
            uint64_t b = VSG_KEY_EMPTY;
#pragma unroll
            for (int r = 0; r < R; ++r) b = B.k[r] < b ? B.k[r] : b;
            b = wave_min64(b);
            if (b == VSG_KEY_EMPTY) break;
            bool live = false;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (B.k[r] == b) {
                    live = (alive >> r) & 1u;
                    B.k[r] = VSG_KEY_EMPTY;
                }
            if (__ballot(live)) {
                if (lane == 0) {
                    od[count] = key_dist(b);
                    sel[count] = (uint32_t)b & VSG_ID_MASK;
                }
                ++count;
            }
        }
        wave_sync();
        for (int j = lane; j < count; j += 64) ok[j] = p.keys[sel[j]];
    }
    for (int j = count + lane; j < p.k; j += 64) {
        ok[j] = ~0ull;
        od[j] = __builtin_inff();
    }
    if (lane == 0) {
        if (p.out_counts) p.out_counts[qi] = (uint32_t)count;
        if (p.stats) {
            atomicAdd(&p.stats[0], (unsigned long long)ndist);
            atomicAdd(&p.stats[1], (unsigned long long)nadj);
            atomicAdd(&p.stats[2], 1ull);
#ifdef VSG_SEARCH_PROFILE
            atomicAdd(&p.stats[10], (unsigned long long)pf.adj);
            atomicAdd(&p.stats[11], (unsigned long long)pf.dist);
            atomicAdd(&p.stats[12], (unsigned long long)pf.merge);
#endif
        }
    }
}

// slots per lane: 64 R >= ef + 64 (a compaction leaves room for a full batch)
static inline int reg_rows(int ef) { return ef <= 64 ? 2 : ef <= 192 ? 4 : ef <= 448 ? 8 : 17; }

size_t search_reg_lds_bytes(int hash) { return wave_lds_bytes(hash, 0, false); }

hipError_t launch_search_reg(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s) {
    if (p.nq <= 0) return hipSuccess;
    if (p.ef < 1 || p.ef > 1024 || p.k > p.ef || p.hash_size < p.k) return hipErrorInvalidValue;
    const size_t lds = search_reg_lds_bytes(p.hash_size);
    hipError_t err = hipSuccess;
    const int rows = reg_rows(p.ef);
    dispatch_all(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        constexpr int G = decltype(sh)::G, VM = decltype(sh)::VM, U = decltype(sh)::U;
        using T = typename decltype(tt)::T;
        constexpr int MET = decltype(mt)::MET;
        auto run = [&](auto kern) {
            if (lds > 65536)
                (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            constexpr int CH = 1 << 22;  // 64 work-items each: the AQL grid size is 32-bit
            for (int off = 0; off < p.nq && err == hipSuccess; off += CH) {
                SearchParams c = p;
                c.nq = min(CH, p.nq - off);
                c.queries = p.queries + (size_t)off * p.g.row_bytes;
                c.out_keys = p.out_keys + (size_t)off * p.k;
                c.out_dist = p.out_dist + (size_t)off * p.k;
                c.out_counts = p.out_counts ? p.out_counts + off : nullptr;
                hipLaunchKernelGGL(kern, dim3(c.nq), dim3(64), lds, s, c);
                err = hipGetLastError();
            }
        };
        if (rows == 2) run(hnsw_search_reg_kernel<G, VM, U, T, MET, 2>);
        else if (rows == 4) run(hnsw_search_reg_kernel<G, VM, U, T, MET, 4>);
        else if (rows == 8) run(hnsw_search_reg_kernel<G, VM, U, T, MET, 8>);
        else run(hnsw_search_reg_kernel<G, VM, U, T, MET, 17>);
    });
    return err;
}

}  // namespace vsg
