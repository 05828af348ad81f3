// hnsw_search_filt.hip — HNSW kNN search of an index that holds removed
// entries, with usearch's semantics for them.
//
// The reference tombstones with usearch::Index::remove (src/index/usearch.rs:
// 215, 245) and then searches (:276).  usearch's index_dense (v2 series)
// searches with an `allow` predicate (member.key != free_key_) that
// index_gt::search_to_find_in_base_ applies when a candidate is admitted: a
// removed node is traversed (pushed to `next`, expanded in turn) but never
// enters `top`, the ef-wide result list, so it neither takes a result slot nor
// tightens the radius.  Restated in oracle/vsg_oracle.c beam_filtered(); the
// register-set form of the argument is in hnsw_regset.hpp (beam_reg_filt).
//
// Kernels (selected by launch_search_filt; the index's unfiltered searches
// keep hnsw_search_reg_kernel / hnsw_search_kernel, untouched):
//   hnsw_search_reg_filt_kernel  -- candidate set in VGPRs (live + removed
//       keys), R rows sized from ef and the index's removed fraction;
//   hnsw_search_filt_kernel      -- sorted LDS list holding live and removed
//       entries (VSG_REM_BIT), cut at the ef-th live entry; ef up to MAX_EF or
//       when the register set would be too small.
// A query whose candidate set runs out of room (a high removed fraction at
// large ef: the removed nodes at or below the radius pile up beside the ef
// live ones) stops, is flagged (p.ovf) and counted in stats[16]
// (vsg_stats_t.search_filter_overflow), and
//   hnsw_search_filt_rerun_kernel -- the same sorted-list beam on a list in
//       device memory sized for every slot (it holds distinct nodes only, so
//       it cannot run out of room) -- searches it again, counted in stats[17].
// No query ever returns a degraded answer; without p.ovf
// (probes) a query degrades to the live-only traversal (hnsw_regset.hpp
// FiltState), which always terminates.
#include <hip/hip_runtime.h>

#include "hnsw_common.hpp"
#include "hnsw_regset.hpp"
#include "vsg_dispatch.hpp"

namespace vsg {

__device__ __forceinline__ int xcd_query(const SearchParams& p) {
    if (!p.xcd_map) return blockIdx.x;
    const int nq = p.nq, qd = nq >> 3, rm = nq & 7;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    return x * qd + min(x, rm) + j;
}

__device__ __forceinline__ void filt_stats(const SearchParams& p, uint64_t ndist, uint64_t nadj, uint32_t overflow,
                                           int qi) {
    if (lane_id() == 0) {
        if (p.ovf) p.ovf[qi] = overflow ? 1 : 0;
        if (p.stats) {
            atomicAdd(&p.stats[0], (unsigned long long)ndist);
            atomicAdd(&p.stats[1], (unsigned long long)nadj);
            atomicAdd(&p.stats[2], 1ull);
            if (overflow) atomicAdd(&p.stats[16], p.ovf ? 1ull : (unsigned long long)overflow);
        }
    }
}

template <int G, int VM, int U, typename T, int MET, int R>
__global__ __launch_bounds__(64) void hnsw_search_reg_filt_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int qi = xcd_query(p);
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, 0, p.hash_size, 0);
    uint64_t ndist = 0, nadj = 0;
    uint32_t overflow = 0;
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
        RegSet<R> B;
        FiltState F;
        if (p.upper_ef > 1 && p.max_level >= 1) {
            // opt-in multi-entry descent (not usearch): the level-1 beam's set
            // (removed nodes included) seeds the filtered level-0 beam
            for (int l = p.max_level; l >= 2; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
            beam_reg<G, VM, U, T, MET, R>(g, q, 1, cur, dcur, min(p.upper_ef, p.ef), w, B, ndist, nadj, pf);
            beam_reg_filt<G, VM, U, T, MET, R>(g, q, p.flags, VSG_EMPTY, 0.f, p.ef, w, B, F, ndist, nadj, pf,
                                               p.ovf != nullptr);
        } else {
            // usearch search_for_one_: the upper levels ignore the predicate
            for (int l = p.max_level; l >= 1; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
            beam_reg_filt<G, VM, U, T, MET, R>(g, q, p.flags, cur, dcur, p.ef, w, B, F, ndist, nadj, pf,
                                               p.ovf != nullptr);
        }
        overflow = F.overflow;
        // results: the live keys in ascending order (the first k of `top`)
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((F.remm >> r) & 1u) B.k[r] = VSG_KEY_EMPTY;
        uint32_t* sel = w.vis.tab;  // the (finished) visited table stages the slots
        for (; count < p.k;) {
            uint64_t b = VSG_KEY_EMPTY;
#pragma unroll
            for (int r = 0; r < R; ++r) b = B.k[r] < b ? B.k[r] : b;
            b = wave_min64(b);
            if (b == VSG_KEY_EMPTY) break;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (B.k[r] == b) B.k[r] = VSG_KEY_EMPTY;
            if (lane == 0) {
                od[count] = key_dist(b);
                sel[count] = (uint32_t)b & VSG_ID_MASK;
            }
            ++count;
        }
        wave_sync();
        for (int j = lane; j < count; j += 64) ok[j] = p.keys ? p.keys[sel[j]] : (uint64_t)sel[j];
    }
    for (int j = count + lane; j < p.k; j += 64) {
        ok[j] = ~0ull;
        od[j] = __builtin_inff();
    }
    if (lane == 0 && p.out_counts) p.out_counts[qi] = (uint32_t)count;
    filt_stats(p, ndist, nadj, overflow, qi);
}

// The filtered beam on a sorted LDS list of capacity w.list.cap >= ef + 64:
// live and removed entries (VSG_REM_BIT) in (distance, slot) order.  Once ef
// live entries are in, the list is cut right after the ef-th (the radius), so
// every entry is at or below it; before that the radius is the last live entry
// (the start's key while there is none).
// (The list may live in device memory instead: hnsw_search_filt_rerun_kernel.)
// stop: end the traversal at the first overflow instead of degrading.
template <int G, int VM, int U, typename T, int MET>
__device__ void beam_level_filt(const GraphDev& g, const QReg<G, VM, T>& q, const uint8_t* flags, uint32_t ep,
                                float dep, int ef, WaveLds& w, uint64_t& ndist, uint64_t& nadj, uint32_t& overflow,
                                bool stop = false) {
    const int lane = lane_id();
    const int m = g.M0;
    w.vis.clear();
    List& L = w.list;
    L.cur = 0;
    L.size = 1;
    const bool r0 = flags[ep] & 1;
    bool lossy = false;
    if (lane == 0) {
        bool unrec;
        w.vis.insert(ep, unrec);
        L.d0[0] = dep;
        L.i0[0] = ep | (r0 ? VSG_REM_BIT : 0u);
    }
    int nlive = r0 ? 0 : 1;
    int lastlive = r0 ? -1 : 0;
    bool degraded = false;  // out of room once (see below)
    wave_sync();
    int hint = 0;
    for (;;) {
        const int p = L.first_unexpanded(hint);
        if (p < 0) break;
        if (nlive < ef) {  // beyond the radius: stop
            if (nlive == 0) {
                if (cand_less(dep, ep, L.D()[p], L.I()[p] & VSG_ID_MASK)) break;
            } else if (p > lastlive) {
                break;
            }
        }
        const uint32_t e = L.I()[p];
        const uint32_t node = e & VSG_ID_MASK;
        wave_sync();
        if (lane == 0) L.I()[p] = e | VSG_EXP_BIT;
        hint = p + 1;
        const uint32_t* row = g.row(node, 0);
        ++nadj;
        for (int c0 = 0; c0 < m; c0 += 64) {
            const uint32_t nb = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
            const bool full = __ballot(nb != VSG_EMPTY) == ~0ull;
            bool fresh = false, evicted = false;
            if (nb != VSG_EMPTY) fresh = w.vis.insert(nb, evicted);
            const uint64_t mask = __ballot(fresh);
            lossy = lossy || __ballot(evicted) != 0;
            const int cnt = popc64(mask);
            if (fresh) w.todo[lanes_below(mask)] = nb;
            wave_sync();
            if (cnt) {
                const uint32_t cid = lane < cnt ? w.todo[lane] : 0u;
                const uint8_t cfl = lane < cnt ? flags[cid] : (uint8_t)0;
                rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
                wave_sync();
                ndist += (uint64_t)cnt;
                bool valid = lane < cnt && !(degraded && (cfl & 1));
                const float cd = lane < cnt ? w.tdist[lane] : 0.f;
                wave_sync();
                if (valid && nlive >= ef) {  // a full `top`: below the radius only
                    const float rd = L.D()[L.size - 1];
                    const uint32_t ri = L.I()[L.size - 1] & VSG_ID_MASK;
                    valid = cand_less(cd, cid, rd, ri);
                }
                const int nc = popc64(__ballot(valid));
                const int lost = max(0, L.size + nc - L.cap);  // the largest entries, when the list is full
                hint = min(hint, L.merge(valid, cd, cid, lossy, w.sd, w.si, (cfl & 1) ? VSG_REM_BIT : 0u));
                // recount the live entries; cut after the ef-th
                int nl = 0, last = -1, cut = -1;
                for (int r = 0; r < L.size; r += 64) {
                    const int i = r + lane;
                    const bool live = i < L.size && !(L.I()[i] & VSG_REM_BIT);
                    const uint64_t lm = __ballot(live);
                    const int c = popc64(lm);
                    if (cut < 0 && nl + c >= ef) {
                        const uint64_t at = __ballot(live && lanes_below(lm) == ef - nl - 1);
                        cut = r + __builtin_ctzll(at);
                    }
                    if (lm) last = r + 63 - __builtin_clzll(lm);
                    nl += c;
                }
                if (cut >= 0) {
                    // entries a full list dropped lay beyond the radius: never needed
                    L.size = cut + 1;
                    nlive = ef;
                } else {
                    nlive = nl;
                    lastlive = last;
                    if (lost && stop) {
                        overflow += (uint32_t)lost;  // re-run by the caller
                        return;
                    }
                    if (lost) {
                        // Out of room before ef live entries: degrade (counted).  Every
                        // removed entry leaves the list and removed candidates are
                        // refused from now on -- the live-only traversal, which
                        // terminates.  (Entries are never dropped otherwise: an expanded
                        // removed one must stay to recognise a forgotten id evaluated
                        // again, so no node is expanded twice.)
                        overflow += (uint32_t)lost;
                        degraded = true;
                        const float* dd = L.D();
                        const uint32_t* ii = L.I();
                        float* nd = L.Dn();
                        uint32_t* ni = L.In();
                        int n2 = 0;
                        for (int r = 0; r < L.size; r += 64) {
                            const int i = r + lane;
                            const uint32_t e = i < L.size ? ii[i] : VSG_REM_BIT;
                            const bool keep = !(e & VSG_REM_BIT);
                            const uint64_t km = __ballot(keep);
                            if (keep) {
                                nd[n2 + lanes_below(km)] = dd[i];
                                ni[n2 + lanes_below(km)] = e;
                            }
                            n2 += popc64(km);
                        }
                        overflow += (uint32_t)(L.size - n2);
                        wave_sync();
                        L.size = n2;
                        L.cur ^= 1;
                        lastlive = n2 - 1;
                        hint = 0;
                    }
                }
            }
            if (!full) break;
        }
    }
}

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void hnsw_search_filt_kernel(SearchParams p, int cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int qi = xcd_query(p);
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, cap, p.hash_size, 0);
    uint64_t ndist = 0, nadj = 0;
    uint32_t overflow = 0;
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
        beam_level_filt<G, VM, U, T, MET>(g, q, p.flags, cur, dcur, p.ef, w, ndist, nadj, overflow, p.ovf != nullptr);
        const List& L = w.list;
        for (int r = 0; r < L.size && count < p.k; r += 64) {
            const int i = r + lane;
            const bool valid = i < L.size;
            const uint32_t e = valid ? L.I()[i] : VSG_REM_BIT;
            const bool alive = !(e & VSG_REM_BIT);
            const uint32_t id = e & VSG_ID_MASK;
            const uint64_t mk = __ballot(alive);
            const int pos = count + lanes_below(mk);
            if (alive && pos < p.k) {
                ok[pos] = p.keys ? p.keys[id] : (uint64_t)id;
                od[pos] = L.D()[i];
            }
            count += popc64(mk);
        }
        if (count > p.k) count = p.k;
    }
    for (int j = count + lane; j < p.k; j += 64) {
        ok[j] = ~0ull;
        od[j] = __builtin_inff();
    }
    if (lane == 0 && p.out_counts) p.out_counts[qi] = (uint32_t)count;
    filt_stats(p, ndist, nadj, overflow, qi);
}

// Re-run of the queries that overflowed (p.ovf[qi] set): persistent blocks, one
// wave each, walk the flags; block b's list (d0 | d1 | i0 | i1, cap entries each)
// is list b of p.filt_lists in device memory, cap >= every slot + 64 (the list
// holds distinct nodes: forgotten ids are de-duplicated against it), so it never
// runs out of room.  The visited table stays in LDS.  Same beam, same results as
// the LDS-list kernel would give with room enough: the oracle's beam_filtered().
template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void hnsw_search_filt_rerun_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    const size_t cap = (size_t)p.filt_cap;
    uint8_t* mine = p.filt_lists + (size_t)blockIdx.x * cap * 16;
    for (int qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
        if (!p.ovf[qi]) continue;  // wave-uniform
        WaveLds w = carve(smem, 0, p.hash_size, 0);
        w.list.d0 = reinterpret_cast<float*>(mine);
        w.list.d1 = reinterpret_cast<float*>(mine + cap * 4);
        w.list.i0 = reinterpret_cast<uint32_t*>(mine + cap * 8);
        w.list.i1 = reinterpret_cast<uint32_t*>(mine + cap * 12);
        w.list.cap = (int)cap;
        uint64_t ndist = 0, nadj = 0;
        uint32_t overflow = 0;
        int count = 0;
        uint64_t* ok = p.out_keys + (size_t)qi * p.k;
        float* od = p.out_dist + (size_t)qi * p.k;
        QReg<G, VM, T> q;
        q.load(p.queries + (size_t)qi * g.row_bytes, g.nchunks);
        uint32_t cur = p.entry;
        float dcur = dist_one<G, VM, U, T, MET>(g, q, cur, w);
        ++ndist;
        for (int l = p.max_level; l >= 1; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
        beam_level_filt<G, VM, U, T, MET>(g, q, p.flags, cur, dcur, p.ef, w, ndist, nadj, overflow);
        const List& L = w.list;
        for (int r = 0; r < L.size && count < p.k; r += 64) {
            const int i = r + lane;
            const bool valid = i < L.size;
            const uint32_t e = valid ? L.I()[i] : VSG_REM_BIT;
            const bool alive = !(e & VSG_REM_BIT);
            const uint32_t id = e & VSG_ID_MASK;
            const uint64_t mk = __ballot(alive);
            const int pos = count + lanes_below(mk);
            if (alive && pos < p.k) {
                ok[pos] = p.keys ? p.keys[id] : (uint64_t)id;
                od[pos] = L.D()[i];
            }
            count += popc64(mk);
        }
        if (count > p.k) count = p.k;
        for (int j = count + lane; j < p.k; j += 64) {
            ok[j] = ~0ull;
            od[j] = __builtin_inff();
        }
        if (lane == 0) {
            if (p.out_counts) p.out_counts[qi] = (uint32_t)count;
            if (p.stats) {
                atomicAdd(&p.stats[0], (unsigned long long)ndist);
                atomicAdd(&p.stats[1], (unsigned long long)nadj);
                atomicAdd(&p.stats[17], 1ull);
                if (overflow) atomicAdd(&p.stats[16], (unsigned long long)overflow);  // cannot happen (cap)
            }
        }
        wave_sync();
    }
}

// One list per re-run block: 16 B x (slots + 64) entries; as many lists as fit
// in 32 MiB (at least one, at most 16).  Every search workspace of an index with
// removed entries carries them, for a re-run that is rare by design (ADVICE r5:
// 256 MiB per workspace at 1M slots before); a workspace that cannot get them
// searches in the degraded, counted mode instead of failing (vsg_index.cpp).
void filt_rerun_shape(size_t slots, int* cap, int* nlists) {
    const size_t c = slots + 64;
    const size_t per = c * 16;
    size_t nl = ((size_t)32 << 20) / per;
    nl = nl < 1 ? 1 : nl > 16 ? 16 : nl;
    *cap = (int)c;
    *nlists = (int)nl;
}
size_t filt_rerun_bytes(size_t slots) {
    int cap = 0, nl = 0;
    filt_rerun_shape(slots, &cap, &nl);
    return (size_t)cap * 16 * (size_t)nl;
}

static hipError_t launch_filt_rerun(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s) {
    if (!p.ovf || !p.filt_lists || p.filt_nlists < 1) return hipSuccess;
    SearchParams r = p;
    // the visited table only (the list is in device memory): forgetful at this size
    r.hash_size = std::max(1024, std::min(p.hash_size, 16384));
    const size_t lds = search_reg_lds_bytes(r.hash_size);
    hipError_t err = hipSuccess;
    dispatch_all<SHAPE_SEARCH>(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        constexpr int G = decltype(sh)::G, VM = decltype(sh)::VM, U = decltype(sh)::U;
        using T = typename decltype(tt)::T;
        constexpr int MET = decltype(mt)::MET;
        auto kern = hnsw_search_filt_rerun_kernel<G, VM, U, T, MET>;
        if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)std::min(p.filt_nlists, p.nq)), dim3(64), lds, s, r);
        err = hipGetLastError();
    });
    return err;
}

// Candidate-set size of a filtered search: the ef live keys, the removed ones
// admitted beside them (about ef x f / (1 - f) for a removed fraction f) with
// a 1.5x margin, and one expansion's batch.
static inline int filt_capacity(int ef, float removed_frac) {
    const double f = std::min(0.97, std::max(0.0, (double)removed_frac));
    return (int)std::ceil(1.5 * ef / (1.0 - f)) + 64;
}

hipError_t launch_search_filt(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s) {
    if (p.nq <= 0) return hipSuccess;
    if (p.ef < 1 || p.ef > (int)MAX_EF || p.k > p.ef) return hipErrorInvalidValue;
    const int need = filt_capacity(p.ef, p.removed_frac);
    int rows = need <= 128 ? 2 : need <= 256 ? 4 : need <= 512 ? 8 : need <= 1088 ? 17 : 0;
    if (const char* e = getenv("VSG_SEARCH_FILT_ROWS")) {  // probes / tests: force a class (0 = list)
        const int r = atoi(e);
        if ((r == 0 || r == 2 || r == 4 || r == 8 || r == 17) && 64 * r >= p.ef + 64) rows = r;
        if (r == 0) rows = 0;
    }
    if (!p.reg && p.upper_ef <= 1) rows = 0;  // VSG_SEARCH_REG=0: the list kernel
    if (p.upper_ef > 1 && rows == 0) rows = 17;  // multi-entry descent is register-only
    if (rows && 64 * rows < p.ef + 64) return hipErrorInvalidValue;
    hipError_t err = hipSuccess;
    constexpr int CH = 1 << 20;
    if (rows) {
        const size_t lds = search_reg_lds_bytes(p.hash_size);
        auto body = [&](auto sh, auto tt, auto mt) {
            constexpr int G = decltype(sh)::G, VM = decltype(sh)::VM, U = decltype(sh)::U;
            using T = typename decltype(tt)::T;
            constexpr int MET = decltype(mt)::MET;
            auto run = [&](auto kern) {
                if (lds > 65536)
                    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                for (int off = 0; off < p.nq && err == hipSuccess; off += CH) {
                    SearchParams c = p;
                    c.nq = min(CH, p.nq - off);
                    c.queries = p.queries + (size_t)off * p.g.row_bytes;
                    c.out_keys = p.out_keys + (size_t)off * p.k;
                    c.out_dist = p.out_dist + (size_t)off * p.k;
                    c.out_counts = p.out_counts ? p.out_counts + off : nullptr;
                    c.ovf = p.ovf ? p.ovf + off : nullptr;
                    hipLaunchKernelGGL(kern, dim3(c.nq), dim3(64), lds, s, c);
                    err = hipGetLastError();
                }
            };
            if (rows == 2) run(hnsw_search_reg_filt_kernel<G, VM, U, T, MET, 2>);
            else if (rows == 4) run(hnsw_search_reg_filt_kernel<G, VM, U, T, MET, 4>);
            else if (rows == 8) run(hnsw_search_reg_filt_kernel<G, VM, U, T, MET, 8>);
            else run(hnsw_search_reg_filt_kernel<G, VM, U, T, MET, 17>);
        };
        if (rows == 17) dispatch_all<SHAPE_GENERIC>(st, mk, p.g.nchunks, body);
        else dispatch_all<SHAPE_SEARCH>(st, mk, p.g.nchunks, body);
        if (err == hipSuccess) err = launch_filt_rerun(st, mk, p, s);
        return err;
    }
    // sorted LDS list: 16 B per entry, up to 8,192 entries (ef <= MAX_EF live ones and
    // the removed ones beside them); the visited table gives way to the list within the
    // 160 KB of LDS a workgroup may hold (a smaller table forgets more: more distance
    // evaluations, the same results)
    const int cap = std::min(8192, std::max(p.ef + 64, 2 * need));
    SearchParams pl = p;
    const int hmax = (int)(((160 * 1024) - (size_t)cap * 16 - 64 * 16 - 1024) / 4) & ~63;
    pl.hash_size = std::max(1024, std::min(p.hash_size, hmax));
    const size_t lds = wave_lds_bytes(pl.hash_size, cap, 0);
    dispatch_all<SHAPE_SEARCH>(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        constexpr int G = decltype(sh)::G, VM = decltype(sh)::VM, U = decltype(sh)::U;
        using T = typename decltype(tt)::T;
        constexpr int MET = decltype(mt)::MET;
        auto kern = hnsw_search_filt_kernel<G, VM, U, T, MET>;
        if (lds > 65536)
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        for (int off = 0; off < p.nq && err == hipSuccess; off += CH) {
            SearchParams c = pl;
            c.nq = min(CH, p.nq - off);
            c.queries = p.queries + (size_t)off * p.g.row_bytes;
            c.out_keys = p.out_keys + (size_t)off * p.k;
            c.out_dist = p.out_dist + (size_t)off * p.k;
            c.out_counts = p.out_counts ? p.out_counts + off : nullptr;
            c.ovf = p.ovf ? p.ovf + off : nullptr;
            hipLaunchKernelGGL(kern, dim3(c.nq), dim3(64), lds, s, c, cap);
            err = hipGetLastError();
        }
    });
    if (err == hipSuccess) err = launch_filt_rerun(st, mk, p, s);
    return err;
}

}  // namespace vsg
