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

#include <map>
#include <type_traits>
#include <mutex>
#include <tuple>

#include "hnsw_common.hpp"
#include "hnsw_regset.hpp"
#include "vsg_dispatch.hpp"

namespace vsg {

// occupancy request (probes: -DVSG_SEARCH_ATTR='__attribute__((amdgpu_waves_per_eu(5)))')
#ifndef VSG_SEARCH_ATTR
#define VSG_SEARCH_ATTR
#endif
template <int G, int VM, int U, typename T, int MET, int R>
__device__ __forceinline__ void search_reg_one(const SearchParams& p, int qi, uint8_t* smem) {
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, 0, p.hash_size, 0);
    uint64_t ndist = 0, nadj = 0;
    BeamProf pf;
    [[maybe_unused]] const uint64_t cq0 = VSG_CYC(), tq0 = VSG_CLK();
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
        if (p.upper_ef > 1 && p.max_level >= 1) {
            // opt-in multi-entry descent (not usearch): greedy down to level 2,
            // an upper_ef-wide beam on level 1, and its whole result set seeds
            // the level-0 beam
#ifdef VSG_UPPER_ALL_LEVELS
            beam_reg<G, VM, U, T, MET, R>(g, q, p.max_level, cur, dcur, min(p.upper_ef, p.ef), w, B, ndist, nadj, pf);
            for (int l = p.max_level - 1; l >= 1; --l)
                beam_reg<G, VM, U, T, MET, R>(g, q, l, VSG_EMPTY, 0.f, min(p.upper_ef, p.ef), w, B, ndist, nadj, pf);
#else
            for (int l = p.max_level; l >= 2; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
            beam_reg<G, VM, U, T, MET, R>(g, q, 1, cur, dcur, min(p.upper_ef, p.ef), w, B, ndist, nadj, pf);
#endif
            beam_reg<G, VM, U, T, MET, R>(g, q, 0, VSG_EMPTY, 0.f, p.ef, w, B, ndist, nadj, pf);
        } else {
            [[maybe_unused]] const uint64_t cd0 = VSG_CYC();
            for (int l = p.max_level; l >= 1; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
#ifdef VSG_SEARCH_PROFILE
            pf.c_desc += VSG_CYC() - cd0;
#endif
            beam_reg<G, VM, U, T, MET, R>(g, q, 0, cur, dcur, p.ef, w, B, ndist, nadj, pf);
        }
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
        for (int j = lane; j < count; j += 64) ok[j] = p.keys ? p.keys[sel[j]] : (uint64_t)sel[j];
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
            // per-expansion breakdown, shader cycles (tools/gpu_probe.py --phases)
            atomicAdd(&p.stats[20], (unsigned long long)pf.c_sel);
            atomicAdd(&p.stats[21], (unsigned long long)pf.c_adj);
            atomicAdd(&p.stats[22], (unsigned long long)pf.c_vis);
            atomicAdd(&p.stats[23], (unsigned long long)pf.rows.wait);
            atomicAdd(&p.stats[24], (unsigned long long)pf.rows.valu);
            atomicAdd(&p.stats[25], (unsigned long long)pf.c_admit);
            atomicAdd(&p.stats[26], (unsigned long long)pf.c_comp);
            atomicAdd(&p.stats[27], (unsigned long long)pf.c_desc);
            atomicAdd(&p.stats[28], (unsigned long long)pf.nexp | ((unsigned long long)pf.ncomp << 40));
            atomicAdd(&p.stats[29], (unsigned long long)pf.rows.passes);
            atomicAdd(&p.stats[30], (unsigned long long)(VSG_CYC() - cq0));
            atomicAdd(&p.stats[31], (unsigned long long)(VSG_CLK() - tq0));
#endif
        }
    }
}

// Persistent grid only in the instances for rows of >= 1 KiB (the shape's row span,
// 16-B chunks): compiled into the short-row kernels, the loop's second copy of the
// search cost the C4 shard kernel 15 VGPRs (87 -> 102: 5 -> 4 waves per SIMD, 2.97 ->
// 3.23 ms at ef 192) although it never ran there.  launch_search_reg sizes the grid by
// the same constant.
template <int G, int VM> constexpr bool persist_shape() { return G * VM * 16 >= 1024; }

template <int G, int VM, int U, typename T, int MET, int R>
__global__ __launch_bounds__(64) VSG_SEARCH_ATTR void hnsw_search_reg_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if constexpr (persist_shape<G, VM>()) {
        if (p.qnext) {
            // persistent grid: resident waves take query indices from a counter until
            // the batch is done
            for (;;) {
                int qi = 0;
                if (lane_id() == 0) qi = (int)atomicAdd(p.qnext, 1u);
                qi = __builtin_amdgcn_readfirstlane(qi);
                if (qi >= p.nq) break;
                search_reg_one<G, VM, U, T, MET, R>(p, qi, smem);
                wave_sync();
            }
            return;
        }
    }
    int qi = blockIdx.x;
    if (p.xcd_map) {
        const int nq = p.nq, qd = nq >> 3, rm = nq & 7;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        qi = x * qd + min(x, rm) + j;
    }
    search_reg_one<G, VM, U, T, MET, R>(p, qi, smem);
}

// slots per lane: 64 R >= ef + 64 (a compaction leaves room for a full batch)
static inline int reg_rows(int ef) { return ef <= 64 ? 2 : ef <= 192 ? 4 : ef <= 448 ? 8 : 17; }

size_t search_reg_lds_bytes(int hash) { return wave_lds_bytes(hash, 0, 0); }

static double env_frac(const char* name, double dflt) {
    const char* e = getenv(name);
    return e ? atof(e) : dflt;
}

// one-wave workgroups of `kern` resident on the whole device at `lds` bytes each
// (occupancy x CUs), cached per (device, kernel, lds)
static int resident_blocks(const void* kern, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, size_t>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({dev, kern, lds});
    if (it != cache.end()) return it->second;
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, lds);
    const int r = std::max(1, per_cu * cus);
    cache[{dev, kern, lds}] = r;
    return r;
}

hipError_t launch_search_reg(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s) {
    if (p.nq <= 0) return hipSuccess;
    if (p.ef < 1 || p.ef > 1024 || p.k > p.ef || p.hash_size < p.k) return hipErrorInvalidValue;
    const size_t lds = search_reg_lds_bytes(p.hash_size);
    hipError_t err = hipSuccess;
    // VSG_SEARCH_REG_ROWS (probes): more register rows than the minimum --
    // same results (B is any superset of the top ef), fewer compactions
    int rows = reg_rows(p.ef);
    if (const char* e = getenv("VSG_SEARCH_REG_ROWS")) {
        const int r = atoi(e);
        if ((r == 2 || r == 4 || r == 8 || r == 17) && 64 * r >= p.ef + 64) rows = r;
    }
    // R (register rows) fixed at compile time, so each row shape is instantiated only
    // for the R classes that use it
    auto launch_rows = [&](auto rtag) {
        constexpr int R = decltype(rtag)::value;
        auto body = [&](auto sh, auto tt, auto mt) {
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
                    unsigned grid = (unsigned)c.nq;
                    if (persist_shape<G, VM>() && p.qnext) {  // persistent: one round of resident waves, counter reset per launch
                        // 3/4 of the resident waves: the kernel is throughput-bound below full
                        // occupancy, and fewer waves end the batch sooner.  C2 fractions 0.35 /
                        // 0.5 / 0.75 / 1.0 with the U=4 row shape (2 waves/SIMD resident): 3.01 /
                        // 3.34 / 3.40 / 3.38 M QPS (profiles/r05_pfrac_u4.jsonl); with U=2 (4
                        // waves/SIMD) 0.35-0.6 were level at 3.34 M (r05_pfrac.jsonl);
                        // VSG_SEARCH_PERSIST_FRAC overrides (probes)
                        static const double frac = std::min(1.0, std::max(0.05, env_frac("VSG_SEARCH_PERSIST_FRAC", 0.75)));
                        const int res = std::max(1, (int)(frac * resident_blocks((const void*)kern, lds)));
                        grid = (unsigned)std::max(1, std::min(c.nq, res));
                        err = hipMemsetAsync(p.qnext, 0, sizeof(unsigned), s);
                        if (err != hipSuccess) break;
                    }
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, s, c);
                    err = hipGetLastError();
                }
            };
            run(hnsw_search_reg_kernel<G, VM, U, T, MET, R>);
        };
        // the search row shape (dispatch_shape_search): 4 passes for long rows with 2 register
        // rows (vsg_dispatch.hpp); with 17 (ef > 448) the generic shape, where the 8 x 2 shape
        // of 64-d f32 rows spills registers
        if constexpr (R == 17) dispatch_all<SHAPE_GENERIC>(st, mk, p.g.nchunks, body);
        else if constexpr (R == 2) dispatch_all<SHAPE_SEARCH_SMALL_EF>(st, mk, p.g.nchunks, body);
        else dispatch_all<SHAPE_SEARCH>(st, mk, p.g.nchunks, body);
    };
    if (rows == 2) launch_rows(std::integral_constant<int, 2>{});
    else if (rows == 4) launch_rows(std::integral_constant<int, 4>{});
    else if (rows == 8) launch_rows(std::integral_constant<int, 8>{});
    else launch_rows(std::integral_constant<int, 17>{});
    return err;
}

}  // namespace vsg
