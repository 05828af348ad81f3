// hnsw.hip — HNSW search and batched build kernels for gfx950 (CDNA4).
//
// Semantics follow the CPU restatement oracle/vsg_oracle.c (usearch
// index.hpp, restated): greedy descent on levels > 0, "expand the best
// unexpanded entry of the (distance, slot)-sorted top-ef list" on the beam
// level, heuristic (refine) neighbour selection, reverse links appended while
// there is room and re-selected with the heuristic otherwise.  Reference call
// sites: usearch::Index::search (src/index/usearch.rs:275-277) and
// usearch::Index::add (src/index/usearch.rs:221).
//
// One wave64 per query / inserted node; all per-wave state in LDS (vsg_device.hpp).
// Base rows and adjacency are read straight from HBM into VGPRs (HBM-bound
// traversal).
#include <hip/hip_runtime.h>

#include "vsg_device.hpp"
#include "vsg_dispatch.hpp"
#include "vsg_kernels.hpp"
#include "hnsw_common.hpp"
#include "hnsw_regset.hpp"

namespace vsg {

// Visited-table entries: `factor` x ef (the traversal evaluates ~15-20 x ef
// nodes), multiple of 64, within [1024, 16384].  Smaller tables raise the
// number of co-resident waves per CU (LDS-bound occupancy at large ef) at the
// cost of re-evaluating forgotten nodes (Visited::insert); results do not
// depend on it.
__host__ __device__ int hash_size_for(int ef, int factor) {
    long h = (long)factor * ef;
    h = (h + 63) & ~63L;
    if (h < 1024) h = 1024;
    if (h > 16384) h = 16384;
    return (int)h;
}

// cooperative search: + 8 control words (WgCtl) after the shared wave state
size_t search_lds_bytes(int ef, int hash, int waves) {
    return wave_lds_bytes(hash, ef, 0) + (waves > 1 ? 32 : 0);
}
size_t insert_lds_bytes(int efc, int hash, int m0) { return wave_lds_bytes(hash, efc, sel_entries(m0)); }


// usearch search_to_find_in_base_ restated (oracle beam()).
// `hint`: entries below it are all expanded, so the scan for the next
// candidate starts there (merge() reports the lowest position it filled).
// (Prefetching the next entry's adjacency row during this expansion's distance
// loads measured 2-7% slower: profiles/r01_search_phases.jsonl.)
// self: the node an insert (re)links, never admitted (VSG_EMPTY in searches).
template <int G, int VM, int U, typename T, int MET>
__device__ void beam_level(const GraphDev& g, const QReg<G, VM, T>& q, int l, uint32_t ep, float dep,
                           WaveLds& w, uint64_t& ndist, uint64_t& nadj, BeamProf& pf, uint32_t self = VSG_EMPTY) {
    const int lane = lane_id();
    const int m = l == 0 ? g.M0 : g.M;
    w.vis.clear();
    List& L = w.list;
    L.cur = 0;
    L.size = 1;
    bool lossy = false;  // the visited table has forgotten an id (wave-uniform)
    if (lane == 0) {
        bool unrec;
        w.vis.insert(ep, unrec);
        L.d0[0] = dep;
        L.i0[0] = ep;
    }
    wave_sync();
    int hint = 0;
    for (;;) {
        const uint64_t t0 = VSG_CLK();
        const int p = L.first_unexpanded(hint);
        if (p < 0) break;
        const uint32_t node = L.I()[p] & VSG_ID_MASK;
        wave_sync();
        if (lane == 0) L.I()[p] = node | VSG_EXP_BIT;
        hint = p + 1;
        const uint32_t* row = g.row(node, l);
        ++nadj;
        for (int c0 = 0; c0 < m; c0 += 64) {  // 64-entry pieces of the row (M0 <= 128)
            const uint32_t nb = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
            const bool full = __ballot(nb != VSG_EMPTY) == ~0ull;
            bool fresh = false, evicted = false;
            if (nb != VSG_EMPTY && nb != self) fresh = w.vis.insert(nb, evicted);
            const uint64_t mask = __ballot(fresh);
            lossy = lossy || __ballot(evicted) != 0;
            const int cnt = popc64(mask);
            if (fresh) w.todo[lanes_below(mask)] = nb;
            wave_sync();
            const uint64_t t1 = VSG_CLK();
            pf.adj += t1 - t0;
            if (cnt) {
                rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
                wave_sync();
                ndist += (uint64_t)cnt;
                const bool valid = lane < cnt;
                const float cd = valid ? w.tdist[lane] : 0.f;
                const uint32_t ci = valid ? w.todo[lane] : 0u;
                wave_sync();
                const uint64_t t2 = VSG_CLK();
                pf.dist += t2 - t1;
                hint = min(hint, L.merge(valid, cd, ci, lossy, w.sd, w.si));
                pf.merge += VSG_CLK() - t2;
            }
            if (!full) break;
        }
    }
}

// usearch refine_ restated (oracle select_heuristic()): walk the sorted list,
// keep c unless a kept r has dist(c, r) < dist(c, base).  Returns #kept.
// Fewer than m candidates: all of them, unfiltered (refine_'s early return).
// Candidates go in blocks of NQ held in VGPRs: the block is tested against the
// kept set in one pass over its rows (each row loaded once, rows_test), then
// each candidate, in list order, against the block's earlier kept candidates
// from registers -- the sequential decision for every candidate, with the same
// distance values.  NQ = 2 halves the kept-row loads of one-at-a-time
// (single: insert kernel +20 % time); NQ = 4 halves them again (C2 insert -1 %,
// reverse -13 %; C4 shard insert -2 %, reverse -9 %).
// NQ per row shape: up to 4 candidates, at most ~96 VGPRs of candidate images
// (VM x E floats each: 24 for 768-d f32, 48 for 768-d f16, 8 for 128-d f16).
#ifndef VSG_SEL_VGPRS
#define VSG_SEL_VGPRS 96
#endif
// SU: row passes in flight per kept-set test (rows_test U), capped at the
// shape's U.  The test is a chain of dependent L2 round trips (the kept rows
// were fetched by the beam moments ago): more passes per trip, fewer trips.
#ifndef VSG_SEL_U
#define VSG_SEL_U 1
#endif
// occupancy requests of the selection / reverse kernels (probes: e.g.
// -DVSG_SEL_WAVES='__attribute__((amdgpu_waves_per_eu(3, 3)))')
#ifndef VSG_SEL_WAVES
#define VSG_SEL_WAVES
#endif
#ifndef VSG_REV_WAVES
#define VSG_REV_WAVES
#endif
#ifndef VSG_SEL_U_INSERT
#define VSG_SEL_U_INSERT VSG_SEL_U
#endif
#ifndef VSG_SEL_U_REVERSE
#define VSG_SEL_U_REVERSE VSG_SEL_U
#endif
// register rows of the build's efC beam (64 R >= efC + 64; more rows: fewer
// compactions, more VGPRs)
#ifndef VSG_BUILD_REG_R
#define VSG_BUILD_REG_R 4
#endif
// Selection row shape (probes): VSG_SEL_G64 lays a 32-lane row shape with an even
// VM over the whole wave (G 64, VM / 2: half the candidate image, so twice the
// candidates per block at the same registers); VSG_SEL_NQMAX caps the block.
#ifndef VSG_SEL_G64
#define VSG_SEL_G64 0
#endif
#ifndef VSG_SEL_NQMAX
#define VSG_SEL_NQMAX 4
#endif
template <int G, int VM> struct SelShape {
    static constexpr bool W = VSG_SEL_G64 && G == 32 && VM % 2 == 0;
    static constexpr int G2 = W ? 64 : G, VM2 = W ? VM / 2 : VM;
};
template <int QF> constexpr int sel_nq() {
    int nq = VSG_SEL_NQMAX;
    while (nq > 1 && nq * QF > VSG_SEL_VGPRS) --nq;
    return nq;
}

template <int G0, int VM0, int U, typename T, int MET, int SU = VSG_SEL_U>
__device__ int select_heuristic(const GraphDev& g, WaveLds& w, int n, int m, uint64_t& ndist) {
    constexpr int G = SelShape<G0, VM0>::G2, VM = SelShape<G0, VM0>::VM2;
    constexpr int QF = VM * ChunkT<T>::E;
    constexpr int NQ = sel_nq<QF>();
    constexpr int UT = SU;  // row passes in flight per test
    constexpr int BLK = (64 / G) * UT;
    const int lane = lane_id();
    List& L = w.list;
    if (n < m) {
        // refine_'s early return (top_count < needed): every candidate, unfiltered
        // (a new node's forward links while the level has < M reachable nodes)
        for (int j = lane; j < n; j += 64) {
            w.sel[j] = L.I()[j] & VSG_ID_MASK;
            w.seld[j] = L.D()[j];
        }
        wave_sync();
        return n;
    }
    int kept = 0;
    using Q = QReg<G, VM, T>;
    for (int i = 0; i < n && kept < m; i += NQ) {
        const int nb = min(NQ, n - i);
        Q qc[NQ];
        float cd[NQ];
        uint32_t cid[NQ];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            const int jj = j < nb ? i + j : i;  // a short last block repeats its head (masked off)
            cid[j] = L.I()[jj] & VSG_ID_MASK;
            cd[j] = L.D()[jj];
            qc[j].load(g.vec(cid[j]), g.nchunks);
        }
        uint32_t alive = (1u << nb) - 1u;
        for (int b = 0; b < kept && alive; b += BLK) {
            const int cnt = min(BLK, kept - b);
            ndist += (uint64_t)cnt * (uint64_t)__popc(alive);
            alive &= ~rows_test<NQ, G, VM, UT, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.sel + b, cnt, qc, cd);
        }
        uint32_t kb = 0;  // block members kept so far
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            bool good = ((alive >> j) & 1u) && kept < m;
#pragma unroll
            for (int t = 0; t < j; ++t) {
                if (good && ((kb >> t) & 1u)) {
                    ++ndist;
                    if (reg_dist<G, VM, T, MET>(qc[j], qc[t], g.nchunks) < cd[j]) good = false;
                }
            }
            if (good) {
                if (lane == 0) {
                    w.sel[kept] = cid[j];
                    w.seld[kept] = cd[j];
                }
                kb |= 1u << j;
                ++kept;
            }
        }
        wave_sync();
    }
    return kept;
}

// The selected neighbours (and, when the graph carries them, their distances
// to `node`: the values the selection walked, kept so the reverse-link prune
// need not recompute them) become row(node, l); EMPTY / +inf past nsel.
__device__ inline void write_row(const GraphDev& g, uint32_t node, int l, int m, int nsel, const WaveLds& w) {
    const int lane = lane_id();
    uint32_t* row = g.row(node, l);
    for (int j = lane; j < m; j += 64) row[j] = j < nsel ? w.sel[j] : VSG_EMPTY;
    if (g.adjd0) {
        float* rd = g.rowd(node, l);
        for (int j = lane; j < m; j += 64) rd[j] = j < nsel ? w.seld[j] : __builtin_inff();
    }
}

// ------------------------------------------------------------------ search --

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void hnsw_search_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int qi = blockIdx.x;
    if (p.xcd_map) {
        // bijective: XCD group x = b % 8 takes the contiguous query range
        // [x*q + min(x, r), ...) so neighbouring (similar) queries share an L2
        const int nq = p.nq, qd = nq >> 3, rm = nq & 7;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        qi = x * qd + min(x, rm) + j;
    }
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, p.ef, p.hash_size, 0);
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
        beam_level<G, VM, U, T, MET>(g, q, 0, cur, dcur, w, ndist, nadj, pf);
        const List& L = w.list;
        for (int r = 0; r < L.size && count < p.k; r += 64) {
            const int i = r + lane;
            const bool valid = i < L.size;
            const uint32_t id = valid ? (L.I()[i] & VSG_ID_MASK) : 0u;
            const bool alive = valid && !(p.flags[id] & 1);
            const uint64_t m = __ballot(alive);
            const int pos = count + lanes_below(m);
            if (alive && pos < p.k) {
                ok[pos] = p.keys ? p.keys[id] : (uint64_t)id;
                od[pos] = L.D()[i];
            }
            count += popc64(m);
        }
        if (count > p.k) count = p.k;
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

// ------------------------------------------------------ search: cooperative --
// Large ef: NW waves share ONE query's LDS state (visited hash, list).  Per
// expansion: wave 0 picks the best unexpanded entry, reads its adjacency row and
// records fresh neighbours (serial control, as in beam_level); the fresh rows'
// distances are split over the NW waves (NW x the loads in flight per LDS byte,
// 1/NW of the latency); wave 0 ranks the candidates (List::place) and every
// thread moves the existing entries (List::shift).  Same expansion order and
// same list as hnsw_search_kernel, hence the same results (tested bit-exact
// against the oracle).  Upper levels: wave 0 alone (greedy_level).
//
// Control words in LDS (ctl[8]): [0..3] (done, cnt) double-buffered by
// iteration parity (a wave still reading iteration i's words never sees i+1's:
// wave 0 cannot reach i+2 without the barrier that wave joins after reading),
// [4..5] nc by parity, [6..7] level-0 entry (slot, distance bits).

template <int G, int VM, int U, typename T, int MET, int NW>
__device__ void beam0_wg(const GraphDev& g, const QReg<G, VM, T>& q, WaveLds& w, int* ctl, uint64_t& ndist,
                         uint64_t& nadj) {
    constexpr int NT = 64 * NW;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = lane_id();
    const int m = g.M0;
    List& L = w.list;
    L.cur = 0;
    L.size = 1;
    {
        uint4* t4 = reinterpret_cast<uint4*>(w.vis.tab);
        for (uint32_t i = tid; i < w.vis.size / 4; i += NT)
            t4[i] = make_uint4(VSG_EMPTY, VSG_EMPTY, VSG_EMPTY, VSG_EMPTY);
    }
    __syncthreads();
    bool lossy = false;  // wave 0 only
    if (tid == 0) {
        const uint32_t ep = (uint32_t)ctl[6];
        bool unrec;
        w.vis.insert(ep, unrec);
        L.d0[0] = __int_as_float(ctl[7]);
        L.i0[0] = ep;
    }
    __syncthreads();
    for (int it = 0;; ++it) {
        int* c2 = ctl + 2 * (it & 1);
        if (wave == 0) {
            const int p = L.first_unexpanded();
            int cnt = 0;
            if (p >= 0) {
                const uint32_t node = L.I()[p] & VSG_ID_MASK;
                wave_sync();
                if (lane == 0) L.I()[p] = node | VSG_EXP_BIT;
                const uint32_t* row = g.row(node, 0);
                const uint32_t nb = lane < m ? row[lane] : VSG_EMPTY;
                ++nadj;
                bool fresh = false, evicted = false;
                if (nb != VSG_EMPTY) fresh = w.vis.insert(nb, evicted);
                const uint64_t mask = __ballot(fresh);
                lossy = lossy || __ballot(evicted) != 0;
                cnt = popc64(mask);
                if (fresh) w.todo[lanes_below(mask)] = nb;
            }
            if (lane == 0) {
                c2[0] = p < 0;
                c2[1] = cnt;
            }
        }
        __syncthreads();
        if (c2[0]) break;
        const int cnt = c2[1];
        if (cnt == 0) continue;  // parity double-buffering makes the next write safe
        const int per = (cnt + NW - 1) / NW;
        const int b0 = wave * per;
        const int c = min(cnt - b0, per);
        if (c > 0) rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo + b0, c, q, w.tdist + b0);
        __syncthreads();
        if (wave == 0) {
            ndist += (uint64_t)cnt;
            const bool valid = lane < cnt;
            const float cd = valid ? w.tdist[lane] : 0.f;
            const uint32_t ci = valid ? w.todo[lane] : 0u;
            const int nc = L.place(valid, cd, ci, lossy, w.sd, w.si);
            if (lane == 0) ctl[4 + (it & 1)] = nc;
        }
        __syncthreads();
        const int nc = ctl[4 + (it & 1)];
        if (nc) L.shift(nc, w.sd, w.si, tid, NT);
        L.advance(nc);
        __syncthreads();
    }
}

template <int G, int VM, int U, typename T, int MET, int NW>
__global__ __launch_bounds__(64 * NW) void hnsw_search_wg_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int qi = blockIdx.x;
    if (p.xcd_map) {
        const int nq = p.nq, qd = nq >> 3, rm = nq & 7;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        qi = x * qd + min(x, rm) + j;
    }
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, p.ef, p.hash_size, 0);
    int* ctl = reinterpret_cast<int*>(smem + wave_lds_bytes(p.hash_size, p.ef, 0));
    uint64_t ndist = 0, nadj = 0;
    [[maybe_unused]] BeamProf pf;
    int count = 0;
    uint64_t* ok = p.out_keys + (size_t)qi * p.k;
    float* od = p.out_dist + (size_t)qi * p.k;
    if (p.entry != VSG_EMPTY) {
        QReg<G, VM, T> q;
        q.load(p.queries + (size_t)qi * g.row_bytes, g.nchunks);
        if (wave == 0) {
            uint32_t cur = p.entry;
            float dcur = dist_one<G, VM, U, T, MET>(g, q, cur, w);
            ++ndist;
            for (int l = p.max_level; l >= 1; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj);
            if (lane == 0) {
                ctl[6] = (int)cur;
                ctl[7] = __float_as_int(dcur);
            }
        }
        __syncthreads();
        beam0_wg<G, VM, U, T, MET, NW>(g, q, w, ctl, ndist, nadj);
        if (wave == 0) {
            const List& L = w.list;
            for (int r = 0; r < L.size && count < p.k; r += 64) {
                const int i = r + lane;
                const bool valid = i < L.size;
                const uint32_t id = valid ? (L.I()[i] & VSG_ID_MASK) : 0u;
                const bool alive = valid && !(p.flags[id] & 1);
                const uint64_t m = __ballot(alive);
                const int pos = count + lanes_below(m);
                if (alive && pos < p.k) {
                    ok[pos] = p.keys ? p.keys[id] : (uint64_t)id;
                    od[pos] = L.D()[i];
                }
                count += popc64(m);
            }
            if (count > p.k) count = p.k;
        }
    }
    if (wave != 0) return;
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

// ------------------------------------------------------------ build: fwd --
// One wave per new node of the batch: descend, beam with efC per level,
// select M_l neighbours, write the node's own rows and emit (level, v, u)
// reverse-link pairs at the node's pre-assigned offset (no atomics).

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void hnsw_insert_kernel(InsertParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int bi = blockIdx.x;
    if (p.perm) {  // sorted batch, dealt XCD-contiguously (block b runs on XCD b % 8)
        const int n = p.nnodes, qd = n >> 3, rm = n & 7, x = blockIdx.x & 7, j = blockIdx.x >> 3;
        bi = (int)p.perm[x * qd + min(x, rm) + j];
    }
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, p.efc, p.hash_size, sel_entries(g.M0));
    const uint64_t t_start = wall_clock64();
    const uint32_t node = p.nodes[bi];
    const int L = p.levels[bi];
    uint64_t ndist = 0, nadj = 0, nsel_d = 0;
    BeamProf pf;
    uint64_t tsel = 0;
    QReg<G, VM, T> q;
    q.load(g.vec(node), g.nchunks);
    uint32_t cur = p.entry;
    float dcur = dist_one<G, VM, U, T, MET>(g, q, cur, w);
    ++ndist;
    for (int l = p.max_level; l > L; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj, node);
    uint32_t pos = p.pair_off[bi];
    for (int l = min(L, p.max_level); l >= 0; --l) {
        if (p.efc <= 192) {
            // candidate set in VGPRs (hnsw_regset.hpp), then the sorted top-efc
            // list the selection walks -- the list beam's exact result
            RegSet<VSG_BUILD_REG_R> B;
            beam_reg<G, VM, U, T, MET, VSG_BUILD_REG_R>(g, q, l, cur, dcur, p.efc, w, B, ndist, nadj, pf, node);
            regset_to_list<VSG_BUILD_REG_R>(B, p.efc, w);
        } else {
            beam_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj, pf, node);
        }
        // usearch connect_new_node_: at most M forward links on every level
        // (refine_ with config_.connectivity); level-0 rows reach M0 = 2M only
        // through reverse links (hnsw_reverse_kernel)
        const int m = l == 0 ? g.M0 : g.M;
        const uint64_t ts = VSG_CLK();
        const int nsel = select_heuristic<G, VM, U, T, MET>(g, w, w.list.size, g.M, nsel_d);
        tsel += VSG_CLK() - ts;
        write_row(g, node, l, m, nsel, w);
        for (int j = lane; j < nsel; j += 64) {
            const uint64_t key = ((uint64_t)l << PAIR_L_SHIFT) | ((uint64_t)w.sel[j] << PAIR_V_SHIFT) |
                                 (uint64_t)node;
            p.pair_keys[pos + j] = key;
            p.pair_vals[pos + j] = __float_as_uint(w.seld[j]);
        }
        pos += (uint32_t)nsel;
        cur = w.list.I()[0] & VSG_ID_MASK;
        dcur = w.list.D()[0];
        wave_sync();
    }
    if (lane == 0 && p.stats) {
        atomicAdd(&p.stats[3], (unsigned long long)(ndist + nsel_d));
        atomicAdd(&p.stats[4], (unsigned long long)nadj);
        atomicAdd(&p.stats[5], (unsigned long long)nsel_d);
        const unsigned long long dt = wall_clock64() - t_start;
        atomicAdd(&p.stats[10], dt);
        atomicMax(&p.stats[11], dt);
#ifdef VSG_SEARCH_PROFILE
        // profile build: [14] heuristic selection, [15] beam (adjacency + rows + merge)
        atomicAdd(&p.stats[14], (unsigned long long)tsel);
        atomicAdd(&p.stats[15], (unsigned long long)(pf.adj + pf.dist + pf.merge));
#else
        (void)tsel;
#endif
    }
}

// ------------------------------------------------------------ build: split --
// The insert kernel above in two launches.  Its register footprint is set by the
// heuristic selection (NQ candidate images + row loads: 232 VGPRs at C2, 2
// waves/SIMD) while 2/3 of its time is the efC beam, which needs about half.
// hnsw_insert_beam_kernel runs descent + beam of every level at the beam's own
// occupancy and stores each level's sorted top-efc list (as regset_to_list
// leaves it in LDS) in HBM; hnsw_insert_select_kernel reloads the lists and runs
// the selection, row writes and pair emission in the same level order.  Same
// operations on the same values: the graph is bit-identical to the fused kernel.

__device__ __forceinline__ int insert_index(const InsertParams& p) {
    if (!p.perm) return blockIdx.x;
    const int n = p.nnodes, qd = n >> 3, rm = n & 7, x = blockIdx.x & 7, j = blockIdx.x >> 3;
    return (int)p.perm[x * qd + min(x, rm) + j];
}

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void hnsw_insert_beam_kernel(InsertParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int bi = insert_index(p);
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, p.efc, p.hash_size, 0);
    const uint64_t t_start = wall_clock64();
    const uint32_t node = p.nodes[bi];
    const int L = p.levels[bi];
    uint64_t ndist = 0, nadj = 0;
    BeamProf pf;
    QReg<G, VM, T> q;
    q.load(g.vec(node), g.nchunks);
    uint32_t cur = p.entry;
    float dcur = dist_one<G, VM, U, T, MET>(g, q, cur, w);
    ++ndist;
    for (int l = p.max_level; l > L; --l) greedy_level<G, VM, U, T, MET>(g, q, l, cur, dcur, w, ndist, nadj, node);
    for (int l = min(L, p.max_level); l >= 0; --l) {
        RegSet<VSG_BUILD_REG_R> B;
        beam_reg<G, VM, U, T, MET, VSG_BUILD_REG_R>(g, q, l, cur, dcur, p.efc, w, B, ndist, nadj, pf, node);
        regset_to_list<VSG_BUILD_REG_R>(B, p.efc, w);
        const size_t slot = (size_t)p.list_off[bi] + (size_t)l;
        const int n = w.list.size;
        float* od = p.lst_d + slot * (size_t)p.efc;
        uint32_t* oi = p.lst_i + slot * (size_t)p.efc;
        for (int j = lane; j < n; j += 64) {
            od[j] = w.list.d0[j];
            oi[j] = w.list.i0[j];
        }
        if (lane == 0) p.lst_n[slot] = n;
        cur = w.list.i0[0] & VSG_ID_MASK;
        dcur = w.list.d0[0];
        wave_sync();
    }
    if (lane == 0 && p.stats) {
        atomicAdd(&p.stats[3], (unsigned long long)ndist);
        atomicAdd(&p.stats[4], (unsigned long long)nadj);
        const unsigned long long dt = wall_clock64() - t_start;
        atomicAdd(&p.stats[10], dt);
        atomicMax(&p.stats[11], dt);
    }
}

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) VSG_SEL_WAVES void hnsw_insert_select_kernel(InsertParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int bi = insert_index(p);
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    WaveLds w = carve(smem, p.efc, 0, sel_entries(g.M0));
    const uint32_t node = p.nodes[bi];
    const int L = p.levels[bi];
    uint64_t nsel_d = 0;
    uint32_t pos = p.pair_off[bi];
    for (int l = min(L, p.max_level); l >= 0; --l) {
        const size_t slot = (size_t)p.list_off[bi] + (size_t)l;
        const int n = p.lst_n[slot];
        const float* id = p.lst_d + slot * (size_t)p.efc;
        const uint32_t* ii = p.lst_i + slot * (size_t)p.efc;
        for (int j = lane; j < n; j += 64) {
            w.list.d0[j] = id[j];
            w.list.i0[j] = ii[j];
        }
        w.list.cur = 0;
        w.list.size = n;
        wave_sync();
        const int m = l == 0 ? g.M0 : g.M;  // row width; <= M forward links (connect_new_node_)
        const int nsel = select_heuristic<G, VM, U, T, MET, VSG_SEL_U_INSERT>(g, w, n, g.M, nsel_d);
        write_row(g, node, l, m, nsel, w);
        for (int j = lane; j < nsel; j += 64) {
            const uint64_t key = ((uint64_t)l << PAIR_L_SHIFT) | ((uint64_t)w.sel[j] << PAIR_V_SHIFT) |
                                 (uint64_t)node;
            p.pair_keys[pos + j] = key;
            p.pair_vals[pos + j] = __float_as_uint(w.seld[j]);
        }
        pos += (uint32_t)nsel;
        wave_sync();
    }
    if (lane == 0 && p.stats) {
        atomicAdd(&p.stats[3], (unsigned long long)nsel_d);
        atomicAdd(&p.stats[5], (unsigned long long)nsel_d);
    }
}

// ------------------------------------------------------------ build: rev --
// Pairs sorted by (level, v, u).  Persistent waves scan contiguous chunks for
// segment heads; each segment (level, v) is merged into v's row: append while
// there is room, else heuristic re-selection over existing + incoming.
// Re-linking reused slots (p.flags set: bit 1 marks the call's reused slots),
// an incoming u that v's row already holds -- a link into the slot kept from
// before its removal -- changes nothing (usearch reconnect_neighbor_nodes_,
// oracle add_reverse); only those segments take the checks.

#define VSG_FLAG_RELINK 2  // d_flags bit 1: a reused slot being re-linked by the current add

// does row[0, ne) hold u (one lane; the row was just read, so from L1/L2)
__device__ __forceinline__ bool row_holds(const uint32_t* row, int ne, uint32_t u) {
    bool h = false;
    for (int c = 0; c < ne; ++c) h = h || row[c] == u;
    return h;
}

// Entries in use of an adjacency row (a compact prefix), read by one lane: 16 B
// at a time when rows are 16-B aligned (m % 4 == 0), stopping at the first piece
// that is not full.
#ifndef VSG_REVERSE_LANE_APPEND
#define VSG_REVERSE_LANE_APPEND 1
#endif
__device__ __forceinline__ int row_fill(const uint32_t* row, int m) {
    int ne = 0;
    if ((m & 3) == 0) {
        const uint4* r4 = reinterpret_cast<const uint4*>(row);
        const int m4 = m >> 2;
        for (int c0 = 0; c0 < m4; c0 += 8) {
            int cnt = 0;
            uint4 x[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                x[j] = c0 + j < m4 ? r4[c0 + j] : make_uint4(VSG_EMPTY, VSG_EMPTY, VSG_EMPTY, VSG_EMPTY);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                cnt += (x[j].x != VSG_EMPTY) + (x[j].y != VSG_EMPTY) + (x[j].z != VSG_EMPTY) + (x[j].w != VSG_EMPTY);
            ne += cnt;
            if (cnt < 32) break;
        }
    } else {
        for (int c0 = 0; c0 < m; c0 += 8) {
            int cnt = 0;
            uint32_t x[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = c0 + j < m ? row[c0 + j] : VSG_EMPTY;
#pragma unroll
            for (int j = 0; j < 8; ++j) cnt += x[j] != VSG_EMPTY;
            ne += cnt;
            if (cnt < 8) break;
        }
    }
    return ne;
}

// One instance for both paths (stored distances / recomputed): compiled as two
// instances, the stored-distance one got 185 VGPRs instead of 239 and ran 50 %
// slower (C2 reverse 54 -> 82 ms; profiles/r03_build_probe.jsonl) -- the larger
// allocation keeps more of the selection's row loads in flight.
template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) VSG_REV_WAVES void hnsw_reverse_kernel(ReverseParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = lane_id();
    const GraphDev g = to_dev(p.g);
    const int cap = 2 * g.M0 > 64 ? 2 * g.M0 : 64;
    WaveLds w = carve(smem, cap, 0, sel_entries(g.M0));  // no visited table
    const uint64_t t_start = wall_clock64();
    uint64_t ndist = 0, nadj = 0, nsel_d = 0, nprune = 0, nappend = 0;
    const size_t nw = gridDim.x;
    const size_t chunk = (p.npairs + nw - 1) / nw;  // segments are found by their head pair
    const size_t beg = (size_t)blockIdx.x * chunk;
    const size_t end = min(beg + chunk, p.npairs);
    for (size_t i0 = beg; i0 < end; i0 += 64) {
        const size_t i = i0 + lane;
        const uint64_t key = i < end ? p.keys[i] : ~0ull;
        const uint64_t prev = (i < end && i > 0) ? p.keys[i - 1] : ~0ull;
        const bool head = key != ~0ull && (i == 0 || (key >> PAIR_V_SHIFT) != (prev >> PAIR_V_SHIFT));
        uint64_t heads = __ballot(head);
        nadj += (uint64_t)popc64(heads);
        if (VSG_REVERSE_LANE_APPEND) {
            // Appends, one segment per head lane: each lane reads its own row's
            // fill (one round trip for every segment of the window, where the
            // wave-wide path below pays one per segment) and appends when the
            // segment fits.  Segments touch only their own (level, v) row, so
            // the order they are applied in changes nothing.
            bool fits = false;
            if (head) {
                const uint64_t seg = key >> PAIR_V_SHIFT;
                const int l = (int)(key >> PAIR_L_SHIFT);
                const uint32_t v = (uint32_t)(seg & PAIR_ID_MASK);
                const uint64_t above = heads & ~((2ull << lane) - 1ull);  // later heads of the window
                size_t e;
                if (above) {
                    e = i0 + (size_t)__builtin_ctzll(above);
                } else {  // the window's last segment: scan on (segments are short)
                    e = i + 1;
                    while (e < p.npairs && (p.keys[e] >> PAIR_V_SHIFT) == seg) ++e;
                }
                const int nin = (int)(e - i);
                const int m = l == 0 ? g.M0 : g.M;
                uint32_t* row = g.row(v, l);
                const int ne = row_fill(row, m);
                bool relink = false;  // a reused slot among the incoming: the wave-wide path checks it
                if (p.flags)
                    for (int t = 0; t < nin; ++t)
                        relink = relink || (p.flags[(uint32_t)(p.keys[i + t] & PAIR_ID_MASK)] & VSG_FLAG_RELINK);
                if (!relink && ne + nin <= m) {
                    fits = true;
                    float* rowd = g.adjd0 ? g.rowd(v, l) : nullptr;
                    for (int t = 0; t < nin; ++t) {
                        row[ne + t] = (uint32_t)(p.keys[i + t] & PAIR_ID_MASK);
                        if (rowd) rowd[ne + t] = __uint_as_float(p.vals[i + t]);
                    }
                }
            }
            const uint64_t done = __ballot(fits);
            nappend += (uint64_t)popc64(done);
            heads &= ~done;  // the segments that need a prune
        }
        while (heads) {
            const int hl = __builtin_ctzll(heads);
            heads &= heads - 1;
            const size_t h = i0 + hl;
            const uint64_t hkey = p.keys[h];
            const uint64_t seg = hkey >> PAIR_V_SHIFT;
            const int l = (int)(hkey >> PAIR_L_SHIFT);
            const uint32_t v = (uint32_t)((hkey >> PAIR_V_SHIFT) & PAIR_ID_MASK);
            // segment end
            size_t e = h;
            for (;;) {
                const size_t j = e + lane;
                const bool same = j < p.npairs && (p.keys[j] >> PAIR_V_SHIFT) == seg;
                const uint64_t nm = __ballot(!same);
                if (nm) {
                    e += __builtin_ctzll(nm);
                    break;
                }
                e += 64;
            }
            const int nin = (int)(e - h);
            const int m = l == 0 ? g.M0 : g.M;
            uint32_t* row = g.row(v, l);
            int ne = 0;  // rows are a compact prefix (M0 <= 128: up to two pieces)
            for (int c0 = 0; c0 < m; c0 += 64) {
                const uint32_t x = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
                const uint64_t xm = __ballot(x != VSG_EMPTY);
                ne += popc64(xm);
                if (xm != ~0ull) break;
            }
            float* rowd = g.adjd0 ? g.rowd(v, l) : nullptr;
            // re-linked reused slots: incoming links v's row already holds are dropped
            bool anyrel = false;
            if (p.flags)
                for (int t = 0; t < nin; t += 64) {
                    const bool valid = t + lane < nin;
                    const uint32_t u = valid ? (uint32_t)(p.keys[h + t + lane] & PAIR_ID_MASK) : 0u;
                    anyrel = anyrel || __ballot(valid && (p.flags[u] & VSG_FLAG_RELINK)) != 0;
                }
            auto kept_in = [&](int idx) {  // incoming idx (< nin) survives the check
                if (!anyrel) return true;
                const uint32_t u = (uint32_t)(p.keys[h + idx] & PAIR_ID_MASK);
                return !((p.flags[u] & VSG_FLAG_RELINK) && row_holds(row, ne, u));
            };
            int nkeep = nin;
            if (anyrel) {
                nkeep = 0;
                for (int t = 0; t < nin; t += 64) nkeep += popc64(__ballot(t + lane < nin && kept_in(t + lane)));
                if (nkeep == 0) {
                    ++nappend;
                    continue;
                }
            }
            if (ne + nkeep <= m) {
                if (!anyrel) {
                    for (int t = lane; t < nin; t += 64) {
                        row[ne + t] = (uint32_t)(p.keys[h + t] & PAIR_ID_MASK);
                        if (rowd) rowd[ne + t] = __uint_as_float(p.vals[h + t]);
                    }
                } else {
                    int at = ne;
                    for (int t = 0; t < nin; t += 64) {
                        const bool keep = t + lane < nin && kept_in(t + lane);
                        const uint64_t km = __ballot(keep);
                        wave_sync();  // every lane's row_holds read precedes this chunk's writes
                        if (keep) {
                            const int pos = at + lanes_below(km);
                            row[pos] = (uint32_t)(p.keys[h + t + lane] & PAIR_ID_MASK);
                            if (rowd) rowd[pos] = __uint_as_float(p.vals[h + t + lane]);
                        }
                        at += popc64(km);
                    }
                }
                ++nappend;
                continue;
            }
            ++nprune;
            List& L = w.list;
            L.cur = 0;
            L.size = 0;
            if (rowd) {
                // existing neighbours with their stored distances: the values the
                // insert that wrote them computed -- dist(v, x) or dist(x, v), the
                // same float (operand-symmetric: (a-b)^2, a.b, same lane order)
                for (int c0 = 0; c0 < ne; c0 += 64) {
                    const bool valid = c0 + lane < ne;
                    const uint32_t ci = valid ? row[c0 + lane] : 0u;
                    const float cd = valid ? rowd[c0 + lane] : 0.f;
                    L.merge(valid, cd, ci, false, w.sd, w.si);
                }
            } else {
                QReg<G, VM, T> q;
                q.load(g.vec(v), g.nchunks);
                for (int c0 = 0; c0 < ne; c0 += 64) {  // existing neighbours, distances recomputed
                    const uint32_t x = c0 + lane < ne ? row[c0 + lane] : VSG_EMPTY;
                    const uint64_t xm = __ballot(x != VSG_EMPTY);
                    const int c = popc64(xm);
                    if (x != VSG_EMPTY) w.todo[lanes_below(xm)] = x;
                    wave_sync();
                    rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, c, q, w.tdist);
                    wave_sync();
                    ndist += (uint64_t)c;
                    const bool valid = lane < c;
                    const float cd = valid ? w.tdist[lane] : 0.f;
                    const uint32_t ci = valid ? w.todo[lane] : 0u;
                    wave_sync();
                    L.merge(valid, cd, ci, false, w.sd, w.si);
                }
            }
            for (int t = 0; t < nin; t += 64) {
                const bool valid = t + lane < nin && kept_in(t + lane);
                const size_t idx = h + t + lane;
                const float cd = valid ? __uint_as_float(p.vals[idx]) : 0.f;
                const uint32_t ci = valid ? (uint32_t)(p.keys[idx] & PAIR_ID_MASK) : 0u;
                L.merge(valid, cd, ci, false, w.sd, w.si);
            }
            const int nsel = select_heuristic<G, VM, U, T, MET, VSG_SEL_U_REVERSE>(g, w, L.size, m, nsel_d);
            write_row(g, v, l, m, nsel, w);
            wave_sync();
        }
    }
    if (lane == 0 && p.stats) {
        atomicAdd(&p.stats[3], (unsigned long long)(ndist + nsel_d));
        atomicAdd(&p.stats[4], (unsigned long long)nadj);
        atomicAdd(&p.stats[6], (unsigned long long)ndist);
        atomicAdd(&p.stats[7], (unsigned long long)nsel_d);
        atomicAdd(&p.stats[8], (unsigned long long)nprune);
        atomicAdd(&p.stats[9], (unsigned long long)nappend);
        const unsigned long long dt = wall_clock64() - t_start;
        atomicAdd(&p.stats[12], dt);
        atomicMax(&p.stats[13], dt);
    }
}

// ------------------------------------------------------- edge distances --
// Per-edge distances of a graph that arrived without them (import, load): one
// wave per slot, dist(slot, neighbour) for every entry of every level's row --
// the value rows_dist gives with the slot as query, as the build stores it.

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void edge_dist_fill_kernel(DevGraph gd, const int8_t* levels, uint32_t n) {
    __shared__ uint32_t todo[64];
    __shared__ float tdist[64];
    const uint32_t s = blockIdx.x;
    if (s >= n) return;
    const int lane = lane_id();
    const GraphDev g = to_dev(gd);
    QReg<G, VM, T> q;
    q.load(g.vec(s), g.nchunks);
    for (int l = 0; l <= levels[s]; ++l) {
        const int m = l == 0 ? g.M0 : g.M;
        const uint32_t* row = g.row(s, l);
        float* rd = g.rowd(s, l);
        for (int c0 = 0; c0 < m; c0 += 64) {
            const uint32_t x = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
            const uint64_t xm = __ballot(x != VSG_EMPTY);
            const int c = popc64(xm);  // compact prefix: the first c lanes
            if (x != VSG_EMPTY) todo[lane] = x;
            wave_sync();
            if (c) rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, todo, c, q, tdist);
            wave_sync();
            if (c0 + lane < m) rd[c0 + lane] = lane < c ? tdist[lane] : __builtin_inff();
            wave_sync();
            if (xm != ~0ull) break;
        }
    }
}

// ----------------------------------------------------------- slot reuse --
// An add that reuses removed slots (usearch index_dense_gt::add_ popping
// free_keys_ -> index_gt::update; oracle orc_hnsw_add) stages them before its
// first batch: prepared row, |x|^2 and key into the slot, every row of the
// slot cleared (its level and upper rows are kept), flags = removed | relink
// until the add publishes (searches keep treating it as removed; the reverse
// kernel sees the relink bit).  One wave per reused slot.
__global__ __launch_bounds__(64) void reuse_stage_kernel(DevGraph g, uint8_t* __restrict__ vecs,
                                                         float* __restrict__ sqnorm, uint64_t* __restrict__ okeys,
                                                         uint8_t* __restrict__ flags, const uint8_t* __restrict__ rows,
                                                         const float* __restrict__ sq, const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ slots,
                                                         const int8_t* __restrict__ levels, uint32_t n) {
    const int lane = lane_id();
    const size_t n16 = g.row_bytes / 16;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t s = slots[i];
        const uint4* a = reinterpret_cast<const uint4*>(rows + (size_t)i * g.row_bytes);
        uint4* b = reinterpret_cast<uint4*>(vecs + (size_t)s * g.row_bytes);
        for (size_t c = lane; c < n16; c += 64) b[c] = a[c];
        if (lane == 0) {
            if (sqnorm) sqnorm[s] = sq[i];
            okeys[s] = keys[i];
            flags[s] = 1 | VSG_FLAG_RELINK;
        }
        for (int l = 0; l <= levels[i]; ++l) {
            const int m = l == 0 ? g.M0 : g.M;
            uint32_t* row = l == 0 ? g.adj0 + (size_t)s * g.M0 : g.upper + ((size_t)g.upper_off[s] + (size_t)(l - 1)) * g.M;
            for (int j = lane; j < m; j += 64) row[j] = VSG_EMPTY;
            if (g.adjd0) {
                float* rd = l == 0 ? g.adjd0 + (size_t)s * g.M0 : g.upperd + ((size_t)g.upper_off[s] + (size_t)(l - 1)) * g.M;
                for (int j = lane; j < m; j += 64) rd[j] = __builtin_inff();
            }
        }
    }
}

hipError_t launch_reuse_stage(const DevGraph& g, uint8_t* vecs, float* sqnorm, uint64_t* keys_out, uint8_t* flags,
                              const uint8_t* rows, const float* sq, const uint64_t* keys, const uint32_t* slots,
                              const int8_t* levels, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>(n, 1u << 20);
    hipLaunchKernelGGL(reuse_stage_kernel, dim3(grid), dim3(64), 0, s, g, vecs, sqnorm, keys_out, flags, rows, sq,
                       keys, slots, levels, (uint32_t)n);
    return hipGetLastError();
}

// The stored distance of every link INTO a reused slot (kept from before its
// removal) was computed against the slot's old vector: recompute it against the
// new one, dist(v, slot) with v as the query -- the value an insert stores
// (operand-symmetric, same lane order), so the reverse prune reads exactly the
// distances the oracle recomputes.  One wave per slot v (grid-stride); only
// rows that hold a relink-flagged id load v's vector.
template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void edge_dist_refresh_kernel(DevGraph gd, const int8_t* levels, const uint8_t* flags,
                                                               uint32_t n) {
    __shared__ uint32_t todo[64];
    __shared__ float tdist[64];
    __shared__ int pos[64];
    const int lane = lane_id();
    const GraphDev g = to_dev(gd);
    for (uint32_t s = blockIdx.x; s < n; s += gridDim.x) {
        if (flags[s] & VSG_FLAG_RELINK) continue;  // a reused slot itself: its rows were cleared
        QReg<G, VM, T> q;
        bool loaded = false;
        for (int l = 0; l <= levels[s]; ++l) {
            const int m = l == 0 ? g.M0 : g.M;
            const uint32_t* row = g.row(s, l);
            float* rd = g.rowd(s, l);
            for (int c0 = 0; c0 < m; c0 += 64) {
                const uint32_t x = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
                const uint64_t xm = __ballot(x != VSG_EMPTY);
                const bool hit = x != VSG_EMPTY && (flags[x] & VSG_FLAG_RELINK);
                const uint64_t hm = __ballot(hit);
                if (hm) {
                    if (!loaded) {
                        q.load(g.vec(s), g.nchunks);
                        loaded = true;
                    }
                    const int cnt = popc64(hm);
                    if (hit) {
                        todo[lanes_below(hm)] = x;
                        pos[lanes_below(hm)] = c0 + lane;
                    }
                    wave_sync();
                    rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, todo, cnt, q, tdist);
                    wave_sync();
                    if (lane < cnt) rd[pos[lane]] = tdist[lane];
                    wave_sync();
                }
                if (xm != ~0ull) break;
            }
        }
    }
}

hipError_t launch_edge_dist_refresh(Storage st, MetricKind mk, const DevGraph& g, const int8_t* levels,
                                    const uint8_t* flags, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!g.adjd0) return hipErrorInvalidValue;
    hipError_t err = hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>(n, 1u << 20);
    dispatch_all<SHAPE_BUILD>(st, mk, g.nchunks, [&](auto sh, auto tt, auto mt) {
        auto kern = VSG_KERNEL_OF(edge_dist_refresh_kernel, sh, tt, mt);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, s, g, levels, flags, (uint32_t)n);
        err = hipGetLastError();
    });
    return err;
}

hipError_t launch_edge_dist_fill(Storage st, MetricKind mk, const DevGraph& g, const int8_t* levels, size_t n,
                                 hipStream_t s) {
    if (n == 0) return hipSuccess;
    // upperd is read only for slots with levels > 0, which exist only when the
    // graph has upper rows (and then ensure_upper allocated it): a graph without
    // upper rows (a small loaded / imported index) has none to fill
    if (!g.adjd0) return hipErrorInvalidValue;
    hipError_t err = hipSuccess;
    dispatch_all<SHAPE_BUILD>(st, mk, g.nchunks, [&](auto sh, auto tt, auto mt) {
        auto kern = VSG_KERNEL_OF(edge_dist_fill_kernel, sh, tt, mt);
        hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(64), 0, s, g, levels, (uint32_t)n);
        err = hipGetLastError();
    });
    return err;
}

// ------------------------------------------------------------------ launch --

bool shape_supported(int nchunks) { return nchunks >= 1 && nchunks <= 1024; }

hipError_t launch_search(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s) {
    if (p.nq <= 0) return hipSuccess;
    // an index with removed entries: usearch's filtered base-level search
    if (p.filt) return launch_search_filt(st, mk, p, s);
    // register kernel up to ef 1024 (multi-entry descent: register kernel only);
    // above it the sorted LDS list (ef <= MAX_EF)
    if ((p.reg && p.ef <= (int)MAX_REG_EF) || p.upper_ef > 1) return launch_search_reg(st, mk, p, s);
    if (p.ef < 1 || p.ef > (int)MAX_EF || p.k > p.ef) return hipErrorInvalidValue;
    // the cooperative kernel stages one 64-entry row piece per expansion: M0 <= 64 only
    const int nw = (p.waves == 2 || p.waves == 4) && p.g.M0 <= 64 ? p.waves : 1;
    const size_t lds = search_lds_bytes(p.ef, p.hash_size, nw);
    hipError_t err = hipSuccess;
    dispatch_all<SHAPE_SEARCH>(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        auto run = [&](auto kern) {
            if (lds > 65536)
                (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            // <= 1M queries per dispatch (<= 256 work-items each: the AQL grid size is 32-bit)
            constexpr int CH = 1 << 20;
            for (int off = 0; off < p.nq && err == hipSuccess; off += CH) {
                SearchParams c = p;
                c.nq = min(CH, p.nq - off);
                c.queries = p.queries + (size_t)off * p.g.row_bytes;
                c.out_keys = p.out_keys + (size_t)off * p.k;
                c.out_dist = p.out_dist + (size_t)off * p.k;
                c.out_counts = p.out_counts ? p.out_counts + off : nullptr;
                hipLaunchKernelGGL(kern, dim3(c.nq), dim3(64 * nw), lds, s, c);
                err = hipGetLastError();
            }
        };
        constexpr int G = decltype(sh)::G, VM = decltype(sh)::VM, U = decltype(sh)::U;
        using T = typename decltype(tt)::T;
        constexpr int MET = decltype(mt)::MET;
        if (nw == 1) run(hnsw_search_kernel<G, VM, U, T, MET>);
        else if (nw == 2) run(hnsw_search_wg_kernel<G, VM, U, T, MET, 2>);
        else run(hnsw_search_wg_kernel<G, VM, U, T, MET, 4>);
    });
    return err;
}

hipError_t launch_insert(Storage st, MetricKind mk, const InsertParams& p, hipStream_t s) {
    if (p.nnodes <= 0) return hipSuccess;
    const size_t lds = insert_lds_bytes(p.efc, p.hash_size, p.g.M0);
    hipError_t err = hipSuccess;
    dispatch_all<SHAPE_BUILD>(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        auto kern = VSG_KERNEL_OF(hnsw_insert_kernel, sh, tt, mt);
        if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(p.nnodes), dim3(64), lds, s, p);
        err = hipGetLastError();
    });
    return err;
}

hipError_t launch_insert_split(Storage st, MetricKind mk, const InsertParams& p, hipStream_t s, hipEvent_t mid) {
    if (p.nnodes <= 0) return hipSuccess;
    if (p.efc > 192 || !p.list_off || !p.lst_d || !p.lst_i || !p.lst_n) return hipErrorInvalidValue;
    const size_t lds_beam = wave_lds_bytes(p.hash_size, p.efc, 0);
    const size_t lds_sel = wave_lds_bytes(0, p.efc, sel_entries(p.g.M0));
    hipError_t err = hipSuccess;
    dispatch_all<SHAPE_BUILD>(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        auto kb = VSG_KERNEL_OF(hnsw_insert_beam_kernel, sh, tt, mt);
        auto ks = VSG_KERNEL_OF(hnsw_insert_select_kernel, sh, tt, mt);
        if (lds_beam > 65536) (void)hipFuncSetAttribute((const void*)kb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_beam);
        hipLaunchKernelGGL(kb, dim3(p.nnodes), dim3(64), lds_beam, s, p);
        err = hipGetLastError();
        if (err == hipSuccess && mid) err = hipEventRecord(mid, s);
        if (err == hipSuccess) {
            hipLaunchKernelGGL(ks, dim3(p.nnodes), dim3(64), lds_sel, s, p);
            err = hipGetLastError();
        }
    });
    return err;
}

hipError_t launch_reverse(Storage st, MetricKind mk, const ReverseParams& p, int grid, hipStream_t s) {
    if (p.npairs == 0) return hipSuccess;
    const int cap = 2 * p.g.M0 > 64 ? 2 * p.g.M0 : 64;
    const size_t lds = insert_lds_bytes(cap, 0, p.g.M0);
    hipError_t err = hipSuccess;
    dispatch_all<SHAPE_BUILD>(st, mk, p.g.nchunks, [&](auto sh, auto tt, auto mt) {
        auto kern = VSG_KERNEL_OF(hnsw_reverse_kernel, sh, tt, mt);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, s, p);
        err = hipGetLastError();
    });
    return err;
}

}  // namespace vsg
