// hnsw_common.hpp — per-wave search state and the descent shared by the HNSW
// kernels (hnsw.hip: list search, build; hnsw_search_reg.hip: register search).
#pragma once
#include <hip/hip_runtime.h>

#include "vsg_device.hpp"
#include "vsg_kernels.hpp"

namespace vsg {

// sel: entries of the heuristic-selection output (0 = none; >= M0 for the build)
static inline __host__ __device__ int sel_entries(int m0) { return m0 > 64 ? m0 : 64; }
static inline __host__ __device__ size_t wave_lds_bytes(int hash, int cap, int sel) {
    return (size_t)hash * 4 + (size_t)cap * 16 + 64 * 4 * 4 + (size_t)sel * 4 * 2;
}

static __device__ inline GraphDev to_dev(const DevGraph& g) {
    GraphDev d;
    d.vecs = g.vecs;
    d.row_bytes = g.row_bytes;
    d.nchunks = g.nchunks;
    d.adj0 = g.adj0;
    d.upper_off = g.upper_off;
    d.upper = g.upper;
    d.M = g.M;
    d.M0 = g.M0;
    d.adjd0 = g.adjd0;
    d.upperd = g.upperd;
    return d;
}

struct WaveLds {
    Visited vis;
    List list;
    float* sd;
    uint32_t* si;
    uint32_t* todo;
    float* tdist;
    uint32_t* sel;
    float* seld;
};

static __device__ inline WaveLds carve(uint8_t* smem, int cap, int hs, int sel) {
    WaveLds w;
    uint8_t* p = smem;
    w.vis.tab = reinterpret_cast<uint32_t*>(p);
    w.vis.size = (uint32_t)hs;
    p += (size_t)hs * 4;
    w.list.d0 = reinterpret_cast<float*>(p);
    p += (size_t)cap * 4;
    w.list.d1 = reinterpret_cast<float*>(p);
    p += (size_t)cap * 4;
    w.list.i0 = reinterpret_cast<uint32_t*>(p);
    p += (size_t)cap * 4;
    w.list.i1 = reinterpret_cast<uint32_t*>(p);
    p += (size_t)cap * 4;
    w.list.cap = cap;
    w.list.cur = 0;
    w.list.size = 0;
    w.sd = reinterpret_cast<float*>(p);
    p += 256;
    w.si = reinterpret_cast<uint32_t*>(p);
    p += 256;
    w.todo = reinterpret_cast<uint32_t*>(p);
    p += 256;
    w.tdist = reinterpret_cast<float*>(p);
    p += 256;
    if (sel) {
        w.sel = reinterpret_cast<uint32_t*>(p);
        p += (size_t)sel * 4;
        w.seld = reinterpret_cast<float*>(p);
        p += (size_t)sel * 4;
    } else {
        w.sel = nullptr;
        w.seld = nullptr;
    }
    return w;
}

// distance from q to a single slot (result in all lanes)
template <int G, int VM, int U, typename T, int MET>
__device__ inline float dist_one(const GraphDev& g, const QReg<G, VM, T>& q, uint32_t s, WaveLds& w) {
    if (lane_id() == 0) w.todo[0] = s;
    wave_sync();
    rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, 1, q, w.tdist);
    wave_sync();
    const float d = w.tdist[0];
    wave_sync();
    return d;
}

// usearch search_for_one_ restated (oracle greedy()): move to the best
// neighbour (lexicographic (distance, slot)) until none improves.  Rows longer
// than a wave (M0 = 2M > 64, M <= 64) are read in 64-entry pieces; rows are a
// compact prefix, so a piece that ends in EMPTY ends the row (oracle read_row).
// self: the node being (re)linked by an insert, never its own candidate (a
// reused slot is reachable through other nodes' kept links; oracle greedy());
// VSG_EMPTY in searches.
template <int G, int VM, int U, typename T, int MET>
__device__ void greedy_level(const GraphDev& g, const QReg<G, VM, T>& q, int l, uint32_t& cur,
                             float& dcur, WaveLds& w, uint64_t& ndist, uint64_t& nadj, uint32_t self = VSG_EMPTY) {
    const int lane = lane_id();
    const int m = l == 0 ? g.M0 : g.M;
    for (;;) {
        const uint32_t* row = g.row(cur, l);
        float d = __builtin_inff();
        uint32_t id = VSG_EMPTY;
        ++nadj;
        for (int c0 = 0; c0 < m; c0 += 64) {
            const uint32_t nb = c0 + lane < m ? row[c0 + lane] : VSG_EMPTY;
            const uint64_t pm = __ballot(nb != VSG_EMPTY);  // the row's entries in this piece
            const bool ok = nb != VSG_EMPTY && nb != self;
            const uint64_t mask = __ballot(ok);
            const int cnt = popc64(mask);
            if (ok) w.todo[lanes_below(mask)] = nb;
            wave_sync();
            if (pm == 0) break;
            if (cnt) {
                rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
                wave_sync();
                ndist += (uint64_t)cnt;
                const float cd = lane < cnt ? w.tdist[lane] : __builtin_inff();
                const uint32_t ci = lane < cnt ? w.todo[lane] : VSG_EMPTY;
                if (cand_less(cd, ci, d, id)) {
                    d = cd;
                    id = ci;
                }
                wave_sync();
            }
            if (pm != ~0ull) break;  // compact prefix: the row ended inside this piece
        }
        wave_argmin(d, id);
        if (id != VSG_EMPTY && cand_less(d, id, dcur, cur)) {
            cur = id;
            dcur = d;
        } else {
            break;
        }
    }
}

// Search-phase clocks (100 MHz wall clock), summed per wave into stats[10..13]
// when built with -DVSG_SEARCH_PROFILE (tools only; zero cost otherwise).
// The register beam also splits each expansion into shader-clock cycles
// (s_memtime) summed into stats[20..31] (hnsw_search_reg.hip): picking the next
// node, the adjacency-row wait, the visited-table inserts, the row-load wait and
// the distance VALU of rows_dist, admission and compaction.
struct BeamProf {
    uint64_t adj = 0, dist = 0, merge = 0;
    uint64_t c_sel = 0, c_adj = 0, c_vis = 0, c_admit = 0, c_comp = 0, c_desc = 0;
    uint32_t nexp = 0, ncomp = 0;
    RowsProf rows;
};
#ifdef VSG_SEARCH_PROFILE
#define VSG_CLK() wall_clock64()
#else
#define VSG_CLK() 0ull
#endif

}  // namespace vsg
