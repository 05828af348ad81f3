// hnsw_common.hpp — per-wave search state and the descent shared by the HNSW
// kernels (hnsw.hip: list search, build; hnsw_search_reg.hip: register search).
#pragma once
#include <hip/hip_runtime.h>

#include "vsg_device.hpp"
#include "vsg_kernels.hpp"

namespace vsg {

static inline __host__ __device__ size_t wave_lds_bytes(int hash, int cap, bool with_sel) {
    return (size_t)hash * 4 + (size_t)cap * 16 + 64 * 4 * 4 + (with_sel ? 64 * 4 * 2 : 0);
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

static __device__ inline WaveLds carve(uint8_t* smem, int cap, int hs, bool with_sel) {
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
    if (with_sel) {
        w.sel = reinterpret_cast<uint32_t*>(p);
        p += 256;
        w.seld = reinterpret_cast<float*>(p);
        p += 256;
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
// neighbour (lexicographic (distance, slot)) until none improves.
template <int G, int VM, int U, typename T, int MET>
__device__ void greedy_level(const GraphDev& g, const QReg<G, VM, T>& q, int l, uint32_t& cur,
                             float& dcur, WaveLds& w, uint64_t& ndist, uint64_t& nadj) {
    const int lane = lane_id();
    const int m = l == 0 ? g.M0 : g.M;
    for (;;) {
        const uint32_t* row = g.row(cur, l);
        const uint32_t nb = lane < m ? row[lane] : VSG_EMPTY;
        const bool ok = nb != VSG_EMPTY;
        const uint64_t mask = __ballot(ok);
        const int cnt = popc64(mask);
        ++nadj;
        if (ok) w.todo[lanes_below(mask)] = nb;
        wave_sync();
        if (cnt == 0) break;
        rows_dist<G, VM, U, T, MET>(g.vecs, g.row_bytes, g.nchunks, w.todo, cnt, q, w.tdist);
        wave_sync();
        ndist += (uint64_t)cnt;
        float d = lane < cnt ? w.tdist[lane] : __builtin_inff();
        uint32_t id = lane < cnt ? w.todo[lane] : VSG_EMPTY;
        wave_sync();
        wave_argmin(d, id);
        if (cand_less(d, id, dcur, cur)) {
            cur = id;
            dcur = d;
        } else {
            break;
        }
    }
}

// Search-phase clocks (100 MHz wall clock), summed per wave into stats[10..13]
// when built with -DVSG_SEARCH_PROFILE (tools only; zero cost otherwise).
struct BeamProf {
    uint64_t adj = 0, dist = 0, merge = 0;
};
#ifdef VSG_SEARCH_PROFILE
#define VSG_CLK() wall_clock64()
#else
#define VSG_CLK() 0ull
#endif

}  // namespace vsg
