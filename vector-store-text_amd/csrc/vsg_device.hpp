// vsg_device.hpp — wave64 device primitives shared by the HNSW / exact kernels.
//
// Execution model: one wave64 = one workgroup = one query (search)
// or one inserted node (build).  All per-wave state lives in LDS:
//   visited hash (u32, open addressing), a (distance, slot) list sorted
//   lexicographically (double-buffered for merges), candidate scratch.
// Base rows are fetched straight to VGPRs in 16-B chunks: a row is split over
// G lanes (G in {4..64}), each lane holds VM chunks, 64/G rows per pass, U
// passes issued back-to-back before any arithmetic so 8-16 loads per lane are
// in flight; partial sums are reduced across the G lanes (group_sum0: DPP adds).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VSG_EMPTY 0xFFFFFFFFu
#define VSG_EXP_BIT 0x80000000u
// list entry of a removed node (filtered search: traversed, never a result)
#define VSG_REM_BIT 0x40000000u
#define VSG_ID_MASK 0x3FFFFFFFu  // slots < MAX_SLOTS = 2^29

namespace vsg {

enum { MET_L2 = 0, MET_DOT = 1 };

// elements per 16-byte chunk
template <typename T> struct ChunkT;
template <> struct ChunkT<float> { static constexpr int E = 4; };
template <> struct ChunkT<_Float16> { static constexpr int E = 8; };

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));

template <typename T>
__device__ __forceinline__ void load_chunk(const uint8_t* __restrict__ row, int c,
                                           float (&out)[ChunkT<T>::E]) {
    const uint4 raw = *reinterpret_cast<const uint4*>(row + (size_t)c * 16);
    if constexpr (sizeof(T) == 4) {
        out[0] = __uint_as_float(raw.x);
        out[1] = __uint_as_float(raw.y);
        out[2] = __uint_as_float(raw.z);
        out[3] = __uint_as_float(raw.w);
    } else {
        half8_t h = __builtin_bit_cast(half8_t, raw);
#pragma unroll
        for (int e = 0; e < 8; ++e) out[e] = (float)h[e];
    }
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ void wave_sync() {
    // single-wave workgroups: orders this wave's LDS traffic across lanes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// Sum of `a` over each G-lane group, valid in the group's first lane only: the
// value the xor butterfly (offsets G/2, ..., 2, 1) leaves there, bit for bit --
// each step adds lane i + o to lane i for the lanes i < o that still feed lane 0,
// with the same operands in the same order.  The steps inside a 16-lane row are
// DPP modifiers of the adds (row_shl 8 / 4, quad_perm) instead of ds_bpermute
// round trips through the LDS crossbar; 16 is a ds_swizzle (xor within 32
// lanes), 32 one ds_bpermute.  Lanes other than the first hold partial sums.
#ifndef VSG_DPP_REDUCE
#define VSG_DPP_REDUCE 1
#endif
template <int G> __device__ __forceinline__ float group_sum0(float a) {
#if VSG_DPP_REDUCE
    if constexpr (G >= 64) a += __shfl_xor(a, 32);
    if constexpr (G >= 32) a += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(a), 0x401F));
    if constexpr (G >= 16) a += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x108, 0xF, 0xF, true));
    if constexpr (G >= 8) a += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x104, 0xF, 0xF, true));
    if constexpr (G >= 4) a += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x4E, 0xF, 0xF, true));
    if constexpr (G >= 2) a += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0xB1, 0xF, 0xF, true));
#else
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) a += __shfl_xor(a, o);
#endif
    return a;
}

__device__ __forceinline__ bool cand_less(float da, uint32_t ia, float db, uint32_t ib) {
    return da < db || (da == db && ia < ib);
}

__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }

__device__ __forceinline__ int lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

template <typename X> __device__ __forceinline__ X readlane(X x, int l) {
    if constexpr (sizeof(X) == 4) {
        return __builtin_bit_cast(X, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
    } else {
        static_assert(sizeof(X) == 4, "32-bit only");
    }
}

// Lexicographic (d, id) minimum across the wave; result in all lanes.  Exact in
// any order: DPP moves inside each 16-lane row (quad xor 1 / 2, half-row and row
// mirrors), then the four row minima through scalar registers.
template <int CTRL> __device__ __forceinline__ void argmin_dpp_step(float& d, uint32_t& id) {
    const float od = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(d), CTRL, 0xF, 0xF, false));
    const uint32_t oi = (uint32_t)__builtin_amdgcn_mov_dpp((int)id, CTRL, 0xF, 0xF, false);
    if (cand_less(od, oi, d, id)) {
        d = od;
        id = oi;
    }
}
__device__ __forceinline__ void wave_argmin(float& d, uint32_t& id) {
#if VSG_DPP_REDUCE
    argmin_dpp_step<0xB1>(d, id);
    argmin_dpp_step<0x4E>(d, id);
    argmin_dpp_step<0x141>(d, id);
    argmin_dpp_step<0x140>(d, id);
    float bd = readlane(d, 0);
    uint32_t bi = readlane(id, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const float rd = readlane(d, r);
        const uint32_t ri = readlane(id, r);
        if (cand_less(rd, ri, bd, bi)) {
            bd = rd;
            bi = ri;
        }
    }
    d = bd;
    id = bi;
#else
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float od = __shfl_xor(d, o);
        uint32_t oi = (uint32_t)__shfl_xor((int)id, o);
        if (cand_less(od, oi, d, id)) {
            d = od;
            id = oi;
        }
    }
#endif
}

// Query / candidate register image: lane (sub, sl) holds chunks v*G + sl.
template <int G, int VM, typename T> struct QReg {
    static constexpr int E = ChunkT<T>::E;
    float x[VM][E];

    __device__ __forceinline__ void load(const uint8_t* __restrict__ row, int nchunks) {
        const int sl = lane_id() % G;
#pragma unroll
        for (int v = 0; v < VM; ++v) {
            const int c = v * G + sl;
            const int cc = c < nchunks ? c : nchunks - 1;
            load_chunk<T>(row, cc, x[v]);
            if (c >= nchunks) {
#pragma unroll
                for (int e = 0; e < E; ++e) x[v][e] = 0.f;
            }
        }
    }

    // split load: fetch() issues the 16-B loads into `raw` (no use, so no wait),
    // set() converts them later -- lets a row stream in under other work
    __device__ __forceinline__ static void fetch(const uint8_t* __restrict__ row, int nchunks, uint4 (&raw)[VM]) {
        const int sl = lane_id() % G;
#pragma unroll
        for (int v = 0; v < VM; ++v) {
            const int c = v * G + sl;
            const int cc = c < nchunks ? c : nchunks - 1;
            raw[v] = *reinterpret_cast<const uint4*>(row + (size_t)cc * 16);
        }
    }
    __device__ __forceinline__ void set(const uint4 (&raw)[VM], int nchunks) {
        const int sl = lane_id() % G;
#pragma unroll
        for (int v = 0; v < VM; ++v) {
            const int c = v * G + sl;
            if constexpr (sizeof(T) == 4) {
                x[v][0] = __uint_as_float(raw[v].x);
                x[v][1] = __uint_as_float(raw[v].y);
                x[v][2] = __uint_as_float(raw[v].z);
                x[v][3] = __uint_as_float(raw[v].w);
            } else {
                half8_t h = __builtin_bit_cast(half8_t, raw[v]);
#pragma unroll
                for (int e = 0; e < 8; ++e) x[v][e] = (float)h[e];
            }
            if (c >= nchunks) {
#pragma unroll
                for (int e = 0; e < E; ++e) x[v][e] = 0.f;
            }
        }
    }
};

// 16-B chunk -> E floats (f16 converted exactly to f32)
template <typename T>
__device__ __forceinline__ void unpack_chunk(const uint4 raw, float (&out)[ChunkT<T>::E]) {
    if constexpr (sizeof(T) == 4) {
        out[0] = __uint_as_float(raw.x);
        out[1] = __uint_as_float(raw.y);
        out[2] = __uint_as_float(raw.z);
        out[3] = __uint_as_float(raw.w);
    } else {
        half8_t h = __builtin_bit_cast(half8_t, raw);
#pragma unroll
        for (int e = 0; e < 8; ++e) out[e] = (float)h[e];
    }
}

// One element of the metric sum, a single FMA: (x - q)^2 + acc for l2sq, x q + acc
// for the dot products.  Chunks past the row's end (lanes of a partial shape)
// add nothing: every register image (QReg::load / set) is zero there, so a dot
// term is x * 0, and an l2sq term reads a row chunk zeroed first (mask_tail).
template <int MET> __device__ __forceinline__ float metric_fma(float x, float q, float acc) {
    if constexpr (MET == MET_L2) {
        const float df = x - q;
        return __builtin_fmaf(df, df, acc);
    } else {
        return __builtin_fmaf(x, q, acc);
    }
}
// l2sq on a partial row shape (G * VM > nchunks): the clamped loads of the lanes
// past the end repeat the last chunk, so zero them (once per row chunk, not per
// term); a dot product needs nothing (its register image is zero there).
template <int G, int VM, int MET>
__device__ __forceinline__ void mask_tail(uint4 (&raw)[VM], int nchunks, int sl) {
    if constexpr (MET == MET_L2) {
        if (G * VM != nchunks) {
#pragma unroll
            for (int v = 0; v < VM; ++v)
                if (v * G + sl >= nchunks) raw[v] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
}

// Distances from the register image q to `count` rows listed in ids[] (LDS),
// written to out[] (LDS).  Wave-uniform count.  out[r] holds the metric
// distance (l2sq, or 1 - dot).  All U x VM chunk loads of a pass are issued
// before any arithmetic and kept as raw 16-B words (4 VGPRs each; f16 rows are
// widened to f32 only when consumed), so the loads in flight cost half the
// registers for f16 rows.  A pass whose rows all lie past `count` is skipped
// (the last round of a call is mostly short: ~19 fresh rows of a C4 expansion
// filled 2.4 of the 4 passes of 8 rows, and the other 1.6 used to load and
// reduce copies of the last row -- 40 % of the distance VALU; round 6).
// Search-profile clock (shader cycles, s_memtime; the make prof build only).
#ifdef VSG_SEARCH_PROFILE
#define VSG_CYC() __builtin_amdgcn_s_memtime()
#else
#define VSG_CYC() 0ull
#endif
// rows_dist's share of a profiled expansion: cycles waiting for the row loads
// of each pass (an explicit vmcnt(0) after the pass is issued) and in its VALU.
struct RowsProf {
    uint64_t wait = 0, valu = 0;
    uint32_t passes = 0;
};

// Loads of a pass past `count` are skipped only for rows of <= 512 B: with a
// conditional load the compiler can no longer count the loads in flight, so the
// first pass's arithmetic waits for every pass's loads (vmcnt(0)); long rows lose
// that overlap (C2 512 queries 0.52 -> 0.547 ms), short rows gain more from the
// skipped loads than they lose (C4 shard ef 192 3.10 -> 2.87 ms; round 6).
template <int G, int VM> constexpr bool kSkipLoads() { return G * VM * 16 <= 512; }

template <int G, int VM, int U, typename T, int MET>
__device__ __forceinline__ void rows_dist(const uint8_t* __restrict__ vecs, size_t row_bytes,
                                          int nchunks, const uint32_t* ids, int count,
                                          const QReg<G, VM, T>& q, float* out, RowsProf* rp = nullptr) {
    constexpr int R = 64 / G;
    constexpr int E = ChunkT<T>::E;
    const int lane = lane_id();
    const int sub = lane / G;
    const int sl = lane % G;
    (void)rp;
    for (int base = 0; base < count; base += R * U) {
        uint4 raw[U][VM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (kSkipLoads<G, VM>() && base + u * R >= count) break;  // wave-uniform: no row listed
            const int r = base + u * R + sub;
            const int rr = r < count ? r : count - 1;
            const uint8_t* row = vecs + (size_t)ids[rr] * row_bytes;
#pragma unroll
            for (int v = 0; v < VM; ++v) {
                const int c = v * G + sl;
                raw[u][v] = *reinterpret_cast<const uint4*>(row + (size_t)(c < nchunks ? c : nchunks - 1) * 16);
            }
        }
#ifdef VSG_SEARCH_PROFILE
        uint64_t tp = 0;
        if (rp) {
            tp = VSG_CYC();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t tw = VSG_CYC();
            rp->wait += tw - tp;
            rp->passes++;
            tp = tw;
        }
#endif
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (base + u * R >= count) break;
            float acc = 0.f;
            mask_tail<G, VM, MET>(raw[u], nchunks, sl);
#pragma unroll
            for (int v = 0; v < VM; ++v) {
                float x[E];
                unpack_chunk<T>(raw[u][v], x);
#pragma unroll
                for (int e = 0; e < E; ++e) acc = metric_fma<MET>(x[e], q.x[v][e], acc);
            }
            acc = group_sum0<G>(acc);
            const int r = base + u * R + sub;
            if (sl == 0 && r < count) out[r] = (MET == MET_L2) ? acc : 1.f - acc;
        }
#ifdef VSG_SEARCH_PROFILE
        if (rp) rp->valu += VSG_CYC() - tp;
#endif
    }
}

// rows_dist for two register images at once: each row is loaded once and
// reduced against both (out0 from q0, out1 from q1; same values as two
// rows_dist calls).
template <int G, int VM, int U, typename T, int MET>
__device__ __forceinline__ void rows_dist2(const uint8_t* __restrict__ vecs, size_t row_bytes, int nchunks,
                                           const uint32_t* ids, int count, const QReg<G, VM, T>& q0,
                                           const QReg<G, VM, T>& q1, float* out0, float* out1) {
    constexpr int R = 64 / G;
    constexpr int E = ChunkT<T>::E;
    const int lane = lane_id();
    const int sub = lane / G;
    const int sl = lane % G;
    for (int base = 0; base < count; base += R * U) {
        uint4 raw[U][VM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (kSkipLoads<G, VM>() && base + u * R >= count) break;  // wave-uniform: no row listed
            const int r = base + u * R + sub;
            const int rr = r < count ? r : count - 1;
            const uint8_t* row = vecs + (size_t)ids[rr] * row_bytes;
#pragma unroll
            for (int v = 0; v < VM; ++v) {
                const int c = v * G + sl;
                raw[u][v] = *reinterpret_cast<const uint4*>(row + (size_t)(c < nchunks ? c : nchunks - 1) * 16);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (base + u * R >= count) break;
            float a0 = 0.f, a1 = 0.f;
            mask_tail<G, VM, MET>(raw[u], nchunks, sl);
#pragma unroll
            for (int v = 0; v < VM; ++v) {
                float x[E];
                unpack_chunk<T>(raw[u][v], x);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    a0 = metric_fma<MET>(x[e], q0.x[v][e], a0);
                    a1 = metric_fma<MET>(x[e], q1.x[v][e], a1);
                }
            }
            a0 = group_sum0<G>(a0);
            a1 = group_sum0<G>(a1);
            const int r = base + u * R + sub;
            if (sl == 0 && r < count) {
                out0[r] = (MET == MET_L2) ? a0 : 1.f - a0;
                out1[r] = (MET == MET_L2) ? a1 : 1.f - a1;
            }
        }
    }
}

// The heuristic selection's test for NQ register-held candidates at once: bit j
// of the result is set if some listed row r has dist(q[j], r) < lim[j].  Each
// row is loaded once for all NQ candidates; distances are the values rows_dist
// computes (same per-lane order and shuffle tree), reduced to a ballot instead
// of an LDS write.  Wave-uniform count.
template <int NQ, int G, int VM, int U, typename T, int MET>
__device__ __forceinline__ uint32_t rows_test(const uint8_t* __restrict__ vecs, size_t row_bytes, int nchunks,
                                              const uint32_t* ids, int count, const QReg<G, VM, T> (&q)[NQ],
                                              const float (&lim)[NQ]) {
    constexpr int R = 64 / G;
    constexpr int E = ChunkT<T>::E;
    const int lane = lane_id();
    const int sub = lane / G;
    const int sl = lane % G;
    uint32_t hit = 0;
    for (int base = 0; base < count; base += R * U) {
        uint4 raw[U][VM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (kSkipLoads<G, VM>() && base + u * R >= count) break;  // wave-uniform: no row listed
            const int r = base + u * R + sub;
            const int rr = r < count ? r : count - 1;
            const uint8_t* row = vecs + (size_t)ids[rr] * row_bytes;
#pragma unroll
            for (int v = 0; v < VM; ++v) {
                const int c = v * G + sl;
                raw[u][v] = *reinterpret_cast<const uint4*>(row + (size_t)(c < nchunks ? c : nchunks - 1) * 16);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (base + u * R >= count) break;
            float a[NQ];
#pragma unroll
            for (int j = 0; j < NQ; ++j) a[j] = 0.f;
            mask_tail<G, VM, MET>(raw[u], nchunks, sl);
#pragma unroll
            for (int v = 0; v < VM; ++v) {
                float x[E];
                unpack_chunk<T>(raw[u][v], x);
#pragma unroll
                for (int e = 0; e < E; ++e) {
#pragma unroll
                    for (int j = 0; j < NQ; ++j) a[j] = metric_fma<MET>(x[e], q[j].x[v][e], a[j]);
                }
            }
            const int r = base + u * R + sub;
            const bool ok = sl == 0 && r < count;
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                a[j] = group_sum0<G>(a[j]);
                const float d = (MET == MET_L2) ? a[j] : 1.f - a[j];
                if (__ballot(ok && d < lim[j])) hit |= 1u << j;
            }
        }
    }
    return hit;
}

// Distance between two register images (candidate vs. an already kept candidate
// of the same selection block): the value rows_dist gives for row b, query a.
template <int G, int VM, typename T, int MET>
__device__ __forceinline__ float reg_dist(const QReg<G, VM, T>& a, const QReg<G, VM, T>& b, int nchunks) {
    constexpr int E = ChunkT<T>::E;
    const int sl = lane_id() % G;
    float acc = 0.f;
    (void)sl;
    (void)nchunks;  // both images are zero past the row's end
#pragma unroll
    for (int v = 0; v < VM; ++v) {
#pragma unroll
        for (int e = 0; e < E; ++e) acc = metric_fma<MET>(b.x[v][e], a.x[v][e], acc);
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    return (MET == MET_L2) ? acc : 1.f - acc;
}

// ----------------------------------------------------------------- visited --

struct Visited {
    uint32_t* tab;
    uint32_t size;  // entries (multiple of 8; buckets via multiply-high)

    __device__ __forceinline__ void clear() {
        const int lane = lane_id();
        uint4* t4 = reinterpret_cast<uint4*>(tab);
        const uint32_t n4 = size / 4;
        for (uint32_t i = lane; i < n4; i += 64) t4[i] = make_uint4(VSG_EMPTY, VSG_EMPTY, VSG_EMPTY, VSG_EMPTY);
        wave_sync();
    }

    // true if id was not present (it is recorded now).  The id's home is an
    // aligned bucket of 8 slots, read with two 16-B LDS loads; a free slot is
    // claimed with one CAS (re-read if another lane took it).  A table that is
    // too small forgets: a full bucket overwrites one of its ids (slot chosen
    // by the new id) and `evicted` is set; from then on the caller must treat
    // every fresh id as possibly seen before and de-duplicate against the
    // top-ef set.  Forgetting never changes the traversal, it only adds
    // distance evaluations: a node seen before is either still in the top-ef
    // set (de-duplicated there) or worse than its current worst entry
    // (rejected by the admission threshold; entries only leave a full set).
    // One LDS round trip + one atomic per id (linear probing needed up to 16
    // dependent atomics once the table was crowded: profiles/r01_search_phases.jsonl).
    __device__ __forceinline__ bool insert(uint32_t id, bool& evicted) {
        const uint32_t b0 = __umulhi(id * 2654435761u, size >> 3) << 3;
        const uint4* t4 = reinterpret_cast<const uint4*>(tab + b0);
        evicted = false;
#pragma unroll 1
        for (int attempt = 0; attempt < 8; ++attempt) {
            const uint4 x = t4[0], y = t4[1];
            const uint32_t v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
            int fs = -1;
            bool hit = false;
#pragma unroll
            for (int i = 7; i >= 0; --i) {
                hit = hit || v[i] == id;
                if (v[i] == VSG_EMPTY) fs = i;
            }
            if (hit) return false;
            if (fs < 0) break;
            const uint32_t old = atomicCAS(&tab[b0 + fs], VSG_EMPTY, id);
            if (old == VSG_EMPTY) return true;
            if (old == id) return false;
        }
        atomicExch(&tab[b0 + (id & 7)], id);
        evicted = true;
        return true;
    }

    // lookup only: !insert() without recording
    __device__ __forceinline__ bool contains(uint32_t id) const {
        const uint32_t b0 = __umulhi(id * 2654435761u, size >> 3) << 3;
        const uint4* t4 = reinterpret_cast<const uint4*>(tab + b0);
        const uint4 x = t4[0], y = t4[1];
        return x.x == id || x.y == id || x.z == id || x.w == id || y.x == id || y.y == id || y.z == id || y.w == id;
    }
};

// ------------------------------------------------------------- sorted list --
// (distance, slot) ascending; slot high bit = "expanded", bit 30 = removed node
// (filtered search).  cap <= MAX_EF (4096), 8192 for the filtered search.

struct List {
    float* d0;
    float* d1;
    uint32_t* i0;
    uint32_t* i1;
    int cur;
    int size;
    int cap;

    // explicit selects: a runtime-indexed pointer array would live in scratch
    __device__ __forceinline__ float* D() const { return cur ? d1 : d0; }
    __device__ __forceinline__ uint32_t* I() const { return cur ? i1 : i0; }
    __device__ __forceinline__ float* Dn() const { return cur ? d0 : d1; }
    __device__ __forceinline__ uint32_t* In() const { return cur ? i0 : i1; }

    // first entry not yet expanded, or -1 (entries below `start` are known to
    // be expanded)
    __device__ __forceinline__ int first_unexpanded(int start = 0) const {
        const int lane = lane_id();
        for (int r = start; r < size; r += 64) {
            const int i = r + lane;
            const bool un = i < size && !(I()[i] & VSG_EXP_BIT);
            const uint64_t m = __ballot(un);
            if (m) return r + __builtin_ctzll(m);
        }
        return -1;
    }

    // #entries strictly less than (cd, ci), binary search in LDS
    __device__ __forceinline__ int lower_bound(float cd, uint32_t ci) const {
        int lo = 0, hi = size;
        const float* dd = D();
        const uint32_t* ii = I();
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cand_less(dd[mid], ii[mid] & VSG_ID_MASK, cd, ci)) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }

    // Merge one candidate per lane (valid lanes only).  Candidates must have
    // distinct ids that are not in the list unless `maybe_dup` is set for them.
    // sd/si: 64-entry LDS scratch.  Returns the lowest position a candidate
    // took (entries below it are unchanged), or INT_MAX if none was placed.
    // cflag: bits stored with this lane's entry (VSG_REM_BIT; never compared).
    __device__ int merge(bool valid, float cd, uint32_t ci, bool maybe_dup, float* sd, uint32_t* si,
                         uint32_t cflag = 0) {
        const int lane = lane_id();
        if (valid && size == cap) {
            const float wd = D()[size - 1];
            const uint32_t wi = I()[size - 1] & VSG_ID_MASK;
            valid = cand_less(cd, ci, wd, wi);
        }
        if (valid && maybe_dup) {
            const int p = lower_bound(cd, ci);
            if (p < size && D()[p] == cd && (I()[p] & VSG_ID_MASK) == ci) valid = false;
        }
        const uint64_t mask = __ballot(valid);
        const int nc = popc64(mask);
        if (nc == 0) return 0x7fffffff;
        // rank among candidates
        int rank = 0;
        for (uint64_t m = mask; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            const float dj = readlane(cd, j);
            const uint32_t ij = readlane(ci, j);
            rank += cand_less(dj, ij, cd, ci) ? 1 : 0;
        }
        if (valid) {
            sd[rank] = cd;
            si[rank] = ci;
        }
        const int pos_new = valid ? rank + lower_bound(cd, ci) : 0;
        const int first = readlane(pos_new, __builtin_ctzll(__ballot(valid && rank == 0)));
        wave_sync();
        float* dd = D();
        uint32_t* ii = I();
        float* nd = Dn();
        uint32_t* ni = In();
        // existing entries shift by #candidates below them
        for (int e = lane; e < size; e += 64) {
            const float ed = dd[e];
            const uint32_t ei = ii[e];
            int lo = 0, hi = nc;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (cand_less(sd[mid], si[mid], ed, ei & VSG_ID_MASK)) lo = mid + 1;
                else hi = mid;
            }
            const int p = e + lo;
            if (p < cap) {
                nd[p] = ed;
                ni[p] = ei;
            }
        }
        if (valid && pos_new < cap) {
            nd[pos_new] = cd;
            ni[pos_new] = ci | cflag;
        }
        size = min(size + nc, cap);
        cur ^= 1;
        wave_sync();
        return first;
    }

    // merge() split for a multi-wave workgroup sharing this list (every wave
    // holds an identical copy of cur / size).  place(): ONE wave filters and
    // ranks its candidates, writes them sorted to sd/si and into the next
    // buffer, and returns nc (wave-uniform).  After a workgroup barrier, every
    // thread of the group calls shift() (existing entries -> next buffer), then
    // advance(nc) and another barrier.  Same result as merge().
    __device__ int place(bool valid, float cd, uint32_t ci, bool maybe_dup, float* sd, uint32_t* si) const {
        if (valid && size == cap) {
            const float wd = D()[size - 1];
            const uint32_t wi = I()[size - 1] & VSG_ID_MASK;
            valid = cand_less(cd, ci, wd, wi);
        }
        if (valid && maybe_dup) {
            const int p = lower_bound(cd, ci);
            if (p < size && D()[p] == cd && (I()[p] & VSG_ID_MASK) == ci) valid = false;
        }
        const uint64_t mask = __ballot(valid);
        const int nc = popc64(mask);
        if (nc == 0) return 0;
        int rank = 0;
        for (uint64_t m = mask; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            rank += cand_less(readlane(cd, j), readlane(ci, j), cd, ci) ? 1 : 0;
        }
        if (valid) {
            sd[rank] = cd;
            si[rank] = ci;
            const int pos_new = rank + lower_bound(cd, ci);
            if (pos_new < cap) {
                Dn()[pos_new] = cd;
                In()[pos_new] = ci;
            }
        }
        return nc;
    }

    __device__ void shift(int nc, const float* sd, const uint32_t* si, int tid, int nthreads) const {
        const float* dd = D();
        const uint32_t* ii = I();
        float* nd = Dn();
        uint32_t* ni = In();
        for (int e = tid; e < size; e += nthreads) {
            const float ed = dd[e];
            const uint32_t ei = ii[e];
            int lo = 0, hi = nc;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (cand_less(sd[mid], si[mid], ed, ei & VSG_ID_MASK)) lo = mid + 1;
                else hi = mid;
            }
            const int p = e + lo;
            if (p < cap) {
                nd[p] = ed;
                ni[p] = ei;
            }
        }
    }

    __device__ __forceinline__ void advance(int nc) {
        if (nc == 0) return;
        size = min(size + nc, cap);
        cur ^= 1;
    }
};

// ----------------------------------------------------------- graph access --

struct GraphDev {
    const uint8_t* vecs;
    size_t row_bytes;
    int nchunks;
    uint32_t* adj0;
    const uint32_t* upper_off;
    uint32_t* upper;
    int M, M0;
    float* adjd0;   // per-edge distances (build kernels; nullptr otherwise)
    float* upperd;

    __device__ __forceinline__ uint32_t* row(uint32_t s, int l) const {
        return l == 0 ? adj0 + (size_t)s * M0 : upper + ((size_t)upper_off[s] + (size_t)(l - 1)) * M;
    }
    // the distances of row(s, l)'s entries (same layout)
    __device__ __forceinline__ float* rowd(uint32_t s, int l) const {
        return l == 0 ? adjd0 + (size_t)s * M0 : upperd + ((size_t)upper_off[s] + (size_t)(l - 1)) * M;
    }
    __device__ __forceinline__ const uint8_t* vec(uint32_t s) const { return vecs + (size_t)s * row_bytes; }
};

}  // namespace vsg
