// rerank.hip — f16 traversal with exact f32 re-rank (opt-in, vsg_index_set_f16_traversal).
//
// The HNSW search (same kernels, same graph) walks an f16 copy of the f32
// image, so every distance evaluation of the traversal reads half the bytes
// (C2: 1.5 KB instead of 3 KB per row) -- the traversal is bound by row-gather
// bandwidth.  Its final beam (ef slots) is then re-scored here
// against the f32 image with the same distance code as the f32 search
// (rows_dist, f32 shape), and the best k by (distance, slot) are returned, so
// every returned distance is the exact f32 metric value.  Which nodes are
// found can differ from an f32 traversal (f16 rounding reorders near-ties
// inside the beam); recall is measured, not assumed (bench.py
// `f16_traversal_rerank`, tests/test_gpu_parity.py).  usearch has no such
// mode: the reference path (src/index/usearch.rs:275-277) is the f32 search.
#include <hip/hip_runtime.h>

#include "vsg_dispatch.hpp"

namespace vsg {

constexpr int RERANK_MAX = 1024;

template <int G, int VM, int U, int MET>
__global__ __launch_bounds__(64) void rerank_kernel(RerankParams p) {
    __shared__ uint32_t ids[RERANK_MAX];
    __shared__ float dist[RERANK_MAX];
    const int qi = blockIdx.x;
    const int lane = lane_id();
    const uint64_t* cand = p.cand + (size_t)qi * p.kc;
    const int n = min((int)p.cand_counts[qi], p.kc);
    for (int j = lane; j < n; j += 64) ids[j] = (uint32_t)cand[j];
    wave_sync();
    if (n > 0) {
        QReg<G, VM, float> q;
        q.load(p.queries + (size_t)qi * p.row_bytes, p.nchunks);
        rows_dist<G, VM, U, float, MET>(p.vecs, p.row_bytes, p.nchunks, ids, n, q, dist);
    }
    wave_sync();
    // rank of each candidate under (distance, slot); slots are distinct, so
    // ranks are a permutation and the best k land at positions 0..k-1
    const int kk = min(n, p.k);
    uint64_t* ok = p.out_keys + (size_t)qi * p.k;
    float* od = p.out_dist + (size_t)qi * p.k;
    for (int j = lane; j < n; j += 64) {
        const float dj = dist[j];
        const uint32_t ij = ids[j];
        int rank = 0;
        for (int i = 0; i < n; ++i) rank += cand_less(dist[i], ids[i], dj, ij) ? 1 : 0;
        if (rank < kk) {
            ok[rank] = p.keys[ij];
            od[rank] = dj;
        }
    }
    for (int j = kk + lane; j < p.k; j += 64) {
        ok[j] = ~0ull;
        od[j] = __builtin_inff();
    }
    if (lane == 0 && p.out_counts) p.out_counts[qi] = (uint32_t)kk;
}

hipError_t launch_rerank(MetricKind mk, const RerankParams& p, hipStream_t s) {
    if (p.nq <= 0) return hipSuccess;
    if (p.kc < 1 || p.kc > RERANK_MAX || p.k < 1 || p.k > p.kc) return hipErrorInvalidValue;
    hipError_t err = hipSuccess;
    dispatch_all(ST_F32, mk, p.nchunks, [&](auto sh, auto, auto mt) {
        constexpr int G = decltype(sh)::G, VM = decltype(sh)::VM, U = decltype(sh)::U;
        constexpr int MET = decltype(mt)::MET;
        constexpr int CH = 1 << 22;
        for (int off = 0; off < p.nq && err == hipSuccess; off += CH) {
            RerankParams c = p;
            c.nq = min(CH, p.nq - off);
            c.queries = p.queries + (size_t)off * p.row_bytes;
            c.cand = p.cand + (size_t)off * p.kc;
            c.cand_counts = p.cand_counts + off;
            c.out_keys = p.out_keys + (size_t)off * p.k;
            c.out_dist = p.out_dist + (size_t)off * p.k;
            c.out_counts = p.out_counts ? p.out_counts + off : nullptr;
            hipLaunchKernelGGL((rerank_kernel<G, VM, U, MET>), dim3(c.nq), dim3(64), 0, s, c);
            err = hipGetLastError();
        }
    });
    return err;
}

// one work-item per 16-B f16 chunk (8 elements); elements >= dim are zero
__global__ __launch_bounds__(256) void shadow_f16_kernel(const uint8_t* __restrict__ vecs, size_t row_bytes,
                                                         size_t r0, size_t r1, int dim, uint8_t* __restrict__ out,
                                                         size_t row_bytes16) {
    const size_t nc = row_bytes16 / 16;
    const size_t tot = (r1 - r0) * nc;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = r0 + i / nc;
        const int c = (int)(i % nc);
        const float* src = reinterpret_cast<const float*>(vecs + r * row_bytes);
        half8_t h;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int j = c * 8 + e;
            h[e] = (_Float16)(j < dim ? src[j] : 0.f);
        }
        *reinterpret_cast<uint4*>(out + r * row_bytes16 + (size_t)c * 16) = __builtin_bit_cast(uint4, h);
    }
}

hipError_t launch_shadow_f16(const uint8_t* vecs, size_t row_bytes, size_t r0, size_t r1, int dim, uint8_t* out,
                             size_t row_bytes16, hipStream_t s) {
    if (r1 <= r0) return hipSuccess;
    const size_t tot = (r1 - r0) * (row_bytes16 / 16);
    const unsigned grid = (unsigned)std::min<size_t>((tot + 255) / 256, 1u << 20);
    hipLaunchKernelGGL(shadow_f16_kernel, dim3(grid), dim3(256), 0, s, vecs, row_bytes, r0, r1, dim, out,
                       row_bytes16);
    return hipGetLastError();
}

// the f16 copy of listed rows only (rows rewritten in place by a slot-reusing add)
__global__ __launch_bounds__(256) void shadow_f16_slots_kernel(const uint8_t* __restrict__ vecs, size_t row_bytes,
                                                               const uint32_t* __restrict__ slots, size_t n,
                                                               size_t limit, int dim, uint8_t* __restrict__ out,
                                                               size_t row_bytes16) {
    const size_t nc = row_bytes16 / 16;
    const size_t tot = n * nc;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = slots[i / nc];
        if (r >= limit) continue;  // beyond the converted rows: the next incremental pass covers it
        const int c = (int)(i % nc);
        const float* src = reinterpret_cast<const float*>(vecs + r * row_bytes);
        half8_t h;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int j = c * 8 + e;
            h[e] = (_Float16)(j < dim ? src[j] : 0.f);
        }
        *reinterpret_cast<uint4*>(out + r * row_bytes16 + (size_t)c * 16) = __builtin_bit_cast(uint4, h);
    }
}

hipError_t launch_shadow_f16_slots(const uint8_t* vecs, size_t row_bytes, const uint32_t* slots, size_t n,
                                   size_t limit, int dim, uint8_t* out, size_t row_bytes16, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t tot = n * (row_bytes16 / 16);
    const unsigned grid = (unsigned)std::min<size_t>((tot + 255) / 256, 1u << 20);
    hipLaunchKernelGGL(shadow_f16_slots_kernel, dim3(grid), dim3(256), 0, s, vecs, row_bytes, slots, n, limit, dim,
                       out, row_bytes16);
    return hipGetLastError();
}

}  // namespace vsg
