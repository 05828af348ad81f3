// exact.hip — brute-force (exact) k-NN on gfx950, VALU path.
//
// Absent from the reference (only HNSW search is called at
// src/index/usearch.rs:276); provided behind the same ABI for ground truth and
// small indexes.  Grid x = query, y = row block, so consecutive workgroups read
// the same row block and share it through L2 / Infinity Cache.  One wave per
// (query, row block) keeps a (distance, slot)-sorted top-k list in LDS; a
// second kernel merges the per-block lists and maps slots to keys.
#include <hip/hip_runtime.h>

#include "vsg_device.hpp"
#include "vsg_dispatch.hpp"
#include "vsg_kernels.hpp"

namespace vsg {

static size_t exact_lds_bytes(int k) { return (size_t)k * 16 + 64 * 4 * 4; }

template <int G, int VM, int U, typename T, int MET>
__global__ __launch_bounds__(64) void exact_kernel(ExactParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int qi = blockIdx.x;
    const int b = blockIdx.y;
    const int lane = lane_id();
    constexpr int BLK = (64 / G) * U;
    uint8_t* s = smem;
    List L;
    L.d0 = reinterpret_cast<float*>(s);
    s += (size_t)p.k * 4;
    L.d1 = reinterpret_cast<float*>(s);
    s += (size_t)p.k * 4;
    L.i0 = reinterpret_cast<uint32_t*>(s);
    s += (size_t)p.k * 4;
    L.i1 = reinterpret_cast<uint32_t*>(s);
    s += (size_t)p.k * 4;
    L.cap = p.k;
    L.cur = 0;
    L.size = 0;
    float* sd = reinterpret_cast<float*>(s);
    uint32_t* si = reinterpret_cast<uint32_t*>(s + 256);
    uint32_t* todo = reinterpret_cast<uint32_t*>(s + 512);
    float* tdist = reinterpret_cast<float*>(s + 768);

    QReg<G, VM, T> q;
    q.load(p.queries + (size_t)qi * p.row_bytes, p.nchunks);
    const size_t beg = (size_t)b * p.rows_per_block;
    const size_t end = min(beg + (size_t)p.rows_per_block, p.nslots);
    for (size_t r0 = beg; r0 < end; r0 += BLK) {
        const int cnt = (int)min((size_t)BLK, end - r0);
        if (lane < cnt) todo[lane] = (uint32_t)(r0 + lane);
        wave_sync();
        rows_dist<G, VM, U, T, MET>(p.vecs, p.row_bytes, p.nchunks, todo, cnt, q, tdist);
        wave_sync();
        const bool valid = lane < cnt && !(p.flags[r0 + (lane < cnt ? lane : 0)] & 1);
        const float cd = valid ? tdist[lane] : 0.f;
        const uint32_t ci = (uint32_t)(r0 + lane);
        wave_sync();
        L.merge(valid, cd, ci, false, sd, si);
    }
    const size_t o = ((size_t)qi * p.nblocks + b) * p.k;
    for (int j = lane; j < p.k; j += 64) {
        const bool v = j < L.size;
        p.part_d[o + j] = v ? L.D()[j] : __builtin_inff();
        p.part_i[o + j] = v ? (L.I()[j] & VSG_ID_MASK) : VSG_EMPTY;
    }
}

__global__ __launch_bounds__(64) void merge_parts_kernel(MergeParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int qi = blockIdx.x;
    const int lane = lane_id();
    uint8_t* s = smem;
    List L;
    L.d0 = reinterpret_cast<float*>(s);
    s += (size_t)p.k * 4;
    L.d1 = reinterpret_cast<float*>(s);
    s += (size_t)p.k * 4;
    L.i0 = reinterpret_cast<uint32_t*>(s);
    s += (size_t)p.k * 4;
    L.i1 = reinterpret_cast<uint32_t*>(s);
    s += (size_t)p.k * 4;
    L.cap = p.k;
    L.cur = 0;
    L.size = 0;
    float* sd = reinterpret_cast<float*>(s);
    uint32_t* si = reinterpret_cast<uint32_t*>(s + 256);
    const size_t total = (size_t)p.parts * (p.kin ? p.kin : p.k);
    const float* pd = p.part_d + (size_t)qi * total;
    const uint32_t* pi = p.part_i + (size_t)qi * total;
    for (size_t t = 0; t < total; t += 64) {
        const size_t i = t + lane;
        const uint32_t id = i < total ? pi[i] : VSG_EMPTY;
        const bool valid = id != VSG_EMPTY;
        const float cd = valid ? pd[i] : 0.f;
        L.merge(valid, cd, id, false, sd, si);
    }
    if (p.out_part_d) {  // stage 1 of a two-stage merge: a partial list again
        for (int j = lane; j < p.k; j += 64) {
            const bool v = j < L.size;
            p.out_part_d[(size_t)qi * p.k + j] = v ? L.D()[j] : __builtin_inff();
            p.out_part_i[(size_t)qi * p.k + j] = v ? (L.I()[j] & VSG_ID_MASK) : VSG_EMPTY;
        }
        return;
    }
    uint64_t* ok = p.out_keys + (size_t)qi * p.k;
    float* od = p.out_dist + (size_t)qi * p.k;
    for (int j = lane; j < p.k; j += 64) {
        const bool v = j < L.size;
        const uint32_t id = v ? (L.I()[j] & VSG_ID_MASK) : 0u;
        ok[j] = v ? p.keys[id] : ~0ull;
        od[j] = v ? L.D()[j] : __builtin_inff();
    }
    if (lane == 0 && p.out_counts) p.out_counts[qi] = (uint32_t)L.size;
}

hipError_t launch_exact(Storage st, MetricKind mk, const ExactParams& p, hipStream_t s) {
    if (p.nq <= 0 || p.nblocks <= 0) return hipSuccess;
    const size_t lds = exact_lds_bytes(p.k);
    hipError_t err = hipSuccess;
    dispatch_all(st, mk, p.nchunks, [&](auto sh, auto tt, auto mt) {
        auto kern = VSG_KERNEL_OF(exact_kernel, sh, tt, mt);
        if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(p.nq, p.nblocks), dim3(64), lds, s, p);
        err = hipGetLastError();
    });
    return err;
}

hipError_t launch_merge_parts(const MergeParams& p, hipStream_t s) {
    if (p.nq <= 0) return hipSuccess;
    const size_t lds = exact_lds_bytes(p.k);
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)merge_parts_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(merge_parts_kernel, dim3(p.nq), dim3(64), lds, s, p);
    return hipGetLastError();
}

// k-way merge of sorted per-shard rows: one thread per query, (distance, key)
// order.  parts x nq x k_in inputs (all-gathered shard results, SURVEY §8e;
// a shard may return fewer candidates than the final k) -> nq x k_out.
__global__ void merge_topk64_kernel(const uint64_t* __restrict__ keys, const float* __restrict__ dist,
                                    int parts, int nq, int kin, int kout, uint64_t* __restrict__ out_keys,
                                    float* __restrict__ out_dist) {
    const int qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    int ptr[64];
    const int P = parts < 64 ? parts : 64;
    for (int pp = 0; pp < P; ++pp) ptr[pp] = 0;
    for (int j = 0; j < kout; ++j) {
        int best = -1;
        float bd = __builtin_inff();
        uint64_t bk = ~0ull;
        for (int pp = 0; pp < P; ++pp) {
            if (ptr[pp] >= kin) continue;
            const size_t o = ((size_t)pp * nq + qi) * kin + ptr[pp];
            const uint64_t kk = keys[o];
            if (kk == ~0ull) continue;
            const float dd = dist[o];
            if (best < 0 || dd < bd || (dd == bd && kk < bk)) {
                best = pp;
                bd = dd;
                bk = kk;
            }
        }
        out_keys[(size_t)qi * kout + j] = best < 0 ? ~0ull : bk;
        out_dist[(size_t)qi * kout + j] = best < 0 ? __builtin_inff() : bd;
        if (best >= 0) ptr[best]++;
    }
}

hipError_t launch_merge_topk64(const uint64_t* keys, const float* dist, int parts, int nq, int kin, int kout,
                               uint64_t* out_keys, float* out_dist, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(merge_topk64_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, keys, dist, parts, nq, kin,
                       kout, out_keys, out_dist);
    return hipGetLastError();
}

}  // namespace vsg
