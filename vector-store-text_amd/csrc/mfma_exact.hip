// mfma_exact.hip — batched brute-force k-NN on the f32 matrix cores (gfx950).
//
// The only dense contraction on this path:
// D = X . Q^T with `v_mfma_f32_32x32x2_f32` (exact f32 FMA chain, 64 FLOP/clk/SIMD),
// fused with a per-lane register top-KMAX so no distance tile ever reaches HBM.
//
//   block = 256 threads (4 waves, 2 x 2), tile = 128 base rows x 128 queries (or 4 x 1:
//   256 rows x 64 queries for batches <= 64),
//   K stage = 32 dims, two static LDS buffers [rows | queries][32] floats (64 KiB,
//   XOR-swizzled 16-B slots), the next stage streamed in by LDS-DMA
//   (global_load_lds) during the MFMAs of the current one, one barrier per stage.
//   Wave (wr, wq) owns rows [wr*64, +64) x queries [wq*64, +64) = 2 x 2 MFMA tiles.
//   A operand = base rows, B operand = queries, so C lane l holds query (l & 31)
//   against 16 rows: each lane keeps a sorted top-KMAX per query in VGPRs.
//   Within a K stage the half-wave h takes dims [h*16, h*16+16): a lane reads 16
//   contiguous floats per fragment (4 x ds_read_b128) instead of a stride-2 gather.
//
// Grid: (query tile, row split) pairs, mapped XCD-contiguously (blocks b, b+8, ...
// share an XCD) so the query tiles of one row split run on one XCD and share the
// base rows through its L2.  Partial lists [q][part][KMAX], part = (split, wr, h),
// are merged by merge_parts_kernel.  Ties: (distance, slot) as everywhere.
#include <hip/hip_runtime.h>

#include "vsg_device.hpp"
#include "vsg_kernels.hpp"

namespace vsg {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int KT = 32;   // dims per stage = one 128-B LDS row
constexpr int LDK = 32;  // LDS row stride (floats), unpadded: glds writes lane-linear 1-KiB pieces
// WQ = waves along the query axis, WR = along the row axis (64 x 64 per wave):
//   WQ 2, WR 2 -> 128 rows x 128 queries, 256 threads (batches > 64);
//   WQ 1, WR 4 -> 256 rows x 64 queries, 256 threads (batches <= 64: the 128-query
//   tile computed half of its MFMAs for padding queries, 0.28 of peak at 64; the
//   128 x 64 tile of 2 waves left one wave per SIMD and re-staged the queries
//   for every 128 rows)
template <int WQ, int WR> struct MfmaTile {
    static constexpr int BQ = 64 * WQ, BR = 64 * WR, NW = WQ * WR, STAGE = (BR + BQ) * LDK;
};

// 16-B slot of logical chunk c (0..7) in LDS row R: XOR swizzle so the sixteen
// lanes of a ds_read_b128 group (rows R..R+15, same chunk) hit distinct slots of
// the 64-bank row (conflict-free); applied to the glds SOURCE and to the read.
__device__ __forceinline__ int swz(int R, int c) { return c ^ ((R >> 1) & 7); }

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

template <int KMAX>
__device__ __forceinline__ void topk_insert(float (&ld)[KMAX], uint32_t (&li)[KMAX], float d, uint32_t id) {
    // ascending list, strict < : an equal distance from a later (larger) slot goes after
#pragma unroll
    for (int t = KMAX - 1; t >= 1; --t) {
        const bool shift = d < ld[t - 1];
        const bool here = !shift && d < ld[t];
        ld[t] = shift ? ld[t - 1] : (here ? d : ld[t]);
        li[t] = shift ? li[t - 1] : (here ? id : li[t]);
    }
    if (d < ld[0]) {
        ld[0] = d;
        li[0] = id;
    }
}

template <int KMAX, int MET, int WQ, int WR>
__global__ __launch_bounds__(64 * WQ * WR, 2) void mfma_exact_kernel(MfmaExactParams p) {
    using TL = MfmaTile<WQ, WR>;
    constexpr int BQ = TL::BQ, BR = TL::BR, NW = TL::NW;
    __shared__ __attribute__((aligned(16))) float lds_a[TL::STAGE];
    __shared__ __attribute__((aligned(16))) float lds_b[TL::STAGE];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int wq = w % WQ, wr = w / WQ;
    const int h = lane >> 5, r = lane & 31;

    // XCD-contiguous block -> (split, query tile)
    const int nb = gridDim.x;
    const int per = nb >> 3;
    const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (L >= p.qtiles * p.splits) return;
    const int split = L / p.qtiles;
    const int qt = L % p.qtiles;
    const int q0 = qt * BQ;
    const size_t ntiles = (p.nslots + BR - 1) / BR;
    const size_t t_beg = (size_t)split * p.tiles_per_split;
    const size_t t_end = min(t_beg + (size_t)p.tiles_per_split, ntiles);
    const int nst = (p.row_floats + KT - 1) / KT;

    float ld[2][KMAX];
    uint32_t li[2][KMAX];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int t = 0; t < KMAX; ++t) {
            ld[b][t] = __builtin_inff();
            li[b][t] = VSG_EMPTY;
        }

    float qs2[2] = {0.f, 0.f};
    if constexpr (MET == MET_L2) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int qi = q0 + wq * 64 + b * 32 + r;
            qs2[b] = qi < p.nq ? p.qsqnorm[qi] : 0.f;
        }
    }

    for (size_t tile = t_beg; tile < t_end; ++tile) {
        const size_t r0 = tile * BR;
        floatx16 acc[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[a][b][g] = 0.f;

        // LDS-DMA staging: the NW waves fill the 1-KiB pieces (8 rows x 128 B) of the
        // base-row tile (16 pieces) and the query tile (BQ / 8 pieces) round-robin;
        // out-of-range rows read a clamped valid row (masked in the epilogue / never
        // written out).
        const int prow = lane >> 3, pslot = lane & 7;
        // Addresses: a wave-uniform stage base + a 32-bit per-lane offset (row within
        // the tile, clamped, x row_floats + swizzled chunk), so no 64-bit address per
        // piece stays live across the K loop (the 64-query tile spilled with them).
        const int xlast = (int)min((size_t)(BR - 1), p.nslots - 1 - r0);
        const int qlast = min(BQ - 1, p.nq - 1 - q0);
        // base rows: row-major (stride row_floats) or the K-tiled copy, where the
        // stage's rows are consecutive 128-B rows of one contiguous block
        const bool kt = p.ktile != nullptr;
        const uint32_t xstride = kt ? (uint32_t)KT : (uint32_t)p.row_floats;
        auto load_stage = [&](int s, float* xs) {
            const int k0 = s * KT;
            float* qs = xs + BR * LDK;
            const float* xb = kt ? p.ktile + (((r0 / KTILE_ROWS) * (size_t)nst + s) * KTILE_ROWS + r0 % KTILE_ROWS) * KT
                                 : p.vecs + r0 * p.row_floats + k0;
            const float* qb = p.queries + (size_t)q0 * p.row_floats + k0;
#pragma unroll
            for (int u = 0; u < BR / 8 / NW; ++u) {
                const int piece = w * (BR / 8 / NW) + u;
                const int R = piece * 8 + prow;
                const uint32_t off = (uint32_t)min(R, xlast) * xstride + (uint32_t)swz(R, pslot) * 4;
                __builtin_amdgcn_global_load_lds((gptr_t)(xb + off), (lptr_t)(xs + piece * 8 * LDK), 16, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < BQ / 8 / NW; ++u) {
                const int piece = w * (BQ / 8 / NW) + u;
                const int R = piece * 8 + prow;
                const uint32_t off = (uint32_t)min(R, qlast) * (uint32_t)p.row_floats + (uint32_t)swz(R, pslot) * 4;
                __builtin_amdgcn_global_load_lds((gptr_t)(qb + off), (lptr_t)(qs + piece * 8 * LDK), 16, 0, 0);
            }
        };
        // one K stage: MFMAs on `cur` while the next stage streams into `nxt`.
        // cur / nxt are two distinct __shared__ arrays named statically (the loop
        // is unrolled by two), so the compiler can tell the DMA target from the
        // ds_read source; through one runtime-indexed buffer it waited for the
        // DMA (vmcnt(0)) before the stage's first ds_read.
        auto stage = [&](int s, const float* cur, float* nxt) __attribute__((always_inline)) {
            if (s + 1 < nst) load_stage(s + 1, nxt);  // nxt was last read before the previous barrier
            const float* xs = cur;
            const float* qs = cur + BR * LDK;
#pragma unroll
            for (int tq = 0; tq < 4; ++tq) {
                float4 xa[2], qb[2];
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    const int R = wr * 64 + a * 32 + r;
                    xa[a] = *reinterpret_cast<const float4*>(xs + R * LDK + swz(R, h * 4 + tq) * 4);
                }
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int R = wq * 64 + b * 32 + r;
                    qb[b] = *reinterpret_cast<const float4*>(qs + R * LDK + swz(R, h * 4 + tq) * 4);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int b = 0; b < 2; ++b) {
                            const float av = e == 0 ? xa[a].x : e == 1 ? xa[a].y : e == 2 ? xa[a].z : xa[a].w;
                            const float bv = e == 0 ? qb[b].x : e == 1 ? qb[b].y : e == 2 ? qb[b].z : qb[b].w;
                            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[a][b], 0, 0, 0);
                        }
                }
            }
            __syncthreads();
        };

        load_stage(0, lds_a);
        __syncthreads();  // drains the LDS-DMA (vmcnt(0)) and publishes stage 0
        for (int s = 0; s < nst; s += 2) {
            stage(s, lds_a, lds_b);
            if (s + 1 < nst) stage(s + 1, lds_b, lds_a);
        }

        // epilogue: distances + register top-KMAX (rows arrive in increasing slot order)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const size_t row = r0 + wr * 64 + a * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
                const bool valid = row < p.nslots && !(p.flags[row < p.nslots ? row : 0] & 1);
                float xs2 = 0.f;
                if constexpr (MET == MET_L2) xs2 = valid ? p.sqnorm[row] : 0.f;
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const float dot = acc[a][b][g];
                    float d = (MET == MET_L2) ? (xs2 + qs2[b]) - 2.f * dot : 1.f - dot;
                    if (!valid) d = __builtin_inff();
                    if (d < ld[b][KMAX - 1]) topk_insert<KMAX>(ld[b], li[b], d, (uint32_t)row);
                }
            }
        }
    }

    const int nparts = p.splits * WR * 2;
    const int part = (split * WR + wr) * 2 + h;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int qi = q0 + wq * 64 + b * 32 + r;
        if (qi >= p.nq) continue;
        const size_t o = ((size_t)qi * nparts + part) * KMAX;
#pragma unroll
        for (int t = 0; t < KMAX; ++t) {
            p.part_d[o + t] = ld[b][t];
            p.part_i[o + t] = ld[b][t] < __builtin_inff() ? li[b][t] : VSG_EMPTY;
        }
    }
}

// one work-item per 16-B chunk of a row: chunk c of row r goes to stage c / 8,
// slot c % 8 of row r % 256 in tile r / 256
__global__ __launch_bounds__(256) void ktile_rows_kernel(const float* __restrict__ vecs, int row_floats, size_t r0,
                                                          size_t r1, float* __restrict__ ktile) {
    const int nc = row_floats / 4, nst = row_floats / KT;
    const size_t tot = (r1 - r0) * (size_t)nc;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = r0 + i / nc;
        const int c = (int)(i % nc);
        const float4 v = *reinterpret_cast<const float4*>(vecs + r * row_floats + (size_t)c * 4);
        const size_t o = (((r / KTILE_ROWS) * (size_t)nst + c / 8) * KTILE_ROWS + r % KTILE_ROWS) * KT + (c % 8) * 4;
        *reinterpret_cast<float4*>(ktile + o) = v;
    }
}

hipError_t launch_ktile_rows(const float* vecs, int row_floats, size_t r0, size_t r1, float* ktile, hipStream_t s) {
    if (r1 <= r0) return hipSuccess;
    if (row_floats % KT) return hipErrorInvalidValue;
    const size_t tot = (r1 - r0) * (size_t)(row_floats / 4);
    const unsigned grid = (unsigned)std::min<size_t>((tot + 255) / 256, 1u << 20);
    hipLaunchKernelGGL(ktile_rows_kernel, dim3(grid), dim3(256), 0, s, vecs, row_floats, r0, r1, ktile);
    return hipGetLastError();
}

hipError_t launch_mfma_exact(MetricKind mk, const MfmaExactParams& p, hipStream_t s) {
    // (bq, br) = (128, 128) or (64, 256); both 256-thread blocks
    if (p.kmax != 16 || !((p.bq == 128 && p.br == 128) || (p.bq == 64 && p.br == 256))) return hipErrorNotSupported;
    const int total = p.qtiles * p.splits;
    const int nb = (total + 7) / 8 * 8;
    if (p.bq == 128) {
        auto kern = mk == MK_L2 ? mfma_exact_kernel<16, MET_L2, 2, 2> : mfma_exact_kernel<16, MET_DOT, 2, 2>;
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, s, p);
    } else {
        auto kern = mk == MK_L2 ? mfma_exact_kernel<16, MET_L2, 1, 4> : mfma_exact_kernel<16, MET_DOT, 1, 4>;
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, s, p);
    }
    return hipGetLastError();
}

}  // namespace vsg
