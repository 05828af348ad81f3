// cells.hip — nearest of P pivot rows for every row of an add (the locality
// launch order of the batched build): a heuristic key that only
// orders a batch's waves (no output depends on it), so it runs on the bf16
// matrix cores (v_mfma_f32_32x32x16_bf16, 16x the f32 rate) instead of the
// f32 exact kernel + top-16 partial lists it replaced (C2: ~18 ms per 1M-row add).
//
// One wave = 32 rows (the B operand, N) against pivot groups of 256 (eight
// 32-pivot A tiles, 8 x 16 accumulators); K = the padded row in steps of 16; a
// block's 4 waves share each pivot chunk through LDS.
// Lane l holds row (l % 32) of every C tile and 16 of each tile's pivots, keeps
// its own best (distance, pivot) and the two half-waves combine at the end.
// Rows stay f32 in HBM and are rounded to bf16 as they are loaded; pivots are
// converted once per call (pivots_bf16_kernel).  Distances: |p|^2 - 2 p.x (l2sq;
// |x|^2 is common to all pivots of a row) or -p.x (cos rows are normalised; ip).
#include <hip/hip_runtime.h>

#include "vsg_device.hpp"
#include "vsg_kernels.hpp"

namespace vsg {

typedef float cfloatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int CELL_GROUP = 8;  // 32-pivot tiles per pass (256 pivots)

__device__ __forceinline__ uint32_t bf16_bits(float x) {  // round to nearest even
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) { return bf16_bits(a) | (bf16_bits(b) << 16); }

// pivots (P x D f32) -> pb (Ppad x D bf16, rows >= P zero)
__global__ __launch_bounds__(256) void pivots_bf16_kernel(const float* __restrict__ piv, int P, int Ppad, int D,
                                                          uint32_t* __restrict__ pb) {
    const size_t pairs = (size_t)Ppad * D / 2;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < pairs; i += (size_t)gridDim.x * blockDim.x) {
        const size_t e = 2 * i;
        const size_t p = e / D;
        pb[i] = p < (size_t)P ? pack_bf16(piv[e], piv[e + 1]) : 0u;
    }
}

// The pivots of a pass are shared by the block's 4 waves through LDS: 32-dim
// chunks (256 pivots x 64 B, rows padded to 80 B so the 16 lanes of a ds_read_b128
// hit distinct 16-B slots), double-buffered, one barrier per chunk -- each pivot
// byte leaves L2 once per 128 rows instead of once per 32.
constexpr int CELL_PROW = 40;  // bf16 per padded LDS pivot row (32 + 8)

template <int MET>
__global__ __launch_bounds__(256, 2) void cells_kernel(const uint4* __restrict__ pb, const float* __restrict__ psq,
                                                       int P, int Ppad, const float* __restrict__ rows, size_t nrows,
                                                       int D, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint16_t sp[2][32 * CELL_GROUP * CELL_PROW];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const size_t r0 = ((size_t)blockIdx.x * 4 + (tid >> 6)) * 32;
    const bool live = r0 < nrows;  // every wave takes part in the block's barriers
    const int n = lane & 31, kb = lane >> 5;
    const size_t row = live ? min(r0 + (size_t)n, nrows - 1) : 0;
    const float* xr = rows + row * (size_t)D + 8 * kb;
    const int dq = D / 8;  // 16-B pieces per pivot row
    const int nch = D / 32;
    float best = __builtin_inff();
    uint32_t bid = 0xFFFFFFFFu;
    // chunk c of pass t0 -> buffer: 256 pivots x 4 pieces, 4 per thread
    auto stage = [&](int t0, int c, uint16_t* dst) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;  // (pivot, piece)
            const int pv = e >> 2, pc = e & 3;
            const uint4 v = pb[(size_t)(t0 + pv) * dq + (size_t)c * 4 + pc];
            *reinterpret_cast<uint4*>(dst + pv * CELL_PROW + pc * 8) = v;
        }
    };
    for (int t0 = 0; t0 < Ppad; t0 += 32 * CELL_GROUP) {
        cfloatx16 acc[CELL_GROUP];
#pragma unroll
        for (int t = 0; t < CELL_GROUP; ++t)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[t][g] = 0.f;
        __syncthreads();  // the previous pass's last reads of sp[0] are done
        stage(t0, 0, sp[0]);
        for (int c = 0; c < nch; ++c) {
            __syncthreads();  // chunk c in sp[c & 1]; sp[(c + 1) & 1] free
            if (c + 1 < nch) stage(t0, c + 1, sp[(c + 1) & 1]);
            const uint16_t* cur = sp[c & 1];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int k = c * 32 + kk * 16;
                const float4 x0 = *reinterpret_cast<const float4*>(xr + k);
                const float4 x1 = *reinterpret_cast<const float4*>(xr + k + 4);
                const uint4 xb = make_uint4(pack_bf16(x0.x, x0.y), pack_bf16(x0.z, x0.w), pack_bf16(x1.x, x1.y),
                                            pack_bf16(x1.z, x1.w));
                const bf16x8 b = __builtin_bit_cast(bf16x8, xb);
#pragma unroll
                for (int t = 0; t < CELL_GROUP; ++t) {
                    const uint4 pv =
                        *reinterpret_cast<const uint4*>(cur + (t * 32 + n) * CELL_PROW + kk * 16 + kb * 8);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, pv), b, acc[t], 0, 0, 0);
                }
            }
        }
        // C[m = pivot][n = row]: register g of lane l holds pivot 8 (g / 4) + 4 (l / 32) + g % 4
#pragma unroll
        for (int t = 0; t < CELL_GROUP; ++t)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int pid = t0 + t * 32 + 8 * (g >> 2) + 4 * kb + (g & 3);
                if (pid < P) {
                    const float dot = acc[t][g];
                    const float d = MET == MET_L2 ? psq[pid] - 2.f * dot : -dot;
                    if (d < best || (d == best && (uint32_t)pid < bid)) {
                        best = d;
                        bid = (uint32_t)pid;
                    }
                }
            }
    }
    const float ob = __shfl_xor(best, 32);
    const uint32_t oi = (uint32_t)__shfl_xor((int)bid, 32);
    if (ob < best || (ob == best && oi < bid)) bid = oi;
    if (live && kb == 0 && r0 + n < nrows) out[r0 + n] = bid;
}

size_t cells_pivot_bytes(int P, int D) { return (size_t)((P + 255) / 256 * 256) * D * 2; }

hipError_t launch_cells(MetricKind mk, const float* piv, const float* psq, int P, const float* rows, size_t nrows,
                        int D, void* pb_scratch, bool convert, uint32_t* out, hipStream_t s) {
    if (P <= 0 || D % 32 || nrows == 0) return P <= 0 || D % 32 ? hipErrorInvalidValue : hipSuccess;
    const int Ppad = (P + 255) / 256 * 256;
    uint32_t* pb = reinterpret_cast<uint32_t*>(pb_scratch);
    if (convert) {
        const size_t pairs = (size_t)Ppad * D / 2;
        const unsigned g = (unsigned)std::min<size_t>((pairs + 255) / 256, 4096);
        hipLaunchKernelGGL(pivots_bf16_kernel, dim3(g), dim3(256), 0, s, piv, P, Ppad, D, pb);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const size_t waves = (nrows + 31) / 32;
    const unsigned grid = (unsigned)((waves + 3) / 4);
    auto kern = mk == MK_L2 ? cells_kernel<MET_L2> : cells_kernel<MET_DOT>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(pb), psq, P, Ppad, rows,
                       nrows, D, out);
    return hipGetLastError();
}

}  // namespace vsg
