// vsg_dispatch.hpp — runtime (storage, metric, row shape) -> template instance.
//
// Row shape (G lanes per row, VM 16-B chunks per lane, U passes in flight)
// is chosen from the row's 16-B chunk count so that a pass keeps 8-16 chunk
// loads per lane outstanding:
//   chunks <=   4: G 4,  VM 1,  U 4   (16 rows / pass)
//   chunks <=  16: G 16, VM 1,  U 4
//   chunks <=  32: G 32, VM 1,  U 8   (D=128 f32, D=256 f16)
//   chunks <=  64: G 64, VM 1,  U 8
//   chunks <=  96: G 32, VM 3,  U 4   (D=384 f32, D=768 f16)
//   chunks <= 128: G 64, VM 2,  U 4
//   chunks <= 192: G 32, VM 6,  U 2   (D=768 f32; was G 64 VM 3 U 4: search +1.7 %, build +6 %,
//                                      profiles/r01_shape192_probe.jsonl; the build and
//                                      search kernels take U 4, below)
//   chunks <= 256: G 64, VM 4,  U 2
//   chunks <= 384: G 64, VM 6,  U 2   (D=1536 f32)
//   chunks <= 512: G 64, VM 8,  U 2
//   chunks <=1024: G 64, VM 16, U 1
#pragma once
#include "vsg_device.hpp"
#include "vsg_kernels.hpp"

namespace vsg {

// 65..96 chunks (D=384 f32, D=768 f16): two 32-lane rows with 3 chunks per lane
// instead of one 64-lane row whose second chunk is idle on a quarter of the lanes.
// Measured on the f16 walk of C2: U=4 +13 %, U=2 +10 % (profiles/r01_shape96_probe.jsonl)
#ifndef VSG_SHAPE96_U
#define VSG_SHAPE96_U 4
#endif

template <int G_, int VM_, int U_> struct Shape {
    static constexpr int G = G_, VM = VM_, U = U_;
};
template <typename T_> struct TypeTag {
    using T = T_;
};
template <int M_> struct MetTag {
    static constexpr int MET = M_;
};

template <typename F>
inline void dispatch_shape(int nc, F&& f) {
    if (nc <= 4) f(Shape<4, 1, 4>{});
#ifdef VSG_SHAPE16
    else if (nc <= 16) f(Shape<VSG_SHAPE16>{});  // probe builds only
#else
    else if (nc <= 16) f(Shape<16, 1, 4>{});
#endif
    else if (nc <= 32) f(Shape<32, 1, 8>{});
    else if (nc <= 64) f(Shape<64, 1, 8>{});
#if VSG_SHAPE96_U
    else if (nc <= 96) f(Shape<32, 3, VSG_SHAPE96_U>{});
#endif
    else if (nc <= 128) f(Shape<64, 2, 4>{});
#ifdef VSG_SHAPE192
    else if (nc <= 192) f(Shape<VSG_SHAPE192>{});  // probe builds only
#else
    else if (nc <= 192) f(Shape<32, 6, 2>{});
#endif
    else if (nc <= 256) f(Shape<64, 4, 2>{});
    else if (nc <= 384) f(Shape<64, 6, 2>{});
    else if (nc <= 512) f(Shape<64, 8, 2>{});
    else f(Shape<64, 16, 1>{});
}

// The search kernels' shape: as dispatch_shape, except 5..16-chunk rows (128-d f16 --
// C4 -- and 64-d f32) run 8 lanes x 2 chunks, 8 rows per pass: with the DPP group sums
// one 32-row pass covers an expansion's ~20 fresh rows where 16 x 1 took two round
// trips (C4 shard at 10k queries: -9 % at ef 64, -7 % at ef 192;
// profiles/r03_c4_shape_probe.jsonl).  The build keeps 16 x 1 (8 x 2: +9 % build
// time, more selection rows per pass).  Distances are the same sums in another lane
// order: exact on integer data, within rounding otherwise.
//
// 4 passes in flight for 768-d and 1536-d f32 rows (C2 / C3, C5) in the search kernels
// at ef <= 64 (round 5): a query's chain is ~22 expansions of ~30 fresh 3- / 6-KiB rows, and one
// wave with 4 rows in flight needs half the round trips per expansion.  Kernel ms at
// ef 36 / 30, U 2 -> 4 (profiles/r05_shape_u4.jsonl, r05_c5u4.jsonl): C2 512 queries
// 0.593 -> 0.509, 2,048 0.923 -> 0.854, 10,000 2.993 -> 2.998; C5 512 0.593 -> 0.500,
// 10,000 4.237 -> 4.172 -- small batches (the actor's) gain, the full chip does not
// lose.  Same sums in the same order: identical results.  Only the 2-row register
// kernels (ef <= 64) take it: with 4 register rows the extra VGPRs cost a wave per SIMD,
// C2 at ef 128 1.83 -> 1.70 M QPS; the list kernels and the 17-row register kernels
// (ef > 448, whose key set leaves no room) keep U=2.
#ifndef VSG_SEARCH_SHAPE16
#define VSG_SEARCH_SHAPE16 8, 2, 4
#endif
#ifndef VSG_SEARCH_SHAPE192
#define VSG_SEARCH_SHAPE192 32, 6, 4
#endif
#ifndef VSG_SEARCH_SHAPE384
#define VSG_SEARCH_SHAPE384 64, 6, 4
#endif
template <bool LONG_U4, typename F>
inline void dispatch_shape_search(int nc, F&& f) {
    if (nc > 4 && nc <= 16) f(Shape<VSG_SEARCH_SHAPE16>{});
    else if (LONG_U4 && nc > 128 && nc <= 192) f(Shape<VSG_SEARCH_SHAPE192>{});
    else if (LONG_U4 && nc > 256 && nc <= 384) f(Shape<VSG_SEARCH_SHAPE384>{});
    else dispatch_shape(nc, f);
}

// The build kernels' shape (insert beam / selection, reverse links, edge distances):
// 768-d and 1536-d f32 rows with 4 passes in flight too -- C2 build 0.485 -> 0.468 s
// (insert 0.435 -> 0.418 s), C5 1M x 1536 IP 1.04 -> 0.985 s (insert 0.971 -> 0.913 s),
// same graphs (profiles/r05_b4_build.jsonl, r05_c5b4_build.jsonl).
#ifndef VSG_BUILD_SHAPE192
#define VSG_BUILD_SHAPE192 32, 6, 4
#endif
#ifndef VSG_BUILD_SHAPE384
#define VSG_BUILD_SHAPE384 64, 6, 4
#endif
template <typename F>
inline void dispatch_shape_build(int nc, F&& f) {
    if (nc > 128 && nc <= 192) f(Shape<VSG_BUILD_SHAPE192>{});
    else if (nc > 256 && nc <= 384) f(Shape<VSG_BUILD_SHAPE384>{});
    else dispatch_shape(nc, f);
}

// SHAPE_SEARCH_SMALL_EF: the 2-row register search kernels (long rows with U=4)
enum ShapeMode { SHAPE_GENERIC = 0, SHAPE_SEARCH = 1, SHAPE_BUILD = 2, SHAPE_SEARCH_SMALL_EF = 3 };

// f(Shape, TypeTag, MetTag); MODE selects the search / build shapes
template <int MODE = SHAPE_GENERIC, typename F>
inline void dispatch_all(Storage st, MetricKind mk, int nc, F&& f) {
    auto pick = [&](auto&& g) {
        if constexpr (MODE == SHAPE_SEARCH) dispatch_shape_search<false>(nc, g);
        else if constexpr (MODE == SHAPE_SEARCH_SMALL_EF) dispatch_shape_search<true>(nc, g);
        else if constexpr (MODE == SHAPE_BUILD) dispatch_shape_build(nc, g);
        else dispatch_shape(nc, g);
    };
    pick([&](auto sh) {
        if (st == ST_F32) {
            if (mk == MK_L2) f(sh, TypeTag<float>{}, MetTag<MET_L2>{});
            else f(sh, TypeTag<float>{}, MetTag<MET_DOT>{});
        } else {
            if (mk == MK_L2) f(sh, TypeTag<_Float16>{}, MetTag<MET_L2>{});
            else f(sh, TypeTag<_Float16>{}, MetTag<MET_DOT>{});
        }
    });
}

}  // namespace vsg

#define VSG_KERNEL_OF(TEMPLATE, sh, tt, mt) \
    TEMPLATE<decltype(sh)::G, decltype(sh)::VM, decltype(sh)::U, typename decltype(tt)::T, decltype(mt)::MET>
