// vsg_kernels.hpp — host-side launch interface of the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace vsg {

enum Storage { ST_F32 = 0, ST_F16 = 1 };
enum MetricKind { MK_L2 = 0, MK_DOT = 1 };  // cos = DOT on normalised rows

struct DevGraph {
    const uint8_t* vecs;
    size_t row_bytes;
    int nchunks;
    uint32_t* adj0;
    const uint32_t* upper_off;
    uint32_t* upper;
    int M, M0;
    // per-edge distances beside the adjacency (build only; nullptr in searches):
    // adjd0[s * M0 + j] = dist(s, adj0[s * M0 + j]), upperd likewise for upper rows
    float* adjd0;
    float* upperd;
};

struct SearchParams {
    DevGraph g;
    const uint8_t* queries;  // prepared rows, g.row_bytes stride
    int nq, k, ef;
    uint32_t entry;
    int max_level;
    const uint8_t* flags;
    const uint64_t* keys;       // slot -> key (NULL: emit slots, f16-traversal candidates)
    uint64_t* out_keys;
    float* out_dist;
    uint32_t* out_counts;
    unsigned long long* stats;  // [0] n_dist, [1] n_adj, [2] queries
    int xcd_map;                // 1: workgroups b, b+8, ... (one XCD) take consecutive queries
    int hash_size;              // visited-table entries (hash_size_for)
    int waves;                  // waves per query: 1 (hnsw_search_kernel), 2 or 4 (cooperative)
    int reg;                    // 1: hnsw_search_reg_kernel (candidate set in VGPRs; ignores waves)
    int upper_ef;               // > 1: level-1 beam of this width seeds level 0 (reg kernel; opt-in)
    // The index holds removed entries: usearch's filtered base-level search
    // (index_dense `allow` predicate: removed nodes traversed, never results;
    // hnsw_search_filt.hip).  removed_frac sizes the candidate set.
    int filt;
    float removed_frac;
    // Filtered searches only.  ovf[qi] = 1: query qi's candidate set ran out of
    // room (registers / LDS list) and the query stopped; launch_search_filt then
    // searches it again on a sorted list in device memory (filt_lists, filt_cap
    // entries per list, filt_nlists lists) that holds every slot, so no result is
    // ever a degraded one.  ovf == nullptr: no re-run (degrades, counted).
    uint8_t* ovf;
    uint8_t* filt_lists;
    int filt_cap, filt_nlists;
    // register kernel, probes (VSG_SEARCH_PERSIST=1): a persistent grid of resident
    // waves pulling query indices from this counter (zeroed per launch); nullptr:
    // one workgroup per query
    unsigned* qnext;
};

struct InsertParams {
    DevGraph g;
    const uint32_t* nodes;     // slots of the batch (insertion order is a random permutation)
    int nnodes;
    const int8_t* levels;      // per batch node
    const uint32_t* pair_off;  // per batch node
    uint64_t* pair_keys;
    uint32_t* pair_vals;
    uint32_t entry;
    int max_level;
    int efc;
    int hash_size;              // visited-table entries (hash_size_for)
    unsigned long long* stats;  // [3] n_dist, [4] n_adj, [5] selection
    // Locality launch order (vsg_index.cpp build_slots): block b inserts batch
    // node perm[xcd_pos(b)] (nullptr: node b)
    const uint32_t* perm;
    // Split insert (hnsw_insert_beam_kernel + hnsw_insert_select_kernel): the
    // beam kernel stores each level's sorted top-efc list in HBM, the selection
    // kernel reads it back.  List (node bi, level l) = slot list_off[bi] + l:
    // lst_n[slot] entries at lst_d / lst_i[slot * efc ...].
    const uint32_t* list_off;
    float* lst_d;
    uint32_t* lst_i;
    int* lst_n;
};

struct ReverseParams {
    DevGraph g;
    const uint64_t* keys;  // sorted (level:5 | v:29 | u:29 | pad)
    const uint32_t* vals;  // f32 bits: dist(u, v)
    size_t npairs;
    unsigned long long* stats;
    // re-link pass of an add that reuses removed slots: the index flags, bit 1 =
    // a reused slot of this add (incoming links a row already holds are
    // dropped); nullptr otherwise (no check)
    const uint8_t* flags;
};

struct ExactParams {
    const uint8_t* vecs;
    size_t row_bytes;
    int nchunks;
    const uint8_t* queries;
    int nq, k;
    size_t nslots;
    int rows_per_block;
    int nblocks;
    const uint8_t* flags;
    float* part_d;     // nq x nblocks x k
    uint32_t* part_i;  // nq x nblocks x k
};

// Brute force on MFMA (f32 storage): Q (nq x D) . X^T (N x D) with a fused
// per-lane register top-KMAX; partial lists [q][part][KMAX], part = (split, wr, half).
struct MfmaExactParams {
    const float* vecs;      // N x row_floats (prepared rows)
    const float* sqnorm;    // N (L2 only)
    const float* queries;   // nq x row_floats (prepared)
    const float* qsqnorm;   // nq (L2 only)
    int row_floats;
    int nq;
    size_t nslots;
    const uint8_t* flags;
    int qtiles, splits;
    int tiles_per_split;    // br-row tiles per split
    int kmax;
    int bq;                 // queries per tile: 128, or 64 (batches <= 64)
    int br;                 // base rows per tile: 128 with bq 128, 256 with bq 64
    float* part_d;
    uint32_t* part_i;
    // K-tiled copy of `vecs` (exact-only f32 indexes; nullptr: row-major `vecs`):
    // 256-row tiles, each stored stage-major -- [tile][K stage of 32 dims][256 rows][32
    // floats] -- so one K stage of a row tile is one contiguous block (32 KiB for 256
    // rows; a 128-row tile reads half of one) instead of 128-B pieces of 256 rows
    // 4-6 KiB apart.
    const float* ktile;
};

struct MergeParams {
    const float* part_d;
    const uint32_t* part_i;
    int nq, parts, k;
    int kin;  // entries per partial list (0 => k)
    const uint64_t* keys;  // slot -> key (NULL: ids are already keys, 64-bit inputs)
    uint64_t* out_keys;
    float* out_dist;
    uint32_t* out_counts;
    // set: write the merged list as (distance, slot) partial-list entries
    // (nq x k, EMPTY padded) instead of keys -- stage 1 of a two-stage merge
    float* out_part_d;
    uint32_t* out_part_i;
};

// f16-traversal re-rank (rerank.hip): exact f32 distances of each query's
// traversal candidates (slots from the f16 search), best k by (distance, slot)
struct RerankParams {
    const uint8_t* vecs;  // f32 image
    size_t row_bytes;
    int nchunks;
    const uint8_t* queries;  // prepared f32 rows, row_bytes stride
    const uint64_t* cand;    // nq x kc slots (~0 = none)
    const uint32_t* cand_counts;
    int nq, kc, k;
    const uint64_t* keys;  // slot -> key
    uint64_t* out_keys;
    float* out_dist;
    uint32_t* out_counts;
};

// kernel counter block (d_stats): [0..2] search, [3..9] build, [10..15] wave
// clocks (tools), [16] filtered-search overflow
constexpr int VSG_NSTATS = 32;

// key layout of the reverse-link pairs
constexpr int PAIR_U_BITS = 29;
constexpr int PAIR_V_SHIFT = 29;
constexpr int PAIR_L_SHIFT = 58;
constexpr uint64_t PAIR_ID_MASK = (1ull << 29) - 1;
constexpr uint32_t MAX_SLOTS = 1u << 29;
// Limits of the kernels (explicit VSG_EUNSUPPORTED above them, never a clamp):
constexpr size_t MAX_EF = 4096;       // search ef / build efC: sorted list in LDS (16 B per entry)
constexpr size_t MAX_REG_EF = 1024;   // register candidate set (hnsw_search_reg.hip), re-rank beam
constexpr size_t MAX_EXACT_K = 8192;  // exact search: per-block top-k list in LDS
constexpr int MAX_CONNECTIVITY = 64;  // M; level-0 rows of M0 = 2M <= 128 entries

bool shape_supported(int nchunks);
__host__ __device__ int hash_size_for(int ef, int factor);
size_t search_lds_bytes(int ef, int hash, int waves = 1);
size_t insert_lds_bytes(int efc, int hash, int m0);

hipError_t launch_search(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s);
hipError_t launch_search_reg(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s);
// filtered search (p.filt): register set when it fits, else the sorted LDS list;
// overflowed queries re-run on device-memory lists (p.ovf, p.filt_lists)
hipError_t launch_search_filt(Storage st, MetricKind mk, const SearchParams& p, hipStream_t s);
// device-memory list scratch of the re-run: bytes for `slots`, and the list count / capacity it holds
size_t filt_rerun_bytes(size_t slots);
void filt_rerun_shape(size_t slots, int* cap, int* nlists);
size_t search_reg_lds_bytes(int hash);
// split insert: beam kernel then selection kernel (efc <= 192: register beam)
hipError_t launch_insert_split(Storage st, MetricKind mk, const InsertParams& p, hipStream_t s,
                               hipEvent_t mid = nullptr);  // recorded between the two kernels
hipError_t launch_insert(Storage st, MetricKind mk, const InsertParams& p, hipStream_t s);
hipError_t launch_reverse(Storage st, MetricKind mk, const ReverseParams& p, int grid, hipStream_t s);
// per-edge distances of slots [0, n) of an imported / loaded graph (levels: per slot)
hipError_t launch_edge_dist_fill(Storage st, MetricKind mk, const DevGraph& g, const int8_t* levels, size_t n,
                                 hipStream_t s);
// slot reuse (hnsw.hip): stage n reused slots (prepared rows | |x|^2 | keys ->
// their slots; rows of every level cleared; flags = removed | relink), then
// refresh the stored distances of links into them (slots [0, n) scanned;
// levels: per slot)
hipError_t launch_reuse_stage(const DevGraph& g, uint8_t* vecs, float* sqnorm, uint64_t* keys_out, uint8_t* flags,
                              const uint8_t* rows, const float* sq, const uint64_t* keys, const uint32_t* slots,
                              const int8_t* levels, size_t n, hipStream_t s);
hipError_t launch_edge_dist_refresh(Storage st, MetricKind mk, const DevGraph& g, const int8_t* levels,
                                    const uint8_t* flags, size_t n, hipStream_t s);
hipError_t launch_exact(Storage st, MetricKind mk, const ExactParams& p, hipStream_t s);
hipError_t launch_merge_parts(const MergeParams& p, hipStream_t s);
hipError_t launch_rerank(MetricKind mk, const RerankParams& p, hipStream_t s);
// f32 image rows [r0, r1) -> f16 traversal copy (row_bytes16 stride, padding zeroed)
hipError_t launch_shadow_f16(const uint8_t* vecs, size_t row_bytes, size_t r0, size_t r1, int dim,
                             uint8_t* out, size_t row_bytes16, hipStream_t s);
// rows `slots[0..n)` (those < limit) of the f16 traversal copy, re-converted in place
hipError_t launch_shadow_f16_slots(const uint8_t* vecs, size_t row_bytes, const uint32_t* slots, size_t n,
                                   size_t limit, int dim, uint8_t* out, size_t row_bytes16, hipStream_t s);
// rows [r0, r1) of row-major f32 `vecs` (row_floats % 32 == 0) -> the K-tiled layout
// of MfmaExactParams::ktile
hipError_t launch_ktile_rows(const float* vecs, int row_floats, size_t r0, size_t r1, float* ktile,
                             hipStream_t s);
constexpr int KTILE_ROWS = 256;
// returns hipErrorNotSupported when the MFMA path does not apply (k > 32)
hipError_t launch_mfma_exact(MetricKind mk, const MfmaExactParams& p, hipStream_t s);
constexpr int MFMA_BQ = 128, MFMA_BR = 128;
hipError_t launch_merge_topk64(const uint64_t* keys, const float* dist, int parts, int nq, int kin, int kout,
                               uint64_t* out_keys, float* out_dist, hipStream_t s);
// f32 rows (stride dim) -> storage rows (row_bytes), normalised when `normalize`
hipError_t launch_prepare(Storage st, const float* in, size_t n, int dim, bool normalize,
                          uint8_t* out, size_t row_bytes, hipStream_t s, float* sqnorm_out = nullptr);
// storage rows -> f32 rows (stride dim)
hipError_t launch_unprepare(Storage st, const uint8_t* in, size_t n, int dim, size_t row_bytes,
                            float* out, hipStream_t s);
hipError_t launch_set_flags(uint8_t* flags, const uint32_t* slots, size_t n, uint8_t value,
                            hipStream_t s);
// rows / |x|^2 / keys of slots idx[0..n) -> dense outputs (compaction)
hipError_t launch_gather_rows(const uint8_t* vecs, const float* sqnorm, const uint64_t* keys,
                              const uint32_t* idx, size_t n, size_t row_bytes, uint8_t* out_vecs,
                              float* out_sq, uint64_t* out_keys, hipStream_t s);
// locality cells (build launch order): out[r] = the nearest of the partial-list
// entries of row r (MFMA exact search of the rows against pivot rows)
// locality cells (cells.hip): out[r] = the nearest of P pivot rows (P x D f32,
// |p|^2 in psq for l2sq) for nrows f32 rows of D floats (D % 32 == 0), on bf16
// MFMA.  pb_scratch holds cells_pivot_bytes(P, D); convert = (re)fill it from piv.
size_t cells_pivot_bytes(int P, int D);
hipError_t launch_cells(MetricKind mk, const float* piv, const float* psq, int P, const float* rows, size_t nrows,
                        int D, void* pb_scratch, bool convert, uint32_t* out, hipStream_t s);
hipError_t launch_nearest_part(const float* part_d, const uint32_t* part_i, int nq, int parts, int kin,
                               uint32_t* out, hipStream_t s);
// okey[b] = cell[nodes[b] - s0] << 32 | b, oidx[b] = b for the n nodes of one batch
hipError_t launch_batch_keys(const uint32_t* nodes, int n, uint32_t s0, const uint32_t* cell, uint64_t* okey,
                             uint32_t* oidx, hipStream_t s);

hipError_t launch_datagen(int kind, size_t n, size_t dim, uint64_t seed, uint64_t model_seed,
                          size_t start_row, float* out, float* scratch_w, float* scratch_c,
                          hipStream_t s);

}  // namespace vsg
