/*
 * vsg_oracle.h — CPU restatement of the reference's ANN hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the
 * CPU-baseline leg of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (libvsg.so) never
 * links it and never falls back to it.
 *
 * What it restates (all citations relative to /root/reference):
 *   - the usearch-backed index actor src/index/usearch.rs:82-311
 *     (new/reserve :89-99, add :221, remove :215/:245, search :275-277,
 *      size :309, duplicate-key error => remove-first at :214-221);
 *   - the external usearch C++ library those call sites reach (unum-cloud/usearch,
 *     NOT vendored and NOT version-pinned: absent from Cargo.toml/Cargo.lock).
 *     Its published HNSW algorithm is restated from its index.hpp /
 *     index_plugins.hpp: connectivity M (default 16), base-layer degree
 *     M0 = 2M, expansion_add efC (default 128), expansion_search ef
 *     (default 64), level multiplier 1/ln(M), greedy descent on upper
 *     levels, ef-beam on level 0 with ef = max(ef, k), heuristic
 *     ("refine") neighbour selection on both forward and reverse links,
 *     tombstone removal, metrics l2sq / ip (1 - a.b) / cos.
 *
 * Parity status: the exact (brute-force) path is pinned by numpy-f64 golden
 * vectors and the reference's own known-answer tests
 * (src/index/usearch.rs:322-425, tests/integration/usearch.rs:74-123).
 * The HNSW restatement is "parity unpinned" against upstream usearch: usearch
 * cannot be built or imported here (no cargo, no network, no vendored copy).
 *
 * Canonical tie-breaking (defined here, reproduced by the GPU path): every
 * candidate list is ordered by (distance, slot) lexicographically.
 */
#ifndef VSG_ORACLE_H
#define VSG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_METRIC_L2SQ 0
#define ORC_METRIC_IP 1
#define ORC_METRIC_COS 2

#define ORC_EMPTY 0xFFFFFFFFu

/* splitmix64 / level sampling shared bit-for-bit with the product's host code */
uint64_t orc_splitmix64(uint64_t x);
int orc_sample_level(uint64_t seed, uint64_t slot, uint32_t connectivity);

/* usearch metric_*_gt restated: f32 serial accumulation. */
float orc_distance(int metric, const float* a, const float* b, size_t dim);
/* 1 => SIMD multi-accumulator metrics with FMA at the host's widest ISA
 * (CPU-baseline timing only; vsg_fast.c). */
void orc_set_fast_metric(int on);
/* ISA the fast metrics dispatch to: "avx512f+fma", "avx2+fma" or "scalar" */
const char* orc_fast_isa(void);

/* Exact top-k.  base: n x dim row-major, keys: n (NULL => key = row index),
 * removed: n flags or NULL.  Output rows of k, ascending (distance, key);
 * padded with key UINT64_MAX / +inf.  threads <= 0 => all cores. */
int orc_exact_search(int metric, const float* base, const uint64_t* keys,
                     const uint8_t* removed, size_t n, size_t dim,
                     const float* queries, size_t nq, size_t k,
                     uint64_t* out_keys, float* out_dist, size_t* out_counts,
                     int threads);

typedef struct orc_hnsw orc_hnsw;

orc_hnsw* orc_hnsw_new(size_t dim, int metric, size_t connectivity,
                       size_t expansion_add, size_t expansion_search,
                       uint64_t seed);
void orc_hnsw_free(orc_hnsw* h);
int orc_hnsw_reserve(orc_hnsw* h, size_t capacity);
size_t orc_hnsw_size(const orc_hnsw* h);      /* live (non-removed) */
size_t orc_hnsw_slots(const orc_hnsw* h);     /* slots incl. tombstones */
size_t orc_hnsw_capacity(const orc_hnsw* h);
void orc_hnsw_params(const orc_hnsw* h, size_t* M, size_t* M0, size_t* efC,
                     size_t* ef);

/* Insert n vectors.  Duplicate live key => returns 3 (usearch: "Duplicate
 * keys not allowed"), nothing inserted.  threads > 1 inserts concurrently
 * (hnswlib-style per-node locks; non-deterministic graph); threads == 1 is
 * the deterministic sequential build.
 *
 * Free-slot reuse (usearch index_dense_gt::add_ -> index_gt::update): the
 * first keys of the call take removed slots from the free ring, oldest
 * removal first (usearch free_keys_ is a FIFO ring_gt), skipping the slot of
 * the current entry point; the rest are appended.  A reused slot keeps its
 * level; other nodes' links into it stay.  The call is a sequence of single
 * adds (usearch's add_ pops one slot per call): in call order, each reused slot
 * gets its new key and vector, its rows (every level) are cleared, it is live
 * again and it is re-linked -- before the next key's slot is touched, so later
 * reused slots still hold their old vectors and links meanwhile (round 6; round
 * 5 staged every reused slot of the call first).  Then the appended slots are
 * inserted -- each as connect_node_across_levels_ from the entry point.
 * Rules beyond a plain insert (the usearch v2 series restated):
 *   - a node is never a candidate of its own insertion (greedy descent and
 *     beam skip it; usearch asserts "Self-loops are impossible");
 *   - a reverse link into a row that already holds the node changes nothing
 *     (reconnect_neighbor_nodes_: "If new_slot is already present in the
 *     neighboring connections of close_slot then no need to modify any
 *     connections or run the heuristics");
 *   - the entry point's own slot is not reused while it is the entry point:
 *     index_gt::update clears a node's rows before connect_node_across_levels_
 *     starts from entry_slot_, which would leave the entry point linked only to
 *     itself (the documented deviation; it stays in the ring, in place). */
int orc_hnsw_add(orc_hnsw* h, const uint64_t* keys, const float* vecs,
                 size_t n, int threads);
/* Tombstone keys; returns number removed.  Each removed slot joins the back of
 * the free ring (usearch index_dense_gt::remove: free_keys_.push(slot)). */
size_t orc_hnsw_remove(orc_hnsw* h, const uint64_t* keys, size_t n);
/* The reference's upsert stream strictly one message at a time
 * (src/index/usearch.rs:214-221): per key, remove it if live, then add it
 * (sequential, single-threaded).  status[i] (optional) = that add's code;
 * returns the first non-zero code (a failed add fails only its own vector). */
int orc_hnsw_replace(orc_hnsw* h, const uint64_t* keys, const float* vecs, size_t n, int* status);
/* The free ring, oldest first: writes min(count, cap) slots, returns count.
 * Invariant: the ring holds exactly the removed slots. */
size_t orc_hnsw_free_list(const orc_hnsw* h, uint32_t* out, size_t cap);
/* 0 => append-only adds (removed slots stay tombstones; the GPU index's
 * VSG_FLAG_NO_SLOT_REUSE); 1 (default) => free-slot reuse */
void orc_hnsw_set_slot_reuse(orc_hnsw* h, int on);

/* k-NN search, ef_override 0 => index expansion_search.  One query per task
 * over `threads` workers (reference granularity, usearch.rs:275-277).
 * Outputs ascending, padded with UINT64_MAX / +inf. */
int orc_hnsw_search(const orc_hnsw* h, const float* queries, size_t nq,
                    size_t k, size_t ef_override, uint64_t* out_keys,
                    float* out_dist, size_t* out_counts, int threads,
                    uint64_t* out_ndist);

/* Graph interchange (same layout as the GPU index's HBM image):
 *   levels[slots] int8; adj0[slots*M0] u32 (ORC_EMPTY padded);
 *   upper_off[slots] u32 (first upper row or ORC_EMPTY);
 *   upper[n_upper_rows*M] u32, row (upper_off[s] + l - 1) holds level l. */
size_t orc_hnsw_upper_rows(const orc_hnsw* h);
void orc_hnsw_entry(const orc_hnsw* h, uint32_t* entry, int* max_level);
/* Import takes the removed slots as the free ring in ascending slot order (the
 * interchange carries no removal order; the GPU index's import does the same). */
int orc_hnsw_export(const orc_hnsw* h, float* vecs, uint64_t* keys,
                    uint8_t* removed, int8_t* levels, uint32_t* adj0,
                    uint32_t* upper_off, uint32_t* upper);
int orc_hnsw_import(orc_hnsw* h, size_t slots, const float* vecs,
                    const uint64_t* keys, const uint8_t* removed,
                    const int8_t* levels, const uint32_t* adj0,
                    const uint32_t* upper_off, const uint32_t* upper,
                    size_t n_upper_rows, uint32_t entry, int max_level);

#ifdef __cplusplus
}
#endif
#endif
