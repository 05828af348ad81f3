/*
 * vsg.h — C ABI of the MI355X-native ANN index (libvsg.so, gfx950 HIP).
 *
 * Drop-in replacement for the usearch-backed index path of the reference
 * (swasik/vector-store-text @ 2025-06-20, paths relative to /root/reference):
 * every entry point below replaces one call the reference makes into the
 * external `usearch` crate from src/index/usearch.rs (cited per function).
 * Plain pointers and sizes only; no torch / HIP types in the signatures
 * (streams are passed as void*: a hipStream_t, NULL = the HIP default stream).
 *
 * Ownership: the caller owns every host buffer for the duration
 * of a call; the library copies inputs before returning.  The library owns all
 * device memory (vectors, graph, keys, tombstones).  The PrimaryKey<->u64 map
 * stays in the caller (src/index/usearch.rs:109-113); the ABI sees u64 keys.
 *
 * Errors: int status, 0 = OK; vsg_last_error() returns a thread-local message
 * for the last failing call on this thread (the host shim maps it to
 * anyhow!, like src/index/usearch.rs:259-272, :281-295).
 *
 * Threading: every call is thread-safe.  Writers (add/remove/reserve/compact/
 * import) serialise among themselves.  Searches may run concurrently with each
 * other AND with an add (the reference runs add and search together under its
 * RwLock read side and usearch's own thread safety, usearch.rs:201-221, 276):
 * an add holds the index-wide lock only to stage its slots and to publish them,
 * not while the graph is built, so a search issued during a long batched build
 * answers at once from the last completed state (plus any rows of the build in
 * flight it reaches through new links -- a prefix of the writes).
 *
 * Memory: every device buffer comes from one stream-ordered memory pool per
 * device and is returned with hipFreeAsync on its owner's stream; streams and
 * pinned staging are recycled process-wide.  No call waits for another index's
 * device work: freeing or growing an index beside another index's build or
 * search returns in milliseconds (tests/test_gpu_concurrency.py).
 */
#ifndef VSG_H
#define VSG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VSG_OK 0
#define VSG_EINVAL 1     /* bad argument (dimension mismatch, k == 0, reserved key) */
#define VSG_ENOMEM 2     /* device or host allocation failed */
#define VSG_EDUPKEY 3    /* key already present (usearch: duplicate keys not allowed) */
#define VSG_EDEVICE 4    /* HIP runtime error */
#define VSG_EUNSUPPORTED 5

#define VSG_METRIC_L2SQ 0 /* sum (a-b)^2, no sqrt */
#define VSG_METRIC_IP 1   /* 1 - a.b */
#define VSG_METRIC_COS 2  /* 1 - a.b / (|a| |b|) */

#define VSG_SCALAR_F32 0
#define VSG_SCALAR_F16 1

#define VSG_NO_KEY UINT64_MAX /* padding key for short result rows */

/* flags: store vectors only (no HNSW graph); exact_search works, search returns
 * VSG_EUNSUPPORTED.  The brute-force MFMA configuration. */
#define VSG_FLAG_EXACT_ONLY 1u
/* flags: HNSW search walks an f16 copy of the (f32) rows and re-ranks its beam
 * of ef candidates with exact f32 distances (rerank.hip).  Returned distances
 * are the f32 metric values; the candidate set can differ from an f32 walk.
 * No usearch equivalent (opt-in; f32 storage only). */
#define VSG_FLAG_F16_TRAVERSAL 2u
/* flags: append-only adds -- removed slots stay tombstones until
 * vsg_index_compact (round-4 behaviour) instead of being re-linked by the next
 * adds (usearch's free-slot reuse, vsg_index_add).  Exact-only indexes are
 * always append-only. */
#define VSG_FLAG_NO_SLOT_REUSE 4u

typedef struct vsg_index vsg_index_t;

/* Mirrors usearch::IndexOptions as built at src/index/usearch.rs:89-96.
 * The reference leaves `metric` to the crate default, which this ABI makes
 * explicit.  0 for connectivity / expansion_* means "usearch
 * default" (16 / 128 / 64), which is what src/db.rs:400-410 passes. */
typedef struct {
    uint32_t dimensions;       /* Dimensions, src/lib.rs:146-147 */
    uint32_t metric;           /* VSG_METRIC_* */
    uint32_t quantization;     /* VSG_SCALAR_* storage in HBM (ScalarKind::F32, :95) */
    uint32_t connectivity;     /* Connectivity (M), src/lib.rs:163-164; 0 => 16, 2..64 (level-0 rows of 2M) */
    uint32_t expansion_add;    /* ExpansionAdd (efC), src/lib.rs:181-182; 0 => 128 */
    uint32_t expansion_search; /* ExpansionSearch (ef), src/lib.rs:199-200; 0 => 64 */
    int32_t device;            /* HIP device ordinal (one shard per GPU) */
    uint32_t flags;            /* VSG_FLAG_*, 0 = HNSW index */
    uint64_t seed;             /* level-sampling seed */
} vsg_index_options_t;

/* Per-index counters for the roofline: every distance
 * evaluation and adjacency-row read performed by the kernels. */
typedef struct {
    uint64_t search_queries;
    uint64_t search_distances;   /* n_dist, summed over queries */
    uint64_t search_adjacency;   /* n_adj rows read */
    uint64_t build_vectors;
    uint64_t build_distances;    /* all build distance evaluations (sum of the next three + beam) */
    uint64_t build_adjacency;
    uint64_t build_batches;
    uint64_t build_select_distances;   /* forward heuristic neighbour selection */
    uint64_t reverse_recompute_distances; /* reverse links: distances to existing neighbours */
    uint64_t reverse_select_distances; /* reverse links: heuristic re-selection */
    uint64_t reverse_prunes;           /* (level, node) segments that overflowed and were re-selected */
    uint64_t reverse_appends;          /* segments appended without re-selection */
    uint64_t build_insert_ns;          /* device time of the build kernels (HIP events on the build */
    uint64_t build_sort_ns;            /*   stream): insert (descent + beam + selection), pair sort, */
    uint64_t build_reverse_ns;         /*   reverse links -- the build roofline's time base */
    uint64_t build_select_ns;          /* the selection kernel's share of build_insert_ns (split insert) */
    uint64_t search_filter_overflow;   /* filtered searches (index with removed entries): queries whose
                                          candidate set (registers / LDS list) ran out of room ... */
    uint64_t search_filter_reruns;     /* ... and were searched again on a list in device memory sized
                                          for every slot: results are usearch's either way */
    uint64_t slots_reused;             /* removed slots re-linked by adds (free-slot reuse) */
    uint64_t ktile_copy_failures;      /* exact-only adds whose K-tiled copy failed (completed by the
                                          next exact search; the add itself succeeded) */
    uint64_t host_searches;            /* host-buffer searches (vsg_index_search / _exact_search) ... */
    uint64_t host_search_ns;           /* ... their wall time inside the library, and with
                                          VSG_PROFILE_HOST_SEARCH=1 the device-timeline split of it: */
    uint64_t host_h2d_ns;              /*   query upload, */
    uint64_t host_device_ns;           /*   search kernels (prepare .. merge), */
    uint64_t host_d2h_ns;              /*   result download (HIP events on the call's stream) */
} vsg_stats_t;

/* replaces usearch::Index::new(&options) — src/index/usearch.rs:98 */
int vsg_index_new(const vsg_index_options_t* options, vsg_index_t** out);
void vsg_index_free(vsg_index_t* index);

/* replaces usearch::Index::reserve — src/index/usearch.rs:99, :206 */
int vsg_index_reserve(vsg_index_t* index, size_t capacity);
/* replaces usearch::Index::capacity — src/index/usearch.rs:201 */
size_t vsg_index_capacity(const vsg_index_t* index);
/* replaces usearch::Index::size (live, excludes removed) — usearch.rs:202, :309 */
size_t vsg_index_size(const vsg_index_t* index);
size_t vsg_index_dimensions(const vsg_index_t* index);
int vsg_index_contains(const vsg_index_t* index, uint64_t key);

/* replaces usearch::Index::add(key, &[f32]) — src/index/usearch.rs:221.
 * Batched: n vectors of `dimensions` f32, row-major.  Any live duplicate
 * (or a duplicate inside the batch) => VSG_EDUPKEY and nothing is inserted.
 * Grows capacity automatically when needed (the reference reserves ahead,
 * usearch.rs:200-212; growth here is the same operation).
 * Free-slot reuse (usearch index_dense: add_ pops free_keys_ and runs
 * index_gt::update on the slot): the first keys of the call take removed slots,
 * oldest removal first (the entry point's slot is skipped while it is the entry
 * point); such a slot keeps its level and the other nodes' links into it, gets
 * the new key and vector and is re-linked in place, before the rest of the call
 * is appended.  The call acts as that many single adds: the reused slots are
 * re-linked in call order, in consecutive batches each staged right before it
 * (later reused slots keep their old vectors and links meanwhile).  The
 * reference's replace is remove + add (usearch.rs:214-221), so an upsert stream
 * recycles slots instead of growing (vsg_index_replace).  Rules in
 * oracle/vsg_oracle.h orc_hnsw_add; VSG_FLAG_NO_SLOT_REUSE turns it off. */
int vsg_index_add(vsg_index_t* index, const uint64_t* keys, const float* vectors, size_t n);
/* Same, with `vectors` already in device memory (f32, n x dimensions). */
int vsg_index_add_device(vsg_index_t* index, const uint64_t* keys, const float* vectors_device,
                         size_t n, void* stream);

/* replaces usearch::Index::remove(key) — src/index/usearch.rs:215, :245.
 * Tombstones (traversed by searches, never returned) and queues each slot at
 * the back of the free ring for reuse by later adds; *n_removed (optional)
 * counts keys that were live. */
int vsg_index_remove(vsg_index_t* index, const uint64_t* keys, size_t n, size_t* n_removed);
/* replaces the AddOrReplace body of src/index/usearch.rs:214-221 (`if remove {
 * idx.remove(key) }` then `idx.add(key, &embedding)`, one message before the next,
 * fed per key by src/monitor_items.rs:56-80), batched: for each i in order, key
 * i is removed if live and then added with vector i.  Results follow the
 * one-message-at-a-time sequence -- every key takes the slot that sequence gives
 * it (free ring, oldest first), keys may repeat (a later message wins) -- while the
 * GPU applies the messages in chunks of consecutive keys: a chunk removes its live
 * keys and re-links their freed slots as one batch, so the rest of the stream
 * stays live with its old vectors meanwhile.  Chunk sizes: batch != 0 => at most
 * `batch`; 0 => max(1, size / 4096) for keys re-linked into free slots (every key
 * alone below 8,192 live rows: exactly the sequence) and max(1, size / 8) for keys
 * appended as new rows (the bulk build's batching).  Chunk boundaries depend on
 * the keys and the index state only, never on timing.  flags
 * VSG_REPLACE_HOLD_TAIL: an incomplete last chunk (fewer keys than its size, and
 * not ended by a following key) is left unapplied: its keys get status
 * VSG_HELD and *n_applied (optional) counts the keys applied -- a caller
 * streaming messages in pieces re-submits the held ones, in order, ahead of the
 * next piece and gets the chunks an uncut stream gets (the actor does).  status
 * (optional, n entries): per key VSG_OK, VSG_HELD or the
 * error of its chunk; a failed chunk does not stop the others (the reference
 * fails per vector, usearch.rs:221-232); returns the first error.  A key whose
 * add failed is absent afterwards (the reference drops its mapping, :230-232). */
#define VSG_REPLACE_HOLD_TAIL 1u
#define VSG_HELD 6 /* status of a key left unapplied under VSG_REPLACE_HOLD_TAIL (not an error) */
int vsg_index_replace(vsg_index_t* index, const uint64_t* keys, const float* vectors, size_t n, size_t batch,
                      uint32_t flags, int* status, size_t* n_applied);
/* Same, with `vectors` in device memory (f32, n x dimensions) ordered after `stream`. */
int vsg_index_replace_device(vsg_index_t* index, const uint64_t* keys, const float* vectors_device, size_t n,
                             size_t batch, int* status, void* stream);
/* The free ring (usearch index_dense free_keys_): removed slots, oldest removal
 * first -- exactly the index's removed slots.  Copies up to `cap` slot ids to
 * `out` (may be NULL) and returns how many there are. */
size_t vsg_index_free_slots(const vsg_index_t* index, uint32_t* out, size_t cap);

/* replaces usearch::Index::search(&[f32], k) — src/index/usearch.rs:275-277.
 * HNSW k-NN for nq queries; ef = max(ef ? ef : expansion_search, k).
 * out_keys / out_distances: nq x k row-major, ascending distance, rows padded
 * with VSG_NO_KEY / +inf past out_counts[i] (optional). */
int vsg_index_search(vsg_index_t* index, const float* queries, size_t nq, size_t k, size_t ef,
                     uint64_t* out_keys, float* out_distances, size_t* out_counts);
/* Exact brute force over all live vectors (absent in the reference);
 * same signature; ties broken by insertion slot. */
int vsg_index_exact_search(vsg_index_t* index, const float* queries, size_t nq, size_t k,
                           uint64_t* out_keys, float* out_distances, size_t* out_counts);

/* Switch the f16 traversal + f32 re-rank mode (VSG_FLAG_F16_TRAVERSAL) on an
 * existing index; the f16 copy is built by the next search (and freed when
 * switched off).  VSG_EINVAL unless the storage is f32.  Not in usearch. */
int vsg_index_set_f16_traversal(vsg_index_t* index, int enable);

/* Opt-in multi-entry descent (not usearch): upper_ef > 1 replaces the greedy
 * step on level 1 by a beam of width min(upper_ef, ef) whose whole result set
 * seeds the level-0 beam (register search kernel).  0 or 1 = usearch's greedy
 * descent (default).  Raises recall at a given ef; results are no longer the
 * usearch traversal's, so parity is by recall, not bit-exact.  An index holding
 * removed entries searches with the greedy descent (its overflow re-run walks a
 * sorted list in device memory that has no multi-entry form). */
int vsg_index_set_upper_ef(vsg_index_t* index, size_t upper_ef);

/* Device-resident variants: queries (f32 nq x dimensions), outputs and counts
 * (u32, optional) in device memory; enqueued on `stream` (NULL => the HIP
 * default stream) and NOT synchronised.  Used by bench.py and the multi-GPU
 * merge.  Writers may run beside an enqueued search: each one records a
 * completion event, and a writer that frees or rewrites memory the search may
 * read (capacity growth, compaction, the f16 copy's reallocation) first waits
 * for every such event; appends and removes do not wait (the search sees a
 * prefix of them, as with vsg_index_search).  Searches enqueued on different
 * streams run concurrently on the device (each takes its own scratch set, up
 * to 4 per index), so a second stream fills the tail of a batch's last round
 * of resident waves; on one stream they run in order. */
int vsg_index_search_device(vsg_index_t* index, const float* queries_device, size_t nq, size_t k,
                            size_t ef, uint64_t* out_keys_device, float* out_distances_device,
                            uint32_t* out_counts_device, void* stream);
int vsg_index_exact_search_device(vsg_index_t* index, const float* queries_device, size_t nq,
                                  size_t k, uint64_t* out_keys_device,
                                  float* out_distances_device, uint32_t* out_counts_device,
                                  void* stream);

/* k-way merge of per-shard top-k rows (after an all-gather over xGMI,
 * SURVEY §8e): parts x nq x k_in (keys, distances; rows ascending, padded with
 * VSG_NO_KEY) -> nq x k_out ascending by (distance, key).  k_in < k_out is
 * allowed: a shard may return fewer candidates than the final k. */
int vsg_merge_topk_device(const uint64_t* keys_device, const float* distances_device,
                          size_t parts, size_t nq, size_t k_in, size_t k_out,
                          uint64_t* out_keys_device, float* out_distances_device, void* stream);

int vsg_index_stats(const vsg_index_t* index, vsg_stats_t* out);
int vsg_index_reset_stats(vsg_index_t* index);

/* Graph image, same layout as oracle/vsg_oracle.h "Graph interchange" (and the
 * HBM layout): vectors as stored (f32 rows of `dimensions`,
 * normalised for cos), keys, removed flags, levels, level-0 adjacency
 * slots x 2M, upper_off, upper rows x M.  Sizes via vsg_index_graph_info. */
int vsg_index_graph_info(const vsg_index_t* index, size_t* slots, size_t* upper_rows,
                         size_t* connectivity, uint32_t* entry, int* max_level);
int vsg_index_export(const vsg_index_t* index, float* vectors, uint64_t* keys, uint8_t* removed,
                     int8_t* levels, uint32_t* adj0, uint32_t* upper_off, uint32_t* upper);
int vsg_index_import(vsg_index_t* index, size_t slots, const float* vectors,
                     const uint64_t* keys, const uint8_t* removed, const int8_t* levels,
                     const uint32_t* adj0, const uint32_t* upper_off, const uint32_t* upper,
                     size_t upper_rows, uint32_t entry, int max_level);

/* Compaction (optional since round 5: adds re-link removed
 * slots): tombstoned rows (vsg_index_remove) keep routing the traversal until
 * the next adds reuse them or compaction drops them.  Gathers the live rows in
 * slot order into a dense image and rebuilds the graph over them on the GPU.
 * Keys, live size and capacity are unchanged; *n_dropped (optional) = slots
 * freed.  Takes the writer lock.  usearch compacts through its own
 * `compact`/`isolate` (not called by the reference, src/index/usearch.rs:235-249). */
int vsg_index_compact(vsg_index_t* index, size_t* n_dropped);

/* Persistence (the reference rebuilds from a DB scan instead,
 * src/db_index.rs:213-237).  One file: a 128-byte header (magic "VSGIDX\0\1",
 * version 2, options, sizes, entry point, FNV-1a-64 checksums) followed by the
 * HBM image (stored rows, |x|^2, keys, flags, levels, level-0 adjacency,
 * upper_off, upper rows) and the free ring ((slots - live) u32, oldest removal
 * first).  Version-1 files (no ring) load with the removed slots ascending.  Save writes `path`.tmp then renames.  Load creates a
 * new index on `device` and verifies sizes and both checksums; a loaded index
 * answers searches bit-identically to the saved one. */
typedef struct {
    vsg_index_options_t options; /* as created (device = the saving device) */
    uint32_t version;
    int32_t max_level;
    uint64_t slots;      /* stored rows, tombstones included */
    uint64_t live;       /* vsg_index_size() */
    uint64_t upper_rows;
    uint64_t file_bytes;
} vsg_file_info_t;

int vsg_index_save(const vsg_index_t* index, const char* path);
int vsg_index_load(const char* path, int device, vsg_index_t** out);
/* header check only (magic, version, header checksum, size); no device needed */
int vsg_index_file_info(const char* path, vsg_file_info_t* out);

/* Synthetic inputs generated in HBM (vsg/datagen.py formulas): kind 0 =
 * clustered-latent, 1 = iid gaussian, 2 = uint8-valued, 3 = SIFT-like
 * (clustered, ReLU, x48, rounded into 0..255). */
int vsg_datagen_device(int kind, size_t n, size_t dim, uint64_t seed, uint64_t model_seed,
                       size_t start_row, float* out_device, void* stream);

/* ---------------------------------------------------------- Sharded index --
 * One logical index row-sharded over the GPUs of a node (SURVEY §8b
 * `create(opts{..., n_gpus, seed})`, §8e; north_star: "the index shards by
 * row-range across the 8 GPUs of one node with per-shard top-k merged over
 * xGMI").  Shard g is a vsg_index_t on devices[g] with its own HNSW graph;
 * several shards may share a device.  A key lives on shard vsg_sharded_route()
 * = splitmix64(key) mod n_shards: balanced for any key stream (the reference
 * allocates monotonic keys, usearch.rs:181), and a duplicate or replaced key
 * always meets its live copy on the same shard.
 *   add     splits the batch by shard, checks every shard for reserved and
 *           duplicate keys first (any => nothing is inserted, as
 *           vsg_index_add), then builds all shards concurrently: one host
 *           thread and stream per shard, no communication.
 *   search  broadcasts the queries to each shard device, searches every shard
 *           concurrently (top-k per shard), gathers the per-shard rows to the
 *           answering device (peer DMA over xGMI; a device-local copy when a
 *           shard lives there) and k-way merges them (merge_topk64_kernel):
 *           rows ascending by (distance, key), padded with VSG_NO_KEY / +inf.
 * Replaces the one-device usearch::Index of src/index/usearch.rs:89-99 when an
 * index is spread over several GPUs.  Thread-safety as vsg_index_t; writers
 * serialise on the sharded index. */
typedef struct vsg_sharded vsg_sharded_t;

#define VSG_MAX_SHARDS 64

typedef struct {
    vsg_index_options_t index; /* every shard's options; index.device is ignored, shard g's
                                  level seed is index.seed + g */
    uint32_t n_shards;         /* 1 .. VSG_MAX_SHARDS */
    int32_t answer_device;     /* device that merges and returns results; -1 => devices[0] */
    const int32_t* devices;    /* n_shards device ordinals (repeats allowed); NULL => shard g
                                  on device g mod (visible device count) */
} vsg_sharded_options_t;

int vsg_sharded_new(const vsg_sharded_options_t* options, vsg_sharded_t** out);
void vsg_sharded_free(vsg_sharded_t* index);
/* each shard reserves ceil(capacity / n_shards) (shards also grow on add) */
int vsg_sharded_reserve(vsg_sharded_t* index, size_t capacity);
size_t vsg_sharded_capacity(const vsg_sharded_t* index); /* sum over shards */
size_t vsg_sharded_size(const vsg_sharded_t* index);     /* live rows, sum over shards */
size_t vsg_sharded_dimensions(const vsg_sharded_t* index);
int vsg_sharded_contains(const vsg_sharded_t* index, uint64_t key);
size_t vsg_sharded_shard_count(const vsg_sharded_t* index);
uint32_t vsg_sharded_route(const vsg_sharded_t* index, uint64_t key);
/* borrowed handle of shard g (stats, export, save); valid until vsg_sharded_free */
vsg_index_t* vsg_sharded_shard(vsg_sharded_t* index, size_t g);
int vsg_sharded_add(vsg_sharded_t* index, const uint64_t* keys, const float* vectors, size_t n);
int vsg_sharded_remove(vsg_sharded_t* index, const uint64_t* keys, size_t n, size_t* n_removed);
/* vsg_index_replace on every shard concurrently (each key's messages meet on its
 * shard, which applies its own sub-stream in order).  With VSG_REPLACE_HOLD_TAIL
 * each shard holds its own tail (status VSG_HELD; re-submitted in order, they
 * lead that shard's next sub-stream). */
int vsg_sharded_replace(vsg_sharded_t* index, const uint64_t* keys, const float* vectors, size_t n, size_t batch,
                        uint32_t flags, int* status, size_t* n_applied);
/* as vsg_index_search / _exact_search: every shard returns its top k */
int vsg_sharded_search(vsg_sharded_t* index, const float* queries, size_t nq, size_t k, size_t ef,
                       uint64_t* out_keys, float* out_distances, size_t* out_counts);
int vsg_sharded_exact_search(vsg_sharded_t* index, const float* queries, size_t nq, size_t k,
                             uint64_t* out_keys, float* out_distances, size_t* out_counts);
/* Device-resident: queries and outputs on the answering device, enqueued on
 * `stream` (a stream of that device) and not synchronised.  exact != 0 =>
 * brute force. */
int vsg_sharded_search_device(vsg_sharded_t* index, const float* queries_device, size_t nq, size_t k,
                              size_t ef, int exact, uint64_t* out_keys_device,
                              float* out_distances_device, void* stream);
int vsg_sharded_compact(vsg_sharded_t* index, size_t* n_dropped);
/* counters summed over shards (device times: the sum of every shard's) */
int vsg_sharded_stats(const vsg_sharded_t* index, vsg_stats_t* out);
int vsg_sharded_reset_stats(vsg_sharded_t* index);

/* ------------------------------------------------------------------ Actor --
 * The reference's per-index actor (src/index/usearch.rs:82-311: an mpsc
 * channel of Index::{AddOrReplace, Remove, Ann, Count} messages served by
 * tokio/rayon tasks) with the GPU index behind it.  One worker thread per actor
 * drains the message FIFO and turns runs of single-vector adds and single-query
 * anns into batched GPU calls; capacity grows like
 * usearch.rs:200-212; tombstones left by removes and replaces are compacted
 * away once they reach compact_percent of the stored rows.  Messages apply in submission order (an ann sees every
 * write submitted before it).  Every function is thread-safe; errors are
 * reported through vsg_last_error() like the index calls.  The PK<->u64
 * bimap stays in the caller, as in the reference (usearch.rs:109-113). */
typedef struct vsg_actor vsg_actor_t;

typedef struct {
    vsg_index_options_t index;
    uint64_t reserve_increment; /* RESERVE_INCREMENT (usearch.rs:63); 0 => 1,000,000 */
    uint64_t reserve_threshold; /* RESERVE_THRESHOLD (:67); 0 => increment / 3 */
    uint32_t max_batch;         /* messages drained per worker wake-up; 0 => 65536 */
    uint32_t max_wait_us;       /* optional coalescing window; 0 => natural batching */
    uint32_t compact_percent;   /* vsg_index_compact once tombstones >= this % of stored
                                   rows; 0 => never (default since round 5: adds re-link
                                   removed slots, as usearch does), >= 100 => never */
    uint32_t concurrent_reads;  /* n >= 1: anns run on n read workers beside the writes and see
                                   a prefix of them (the reference's fire-and-forget adds,
                                   usearch.rs:200-221); n >= 2 keeps n search batches in
                                   flight (capped at 8); 0: submission order (default) */
    uint64_t compact_min_dead;  /* ... and at least this many; 0 => 4096 */
} vsg_actor_options_t;

typedef struct {
    uint64_t messages, writes, anns, counts;
    uint64_t add_calls, remove_calls, search_calls, reserve_calls;
    uint64_t add_errors, remove_errors, search_errors;
    uint64_t max_search_batch, max_add_batch;
    uint64_t compactions, compacted_rows, compact_errors;
    /* serving-path breakdown, steady-clock ns summed: per ann, submission -> its batch
     * starts (coalescing / queueing) and finish -> the caller running again (wake-up);
     * per search batch (search_calls of them), the batched search call and the
     * result copies + completion signals */
    uint64_t ann_queue_ns, ann_wake_ns, batch_search_ns, batch_notify_ns;
} vsg_actor_counters_t;

/* replaces usearch::new (the actor spawn + Index::new + reserve(1M)) — usearch.rs:82-139 */
int vsg_actor_new(const vsg_actor_options_t* options, vsg_actor_t** out);
/* Same actor over a sharded index: options->index is every shard's options,
 * shard g on devices[g] (NULL => g mod device count), results merged on devices[0]. */
int vsg_actor_new_sharded(const vsg_actor_options_t* options, uint32_t n_shards, const int32_t* devices,
                          vsg_actor_t** out);
/* drains queued messages, stops the worker, frees the index (channel close, :129) */
void vsg_actor_free(vsg_actor_t* actor);
/* Index::AddOrReplace — usearch.rs:174-233.  Asynchronous (the reference's
 * channel send); failures inside the worker are counted (add_errors), as the
 * reference logs and swallows them (:207-224). */
int vsg_actor_add_or_replace(vsg_actor_t* actor, uint64_t key, const float* embedding, size_t dims);
/* Same, with a completion: `done(ctx, key, status)` runs on the actor's worker
 * thread once the batched add carrying this message finished (status VSG_OK or
 * the add's error).  The reference awaits every add and drops the new PK<->key
 * mapping when it failed (usearch.rs:198-232); the host shim does that here. */
typedef void (*vsg_add_done_fn)(void* ctx, uint64_t key, int status);
int vsg_actor_add_or_replace_cb(vsg_actor_t* actor, uint64_t key, const float* embedding, size_t dims,
                                vsg_add_done_fn done, void* ctx);
/* Index::Remove — usearch.rs:235-249 (asynchronous; unknown keys are ignored) */
int vsg_actor_remove(vsg_actor_t* actor, uint64_t key);
/* Index::Ann — usearch.rs:251-306.  Blocks until answered.  Dimension errors
 * as :259-272.  out_*: `limit` entries, ascending, padded with VSG_NO_KEY/+inf
 * past *out_count. */
int vsg_actor_ann(vsg_actor_t* actor, const float* embedding, size_t dims, size_t limit,
                  uint64_t* out_keys, float* out_distances, size_t* out_count);
/* Index::Ann with a completion instead of a blocked thread -- the C form of the
 * reference's oneshot reply (usearch.rs:251-306: `ann` sends the query with a
 * oneshot::Sender and the caller awaits the receiver).  Same checks and batching as
 * vsg_actor_ann; returns at once.  `done(ctx, status, count)` runs on an actor worker
 * thread once the batched search carrying this query finished, after out_keys /
 * out_distances (`limit` entries each, caller-owned until then, ascending, padded
 * past count) were written; on failure status is the search's error and
 * vsg_last_error() inside the callback holds its message.  The callback may submit
 * further messages; it must not block on the actor. */
typedef void (*vsg_ann_done_fn)(void* ctx, int status, size_t count);
int vsg_actor_ann_cb(vsg_actor_t* actor, const float* embedding, size_t dims, size_t limit,
                     uint64_t* out_keys, float* out_distances, vsg_ann_done_fn done, void* ctx);
/* Index::Count — usearch.rs:308-311 (live size) */
int vsg_actor_count(vsg_actor_t* actor, size_t* out);
/* Index::Count as the reference computes it (usearch.rs:308-311: a read-lock
 * size() beside fire-and-forget adds): the live size now, without queueing
 * behind pending writes (vsg_actor_count waits for them in submission order) */
size_t vsg_actor_size(const vsg_actor_t* actor);
/* wait until all previously submitted writes (and, in submission-order mode,
 * every other message) are applied */
int vsg_actor_flush(vsg_actor_t* actor);
int vsg_actor_counters(const vsg_actor_t* actor, vsg_actor_counters_t* out);
/* borrowed handle of the actor's index (stats, export); valid until vsg_actor_free.
 * A sharded actor returns its shard 0 here and the whole index from vsg_actor_sharded. */
vsg_index_t* vsg_actor_index(vsg_actor_t* actor);
vsg_sharded_t* vsg_actor_sharded(vsg_actor_t* actor); /* NULL for a one-device actor */

/* splitmix64 level draw; bit-identical to oracle/vsg_oracle.c */
int vsg_sample_level(uint64_t seed, uint64_t slot, uint32_t connectivity);

const char* vsg_last_error(void);
const char* vsg_version(void);

#ifdef __cplusplus
}
#endif
#endif
