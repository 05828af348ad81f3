//! vsg_sys.rs -- raw FFI declarations of libvsg.so (include/vsg.h), the MI355X-native
//! replacement of the `usearch` crate the reference's index actor calls
//! (/root/reference/src/index/usearch.rs:33-34, 89-99, 201-221, 245, 276, 309).
//!
//! Layouts mirror include/vsg.h field for field (`#[repr(C)]`); every function
//! returns a status (`VSG_OK` = 0) and leaves a thread-local message readable with
//! `vsg_last_error()` on the calling thread.
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

pub const VSG_OK: c_int = 0;
pub const VSG_EINVAL: c_int = 1;
pub const VSG_ENOMEM: c_int = 2;
pub const VSG_EDUPKEY: c_int = 3;
pub const VSG_EDEVICE: c_int = 4;
pub const VSG_EUNSUPPORTED: c_int = 5;
pub const VSG_HELD: c_int = 6;
pub const VSG_REPLACE_HOLD_TAIL: u32 = 1;

pub const VSG_METRIC_L2SQ: u32 = 0;
pub const VSG_METRIC_IP: u32 = 1;
pub const VSG_METRIC_COS: u32 = 2;

pub const VSG_SCALAR_F32: u32 = 0;
pub const VSG_SCALAR_F16: u32 = 1;

pub const VSG_NO_KEY: u64 = u64::MAX;
pub const VSG_FLAG_EXACT_ONLY: u32 = 1;
pub const VSG_FLAG_F16_TRAVERSAL: u32 = 2;
pub const VSG_FLAG_NO_SLOT_REUSE: u32 = 4;

#[repr(C)]
pub struct vsg_index_t {
    _opaque: [u8; 0],
}

#[repr(C)]
pub struct vsg_actor_t {
    _opaque: [u8; 0],
}

/// usearch::IndexOptions as built at src/index/usearch.rs:89-96, metric explicit.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct vsg_index_options_t {
    pub dimensions: u32,
    pub metric: u32,
    pub quantization: u32,
    pub connectivity: u32,     // 0 => 16
    pub expansion_add: u32,    // 0 => 128
    pub expansion_search: u32, // 0 => 64
    pub device: i32,
    pub flags: u32,
    pub seed: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct vsg_stats_t {
    pub search_queries: u64,
    pub search_distances: u64,
    pub search_adjacency: u64,
    pub build_vectors: u64,
    pub build_distances: u64,
    pub build_adjacency: u64,
    pub build_batches: u64,
    pub build_select_distances: u64,
    pub reverse_recompute_distances: u64,
    pub reverse_select_distances: u64,
    pub reverse_prunes: u64,
    pub reverse_appends: u64,
    pub build_insert_ns: u64,
    pub build_sort_ns: u64,
    pub build_reverse_ns: u64,
    pub build_select_ns: u64,
    pub search_filter_overflow: u64,
    pub search_filter_reruns: u64,
    pub slots_reused: u64,
    pub ktile_copy_failures: u64,
    pub host_searches: u64,
    pub host_search_ns: u64,
    pub host_h2d_ns: u64,
    pub host_device_ns: u64,
    pub host_d2h_ns: u64,
}

/// The native actor's options (src/index/usearch.rs:60-66, 101-118 constants made knobs).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct vsg_actor_options_t {
    pub index: vsg_index_options_t,
    pub reserve_increment: u64, // 0 => RESERVE_INCREMENT = 1_000_000
    pub reserve_threshold: u64, // 0 => increment / 3
    pub max_batch: u32,         // 0 => 65536 messages per drain
    pub max_wait_us: u32,       // 0 => natural batching
    pub compact_percent: u32,   // 0 => never (slots are reused)
    pub concurrent_reads: u32,  // n >= 1 => anns on n read workers beside writes (the reference's fire-and-forget adds)
    pub compact_min_dead: u64,  // 0 => 4096
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct vsg_actor_counters_t {
    pub messages: u64,
    pub writes: u64,
    pub anns: u64,
    pub counts: u64,
    pub add_calls: u64,
    pub remove_calls: u64,
    pub search_calls: u64,
    pub reserve_calls: u64,
    pub add_errors: u64,
    pub remove_errors: u64,
    pub search_errors: u64,
    pub max_search_batch: u64,
    pub max_add_batch: u64,
    pub compactions: u64,
    pub compacted_rows: u64,
    pub compact_errors: u64,
    pub ann_queue_ns: u64,
    pub ann_wake_ns: u64,
    pub batch_search_ns: u64,
    pub batch_notify_ns: u64,
}

#[repr(C)]
pub struct vsg_sharded_t {
    _opaque: [u8; 0],
}

pub const VSG_MAX_SHARDS: u32 = 64;

/// One logical index row-sharded over the node's GPUs (SURVEY §8b `n_gpus`).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct vsg_sharded_options_t {
    pub index: vsg_index_options_t, // every shard's options (device ignored, seed + g per shard)
    pub n_shards: u32,              // 1 ..= VSG_MAX_SHARDS
    pub answer_device: i32,         // -1 => devices[0]
    pub devices: *const i32,        // n_shards ordinals (repeats allowed); null => g % device count
}

/// Completion of one AddOrReplace (vsg_actor_add_or_replace_cb), on the actor's worker thread.
pub type vsg_add_done_fn = Option<unsafe extern "C" fn(ctx: *mut c_void, key: u64, status: c_int)>;
/// Completion of one Ann (vsg_actor_ann_cb), on an actor worker thread: the oneshot reply.
pub type vsg_ann_done_fn = Option<unsafe extern "C" fn(ctx: *mut c_void, status: c_int, count: usize)>;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct vsg_file_info_t {
    pub options: vsg_index_options_t,
    pub version: u32,
    pub max_level: i32,
    pub slots: u64,
    pub live: u64,
    pub upper_rows: u64,
    pub file_bytes: u64,
}

extern "C" {
    // usearch::Index::new / reserve / capacity / size (usearch.rs:98-99, 201-206, 309)
    pub fn vsg_index_new(options: *const vsg_index_options_t, out: *mut *mut vsg_index_t) -> c_int;
    pub fn vsg_index_free(index: *mut vsg_index_t);
    pub fn vsg_index_reserve(index: *mut vsg_index_t, capacity: usize) -> c_int;
    pub fn vsg_index_capacity(index: *const vsg_index_t) -> usize;
    pub fn vsg_index_size(index: *const vsg_index_t) -> usize;
    pub fn vsg_index_dimensions(index: *const vsg_index_t) -> usize;
    pub fn vsg_index_contains(index: *const vsg_index_t, key: u64) -> c_int;
    // usearch::Index::add (usearch.rs:221), batched
    pub fn vsg_index_add(index: *mut vsg_index_t, keys: *const u64, vectors: *const f32, n: usize) -> c_int;
    pub fn vsg_index_add_device(index: *mut vsg_index_t, keys: *const u64, vectors_device: *const f32,
                                n: usize, stream: *mut c_void) -> c_int;
    // usearch::Index::remove (usearch.rs:215, 245)
    pub fn vsg_index_remove(index: *mut vsg_index_t, keys: *const u64, n: usize, n_removed: *mut usize) -> c_int;
    // the AddOrReplace stream (usearch.rs:214-221): per key remove-if-live then add, in order
    pub fn vsg_index_replace(index: *mut vsg_index_t, keys: *const u64, vectors: *const f32, n: usize, batch: usize,
                             flags: u32, status: *mut c_int, n_applied: *mut usize) -> c_int;
    pub fn vsg_index_replace_device(index: *mut vsg_index_t, keys: *const u64, vectors_device: *const f32, n: usize,
                                    batch: usize, status: *mut c_int, stream: *mut c_void) -> c_int;
    pub fn vsg_index_free_slots(index: *const vsg_index_t, out: *mut u32, cap: usize) -> usize;
    // usearch::Index::search (usearch.rs:276), batched; rows padded with VSG_NO_KEY / +inf
    pub fn vsg_index_search(index: *mut vsg_index_t, queries: *const f32, nq: usize, k: usize, ef: usize,
                            out_keys: *mut u64, out_distances: *mut f32, out_counts: *mut usize) -> c_int;
    pub fn vsg_index_exact_search(index: *mut vsg_index_t, queries: *const f32, nq: usize, k: usize,
                                  out_keys: *mut u64, out_distances: *mut f32, out_counts: *mut usize) -> c_int;
    pub fn vsg_index_search_device(index: *mut vsg_index_t, queries_device: *const f32, nq: usize, k: usize,
                                   ef: usize, out_keys_device: *mut u64, out_distances_device: *mut f32,
                                   out_counts_device: *mut u32, stream: *mut c_void) -> c_int;
    pub fn vsg_index_exact_search_device(index: *mut vsg_index_t, queries_device: *const f32, nq: usize,
                                         k: usize, out_keys_device: *mut u64, out_distances_device: *mut f32,
                                         out_counts_device: *mut u32, stream: *mut c_void) -> c_int;
    pub fn vsg_merge_topk_device(keys_device: *const u64, distances_device: *const f32, parts: usize,
                                 nq: usize, k_in: usize, k_out: usize, out_keys_device: *mut u64,
                                 out_distances_device: *mut f32, stream: *mut c_void) -> c_int;
    pub fn vsg_index_set_f16_traversal(index: *mut vsg_index_t, enable: c_int) -> c_int;
    pub fn vsg_index_set_upper_ef(index: *mut vsg_index_t, upper_ef: usize) -> c_int;
    pub fn vsg_index_stats(index: *const vsg_index_t, out: *mut vsg_stats_t) -> c_int;
    pub fn vsg_index_reset_stats(index: *mut vsg_index_t) -> c_int;
    pub fn vsg_index_graph_info(index: *const vsg_index_t, slots: *mut usize, upper_rows: *mut usize,
                                connectivity: *mut usize, entry: *mut u32, max_level: *mut c_int) -> c_int;
    pub fn vsg_index_export(index: *const vsg_index_t, vectors: *mut f32, keys: *mut u64, removed: *mut u8,
                            levels: *mut i8, adj0: *mut u32, upper_off: *mut u32, upper: *mut u32) -> c_int;
    pub fn vsg_index_import(index: *mut vsg_index_t, slots: usize, vectors: *const f32, keys: *const u64,
                            removed: *const u8, levels: *const i8, adj0: *const u32, upper_off: *const u32,
                            upper: *const u32, upper_rows: usize, entry: u32, max_level: c_int) -> c_int;
    pub fn vsg_index_compact(index: *mut vsg_index_t, n_dropped: *mut usize) -> c_int;
    pub fn vsg_index_save(index: *const vsg_index_t, path: *const c_char) -> c_int;
    pub fn vsg_index_load(path: *const c_char, device: c_int, out: *mut *mut vsg_index_t) -> c_int;
    pub fn vsg_index_file_info(path: *const c_char, out: *mut vsg_file_info_t) -> c_int;
    pub fn vsg_datagen_device(kind: c_int, n: usize, dim: usize, seed: u64, model_seed: u64, start_row: usize,
                              out_device: *mut f32, stream: *mut c_void) -> c_int;

    // one index row-sharded over several GPUs
    pub fn vsg_sharded_new(options: *const vsg_sharded_options_t, out: *mut *mut vsg_sharded_t) -> c_int;
    pub fn vsg_sharded_free(index: *mut vsg_sharded_t);
    pub fn vsg_sharded_reserve(index: *mut vsg_sharded_t, capacity: usize) -> c_int;
    pub fn vsg_sharded_capacity(index: *const vsg_sharded_t) -> usize;
    pub fn vsg_sharded_size(index: *const vsg_sharded_t) -> usize;
    pub fn vsg_sharded_dimensions(index: *const vsg_sharded_t) -> usize;
    pub fn vsg_sharded_contains(index: *const vsg_sharded_t, key: u64) -> c_int;
    pub fn vsg_sharded_shard_count(index: *const vsg_sharded_t) -> usize;
    pub fn vsg_sharded_route(index: *const vsg_sharded_t, key: u64) -> u32;
    pub fn vsg_sharded_shard(index: *mut vsg_sharded_t, g: usize) -> *mut vsg_index_t;
    pub fn vsg_sharded_add(index: *mut vsg_sharded_t, keys: *const u64, vectors: *const f32, n: usize) -> c_int;
    pub fn vsg_sharded_remove(index: *mut vsg_sharded_t, keys: *const u64, n: usize, n_removed: *mut usize) -> c_int;
    pub fn vsg_sharded_replace(index: *mut vsg_sharded_t, keys: *const u64, vectors: *const f32, n: usize,
                               batch: usize, flags: u32, status: *mut c_int, n_applied: *mut usize) -> c_int;
    pub fn vsg_sharded_search(index: *mut vsg_sharded_t, queries: *const f32, nq: usize, k: usize, ef: usize,
                              out_keys: *mut u64, out_distances: *mut f32, out_counts: *mut usize) -> c_int;
    pub fn vsg_sharded_exact_search(index: *mut vsg_sharded_t, queries: *const f32, nq: usize, k: usize,
                                    out_keys: *mut u64, out_distances: *mut f32, out_counts: *mut usize) -> c_int;
    pub fn vsg_sharded_search_device(index: *mut vsg_sharded_t, queries_device: *const f32, nq: usize, k: usize,
                                     ef: usize, exact: c_int, out_keys_device: *mut u64,
                                     out_distances_device: *mut f32, stream: *mut c_void) -> c_int;
    pub fn vsg_sharded_compact(index: *mut vsg_sharded_t, n_dropped: *mut usize) -> c_int;
    pub fn vsg_sharded_stats(index: *const vsg_sharded_t, out: *mut vsg_stats_t) -> c_int;
    pub fn vsg_sharded_reset_stats(index: *mut vsg_sharded_t) -> c_int;

    // the per-index actor (usearch.rs:82-311) with request coalescing
    pub fn vsg_actor_new(options: *const vsg_actor_options_t, out: *mut *mut vsg_actor_t) -> c_int;
    pub fn vsg_actor_free(actor: *mut vsg_actor_t);
    pub fn vsg_actor_new_sharded(options: *const vsg_actor_options_t, n_shards: u32, devices: *const i32,
                                 out: *mut *mut vsg_actor_t) -> c_int;
    pub fn vsg_actor_add_or_replace(actor: *mut vsg_actor_t, key: u64, embedding: *const f32, dims: usize) -> c_int;
    pub fn vsg_actor_add_or_replace_cb(actor: *mut vsg_actor_t, key: u64, embedding: *const f32, dims: usize,
                                       done: vsg_add_done_fn, ctx: *mut c_void) -> c_int;
    pub fn vsg_actor_ann_cb(actor: *mut vsg_actor_t, embedding: *const f32, dims: usize, limit: usize,
                            out_keys: *mut u64, out_distances: *mut f32, done: vsg_ann_done_fn,
                            ctx: *mut c_void) -> c_int;
    pub fn vsg_actor_size(actor: *const vsg_actor_t) -> usize;
    pub fn vsg_actor_remove(actor: *mut vsg_actor_t, key: u64) -> c_int;
    pub fn vsg_actor_ann(actor: *mut vsg_actor_t, embedding: *const f32, dims: usize, limit: usize,
                         out_keys: *mut u64, out_distances: *mut f32, out_count: *mut usize) -> c_int;
    pub fn vsg_actor_count(actor: *mut vsg_actor_t, out: *mut usize) -> c_int;
    pub fn vsg_actor_flush(actor: *mut vsg_actor_t) -> c_int;
    pub fn vsg_actor_counters(actor: *const vsg_actor_t, out: *mut vsg_actor_counters_t) -> c_int;
    pub fn vsg_actor_index(actor: *mut vsg_actor_t) -> *mut vsg_index_t;
    pub fn vsg_actor_sharded(actor: *mut vsg_actor_t) -> *mut vsg_sharded_t;

    pub fn vsg_sample_level(seed: u64, slot: u64, connectivity: u32) -> c_int;
    pub fn vsg_last_error() -> *const c_char;
    pub fn vsg_version() -> *const c_char;
}
