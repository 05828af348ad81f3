//! gpu.rs -- the vector index actor of the reference, on libvsg.so (MI355X, HIP).
//!
//! Replaces /root/reference/src/index/usearch.rs:36-311 (`UsearchIndexFactory`, `new`,
//! `process`, `add_or_replace`, `remove`, `ann`, `count`) behind the unchanged plugin
//! boundary: `IndexFactory::create_index` returns an `mpsc::Sender<Index>` and the
//! `Index::{AddOrReplace, Remove, Ann, Count}` messages mean what they meant there.
//!
//! What moved into native code: the usearch HNSW (GPU batched build + search kernels)
//! and the per-message work queue, now `vsg_actor_*` (csrc/actor.hpp), which coalesces
//! concurrent single-vector adds and single-query anns into batched GPU calls and keeps
//! the reserve policy of usearch.rs:200-212 (RESERVE_INCREMENT / RESERVE_THRESHOLD).
//! What stays here, as in the reference: the PrimaryKey <-> u64 BiMap (usearch.rs:109-113),
//! the dimension checks of `ann` (:259-272) and the key -> PrimaryKey mapping of its result
//! (:285-301).  Key allocation is monotonic: a replace reuses the live key, a new primary
//! key takes the next one, nothing is rolled back (the reference's `fetch_sub`
//! rollback at :191 can hand one key to two primary keys).
//!
//! A failed add drops its PK <-> key mapping again, as usearch.rs:230-232 does: the add
//! goes through vsg_actor_add_or_replace_cb, whose completion runs `add_done` on the native
//! worker thread.  Count is the reference's read-lock size() (usearch.rs:308-311):
//! vsg_actor_size, which does not queue behind pending writes.
//!
//! One index may span several GPUs: `new_gpu_sharded(devices)` creates every index as a
//! row-sharded vsg_sharded_t (one HNSW shard per entry of `devices`, keys routed by hash,
//! per-shard top-k merged on devices[0] over xGMI; include/vsg.h "Sharded index").
//!
//! Symbol sequence a lifecycle drives (mirrored by tests/cpp/test_rust_call_sequence.cpp):
//!   vsg_actor_new | vsg_actor_new_sharded (index(es) + reserve(1M)) ->
//!   vsg_actor_add_or_replace_cb* -> vsg_actor_remove -> vsg_actor_ann_cb -> vsg_actor_size ->
//!   vsg_actor_free.
//!
//! Ann is asynchronous end to end (round 5): `vsg_actor_ann_cb` queues the query and its
//! completion `ann_done` -- run on the native worker once the batched GPU search returned --
//! maps the keys and sends the oneshot reply, as the reference's `ann` answers through a
//! oneshot (usearch.rs:251-306).  No thread blocks per query (round 4 parked a
//! `spawn_blocking` thread in `vsg_actor_ann` for every in-flight query).

use crate::Connectivity;
use crate::Dimensions;
use crate::Embedding;
use crate::ExpansionAdd;
use crate::ExpansionSearch;
use crate::IndexFactory;
use crate::IndexId;
use crate::Limit;
use crate::PrimaryKey;
use crate::index::actor::AnnR;
use crate::index::actor::CountR;
use crate::index::actor::Index;
use crate::index::vsg_sys as sys;
use anyhow::anyhow;
use bimap::BiMap;
use std::ffi::CStr;
use std::os::raw::c_int;
use std::os::raw::c_void;
use std::sync::Arc;
use std::sync::RwLock;
use tokio::sync::mpsc;
use tokio::sync::oneshot;
use tracing::Instrument;
use tracing::debug;
use tracing::debug_span;
use tracing::trace;

/// Status + thread-local message -> anyhow (include/vsg.h "Errors").
fn check(rc: c_int) -> anyhow::Result<()> {
    if rc == sys::VSG_OK {
        return Ok(());
    }
    let msg = unsafe { CStr::from_ptr(sys::vsg_last_error()) }.to_string_lossy().into_owned();
    Err(anyhow!("vsg error {rc}: {msg}"))
}

/// Owned native actor.  Every vsg_actor_* entry point is thread-safe (vsg.h).
/// `keys` is the context of the add completions: declared after `ptr`, it outlives
/// the actor's drain in `drop` (fields drop after `Drop::drop` returns).
struct GpuActor {
    ptr: *mut sys::vsg_actor_t,
    keys: Keys,
}
unsafe impl Send for GpuActor {}
unsafe impl Sync for GpuActor {}

impl Drop for GpuActor {
    fn drop(&mut self) {
        // drains queued messages (running their completions), joins the worker, frees HBM
        unsafe { sys::vsg_actor_free(self.ptr) }
    }
}

/// Completion of one add (worker thread): a failed add forgets its mapping, usearch.rs:230-232.
unsafe extern "C" fn add_done(ctx: *mut c_void, key: u64, status: c_int) {
    if status == sys::VSG_OK {
        return;
    }
    debug!("add_or_replace: unable to add embedding for key {key}: vsg error {status}");
    let keys = unsafe { &*(ctx as *const RwLock<KeyMap>) };
    keys.write().unwrap().map.remove_by_right(&key);
}

/// One ann in flight: its reply channel and the buffers the native actor fills before
/// `ann_done` runs (heap-owned, so the pointers stay valid while the query is queued).
struct AnnCtx {
    tx: Option<oneshot::Sender<AnnR>>,
    keys: Keys,
    out_keys: Vec<u64>,
    out_dist: Vec<f32>,
}

/// Completion of one ann (a native worker thread): keys -> primary keys (usearch.rs:285-296),
/// distances (:297-301), the oneshot reply.  On failure vsg_last_error() is the search's.
unsafe extern "C" fn ann_done(ctx: *mut c_void, status: c_int, count: usize) {
    let mut c = unsafe { Box::from_raw(ctx as *mut AnnCtx) };
    let result = if status != sys::VSG_OK {
        let msg = unsafe { CStr::from_ptr(sys::vsg_last_error()) }.to_string_lossy().into_owned();
        Err(anyhow!("ann: search failed: vsg error {status}: {msg}"))
    } else {
        let k = c.keys.read().unwrap();
        c.out_keys[..count]
            .iter()
            .map(|key| k.map.get_by_right(key).cloned().ok_or(anyhow!("not defined primary key column {key}")))
            .collect::<anyhow::Result<Vec<_>>>()
            .map(|pks| (pks, c.out_dist[..count].iter().map(|d| (*d).into()).collect()))
    };
    if let Some(tx) = c.tx.take() {
        tx.send(result).unwrap_or_else(|_| trace!("ann: unable to send response"));
    }
}

impl GpuActor {
    fn new(options: &sys::vsg_actor_options_t, devices: &[i32], keys: Keys) -> anyhow::Result<Self> {
        let mut a = std::ptr::null_mut();
        if devices.len() > 1 {
            check(unsafe { sys::vsg_actor_new_sharded(options, devices.len() as u32, devices.as_ptr(), &mut a) })?;
        } else {
            check(unsafe { sys::vsg_actor_new(options, &mut a) })?;
        }
        Ok(Self { ptr: a, keys })
    }

    fn add_or_replace(&self, key: u64, embedding: &[f32]) -> anyhow::Result<()> {
        let ctx = Arc::as_ptr(&self.keys) as *mut c_void;
        check(unsafe {
            sys::vsg_actor_add_or_replace_cb(self.ptr, key, embedding.as_ptr(), embedding.len(), Some(add_done), ctx)
        })
    }

    fn remove(&self, key: u64) -> anyhow::Result<()> {
        check(unsafe { sys::vsg_actor_remove(self.ptr, key) })
    }

    /// Queues the query; `ann_done` sends the reply on `tx` once its batch returned.
    fn ann(&self, embedding: &[f32], limit: usize, tx: oneshot::Sender<AnnR>) {
        let mut ctx = Box::new(AnnCtx {
            tx: Some(tx),
            keys: Arc::clone(&self.keys),
            out_keys: vec![sys::VSG_NO_KEY; limit],
            out_dist: vec![f32::INFINITY; limit],
        });
        let (ok, od) = (ctx.out_keys.as_mut_ptr(), ctx.out_dist.as_mut_ptr());
        let raw = Box::into_raw(ctx);
        let rc = unsafe {
            sys::vsg_actor_ann_cb(self.ptr, embedding.as_ptr(), embedding.len(), limit, ok, od, Some(ann_done),
                                  raw as *mut c_void)
        };
        if let Err(err) = check(rc) {
            // not queued: the completion will not run, the reply goes out here
            ctx = unsafe { Box::from_raw(raw) };
            if let Some(tx) = ctx.tx.take() {
                tx.send(Err(anyhow!("ann: search failed: {err}"))).unwrap_or_else(|_| trace!("ann: unable to send response"));
            }
        }
    }

    /// live size now, under the index's shared lock (does not wait for queued writes)
    fn size(&self) -> usize {
        unsafe { sys::vsg_actor_size(self.ptr) }
    }
}

/// `IndexFactory` for GPU-backed vector indexes (replaces `UsearchIndexFactory`,
/// usearch.rs:36-58).  Every index it creates lives on `devices`: one GPU's HBM, or one
/// row shard per listed GPU (vsg_sharded_t, merged on devices[0]).
pub struct GpuIndexFactory {
    devices: Vec<i32>,
    metric: u32,
}

impl IndexFactory for GpuIndexFactory {
    fn create_index(
        &self,
        id: IndexId,
        dimensions: Dimensions,
        connectivity: Connectivity,
        expansion_add: ExpansionAdd,
        expansion_search: ExpansionSearch,
    ) -> anyhow::Result<mpsc::Sender<Index>> {
        new(id, dimensions, connectivity, expansion_add, expansion_search, &self.devices, self.metric)
    }
}

/// GPU `device`, cosine metric.  usearch left the metric to its crate default
/// (usearch.rs:89-96); here it is explicit.
pub fn new_gpu(device: i32) -> anyhow::Result<GpuIndexFactory> {
    Ok(GpuIndexFactory { devices: vec![device], metric: sys::VSG_METRIC_COS })
}

pub fn new_gpu_with_metric(device: i32, metric: u32) -> anyhow::Result<GpuIndexFactory> {
    if metric > sys::VSG_METRIC_COS {
        return Err(anyhow!("unknown metric {metric}"));
    }
    Ok(GpuIndexFactory { devices: vec![device], metric })
}

/// Every index row-sharded over `devices` (e.g. the node's 8 GPUs: `&[0, 1, .., 7]`),
/// cosine metric; results are merged on `devices[0]`.
pub fn new_gpu_sharded(devices: &[i32]) -> anyhow::Result<GpuIndexFactory> {
    if devices.is_empty() || devices.len() > sys::VSG_MAX_SHARDS as usize {
        return Err(anyhow!("between 1 and {} shard devices", sys::VSG_MAX_SHARDS));
    }
    Ok(GpuIndexFactory { devices: devices.to_vec(), metric: sys::VSG_METRIC_COS })
}

const CHANNEL_SIZE: usize = 10; // as usearch.rs:102

type Keys = Arc<RwLock<KeyMap>>;

/// PrimaryKey <-> u64 key of the GPU index, with the next free key.
struct KeyMap {
    map: BiMap<PrimaryKey, u64>,
    next: u64,
}

pub(crate) fn new(
    id: IndexId,
    dimensions: Dimensions,
    connectivity: Connectivity,
    expansion_add: ExpansionAdd,
    expansion_search: ExpansionSearch,
    devices: &[i32],
    metric: u32,
) -> anyhow::Result<mpsc::Sender<Index>> {
    let options = sys::vsg_actor_options_t {
        index: sys::vsg_index_options_t {
            dimensions: dimensions.0.get() as u32,
            metric,
            quantization: sys::VSG_SCALAR_F32, // ScalarKind::F32, usearch.rs:94
            connectivity: connectivity.0 as u32, // 0 => usearch defaults (src/db.rs:400-410)
            expansion_add: expansion_add.0 as u32,
            expansion_search: expansion_search.0 as u32,
            device: devices[0],
            flags: 0,
            seed: 0,
        },
        // reserve(RESERVE_INCREMENT) up front and the growth rule of usearch.rs:200-212
        reserve_increment: 1_000_000,
        reserve_threshold: 1_000_000 / 3,
        // anns on one read worker beside the writes, as the reference's fire-and-forget
        // adds allow.  With completions (vsg_actor_ann_cb) one worker keeps the batches
        // largest: 512 closed-loop clients 640 k QPS on 1, 482 k on 2, 448 k on 3 read
        // workers (profiles/r05_actor_completions.jsonl)
        concurrent_reads: 1,
        ..Default::default()
    };
    let keys: Keys = Arc::new(RwLock::new(KeyMap { map: BiMap::new(), next: 0 }));
    let actor = Arc::new(GpuActor::new(&options, devices, Arc::clone(&keys))?);
    let (tx, mut rx) = mpsc::channel(CHANNEL_SIZE);
    tokio::spawn(
        async move {
            debug!("starting");
            while let Some(msg) = rx.recv().await {
                process(msg, dimensions, Arc::clone(&actor), Arc::clone(&keys)).await;
            }
            debug!("finished");
        }
        .instrument(debug_span!("gpu", "{id}")),
    );
    Ok(tx)
}

async fn process(msg: Index, dimensions: Dimensions, actor: Arc<GpuActor>, keys: Keys) {
    match msg {
        Index::AddOrReplace { primary_key, embedding } => add_or_replace(&actor, &keys, primary_key, embedding),
        Index::Remove { primary_key } => remove(&actor, &keys, primary_key),
        // queued with a completion: the reply is sent from the native worker (ann_done)
        Index::Ann { embedding, limit, tx } => ann(&actor, tx, embedding, dimensions, limit),
        Index::Count { tx } => count(&actor, tx),
    }
}

/// usearch.rs:174-233.  The native actor removes the live row of a replaced key before
/// adding (:214-221) and grows capacity; failures are counted there and logged here,
/// as the reference logs and swallows them (:207-224).
fn add_or_replace(actor: &GpuActor, keys: &Keys, primary_key: PrimaryKey, embedding: Embedding) {
    let key = {
        let mut k = keys.write().unwrap();
        match k.map.get_by_left(&primary_key) {
            Some(key) => *key,
            None => {
                let key = k.next;
                k.next += 1;
                k.map.insert(primary_key, key);
                key
            }
        }
    };
    // a failure inside the batched add arrives in `add_done`; a rejected message here
    if let Err(err) = actor.add_or_replace(key, &embedding.0) {
        debug!("add_or_replace: unable to add embedding for key {key}: {err}");
        keys.write().unwrap().map.remove_by_right(&key); // usearch.rs:230-232
    }
}

/// usearch.rs:235-249
fn remove(actor: &GpuActor, keys: &Keys, primary_key: PrimaryKey) {
    let Some((_, key)) = keys.write().unwrap().map.remove_by_left(&primary_key) else {
        return;
    };
    if let Err(err) = actor.remove(key) {
        debug!("remove: unable to remove embedding for key {key}: {err}");
    }
}

/// usearch.rs:251-306: dimension checks here (:259-272), then the batched search; the
/// key -> primary key mapping and the reply happen in `ann_done`.
fn ann(actor: &GpuActor, tx: oneshot::Sender<AnnR>, embedding: Embedding, dimensions: Dimensions, limit: Limit) {
    let len = embedding.0.len();
    if len == 0 {
        tx.send(Err(anyhow!("ann: embedding dimensions == 0"))).unwrap_or_else(|_| trace!("ann: unable to send response"));
        return;
    }
    if len != dimensions.0.get() {
        tx.send(Err(anyhow!("ann: wrong embedding dimensions: {len} != {dimensions}")))
            .unwrap_or_else(|_| trace!("ann: unable to send response"));
        return;
    }
    actor.ann(&embedding.0, limit.0.get(), tx);
}

/// usearch.rs:308-311: the live size under a read lock, answered at once
fn count(actor: &GpuActor, tx: oneshot::Sender<CountR>) {
    tx.send(Ok(actor.size())).unwrap_or_else(|_| trace!("count: unable to send response"));
}
