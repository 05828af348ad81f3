//! httproutes_vector.rs -- the vector-index HTTP routes over the GPU index actor.
//!
//! UNCOMPILED SOURCE: no Rust toolchain exists in this image, and the file is not wired into
//! a lib.rs here -- tests/test_rust_shim.py checks its routes, fields and statuses against the
//! Python twin (vsg/httproutes.py) by reading the text.  A maintainer adds
//! `pub mod httproutes_vector;` beside the reference's httproutes and `cargo check`s it.
//!
//! The reference's compiled router (/root/reference/src/httproutes.rs:37-150) serves only
//! the text backend; its vector routes survive as the client its integration tests call
//! (/root/reference/tests/integration/httpclient.rs:35-80):
//!
//!   GET  /api/v1/indexes                          -> [IndexId]                  (:35-44)
//!   POST /api/v1/indexes/{keyspace}/{index}/ann   PostIndexAnnRequest
//!                                                 -> PostIndexAnnResponse       (:46-67)
//!   GET  /api/v1/indexes/{keyspace}/{index}/count -> usize                      (:69-80)
//!
//! These handlers serve that shape in the style of the text routes (`post_index_search`,
//! httproutes.rs:132-150): the index comes from `engine.get_index(id)` (404 with an empty
//! body when unknown), the call goes through `IndexExt::{ann, count}` to the index actor
//! (`gpu.rs`: the native vsg_actor coalesces concurrent anns into one GPU launch), an index
//! error is a 500 whose body is the error text, and a body that does not deserialize --
//! a missing `embedding`, a wrong type, `limit: 0` (`Limit` is a `NonZeroUsize`,
//! src/lib.rs:234-256) -- is axum's `Json` rejection, 422.  A missing `limit` is 1
//! (`#[serde(default)]`, as PostIndexSearchRequest has it, httproutes.rs:112-117).
//!
//! The Python twin (`vector-store-text_amd/vsg/httproutes.py`) serves the same routes over
//! the same native actor and is what tests/test_http.py and tests/test_gpu_http.py exercise
//! (no cargo / rustc in this image); tests/test_rust_shim.py checks this file's routes,
//! request / response fields and status mapping against it.
//!
//! Wiring: `mod httproutes_vector;` in src/lib.rs and, in `httproutes::new`
//! (httproutes.rs:37-51), `router.merge(httproutes_vector::new(state))` beside the text
//! routes.  The primary-key column names of an index (the response is column-major,
//! `{column: [values]}`) come from the schema the ingest side already reads
//! (src/db.rs, the table's primary key); `PrimaryKeyColumns` is that lookup.

use crate::ColumnName;
use crate::Distance;
use crate::Embedding;
use crate::IndexId;
use crate::Limit;
use crate::PrimaryKey;
use crate::engine::Engine;
use crate::engine::EngineExt;
use crate::index::IndexExt;
use axum::Router;
use axum::extract;
use axum::extract::Path;
use axum::extract::State;
use axum::http::StatusCode;
use axum::response::IntoResponse;
use axum::response::Response;
use axum::routing::get;
use axum::routing::post;
use scylla::value::CqlValue; // as the reference imports it (src/db_index.rs:22, src/index/usearch.rs:317)
use serde_json::Value;
use std::collections::HashMap;
use std::sync::Arc;
use tokio::sync::mpsc::Sender;
use tracing::debug;

/// Body of `POST .../ann` (client: httpclient.rs:57).
#[derive(serde::Deserialize, serde::Serialize, utoipa::ToSchema)]
pub struct PostIndexAnnRequest {
    pub embedding: Embedding,
    #[serde(default)]
    pub limit: Limit,
}

/// Reply of `POST .../ann` (client: httpclient.rs:62-65): primary keys column-major, one
/// list of values per primary-key column, in ascending-distance order beside `distances`.
#[derive(serde::Deserialize, serde::Serialize, utoipa::ToSchema)]
pub struct PostIndexAnnResponse {
    pub primary_keys: HashMap<ColumnName, Vec<Value>>,
    pub distances: Vec<Distance>,
}

/// Primary-key column names of an index's table, in key order.
pub trait PrimaryKeyColumns: Send + Sync + 'static {
    fn columns(&self, id: &IndexId) -> Option<Vec<ColumnName>>;
}

#[derive(Clone)]
pub struct VectorRoutesState {
    pub engine: Sender<Engine>,
    pub pk_columns: Arc<dyn PrimaryKeyColumns>,
}

pub fn new(state: VectorRoutesState) -> Router {
    Router::new()
        .route("/api/v1/indexes", get(get_indexes))
        .route("/api/v1/indexes/{keyspace}/{index}/ann", post(post_index_ann))
        .route("/api/v1/indexes/{keyspace}/{index}/count", get(get_index_count))
        .with_state(state)
}

/// `IndexId` of `{keyspace}.{index}` (tests/integration/usearch.rs:113 lists "vector.ann").
fn index_id(keyspace: &str, index: &str) -> IndexId {
    IndexId::from(format!("{keyspace}.{index}"))
}

async fn get_indexes(State(state): State<VectorRoutesState>) -> Response {
    (StatusCode::OK, extract::Json(state.engine.get_index_ids().await)).into_response()
}

/// One CQL value of a primary key as JSON (the column types a primary key can have).
fn cql_to_json(v: &CqlValue) -> Value {
    match v {
        CqlValue::TinyInt(x) => Value::from(*x),
        CqlValue::SmallInt(x) => Value::from(*x),
        CqlValue::Int(x) => Value::from(*x),
        CqlValue::BigInt(x) => Value::from(*x),
        CqlValue::Counter(x) => Value::from(x.0),
        CqlValue::Boolean(x) => Value::from(*x),
        CqlValue::Float(x) => Value::from(*x),
        CqlValue::Double(x) => Value::from(*x),
        CqlValue::Text(x) | CqlValue::Ascii(x) => Value::from(x.as_str()),
        CqlValue::Uuid(x) => Value::from(x.to_string()),
        CqlValue::Timeuuid(x) => Value::from(x.to_string()),
        other => Value::from(format!("{other:?}")),
    }
}

async fn post_index_ann(
    State(state): State<VectorRoutesState>,
    Path((keyspace, index)): Path<(String, String)>,
    extract::Json(request): extract::Json<PostIndexAnnRequest>,
) -> Response {
    let id = index_id(&keyspace, &index);
    let Some(actor) = state.engine.get_index(id.clone()).await else {
        return (StatusCode::NOT_FOUND, "").into_response();
    };
    let Some(columns) = state.pk_columns.columns(&id) else {
        return (StatusCode::NOT_FOUND, "").into_response();
    };
    match actor.ann(request.embedding, request.limit).await {
        Err(err) => {
            let msg = format!("index.ann request error: {err}");
            debug!("post_index_ann: {msg}");
            (StatusCode::INTERNAL_SERVER_ERROR, msg).into_response()
        }
        Ok((primary_keys, distances)) => {
            let mut cols: HashMap<ColumnName, Vec<Value>> =
                columns.iter().map(|c| (c.clone(), Vec::with_capacity(primary_keys.len()))).collect();
            for PrimaryKey(values) in primary_keys.iter() {
                if values.len() != columns.len() {
                    let msg = format!("index.ann request error: primary key of {} values, {} columns",
                                      values.len(), columns.len());
                    debug!("post_index_ann: {msg}");
                    return (StatusCode::INTERNAL_SERVER_ERROR, msg).into_response();
                }
                for (c, v) in columns.iter().zip(values.iter()) {
                    cols.get_mut(c).unwrap().push(cql_to_json(v));
                }
            }
            let resp = PostIndexAnnResponse { primary_keys: cols, distances };
            (StatusCode::OK, extract::Json(resp)).into_response()
        }
    }
}

async fn get_index_count(
    State(state): State<VectorRoutesState>,
    Path((keyspace, index)): Path<(String, String)>,
) -> Response {
    let Some(actor) = state.engine.get_index(index_id(&keyspace, &index)).await else {
        return (StatusCode::NOT_FOUND, "").into_response();
    };
    match actor.count().await {
        Err(err) => {
            let msg = format!("index.count request error: {err}");
            debug!("get_index_count: {msg}");
            (StatusCode::INTERNAL_SERVER_ERROR, msg).into_response()
        }
        Ok(count) => (StatusCode::OK, extract::Json(count)).into_response(),
    }
}
