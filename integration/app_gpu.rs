//! Wiring of the GPU plugins into reductionist-rs's router (changes to `src/app.rs`, reference
//! app.rs:46-79 / 123-183).  Not compiled here (no cargo).
//!
//! * start-up: `app::init` (app.rs:46-53) also creates the engine's device pool when the server runs with
//!   `--use-gpu` / `REDUCTIONIST_USE_GPU` (a new clap flag beside `use_rayon`, cli.rs:7-98), listing the
//!   devices in `REDUCTIONIST_GPU_DEVICES` (default: all visible);
//! * routes: `/v2/{count,max,min,select,sum}` go to `operation_handler::<operations_gpu::GpuX>` instead of
//!   `operations::X` (app.rs:63-67);
//! * the synchronous part: `operation_gpu::<T>` replaces `operation::<T>` (app.rs:163-183) for the GPU
//!   plugins, which take the RAW chunk — the engine runs filter_pipeline and validate_raw_size itself.

use bytes::Bytes;
use tracing::debug_span;

use crate::{compression, error::ActiveStorageError, models, operation, operations_gpu};

/// In `app::init` (app.rs:46-53).
pub fn init_gpu(args: &crate::cli::CommandLineArgs) {
    if args.use_gpu {
        operations_gpu::init(&args.gpu_devices).expect("no usable gfx950 device");
    }
}

/// In `router` (app.rs:60-79): the GPU routes.
pub fn gpu_routes() -> axum::Router<crate::app_state::SharedAppState> {
    use axum::routing::post;
    axum::Router::new()
        .route("/count", post(operation_handler::<operations_gpu::GpuCount>))
        .route("/max", post(operation_handler::<operations_gpu::GpuMax>))
        .route("/min", post(operation_handler::<operations_gpu::GpuMin>))
        .route("/select", post(operation_handler::<operations_gpu::GpuSelect>))
        .route("/sum", post(operation_handler::<operations_gpu::GpuSum>))
}

/// Replaces `operation::<T>` (app.rs:163-183) for the GPU plugins; `operation_handler` (app.rs:123-153)
/// calls it in place of `operation` (under the same task permit / rayon spawn).
pub fn operation_gpu<T: operation::Operation + operations_gpu::GpuOp>(
    request_data: models::RequestData,
    data: Bytes,
) -> Result<models::Response, ActiveStorageError> {
    // gzip / zlib: a lone request's DEFLATE stream is decoded by the whole device (k_pinflate, DESIGN.md
    // §9.1: candidate block starts, blocks and the symbols inside them decoded in parallel, then the copies
    // resolved): a 4 MiB zlib-1 chunk in 0.59 ms against 3.5 ms for zlib on one host core
    // (profiles/r05_pinflate_probe.jsonl, r05_bench.json).  A stream the device declines (a block chain it
    // does not follow, e.g. many fixed-Huffman blocks, a corrupt stream, device memory) comes back within
    // 0.2-0.8 ms as UnsupportedOperation (rdx_last_unsupported_reason() == RDX_UNSUPPORTED_INFLATE_DECLINED)
    // and is decompressed here, by the reference's own decoder (its bytes or its error).  A stream whose request states it expands more than
    // 16-fold keeps the host path, as does any request when REDUCTIONIST_GPU_INFLATE=0.
    // blosc2: a chunk is hundreds of independent block streams that the device decodes in parallel
    // (k_blosc2), but a lone 4 MiB chunk takes 1.6 ms (LZ4) / 3.3 ms (zstd) there against
    // 0.75 / 1.5 ms for liblz4 / libzstd on one host thread; so a lone blosc2 request
    // is decompressed on the host unless the operator opts in (REDUCTIONIST_GPU_BLOSC2=1).  A codec the
    // device does not decode comes back as UnsupportedOperation and is decompressed here instead.
    // (The engine's context is created with inflate_fallback = 0: a declined stream never runs the
    // one-wavefront k_inflate, 100-220 ms per 4 MiB.)
    let on_device = match request_data.compression {
        Some(models::Compression::Blosc2) => gpu_blosc2(),
        Some(_) => gpu_inflate(&request_data, data.len()),
        None => false,
    };
    if on_device {
        match debug_span!("operation_gpu").in_scope(|| operations_gpu::execute_slice(&request_data, &data, T::OP)) {
            Err(ActiveStorageError::UnsupportedOperation { .. }) => {}
            other => return other,
        }
    }
    let (request_data, data) = match request_data.compression {
        Some(c) => (host_decompressed(request_data), compression::decompress(c, &data)?),
        None => (request_data, data),
    };
    // the chunk as downloaded — page-locked when the downloader filled a pinned_gpu::PinnedBuf — straight
    // to the engine: no Bytes -> Vec conversion (zero copies, app.rs:173-181's intent)
    debug_span!("operation_gpu").in_scope(|| operations_gpu::execute_slice(&request_data, &data, T::OP))
}

/// Lone gzip / zlib requests decoded on the device (see operation_gpu): on unless REDUCTIONIST_GPU_INFLATE=0,
/// and not for a request whose shape says the chunk expands more than 16-fold.
fn gpu_inflate(request_data: &models::RequestData, compressed_len: usize) -> bool {
    static ON: std::sync::OnceLock<bool> = std::sync::OnceLock::new();
    if !*ON.get_or_init(|| std::env::var("REDUCTIONIST_GPU_INFLATE").map(|v| v != "0").unwrap_or(true)) {
        return false;
    }
    match &request_data.shape {
        Some(shape) => {
            let raw = shape.iter().product::<usize>().saturating_mul(request_data.dtype.size_of());
            raw <= compressed_len.saturating_mul(16)
        }
        None => true,
    }
}

/// Lone blosc2 requests decoded on the device (opt-in: REDUCTIONIST_GPU_BLOSC2=1; see operation_gpu).
fn gpu_blosc2() -> bool {
    static ON: std::sync::OnceLock<bool> = std::sync::OnceLock::new();
    *ON.get_or_init(|| std::env::var("REDUCTIONIST_GPU_BLOSC2").map(|v| v == "1").unwrap_or(false))
}

/// The request that goes to the engine with a chunk this host has already decompressed.  `compression`
/// is cleared and so is `size`: the reference runs validate_raw_size on the decompressed length whenever
/// the request was compressed (app.rs:169-172), and the engine runs it exactly when `size` is absent
/// (`size` of a compressed request is the compressed length, models.rs:244-249, and is no use to it).
fn host_decompressed(request_data: models::RequestData) -> models::RequestData {
    let mut rd = request_data;
    rd.compression = None;
    rd.size = None;
    rd
}

/// A handler variant whose response body the engine serialises (operations_gpu::execute_cbor): the same
/// permits, chunk store and thread-pool choice as `operation_handler` (app.rs:123-153), then the CBOR
/// bytes go out with the header `IntoResponse for models::Response` sets (app.rs:31-43).  Route e.g.
/// `/v2/count` to `operation_handler_cbor::<0>` when responses carry large count vectors.
pub async fn operation_handler_cbor<const OP: u32>(
    axum::extract::State(state): axum::extract::State<crate::app_state::SharedAppState>,
    auth: Option<axum_extra::TypedHeader<headers::Authorization<headers::authorization::Basic>>>,
    crate::validated_json::ValidatedJson(request_data): crate::validated_json::ValidatedJson<models::RequestData>,
) -> Result<axum::response::Response, ActiveStorageError> {
    use axum::response::IntoResponse;
    let memory = request_data.size.unwrap_or(0);
    let mem_permits = state.resource_manager.memory(memory).await?;
    let data = state.chunk_store.get(&auth, &request_data, &state.resource_manager, mem_permits).await?;
    let run = move || -> Result<Bytes, ActiveStorageError> {
        // a lone compressed chunk goes to the device as in operation_gpu (gzip / zlib unless the request
        // says it expands more than 16-fold; blosc2 only with REDUCTIONIST_GPU_BLOSC2=1), else the host
        let on_device = match request_data.compression {
            Some(models::Compression::Blosc2) => gpu_blosc2(),
            Some(_) => gpu_inflate(&request_data, data.len()),
            None => true,
        };
        let (request_data, data) = match request_data.compression {
            Some(c) if !on_device => {
                let d = compression::decompress(c, &data)?;
                (host_decompressed(request_data), d)
            }
            _ => (request_data, data),
        };
        match debug_span!("operation_gpu_cbor").in_scope(|| operations_gpu::execute_cbor::<OP>(&request_data, &data)) {
            // a blosc2 codec the device does not decode: decompress on the host and run again
            Err(ActiveStorageError::UnsupportedOperation { .. }) if request_data.compression.is_some() => {
                let d = compression::decompress(request_data.compression.unwrap(), &data)?;
                operations_gpu::execute_cbor::<OP>(&host_decompressed(request_data), &d)
            }
            other => other,
        }
    };
    let body = if state.args.use_rayon {
        tokio_rayon::spawn(run).await?
    } else {
        let _task_permit = state.resource_manager.task().await?;
        run()?
    };
    Ok((axum::http::StatusCode::OK, [(axum::http::header::CONTENT_TYPE, "application/cbor")], body).into_response())
}

// `operation_handler` body change (app.rs:147-152):
//
//     if state.args.use_rayon {
//         tokio_rayon::spawn(move || operation_gpu::<T>(request_data, data)).await
//     } else {
//         let _task_permit = state.resource_manager.task().await?;
//         operation_gpu::<T>(request_data, data)
//     }
use crate::app::operation_handler;
