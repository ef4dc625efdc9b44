//! FFI declarations of the MI355X engine (`include/rdx.h`, `librdx.so`) for reductionist-rs.
//!
//! New file for the reference crate: `src/rdx_ffi.rs` (add `pub mod rdx_ffi;` to `src/lib.rs`).  Every
//! struct is `#[repr(C)]` and mirrors `include/rdx.h` field for field; the `const _` assertions at the
//! bottom pin the layout, and `tests/test_integration_cpu.py` checks the same numbers against the C
//! compiler's `sizeof` / `offsetof` of `rdx.h` (no Rust toolchain exists in this image, so this file is
//! checked textually there and compiled by a maintainer with `cargo build`).
//!
//! Each entry point replaces (reference file:line):
//!   rdx_execute / rdx_execute_owned   app.rs:163-183 `operation<T>` after the download: filter_pipeline
//!                                     (filter_pipeline.rs:19-34), validate_raw_size (app.rs:169-172),
//!                                     T::execute (operation.rs:78-96 -> operations.rs)
//!   rdx_plan                          the response sizing implied by operations.rs `Response::new` calls
//!   rdx_validate_request              models.rs:242-313 `validate_request_data` (optional)
//!   rdx_missing_from_{i64,u64,f64}    types/dvalue.rs:43-83 `TryFromDValue` (optional)
//!   rdx_context_create / _destroy     new: device pool, built in `app::init` / `AppState::new`
//!                                     (app.rs:46-53, app_state.rs:21-37)
//!   rdx_context_configure / _stats    pool limits (resource_manager.rs:54-89's role on the device) and
//!                                     request coalescing; per-device bookkeeping for metrics.rs
//!   rdx_execute_resident              rdx_execute for a chunk kept in HBM (a device-side chunk_cache.rs)
//!   rdx_execute_device / _batch_device / _multi_device, rdx_workspace_*
//!                                     new: device-resident, batched and heterogeneous entry points
//!   rdx_decompress_batch_device       compression.rs:18-27 `decompress` for a batch of device streams
//!   rdx_inflate_last_error / _string  the detail of RDX_E_DECOMPRESSION (error.rs:33-41)
//!   rdx_decompress_one_device         compression.rs:60-82 for ONE device stream, decoded by the whole device
//!   rdx_inflate_last_path             which decoder ran (k_pinflate; declined; or k_inflate)
//!   rdx_last_unsupported_reason       the cause of RDX_E_UNSUPPORTED: a blosc2 codec or a gzip / zlib stream
//!                                     k_pinflate declined (host decompression), or a request only the
//!                                     reference CPU path plans (operations.rs)
//!   rdx_execute_cbor                  app.rs:163-183 + app.rs:33-40: the response leaves the engine as
//!                                     its CBOR body
//!   rdx_cbor_bound / _encode / _encode_device
//!                                     app.rs:33-40 `serde_cbor::to_vec(&CBORResponse::new(&self))`
//!                                     (models.rs:355-416), host or device-resident outputs

#![allow(non_camel_case_types, dead_code)]

use core::mem::{offset_of, size_of};
use std::os::raw::{c_char, c_int, c_void};

pub const RDX_ABI_VERSION: u32 = 2;
pub const RDX_MAX_NDIM: usize = 32;
/// rdx_cbor_* flags: RequestData.option_shape_as_bytes / option_count_as_bytes (models.rs:173-175)
pub const RDX_CBOR_SHAPE_AS_BYTES: u32 = 1;
pub const RDX_CBOR_COUNT_AS_BYTES: u32 = 2;

/// `rdx_status` (include/rdx.h).
pub mod status {
    pub const OK: i32 = 0;
    pub const E_INVALID_ARGUMENT: i32 = 1;
    pub const E_REQUEST_VALIDATION: i32 = 2;
    pub const E_FROM_BYTES: i32 = 3;
    pub const E_SHAPE_INVALID: i32 = 4;
    pub const E_INCOMPATIBLE_MISSING: i32 = 5;
    pub const E_SHUFFLE_LENGTH: i32 = 6;
    pub const E_NAN_UNORDERED: i32 = 7;
    pub const E_UNSUPPORTED: i32 = 8;
    pub const E_DEVICE: i32 = 9;
    pub const E_OUT_OF_MEMORY: i32 = 10;
    pub const E_BUFFER_TOO_SMALL: i32 = 11;
    pub const E_NO_DEVICE: i32 = 12;
    pub const E_DECOMPRESSION: i32 = 13;
}

/// rdx_inflate_error values of a blosc2 chunk (include/rdx.h; compression.rs:29-57 messages)
pub mod blosc2 {
    pub const INVALID: u32 = 12;      // "invalid blosc2 compressed data"
    pub const FAILED: u32 = 13;       // "failed to decompress blosc2 data"
    pub const SIZE: u32 = 14;         // "unexpected decompressed size for blosc2 data"
    pub const UNSUPPORTED: u32 = 15;  // dictionaries / delta / checksummed zstd: host fallback
}

/// rdx_unsupported_reason (include/rdx.h): why the last RDX_E_UNSUPPORTED of this thread was returned.
pub mod unsupported {
    pub const NONE: u32 = 0;
    pub const BLOSC2_CODEC: u32 = 1;  // decompress on the host, then call the engine again
    pub const RANK: u32 = 2;          // every other reason: serve the request on the reference CPU path
    pub const VIEW_SIZE: u32 = 3;
    pub const VIEW_DIMS: u32 = 4;
    pub const MISSING_LIST: u32 = 5;
    pub const CBOR_SIZE: u32 = 6;
    pub const INFLATE_DECLINED: u32 = 7; // a lone gzip / zlib stream k_pinflate did not accept: host decompression
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RdxSlice {
    pub start: i64,
    pub end: i64,
    pub stride: i64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RdxFilter {
    pub id: u32, // 1 shuffle, 2 shuffle_simd
    pub reserved: u32,
    pub element_size: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct RdxMissing {
    pub kind: u32, // 0 none, 1 missing_value, 2 missing_values, 3 valid_min, 4 valid_max, 5 valid_range
    pub reserved: u32,
    pub n_values: u64,
    pub values: *const c_void, // n_values elements of the request dtype, native byte order
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct RdxRequest {
    pub abi_version: u32,
    pub op: u32,         // 0 count, 1 max, 2 min, 3 select, 4 sum
    pub dtype: u32,      // 0 int32, 1 int64, 2 uint32, 3 uint64, 4 float32, 5 float64
    pub byte_order: u32, // 0 unset, 1 little, 2 big
    pub order: u32,      // 0 unset, 1 C, 2 F
    pub axes_kind: u32,  // 0 all, 1 one, 2 multi
    pub ndim: u32,
    pub n_axes: u32,
    pub shape: *const u64,
    pub selection: *const RdxSlice,
    pub axes: *const u64,
    pub n_filters: u32,
    pub compression: u32, // 0 none, 1 gzip, 2 zlib, 3 blosc2
    pub filters: *const RdxFilter,
    pub missing: RdxMissing,
    pub has_size: u32,
    pub reserved: u32,
    pub size: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct RdxResponseInfo {
    pub dtype: u32,
    pub ndim: u32,
    pub shape: [u64; RDX_MAX_NDIM],
    pub body_bytes: u64,
    pub n_counts: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct RdxMultiItem {
    pub req: *const RdxRequest,
    pub d_chunk: *const c_void,
    pub chunk_len: u64,
    pub d_body: *mut c_void,
    pub d_counts: *mut i64,
    pub d_status: *mut u32,
}

#[repr(C)]
#[derive(Debug)]
pub struct RdxResult {
    pub info: RdxResponseInfo,
    pub body: *mut c_void,
    pub counts: *mut i64,
    pub cbor_bytes: u64,
    pub reserved: u64,
}

/// `rdx_context_config` (include/rdx.h): pool limits and request coalescing.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RdxContextConfig {
    pub max_workspaces: u32,
    pub coalesce: u32,
    pub coalesce_lanes: u32,
    pub inflate_fallback: u32, // 0: declined lone gzip / zlib streams -> E_UNSUPPORTED (INFLATE_DECLINED)
    pub coalesce_max_bytes: u64,
    pub coalesce_host_max_bytes: u64,
}

/// `rdx_device_stats` (include/rdx.h): one pool entry's bookkeeping.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RdxDeviceStats {
    pub device: i32,
    pub workspaces: u32,
    pub workspaces_busy: u32,
    pub max_workspaces: u32,
    pub requests: u64,
    pub coalesced_requests: u64,
    pub coalesced_launches: u64,
    pub outstanding_bytes: u64,
    pub waits: u64,
    pub direct_requests: u64,
    pub placed_bytes: u64,
    pub peak_outstanding_bytes: u64,
    pub host_read_requests: u64,
    pub sleeps: u64,
}

pub enum RdxContext {}
pub enum RdxWorkspace {}

#[link(name = "rdx")]
extern "C" {
    pub fn rdx_abi_version() -> u32;
    pub fn rdx_status_string(status: c_int) -> *const c_char;
    pub fn rdx_device_count() -> c_int;
    pub fn rdx_context_create(devices: *const c_int, n_devices: c_int, out: *mut *mut RdxContext) -> c_int;
    pub fn rdx_context_destroy(ctx: *mut RdxContext);
    pub fn rdx_context_configure(ctx: *mut RdxContext, cfg: *const RdxContextConfig) -> c_int;
    pub fn rdx_context_stats(ctx: *mut RdxContext, index: u32, out: *mut RdxDeviceStats) -> c_int;
    pub fn rdx_validate_request(req: *const RdxRequest) -> c_int;
    pub fn rdx_plan(req: *const RdxRequest, chunk_len: u64, info: *mut RdxResponseInfo) -> c_int;
    pub fn rdx_missing_from_i64(dtype: u32, v: i64, out: *mut c_void) -> c_int;
    pub fn rdx_missing_from_u64(dtype: u32, v: u64, out: *mut c_void) -> c_int;
    pub fn rdx_missing_from_f64(dtype: u32, v: f64, out: *mut c_void) -> c_int;
    pub fn rdx_inflate_error_string(code: u32) -> *const c_char;
    pub fn rdx_inflate_last_error() -> u32;
    pub fn rdx_inflate_last_path() -> u32;
    pub fn rdx_last_unsupported_reason() -> u32;
    pub fn rdx_blosc2_cbuffer_sizes(
        src: *const c_void,
        len: u64,
        nbytes: *mut u64,
        cbytes: *mut u64,
        blocksize: *mut u64,
    ) -> c_int;
    pub fn rdx_host_alloc(ctx: *mut RdxContext, bytes: u64, out: *mut *mut c_void) -> c_int;
    pub fn rdx_host_free(ctx: *mut RdxContext, p: *mut c_void);
    pub fn rdx_execute(
        ctx: *mut RdxContext,
        req: *const RdxRequest,
        chunk: *const c_void,
        chunk_len: u64,
        body: *mut c_void,
        body_capacity: u64,
        counts: *mut i64,
        counts_capacity: u64,
        info: *mut RdxResponseInfo,
    ) -> c_int;
    pub fn rdx_execute_owned(
        ctx: *mut RdxContext,
        req: *const RdxRequest,
        chunk: *const c_void,
        chunk_len: u64,
        out: *mut *mut RdxResult,
    ) -> c_int;
    pub fn rdx_execute_cbor(
        ctx: *mut RdxContext,
        req: *const RdxRequest,
        chunk: *const c_void,
        chunk_len: u64,
        flags: u32,
        out: *mut *mut RdxResult,
    ) -> c_int;
    pub fn rdx_result_free(ctx: *mut RdxContext, result: *mut RdxResult);
    pub fn rdx_execute_resident(
        ctx: *mut RdxContext,
        device: c_int,
        req: *const RdxRequest,
        d_chunk: *const c_void,
        chunk_len: u64,
        body: *mut c_void,
        body_capacity: u64,
        counts: *mut i64,
        counts_capacity: u64,
        info: *mut RdxResponseInfo,
    ) -> c_int;
    pub fn rdx_workspace_create(ctx: *mut RdxContext, device: c_int, out: *mut *mut RdxWorkspace) -> c_int;
    pub fn rdx_workspace_destroy(ws: *mut RdxWorkspace);
    pub fn rdx_execute_device(
        ws: *mut RdxWorkspace,
        req: *const RdxRequest,
        d_chunk: *const c_void,
        chunk_len: u64,
        d_body: *mut c_void,
        d_counts: *mut i64,
        d_status: *mut u32,
        stream: *mut c_void,
        info: *mut RdxResponseInfo,
    ) -> c_int;
    pub fn rdx_execute_batch_device(
        ws: *mut RdxWorkspace,
        req: *const RdxRequest,
        n_chunks: u64,
        h_chunk_ptrs: *const *const c_void,
        chunk_len: u64,
        d_bodies: *mut c_void,
        d_counts: *mut i64,
        d_status: *mut u32,
        stream: *mut c_void,
        info: *mut RdxResponseInfo,
    ) -> c_int;
    pub fn rdx_execute_multi_device(
        ws: *mut RdxWorkspace,
        n: u64,
        items: *const RdxMultiItem,
        stream: *mut c_void,
        statuses: *mut u32,
        infos: *mut RdxResponseInfo,
    ) -> c_int;
    pub fn rdx_decompress_one_device(
        ws: *mut RdxWorkspace,
        compression: u32,
        d_in: *const c_void,
        len: u64,
        d_out: *mut c_void,
        out_cap: u64,
        out_len: *mut u64,
        error: *mut u32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn rdx_decompress_batch_device(
        ws: *mut RdxWorkspace,
        compression: u32,
        n: u64,
        h_in_ptrs: *const *const c_void,
        h_in_lens: *const u64,
        d_out: *mut c_void,
        out_capacity: u64,
        d_out_lens: *mut u64,
        d_errors: *mut u32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn rdx_cbor_bound(info: *const RdxResponseInfo, flags: u32) -> u64;
    pub fn rdx_cbor_encode(
        info: *const RdxResponseInfo,
        body: *const c_void,
        counts: *const i64,
        flags: u32,
        out: *mut c_void,
        out_cap: u64,
        out_len: *mut u64,
    ) -> c_int;
    pub fn rdx_cbor_encode_device(
        ws: *mut RdxWorkspace,
        info: *const RdxResponseInfo,
        d_body: *const c_void,
        d_counts: *const i64,
        flags: u32,
        d_out: *mut c_void,
        out_cap: u64,
        d_out_len: *mut u64,
        d_status: *mut u32,
        stream: *mut c_void,
    ) -> c_int;
}

// ---- layout pins (the same numbers as the C compiler's sizeof / offsetof of include/rdx.h) ----------
const _: () = assert!(size_of::<RdxSlice>() == 24);
const _: () = assert!(size_of::<RdxFilter>() == 16);
const _: () = assert!(size_of::<RdxMissing>() == 24);
const _: () = assert!(size_of::<RdxRequest>() == 112);
const _: () = assert!(size_of::<RdxResponseInfo>() == 280);
const _: () = assert!(size_of::<RdxMultiItem>() == 48);
const _: () = assert!(size_of::<RdxResult>() == 312);
const _: () = assert!(size_of::<RdxContextConfig>() == 32);
const _: () = assert!(size_of::<RdxDeviceStats>() == 96);
const _: () = assert!(offset_of!(RdxContextConfig, coalesce_max_bytes) == 16);
const _: () = assert!(offset_of!(RdxDeviceStats, requests) == 16);
const _: () = assert!(offset_of!(RdxRequest, op) == 4);
const _: () = assert!(offset_of!(RdxRequest, shape) == 32);
const _: () = assert!(offset_of!(RdxRequest, selection) == 40);
const _: () = assert!(offset_of!(RdxRequest, axes) == 48);
const _: () = assert!(offset_of!(RdxRequest, n_filters) == 56);
const _: () = assert!(offset_of!(RdxRequest, compression) == 60);
const _: () = assert!(offset_of!(RdxRequest, filters) == 64);
const _: () = assert!(offset_of!(RdxRequest, missing) == 72);
const _: () = assert!(offset_of!(RdxRequest, has_size) == 96);
const _: () = assert!(offset_of!(RdxRequest, size) == 104);
const _: () = assert!(offset_of!(RdxResponseInfo, shape) == 8);
const _: () = assert!(offset_of!(RdxResponseInfo, body_bytes) == 264);
const _: () = assert!(offset_of!(RdxResponseInfo, n_counts) == 272);
const _: () = assert!(offset_of!(RdxMissing, values) == 16);
const _: () = assert!(offset_of!(RdxMultiItem, d_status) == 40);
const _: () = assert!(offset_of!(RdxResult, body) == 280);
const _: () = assert!(offset_of!(RdxResult, counts) == 288);
