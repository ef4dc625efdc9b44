//! GPU `Operation` plugins for reductionist-rs: the same plugin surface (`operation.rs:53-66`) backed by
//! the MI355X engine through `rdx_ffi` (this directory).  New file for the reference crate:
//! `src/operations_gpu.rs`; `app.rs` routes `/v2/{count,max,min,select,sum}` to `GpuCount` ... `GpuSum`
//! when the server runs with a GPU (see `app_gpu.rs`).  Not compiled in this image (no cargo): checked
//! textually by `tests/test_integration_cpu.py`.
//!
//! Each `execute` takes the RAW chunk (still compressed, still shuffled): the engine runs
//! `filter_pipeline` (`filter_pipeline.rs:19-34`), `validate_raw_size` (`app.rs:169-172`), the byte-order
//! swap and slicing (`array.rs:147-208`, `:93-144`) and the `NumOperation` (`operations.rs`) in the
//! reference's order, and returns the first error the reference would raise.

use std::os::raw::c_void;
use std::sync::OnceLock;

use bytes::Bytes;

use crate::error::ActiveStorageError;
use crate::models::{self, Compression, DType, Filter, Order, ReductionAxes};
use crate::operation::Operation;
use crate::rdx_ffi::*;
use crate::types::{ByteOrder, Missing};

/// The engine's device pool: one per process, created at start-up (`app::init`, app.rs:46-53).
struct Ctx(*mut RdxContext);
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {} // rdx_execute* are thread-safe (include/rdx.h, rdx_context)

static CTX: OnceLock<Ctx> = OnceLock::new();

pub fn init(devices: &[i32]) -> Result<(), ActiveStorageError> {
    // a plugin built against another rdx.h refuses to start: struct sizes differ between ABI versions
    // (version 2: rdx_device_stats grew, rdx_context_config.inflate_fallback)
    let abi = unsafe { rdx_abi_version() };
    if abi != RDX_ABI_VERSION {
        return Err(ActiveStorageError::GpuEngine {
            status: -1,
            error: format!("librdx implements ABI {abi}, the plugin was built for {RDX_ABI_VERSION}"),
        });
    }
    let mut ctx = std::ptr::null_mut();
    check(unsafe { rdx_context_create(devices.as_ptr(), devices.len() as i32, &mut ctx) }, None, DType::Float64)?;
    let _ = CTX.set(Ctx(ctx));
    Ok(())
}

fn ctx() -> *mut RdxContext {
    CTX.get().expect("operations_gpu::init not called").0
}

/// The engine context (pinned_gpu allocates download buffers from it).
pub fn context() -> *mut RdxContext {
    ctx()
}

/// Whether `init` has created the engine (download_gpu: page-locked download buffers only then).
pub fn initialized() -> bool {
    CTX.get().is_some()
}

/// `Gpu<OP>` — OP: 0 count, 1 max, 2 min, 3 select, 4 sum (rdx_op).
pub struct Gpu<const OP: u32>;
pub type GpuCount = Gpu<0>;
pub type GpuMax = Gpu<1>;
pub type GpuMin = Gpu<2>;
pub type GpuSelect = Gpu<3>;
pub type GpuSum = Gpu<4>;

/// The rdx_op code of a GPU plugin (app_gpu::operation_gpu calls execute_slice with it).
pub trait GpuOp {
    const OP: u32;
}
impl<const OP: u32> GpuOp for Gpu<OP> {
    const OP: u32 = OP;
}

impl<const OP: u32> Operation for Gpu<OP> {
    fn execute(rd: &models::RequestData, data: Vec<u8>) -> Result<models::Response, ActiveStorageError> {
        execute_slice(rd, &data, OP)
    }
}

/// The plugin's body over any byte slice: a `Vec` (the `Operation` trait), or the downloader's `Bytes`
/// as it is — page-locked when it came from `pinned_gpu::PinnedBuf` (the engine then DMAs it without a
/// staging copy), so `operation_gpu` never converts it to a `Vec` (that conversion would copy a
/// non-`Vec` owner and break the reference's zero-copy assertion, app.rs:173-181).
pub fn execute_slice(rd: &models::RequestData, data: &[u8], op: u32) -> Result<models::Response, ActiveStorageError> {
    let req = Marshalled::new(rd, op)?;
    let mut res: *mut RdxResult = std::ptr::null_mut();
    // One call, any request (compressed chunks included): the engine sizes and allocates the
    // response in page-locked memory (include/rdx.h rdx_execute_owned).
    let st = unsafe { rdx_execute_owned(ctx(), &req.c, data.as_ptr() as *const c_void, data.len() as u64, &mut res) };
    if planned_on_cpu(st) {
        return cpu_operation(rd, data, op);
    }
    check(st, rd.compression, rd.dtype)?;
    let owner = Owned(res);
    let info = unsafe { (*res).info };
    let shape: Vec<usize> = info.shape[..info.ndim as usize].iter().map(|&s| s as usize).collect();
    let counts: Vec<i64> = owner.counts().to_vec();
    // the body stays in the engine's page-locked block until the HTTP response is dropped
    let body = Bytes::from_owner(owner);
    Ok(models::Response::new(
        body,
        dtype_of(info.dtype),
        shape,
        counts,
        rd.option_shape_as_bytes.unwrap_or(false),
        rd.option_count_as_bytes.unwrap_or(false),
    ))
}

/// RDX_E_UNSUPPORTED for a reason other than the chunk's encoding (a blosc2 codec the device does not
/// decode, a gzip / zlib stream k_pinflate declined — both come back to `app_gpu::operation_gpu` as
/// UnsupportedOperation and are decompressed on the host): a request the reference serves that the engine
/// does not plan (rank above 32, views of 2^32 or more elements; include/rdx.h rdx_unsupported_reason).  It
/// runs on the reference's own CPU path instead of failing.
fn planned_on_cpu(st: i32) -> bool {
    st == status::E_UNSUPPORTED
        && !matches!(unsafe { rdx_last_unsupported_reason() }, unsupported::BLOSC2_CODEC | unsupported::INFLATE_DECLINED)
}

/// The reference's synchronous path for this route, unchanged: `operation::<T>` (app.rs:163-183: the
/// filter pipeline, validate_raw_size, then the CPU plugin of operations.rs).  `app::operation` becomes
/// `pub(crate)` for this.  Rare (see planned_on_cpu), so the one copy of the chunk
/// into a fresh `Bytes` is of no consequence.
fn cpu_operation(rd: &models::RequestData, data: &[u8], op: u32) -> Result<models::Response, ActiveStorageError> {
    use crate::operations;
    let (rd, data) = (rd.clone(), Bytes::copy_from_slice(data));
    match op {
        0 => crate::app::operation::<operations::Count>(rd, data),
        1 => crate::app::operation::<operations::Max>(rd, data),
        2 => crate::app::operation::<operations::Min>(rd, data),
        3 => crate::app::operation::<operations::Select>(rd, data),
        _ => crate::app::operation::<operations::Sum>(rd, data),
    }
}

/// The response of `Gpu<OP>` as the reference's HTTP body — `serde_cbor::to_vec(&CBORResponse::new(..))`
/// (app.rs:33-40, models.rs:355-416) — serialised by the engine on the device (`rdx_execute_cbor`):
/// a large count vector (axis reductions with many outputs, `axis: []`) crosses PCIe as CBOR integers
/// (1 byte for a 0 / 1 count) instead of 8-byte values, and no host-side serialisation runs.  The bytes
/// live in the engine's page-locked block until the HTTP response is dropped.
pub fn execute_cbor<const OP: u32>(rd: &models::RequestData, data: &[u8]) -> Result<Bytes, ActiveStorageError> {
    let req = Marshalled::new(rd, OP)?;
    let flags = if rd.option_shape_as_bytes.unwrap_or(false) { RDX_CBOR_SHAPE_AS_BYTES } else { 0 }
        | if rd.option_count_as_bytes.unwrap_or(false) { RDX_CBOR_COUNT_AS_BYTES } else { 0 };
    let mut res: *mut RdxResult = std::ptr::null_mut();
    let st = unsafe { rdx_execute_cbor(ctx(), &req.c, data.as_ptr() as *const c_void, data.len() as u64, flags, &mut res) };
    if planned_on_cpu(st) {
        // the reference's path and its own serialisation (app.rs:31-43)
        let response = cpu_operation(rd, data, OP)?;
        return Ok(Bytes::from(serde_cbor::to_vec(&models::CBORResponse::new(&response)).unwrap()));
    }
    check(st, rd.compression, rd.dtype)?;
    Ok(Bytes::from_owner(OwnedCbor(res)))
}

/// An `RdxResult` of rdx_execute_cbor owned by a `Bytes`.
struct OwnedCbor(*mut RdxResult);
unsafe impl Send for OwnedCbor {}
unsafe impl Sync for OwnedCbor {}

impl AsRef<[u8]> for OwnedCbor {
    fn as_ref(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts((*self.0).body as *const u8, (*self.0).cbor_bytes as usize) }
    }
}

impl Drop for OwnedCbor {
    fn drop(&mut self) {
        unsafe { rdx_result_free(ctx(), self.0) }
    }
}

/// An `RdxResult` owned by a `Bytes` (freed back to the engine's pool on drop).
struct Owned(*mut RdxResult);
unsafe impl Send for Owned {}
unsafe impl Sync for Owned {}

impl Owned {
    fn counts(&self) -> &[i64] {
        unsafe { std::slice::from_raw_parts((*self.0).counts, (*self.0).info.n_counts as usize) }
    }
}

impl AsRef<[u8]> for Owned {
    fn as_ref(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts((*self.0).body as *const u8, (*self.0).info.body_bytes as usize) }
    }
}

impl Drop for Owned {
    fn drop(&mut self) {
        unsafe { rdx_result_free(ctx(), self.0) }
    }
}

/// `RequestData` (models.rs:133-176) as the plain C request of include/rdx.h; owns the arrays the
/// request points into.
struct Marshalled {
    c: RdxRequest,
    _shape: Vec<u64>,
    _selection: Vec<RdxSlice>,
    _axes: Vec<u64>,
    _filters: Vec<RdxFilter>,
    _missing: Vec<u8>,
}

impl Marshalled {
    fn new(rd: &models::RequestData, op: u32) -> Result<Self, ActiveStorageError> {
        let shape: Vec<u64> = rd.shape.iter().flatten().map(|&s| s as u64).collect();
        let selection: Vec<RdxSlice> = rd
            .selection
            .iter()
            .flatten()
            .map(|s| RdxSlice { start: s.start as i64, end: s.end as i64, stride: s.stride as i64 })
            .collect();
        let (axes_kind, axes): (u32, Vec<u64>) = match &rd.axis {
            ReductionAxes::All => (0, vec![]),
            ReductionAxes::One(a) => (1, vec![*a as u64]),
            ReductionAxes::Multi(v) => (2, v.iter().map(|&a| a as u64).collect()),
        };
        let filters: Vec<RdxFilter> = rd
            .filters
            .iter()
            .flatten()
            .map(|f| match f {
                Filter::Shuffle { element_size } => RdxFilter { id: 1, reserved: 0, element_size: *element_size as u64 },
                Filter::ShuffleSimd { element_size } => {
                    RdxFilter { id: 2, reserved: 0, element_size: *element_size as u64 }
                }
            })
            .collect();
        // Missing<DValue> -> raw values of the request dtype with the reference's own conversion
        // (missing.rs:85-110 / dvalue.rs:43-83), so IncompatibleMissing is raised exactly as today.
        let (kind, missing) = match &rd.missing {
            None => (0, vec![]),
            Some(m) => marshal_missing(rd.dtype, m)?,
        };
        let n_values = match kind {
            0 => 0,
            5 => 2,
            2 => missing.len() as u64 / rd.dtype.size_of() as u64,
            _ => 1,
        };
        let c = RdxRequest {
            abi_version: RDX_ABI_VERSION,
            op,
            dtype: dtype_code(rd.dtype),
            byte_order: match rd.byte_order {
                None => 0,
                Some(ByteOrder::Little) => 1,
                Some(ByteOrder::Big) => 2,
            },
            order: match rd.order {
                None => 0,
                Some(Order::C) => 1,
                Some(Order::F) => 2,
            },
            axes_kind,
            ndim: shape.len() as u32,
            n_axes: axes.len() as u32,
            shape: if shape.is_empty() { std::ptr::null() } else { shape.as_ptr() },
            selection: if selection.is_empty() { std::ptr::null() } else { selection.as_ptr() },
            axes: if axes_kind == 0 { std::ptr::null() } else { axes.as_ptr() },
            n_filters: filters.len() as u32,
            compression: match rd.compression {
                None => 0,
                Some(Compression::Gzip) => 1,
                Some(Compression::Zlib) => 2,
                Some(Compression::Blosc2) => 3,
            },
            filters: if filters.is_empty() { std::ptr::null() } else { filters.as_ptr() },
            missing: RdxMissing { kind, reserved: 0, n_values, values: missing.as_ptr() as *const c_void },
            has_size: rd.size.is_some() as u32,
            reserved: 0,
            size: rd.size.unwrap_or(0) as u64,
        };
        Ok(Marshalled { c, _shape: shape, _selection: selection, _axes: axes, _filters: filters, _missing: missing })
    }
}

fn marshal_missing(dtype: DType, m: &Missing<crate::types::DValue>) -> Result<(u32, Vec<u8>), ActiveStorageError> {
    fn typed<T: crate::operation::Element + zerocopy::AsBytes>(
        m: &Missing<crate::types::DValue>,
    ) -> Result<(u32, Vec<u8>), ActiveStorageError> {
        let t = Missing::<T>::try_from(m)?;
        let mut out = Vec::new();
        let kind = match &t {
            Missing::MissingValue(v) => {
                out.extend_from_slice(v.as_bytes());
                1
            }
            Missing::MissingValues(vs) => {
                vs.iter().for_each(|v| out.extend_from_slice(v.as_bytes()));
                2
            }
            Missing::ValidMin(v) => {
                out.extend_from_slice(v.as_bytes());
                3
            }
            Missing::ValidMax(v) => {
                out.extend_from_slice(v.as_bytes());
                4
            }
            Missing::ValidRange(a, b) => {
                out.extend_from_slice(a.as_bytes());
                out.extend_from_slice(b.as_bytes());
                5
            }
        };
        Ok((kind, out))
    }
    match dtype {
        DType::Int32 => typed::<i32>(m),
        DType::Int64 => typed::<i64>(m),
        DType::Uint32 => typed::<u32>(m),
        DType::Uint64 => typed::<u64>(m),
        DType::Float32 => typed::<f32>(m),
        DType::Float64 => typed::<f64>(m),
    }
}

/// `std::any::type_name::<T>()` of the element type, as array.rs:22-24 reports it in `FromBytes`.
fn type_name_of(d: DType) -> &'static str {
    match d {
        DType::Int32 => std::any::type_name::<i32>(),
        DType::Int64 => std::any::type_name::<i64>(),
        DType::Uint32 => std::any::type_name::<u32>(),
        DType::Uint64 => std::any::type_name::<u64>(),
        DType::Float32 => std::any::type_name::<f32>(),
        DType::Float64 => std::any::type_name::<f64>(),
    }
}

fn dtype_code(d: DType) -> u32 {
    match d {
        DType::Int32 => 0,
        DType::Int64 => 1,
        DType::Uint32 => 2,
        DType::Uint64 => 3,
        DType::Float32 => 4,
        DType::Float64 => 5,
    }
}

fn dtype_of(code: u32) -> DType {
    match code {
        0 => DType::Int32,
        1 => DType::Int64,
        2 => DType::Uint32,
        3 => DType::Uint64,
        4 => DType::Float32,
        _ => DType::Float64,
    }
}

/// rdx_status -> the ActiveStorageError the reference raises for the same condition (error.rs:242-376).
pub fn check(st: i32, compression: Option<Compression>, dtype: DType) -> Result<(), ActiveStorageError> {
    use status::*;
    match st {
        OK => Ok(()),
        // models.rs:242-313 validators / validate_raw_size -> 400
        E_REQUEST_VALIDATION => Err(ActiveStorageError::RequestDataValidationSingle(
            validator::ValidationError::new("request data is not valid"),
        )),
        // array.rs:18-27 zerocopy length / alignment -> 500 (error.rs:271)
        E_FROM_BYTES => Err(ActiveStorageError::FromBytes { type_name: type_name_of(dtype) }),
        // array.rs:58-63 ndarray from_shape -> 400
        E_SHAPE_INVALID => {
            Err(ActiveStorageError::ShapeInvalid(ndarray::ShapeError::from_kind(ndarray::ErrorKind::OutOfBounds)))
        }
        // shuffle.rs:21 assert_eq!(len % element_size, 0): the reference panics; parity
        E_SHUFFLE_LENGTH => panic!("assertion `left == right` failed"),
        // operations.rs:181-183,355-357: NaN in a min/max comparison panics in the reference; parity
        E_NAN_UNORDERED => panic!("unexpected undefined order error for min"),
        // a blosc2 codec / filter the device does not decode (dictionaries, delta, checksummed zstd frames) or
        // a gzip / zlib stream k_pinflate declined: app_gpu::operation_gpu catches this variant and
        // decompresses on the host instead (the reference's decoder: its bytes or its error).  The other
        // reasons never get here: Gpu<OP> serves them on the reference CPU path (planned_on_cpu).
        E_UNSUPPORTED => Err(ActiveStorageError::UnsupportedOperation { operation: "chunk codec on the GPU".into() }),
        // compression.rs:60-82 -> DecompressionFlate2 / DecompressionZune, 400 (error.rs:247-249)
        E_DECOMPRESSION => {
            let code = unsafe { rdx_inflate_last_error() };
            let msg = unsafe { std::ffi::CStr::from_ptr(rdx_inflate_error_string(code)) }.to_string_lossy().into_owned();
            Err(match compression {
                // compression.rs:33-55: DecompressionBlosc2 carries one of three static messages
                Some(Compression::Blosc2) => ActiveStorageError::DecompressionBlosc2 {
                    error: match code {
                        crate::rdx_ffi::blosc2::INVALID => "invalid blosc2 compressed data",
                        crate::rdx_ffi::blosc2::SIZE => "unexpected decompressed size for blosc2 data",
                        _ => "failed to decompress blosc2 data",
                    },
                },
                // compression.rs:184 reads the message back from DecodeErrorStatus::GenericStr
                Some(Compression::Zlib) => ActiveStorageError::DecompressionZune(
                    zune_inflate::errors::InflateDecodeErrors::new_with_error(
                        zune_inflate::errors::DecodeErrorStatus::GenericStr(msg),
                    ),
                ),
                _ => ActiveStorageError::DecompressionFlate2(std::io::Error::new(std::io::ErrorKind::InvalidInput, msg)),
            })
        }
        // device-side failures are the engine's own: a 500 of their own variant (error_gpu.rs)
        E_OUT_OF_MEMORY => Err(ActiveStorageError::GpuEngine { status: st, error: "device or pinned memory exhausted".into() }),
        _ => {
            let msg = unsafe { std::ffi::CStr::from_ptr(rdx_status_string(st)) }.to_string_lossy().into_owned();
            Err(ActiveStorageError::GpuEngine { status: st, error: msg })
        }
    }
}
