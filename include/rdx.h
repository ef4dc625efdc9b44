/*
 * rdx.h — C ABI of the MI355X chunk filter+reduce engine (reductionist-rs drop-in).
 *
 * This is the boundary a Reductionist host (Rust, through `extern "C"`) binds to replace the
 * synchronous part of a request: `operation<T>()` in src/app.rs:163-183, i.e.
 *   filter_pipeline()            src/filter_pipeline.rs:19-34 (gzip / zlib / blosc2 decompression, byte
 *                                unshuffle)
 *   validate_raw_size()          src/app.rs:169-172 -> src/models.rs:214-239
 *   T::execute(&RequestData,..)  src/operation.rs:53-96 -> src/operations.rs (Count/Max/Min/Select/Sum)
 *   build_array + slicing        src/array.rs:18-208 (byte-order swap, hyperslab)
 *   missing-data predicate       src/types/missing.rs:114-122, src/operations.rs:25-33
 *
 * Plain C: no torch / HIP types in any signature. Device streams are passed as `void*`
 * (a hipStream_t); device buffers as plain pointers.  Every entry point returns an rdx_status and
 * never aborts the process; the host shim maps the status onto ActiveStorageError
 * (src/error.rs:30-130) — see rdx_status below and INTEGRATION.md.
 */
#ifndef RDX_H
#define RDX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: rdx_device_stats grew to 80 bytes (round 4) and rdx_context_config.inflate_fallback (round 5).  A host
 * checks rdx_abi_version() == RDX_ABI_VERSION once at load time before passing any struct. */
#define RDX_ABI_VERSION 2u
/* Maximum rank of a request shape (the reference accepts any rank via ndarray IxDyn; 32 matches
 * numpy's NPY_MAXDIMS and is far above any chunk layout seen in practice). */
#define RDX_MAX_NDIM 32u

/* ---- status codes (mapped onto src/error.rs ActiveStorageError by the host shim) ------------- */
typedef enum rdx_status {
    RDX_OK = 0,
    RDX_E_INVALID_ARGUMENT = 1,    /* NULL pointer / bad enum / ABI version mismatch (caller bug)            */
    RDX_E_REQUEST_VALIDATION = 2,  /* models.rs:179-313 validators and validate_raw_size (HTTP 400)          */
    RDX_E_FROM_BYTES = 3,          /* array.rs:18-27 length not a multiple of / misaligned for T (HTTP 500)  */
    RDX_E_SHAPE_INVALID = 4,       /* array.rs:58-63 ndarray from_shape failure (HTTP 400)                  */
    RDX_E_INCOMPATIBLE_MISSING = 5,/* dvalue.rs:43-83 / missing.rs:47-80 conversion failure (HTTP 400)      */
    RDX_E_SHUFFLE_LENGTH = 6,      /* shuffle.rs:21 assert_eq!(len % element_size, 0) — reference panics    */
    RDX_E_NAN_UNORDERED = 7,       /* operations.rs:181-183,355-357 NaN in min/max — reference panics with
                                      "unexpected undefined order error for min"                            */
    RDX_E_UNSUPPORTED = 8,         /* a blosc2 codec / filter not decoded on the device (RDX_BLOSC2_UNSUPPORTED:
                                      dictionaries, delta, checksummed zstd frames) / rank > 32 / views of >= 2^32
                                      elements: the cause is rdx_last_unsupported_reason()             */
    RDX_E_DEVICE = 9,              /* HIP runtime error                                                      */
    RDX_E_OUT_OF_MEMORY = 10,      /* device or pinned allocation failed                                     */
    RDX_E_BUFFER_TOO_SMALL = 11,   /* caller-provided output buffer smaller than rdx_plan() reported        */
    RDX_E_NO_DEVICE = 12,          /* no usable gfx950 device                                                */
    RDX_E_DECOMPRESSION = 13       /* compression.rs:18-82 gzip/zlib/blosc2 stream invalid: ActiveStorageError::
                                      DecompressionFlate2 / DecompressionZune / DecompressionBlosc2 (HTTP
                                      400, error.rs:247-249); the rdx_inflate_error detail:
                                      rdx_inflate_last_error()                                          */
} rdx_status;

/* Why a gzip / zlib / blosc2 stream failed to decompress (RDX_E_DECOMPRESSION).  The reference's messages are
 * reproduced by rdx_inflate_error_string where its tests pin them (compression.rs:166-190). */
typedef enum rdx_inflate_error {
    RDX_INFLATE_OK = 0,
    RDX_INFLATE_GZIP_HEADER = 1,     /* "invalid gzip header" (flate2): bad magic or CM != 8             */
    RDX_INFLATE_ZLIB_METHOD = 2,     /* "Unknown zlib compression method N" (zune-inflate): CM != 8      */
    RDX_INFLATE_ZLIB_HEADER = 3,     /* CINFO > 7, FCHECK not a multiple of 31, or a preset dictionary  */
    RDX_INFLATE_TRUNCATED = 4,       /* the input ends inside the header, a block or the trailer         */
    RDX_INFLATE_BLOCK_TYPE = 5,      /* reserved DEFLATE block type 3                                    */
    RDX_INFLATE_STORED_LENGTH = 6,   /* stored block with LEN != ~NLEN                                    */
    RDX_INFLATE_CODE_LENGTHS = 7,    /* invalid dynamic-block code lengths / incomplete or over-full code */
    RDX_INFLATE_BAD_SYMBOL = 8,      /* a bit pattern with no code, or a length/distance symbol >= 286/30 */
    RDX_INFLATE_DISTANCE = 9,        /* back-reference before the start of the output                    */
    RDX_INFLATE_CHECKSUM = 10,       /* gzip CRC-32 / ISIZE or zlib Adler-32 mismatch                    */
    RDX_INFLATE_OUTPUT_OVERFLOW = 11,/* more output than the capacity given (retry with a larger one)    */
    /* blosc2 (compression.rs:29-57, ActiveStorageError::DecompressionBlosc2, HTTP 400) */
    RDX_BLOSC2_INVALID = 12,         /* "invalid blosc2 compressed data": blosc2_cbuffer_sizes -> nbytes 0 */
    RDX_BLOSC2_FAILED = 13,          /* "failed to decompress blosc2 data": blosc2_decompress <= 0        */
    RDX_BLOSC2_SIZE = 14,            /* "unexpected decompressed size for blosc2 data"                     */
    RDX_BLOSC2_UNSUPPORTED = 15      /* a codec / flag not decoded here (checksummed zstd frames, dictionaries,
                                        user-defined codecs or filters, delta): status RDX_E_UNSUPPORTED */
} rdx_inflate_error;

/* Why this thread's last RDX_E_UNSUPPORTED was returned (rdx_last_unsupported_reason).  BLOSC2_CODEC and
 * INFLATE_DECLINED concern the chunk's encoding (decompress it on the host and call again); every other reason
 * is a request the reference serves that this engine does not plan (run the reference's CPU path for it). */
typedef enum rdx_unsupported_reason {
    RDX_UNSUPPORTED_NONE = 0,
    RDX_UNSUPPORTED_BLOSC2_CODEC = 1, /* RDX_BLOSC2_UNSUPPORTED: dictionaries, delta, user codecs, zstd checksums */
    RDX_UNSUPPORTED_RANK = 2,         /* request rank above RDX_MAX_NDIM                                    */
    RDX_UNSUPPORTED_VIEW_SIZE = 3,    /* a view of 2^32 or more elements, or a dim of 2^32 or more            */
    RDX_UNSUPPORTED_VIEW_DIMS = 4,    /* more than 16 dims left after canonicalisation                       */
    RDX_UNSUPPORTED_MISSING_LIST = 5, /* a missing_values list of 2^32 or more entries                       */
    RDX_UNSUPPORTED_CBOR_SIZE = 6,    /* a CBOR count vector of 2^43 or more entries                          */
    RDX_UNSUPPORTED_INFLATE_DECLINED = 7 /* a lone gzip / zlib stream (> 4 KiB) the parallel decoder (k_pinflate)
                                        did not accept — a block chain it does not follow (e.g. many fixed-
                                        Huffman blocks) or a corrupt stream: decompress it on the host (the
                                        reference's decoder gives its bytes or its error) and call again
                                        uncompressed.  Only with inflate_fallback = 0 (the default).        */
} rdx_unsupported_reason;

/* ---- request enums (src/models.rs) ------------------------------------------------------------ */
typedef enum rdx_op { /* routes /v2/{count,max,min,select,sum}, src/app.rs:61-71 */
    RDX_OP_COUNT = 0, RDX_OP_MAX = 1, RDX_OP_MIN = 2, RDX_OP_SELECT = 3, RDX_OP_SUM = 4
} rdx_op;

typedef enum rdx_dtype { /* DType, src/models.rs:14-27 */
    RDX_DTYPE_INT32 = 0, RDX_DTYPE_INT64 = 1, RDX_DTYPE_UINT32 = 2,
    RDX_DTYPE_UINT64 = 3, RDX_DTYPE_FLOAT32 = 4, RDX_DTYPE_FLOAT64 = 5
} rdx_dtype;

typedef enum rdx_byte_order { /* Option<ByteOrder>, src/types/byte_order.rs:19-24 */
    RDX_BYTE_ORDER_UNSET = 0, RDX_BYTE_ORDER_LITTLE = 1, RDX_BYTE_ORDER_BIG = 2
} rdx_byte_order;

typedef enum rdx_order { /* Option<Order>, src/models.rs:47-52 */
    RDX_ORDER_UNSET = 0, RDX_ORDER_C = 1, RDX_ORDER_F = 2
} rdx_order;

typedef enum rdx_axes_kind { /* ReductionAxes, src/models.rs:122-127 */
    RDX_AXES_ALL = 0, RDX_AXES_ONE = 1, RDX_AXES_MULTI = 2
} rdx_axes_kind;

typedef enum rdx_filter_id { /* Filter, src/models.rs:111-117 */
    RDX_FILTER_SHUFFLE = 1, RDX_FILTER_SHUFFLE_SIMD = 2
} rdx_filter_id;

typedef enum rdx_compression { /* Option<Compression>, src/models.rs:98-105 */
    RDX_COMPRESSION_NONE = 0, RDX_COMPRESSION_GZIP = 1, RDX_COMPRESSION_ZLIB = 2, RDX_COMPRESSION_BLOSC2 = 3
} rdx_compression;

typedef enum rdx_missing_kind { /* Missing<T>, src/types/missing.rs:31-42 */
    RDX_MISSING_NONE = 0, RDX_MISSING_VALUE = 1, RDX_MISSING_VALUES = 2,
    RDX_MISSING_VALID_MIN = 3, RDX_MISSING_VALID_MAX = 4, RDX_MISSING_VALID_RANGE = 5
} rdx_missing_kind;

/* numpy-semantics slice [start, end, stride], src/models.rs:77-92 */
typedef struct rdx_slice {
    int64_t start;
    int64_t end;
    int64_t stride;
} rdx_slice;

typedef struct rdx_filter {
    uint32_t id;           /* rdx_filter_id */
    uint32_t reserved;
    uint64_t element_size; /* NOT validated by the reference; 0 or len % es != 0 -> RDX_E_SHUFFLE_LENGTH */
} rdx_filter;

/* Missing-data descriptor with values ALREADY converted to the request dtype (native byte order)
 * by the host, using the reference's TryFromDValue rules (src/types/dvalue.rs:43-83);
 * rdx_missing_from_f64/i64/u64 below implement those rules for hosts that want them. */
typedef struct rdx_missing {
    uint32_t kind;         /* rdx_missing_kind */
    uint32_t reserved;
    uint64_t n_values;     /* VALUE/VALID_MIN/VALID_MAX: 1, VALID_RANGE: 2 (min,max), VALUES: list length */
    const void *values;    /* n_values elements of the request dtype */
} rdx_missing;

/* One request = one chunk (src/models.rs:133-176 RequestData, minus the transport fields). */
typedef struct rdx_request {
    uint32_t abi_version;  /* RDX_ABI_VERSION */
    uint32_t op;           /* rdx_op */
    uint32_t dtype;        /* rdx_dtype */
    uint32_t byte_order;   /* rdx_byte_order */
    uint32_t order;        /* rdx_order */
    uint32_t axes_kind;    /* rdx_axes_kind */
    uint32_t ndim;         /* 0 => `shape` absent: 1-D of len/sizeof(T) elements (array.rs:40) */
    uint32_t n_axes;       /* ONE: 1; MULTI: list length (may be 0 = numpy axis=()) */
    const uint64_t *shape;         /* ndim entries or NULL */
    const rdx_slice *selection;    /* ndim entries or NULL */
    const uint64_t *axes;          /* n_axes entries or NULL */
    uint32_t n_filters;
    uint32_t compression;          /* rdx_compression: decompressed on the device (k_inflate / k_blosc2) */
    const rdx_filter *filters;     /* n_filters entries, in REQUEST order (decoded in reverse) */
    rdx_missing missing;
    uint32_t has_size;             /* RequestData.size is Some(..): app.rs:169 skips validate_raw_size */
    uint32_t reserved;
    uint64_t size;
} rdx_request;

/* Everything a caller needs to size the response (src/models.rs:316-351 Response). */
typedef struct rdx_response_info {
    uint32_t dtype;        /* response dtype (count -> INT64) */
    uint32_t ndim;         /* rank of the response shape */
    uint64_t shape[RDX_MAX_NDIM];
    uint64_t body_bytes;   /* bytes of the response body (native-endian values) */
    uint64_t n_counts;     /* number of i64 counts */
} rdx_response_info;

/* ---- library / device management -------------------------------------------------------------- */
uint32_t rdx_abi_version(void);
const char *rdx_status_string(rdx_status status);
/* Number of visible gfx950 devices (0 when none / no driver). Never initialises anything else. */
int rdx_device_count(void);

/* A context is a pool over one or more devices — the in-process multi-GPU server of app_state.rs:21-37
 * (one process, requests on worker threads, src/app.rs:147-152).  Every entry of `devices` is one pool
 * entry (a device listed twice is two entries on one GPU).  Thread-safe: rdx_execute* may be called
 * concurrently from any number of host threads.  Each request goes to the entry with the fewest bytes
 * of requests in flight; an entry holds up to max_workspaces workspaces (stream, buffers) and a caller
 * that finds all of them busy waits for one (back-pressure, as the reference's resource manager
 * semaphores, resource_manager.rs:54-89).  Concurrent small all-axes requests on one entry are coalesced:
 * queued, and issued by whichever caller finds a launch lane free as ONE heterogeneous k_multi launch +
 * one result copy; each caller returns when its own result is in host memory.
 * devices == NULL / n_devices == 0 => device 0. */
typedef struct rdx_context rdx_context;
rdx_status rdx_context_create(const int *devices, int n_devices, rdx_context **out);
void rdx_context_destroy(rdx_context *ctx);

typedef struct rdx_context_config {
    uint32_t max_workspaces;        /* per pool entry (0: 16); requests beyond it wait for a free one           */
    uint32_t coalesce;              /* 1 (default): coalesce small all-axes requests into k_multi launches; 0: off */
    uint32_t coalesce_lanes;        /* coalesced launches in flight per pool entry (0: 3)                      */
    uint32_t inflate_fallback;      /* a lone gzip / zlib stream k_pinflate declines: 0 (default) -> RDX_E_UNSUPPORTED
                                       (RDX_UNSUPPORTED_INFLATE_DECLINED; streams up to 4 KiB still decode on the
                                       device), 1 -> the sequential k_inflate decodes it on the device (its bytes
                                       or its error; 100-220 ms per 4 MiB).  Workspaces keep the value they were
                                       created with.                                                          */
    uint64_t coalesce_max_bytes;    /* rdx_execute_resident chunks up to this many bytes coalesce (0: 64 MiB)  */
    uint64_t coalesce_host_max_bytes; /* rdx_execute / _owned host chunks up to this many (0: 1 MiB) coalesce   *
                                       after their H2D copy.  It does not bound page-locked all-axes chunks   *
                                       of up to RDX_HOST_READ_KIB (env, default 4096 KiB): those are read by  *
                                       the kernel over PCIe, direct or in a shared launch whose few readers  *
                                       keep the link, not HBM, the bound                     */
} rdx_context_config;
/* Call it before the context is shared: once a request has been placed the configuration is frozen and
 * this returns RDX_E_INVALID_ARGUMENT (the dispatchers and the placement read it without a lock). */
rdx_status rdx_context_configure(rdx_context *ctx, const rdx_context_config *cfg);

/* Bookkeeping of pool entry `index` (0 .. n_devices-1). */
typedef struct rdx_device_stats {
    int32_t device;                 /* HIP ordinal of the entry                                              */
    uint32_t workspaces;            /* workspaces created (<= max_workspaces)                                */
    uint32_t workspaces_busy;       /* held by a request right now                                            */
    uint32_t max_workspaces;
    uint64_t requests;              /* requests placed on this entry                                          */
    uint64_t coalesced_requests;    /* of which served through a coalesced k_multi launch                     */
    uint64_t coalesced_launches;    /* k_multi launches issued by the coalescer                               */
    uint64_t outstanding_bytes;     /* chunk bytes of the requests in flight on this entry now                */
    uint64_t waits;                 /* requests that waited for a free workspace                              */
    uint64_t direct_requests;       /* coalescible requests that found the coalescer idle and launched on the
                                       caller's own thread (the idle-queue fast path; not in coalesced_*)      */
    uint64_t placed_bytes;          /* chunk bytes of all requests placed on this entry (the placement key,
                                       summed over time)                                                       */
    uint64_t peak_outstanding_bytes;/* high-water mark of outstanding_bytes (each request weighs its chunk
                                       bytes + 64 KiB): least-outstanding placement keeps it near
                                       ceil(concurrent requests / entries) requests' weight                    */
    uint64_t host_read_requests;    /* page-locked host chunks the kernel read over PCIe itself (no H2D copy;
                                       RDX_HOST_READ_KIB), direct or coalesced                                 */
    uint64_t sleeps;                /* callers that slept (futex) instead of spinning until their result          */
} rdx_device_stats;
rdx_status rdx_context_stats(rdx_context *ctx, uint32_t index, rdx_device_stats *out);

/* ---- host logic (no device needed) -------------------------------------------------------------- */
/* models.rs:242-313 validate_request_data (+ missing validation, missing.rs:47-80, with typed values). */
rdx_status rdx_validate_request(const rdx_request *req);
/* Shape / dtype / sizes of the response for a chunk of chunk_len bytes; runs every check
 * operation<T>() would run before touching the data (app.rs:163-183, array.rs:18-63).  For a
 * compressed request chunk_len is the DECOMPRESSED length (the response depends on it). */
rdx_status rdx_plan(const rdx_request *req, uint64_t chunk_len, rdx_response_info *info);
/* TryFromDValue (dvalue.rs:43-83): JSON number -> dtype value bytes (out: 8 bytes). */
rdx_status rdx_missing_from_i64(uint32_t dtype, int64_t v, void *out);
rdx_status rdx_missing_from_u64(uint32_t dtype, uint64_t v, void *out);
rdx_status rdx_missing_from_f64(uint32_t dtype, double v, void *out);
/* Message for an rdx_inflate_error, and the detail of this thread's last RDX_E_DECOMPRESSION. */
const char *rdx_inflate_error_string(uint32_t code);
uint32_t rdx_inflate_last_error(void);
/* How this thread's last compressed request was decompressed: a lone gzip / zlib stream is decoded by the
 * whole device (k_pinflate: block starts found, blocks and the symbols inside them decoded in parallel);
 * a stream that path does not accept (errors, a block chain it cannot follow) goes back to the caller
 * (DECLINED: RDX_E_UNSUPPORTED) or, with inflate_fallback / up to 4 KiB, is decoded again by the
 * sequential k_inflate, whose result and error are the reference's. */
typedef enum rdx_inflate_path {
    RDX_INFLATE_PATH_NONE = 0,
    RDX_INFLATE_PATH_SERIAL = 1,            /* k_inflate (one wavefront per stream) / k_blosc2             */
    RDX_INFLATE_PATH_PARALLEL = 2,          /* k_pinflate                                                   */
    RDX_INFLATE_PATH_PARALLEL_FALLBACK = 3, /* k_pinflate declined, then k_inflate                          */
    RDX_INFLATE_PATH_DECLINED = 4           /* k_pinflate declined: RDX_E_UNSUPPORTED, INFLATE_DECLINED       */
} rdx_inflate_path;
uint32_t rdx_inflate_last_path(void);
/* The rdx_unsupported_reason of this thread's last RDX_E_UNSUPPORTED. */
uint32_t rdx_last_unsupported_reason(void);
/* blosc2_cbuffer_sizes (src/compression.rs:33, blusc 0.0.2 / c-blosc2): the sizes a blosc chunk's
 * 16-byte header states; all three 0 when it is not a valid header (the reference's "invalid blosc2
 * compressed data").  Host only: sizes the output of rdx_decompress_batch_device. */
rdx_status rdx_blosc2_cbuffer_sizes(const void *src, uint64_t len, uint64_t *nbytes, uint64_t *cbytes,
                                    uint64_t *blocksize);

/* Page-locked host buffers: a host that downloads chunks straight into these (s3_client.rs:215-233
 * today copies into an 8-byte aligned Vec) lets rdx_execute DMA them without a staging copy, and
 * large responses (select) come back at full PCIe rate.  Any host pointer is accepted by
 * rdx_execute; pinned ones are detected and used directly. */
rdx_status rdx_host_alloc(rdx_context *ctx, uint64_t bytes, void **out);
void rdx_host_free(rdx_context *ctx, void *p);

/* ---- execution ------------------------------------------------------------------------------------ */
/* Host-resident chunk in, host-resident response out (the drop-in for operation<T>()).
 * `chunk` is borrowed read-only; body/counts are caller-provided with capacities from rdx_plan.
 * Blocks until the response is in host memory.  A gzip/zlib/blosc2 chunk crosses PCIe compressed and is
 * inflated on the device (k_inflate); info describes the response of the decompressed chunk. */
rdx_status rdx_execute(rdx_context *ctx, const rdx_request *req,
                       const void *chunk, uint64_t chunk_len,
                       void *body, uint64_t body_capacity,
                       int64_t *counts, uint64_t counts_capacity,
                       rdx_response_info *info);

/* The same, with response buffers the engine allocates: one call for any request — including a gzip /
 * zlib chunk, whose response size is only known after inflating it (calling rdx_plan + rdx_execute for
 * a compressed chunk would need a sizing call that inflates it twice).  body / counts live in one
 * page-locked block from a per-context pool, so a Rust host can hand them to the HTTP response without
 * a copy (bytes::Bytes::from_owner, freeing with rdx_result_free when the response is dropped); `counts`
 * is exactly CBORResponse's count_as_bytes when option_count_as_bytes is set (models.rs:379-401: the
 * i64 counts in native byte order), and info.shape the u64 array of shape_as_bytes.
 * Select from page-locked input into a page-locked response (this API, or rdx_execute with
 * rdx_host_alloc buffers) is pipelined: the chunk's H2D and the response's D2H overlap. */
typedef struct rdx_result {
    rdx_response_info info;
    void *body;            /* rdx_execute_owned: info.body_bytes bytes (16-byte aligned);
                              rdx_execute_cbor: the CBOR response body, cbor_bytes bytes */
    int64_t *counts;       /* rdx_execute_owned: info.n_counts values; rdx_execute_cbor: NULL */
    uint64_t cbor_bytes;   /* rdx_execute_cbor: length of the CBOR body; otherwise 0 */
    uint64_t reserved;
} rdx_result;
rdx_status rdx_execute_owned(rdx_context *ctx, const rdx_request *req, const void *chunk, uint64_t chunk_len,
                             rdx_result **out);
/* rdx_execute_owned whose response leaves the device already serialised: `body` holds the HTTP body of
 * the reference's success response (serde_cbor::to_vec(&CBORResponse::new(&response)), app.rs:33-40;
 * flags = RDX_CBOR_* from RequestData.option_*_as_bytes), packed on the device by the same encoder as
 * rdx_cbor_encode_device — a large count vector never crosses PCIe as 8-byte integers. */
rdx_status rdx_execute_cbor(rdx_context *ctx, const rdx_request *req, const void *chunk, uint64_t chunk_len,
                            uint32_t flags, rdx_result **out);
void rdx_result_free(rdx_context *ctx, rdx_result *result);

/* rdx_execute for a chunk already resident in HBM of device `device` (a HIP ordinal of the context's pool):
 * a device-side chunk cache (chunk_cache.rs keeps chunks in host memory; on the GPU server they can stay
 * in HBM), or a chunk an earlier call left there.  Response into HOST buffers, synchronously, exactly as
 * rdx_execute; the chunk is borrowed read-only.  Small all-axes requests are coalesced with concurrent
 * callers' (rdx_context). */
rdx_status rdx_execute_resident(rdx_context *ctx, int device, const rdx_request *req,
                                const void *d_chunk, uint64_t chunk_len,
                                void *body, uint64_t body_capacity,
                                int64_t *counts, uint64_t counts_capacity,
                                rdx_response_info *info);

/* Device-resident path: everything already in HBM, nothing copied, asynchronous on `stream`.
 * A workspace holds the per-stream scratch (partials, arrival tickets, unshuffle buffers); use one
 * workspace per concurrently used stream. `d_status` (device, one uint32 per chunk, may be NULL)
 * receives 0 or an rdx_status raised inside the kernels (RDX_E_NAN_UNORDERED). */
typedef struct rdx_workspace rdx_workspace;
rdx_status rdx_workspace_create(rdx_context *ctx, int device, rdx_workspace **out);
void rdx_workspace_destroy(rdx_workspace *ws);

/* A compressed request (gzip/zlib/blosc2) is decompressed into workspace scratch first; the call then waits on
 * `stream` once for the decompressed length before launching the operation. */
rdx_status rdx_execute_device(rdx_workspace *ws, const rdx_request *req,
                              const void *d_chunk, uint64_t chunk_len,
                              void *d_body, int64_t *d_counts, uint32_t *d_status,
                              void *stream, rdx_response_info *info);

/* Batch of n_chunks independent chunks sharing one request (same dtype/shape/filters/selection),
 * e.g. many chunks of one variable: one launch for the whole batch.  h_chunk_ptrs is a HOST array
 * of n_chunks DEVICE pointers; chunk i's response goes to d_bodies + i*body_bytes,
 * d_counts + i*n_counts, d_status + i. */
rdx_status rdx_execute_batch_device(rdx_workspace *ws, const rdx_request *req,
                                    uint64_t n_chunks, const void *const *h_chunk_ptrs,
                                    uint64_t chunk_len,
                                    void *d_bodies, int64_t *d_counts, uint32_t *d_status,
                                    void *stream, rdx_response_info *info);

/* One request of a heterogeneous batch (rdx_execute_multi_device): each carries its own request. */
typedef struct rdx_multi_item {
    const rdx_request *req;   /* its own op, dtype, shape, selection, axes, byte order, filters, missing */
    const void *d_chunk;      /* device pointer to the raw (uncompressed) chunk */
    uint64_t chunk_len;
    void *d_body;             /* device, >= rdx_plan's body_bytes */
    int64_t *d_counts;        /* device, >= rdx_plan's n_counts */
    uint32_t *d_status;       /* device word (may be NULL): 0 or a status raised in the kernels */
} rdx_multi_item;

/* Many independent requests on one stream — the request-level concurrency of src/app.rs:147-152
 * (every HTTP request is its own operation<T>() call) folded into as few launches as possible: every
 * all-axes request (axis unset) over an unshuffled chunk (no filters) whose view has < 2^31 elements
 * in at most 4 canonical dims and whose missing_values list has at most 2 entries runs in a
 * heterogeneous launch (k_multi, up to 24 requests per launch, their descriptors in the kernel
 * arguments), each with its own dtype, op, view, byte order and missing predicate; the others (axis
 * reductions, select, axis = [], shuffled chunks, longer missing lists) run as their own launches on
 * the same stream, after them.
 * statuses[i] (HOST, n entries) receives request i's planning status — an invalid request does not stop
 * the others; infos[i] (HOST, may be NULL) its response shape and sizes.  Compressed requests are
 * refused per item (RDX_E_INVALID_ARGUMENT): decompress them first (rdx_decompress_batch_device).
 * Returns RDX_OK unless the launch itself failed. */
rdx_status rdx_execute_multi_device(rdx_workspace *ws, uint64_t n, const rdx_multi_item *items, void *stream,
                                    uint32_t *statuses, rdx_response_info *infos);

/* compression::decompress (src/compression.rs:18-27: gzip, zlib, blosc2) for a batch of n device-resident
 * compressed streams, asynchronous on `stream`: stream i (h_in_ptrs[i] device pointer, h_in_lens[i]
 * bytes; HOST arrays) is inflated into d_out + i*out_capacity (out_capacity a multiple of 16, d_out
 * 16-byte aligned); d_out_lens[i] = bytes produced, d_errors[i] = rdx_inflate_error (device arrays).
 * RDX_INFLATE_OUTPUT_OVERFLOW means the stream needs more than out_capacity: the caller retries that
 * stream with a larger capacity (for blosc2, d_out_lens[i] then holds the size the header states).
 * gzip / zlib: one wavefront per stream (k_inflate); blosc2: one wavefront per block stream, every chunk
 * spread over many (k_blosc2), so a lone blosc2 chunk decodes in parallel.  rdx_execute / rdx_execute_device call this for a compressed
 * request (then synchronise once to learn the decompressed length) before planning the operation. */
rdx_status rdx_decompress_batch_device(rdx_workspace *ws, uint32_t compression, uint64_t n,
                                       const void *const *h_in_ptrs, const uint64_t *h_in_lens,
                                       void *d_out, uint64_t out_capacity,
                                       uint64_t *d_out_lens, uint32_t *d_errors, void *stream);

/* One device-resident gzip / zlib stream (d_in, len bytes), decoded by the whole device — the lone
 * compressed request of compression.rs:60-82 (k_pinflate; a stream it does not accept returns
 * RDX_E_UNSUPPORTED / RDX_UNSUPPORTED_INFLATE_DECLINED, or with the workspace's inflate_fallback is decoded
 * by k_inflate, whose result and error are the reference's) — SYNCHRONOUSLY on `stream`.  *out_len (host) =
 * the decompressed size; *error (host) = rdx_inflate_error: RDX_INFLATE_OUTPUT_OVERFLOW when that size
 * exceeds out_cap (nothing written), else the bytes are in d_out.  rdx_inflate_last_path() tells which
 * decoder produced them. */
rdx_status rdx_decompress_one_device(rdx_workspace *ws, uint32_t compression, const void *d_in, uint64_t len,
                                     void *d_out, uint64_t out_cap, uint64_t *out_len, uint32_t *error,
                                     void *stream);

/* ---- response serialisation ------------------------------------------------------------------- *
 * The HTTP body of a successful request: serde_cbor::to_vec(&CBORResponse::new(&response))
 * (src/app.rs:33-40, src/models.rs:355-416, serde_cbor 0.11.2): a CBOR map of 7 entries in field order
 * bytes, dtype, shape, shape_as_bytes, count, count_as_bytes, byte_order; integers in their shortest
 * form; `option_shape_as_bytes` / `option_count_as_bytes` move shape / count into native-endian u64 /
 * i64 byte strings and leave empty arrays (models.rs:379-401).  A large count vector (an axis reduction
 * with many outputs, axis = []) is encoded where it was computed: rdx_cbor_encode_device packs the
 * device-resident body and counts into the CBOR body on the device (one pass over the counts: a
 * decoupled look-back scan of the per-count encoded lengths), so only the packed response crosses PCIe. */
#define RDX_CBOR_SHAPE_AS_BYTES 1u   /* RequestData.option_shape_as_bytes (models.rs:173) */
#define RDX_CBOR_COUNT_AS_BYTES 2u   /* RequestData.option_count_as_bytes (models.rs:175) */
/* Upper bound of the encoded size (every count at its longest, 9 bytes). */
uint64_t rdx_cbor_bound(const rdx_response_info *info, uint32_t flags);
/* Host buffers in, host buffer out; *out_len = bytes written.  RDX_E_BUFFER_TOO_SMALL when out_cap is
 * short of the exact size (then *out_len = the size needed). */
rdx_status rdx_cbor_encode(const rdx_response_info *info, const void *body, const int64_t *counts, uint32_t flags,
                           void *out, uint64_t out_cap, uint64_t *out_len);
/* Device buffers in (e.g. rdx_execute_device's outputs), device buffer out (>= rdx_cbor_bound bytes),
 * asynchronous on `stream`: *d_out_len (device u64) receives the encoded length; *d_status (device word,
 * may be NULL) is set to 0 (reserved for device-side failures; the encoder never waits on another
 * workgroup's progress, so it has none today). */
rdx_status rdx_cbor_encode_device(rdx_workspace *ws, const rdx_response_info *info, const void *d_body,
                                  const int64_t *d_counts, uint32_t flags, void *d_out, uint64_t out_cap,
                                  uint64_t *d_out_len, uint32_t *d_status, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* RDX_H */
