"""ctypes mirror of include/rdx.h and the loader for the in-tree librdx.so.

The product path has no CPU fallback: if librdx.so is missing this module raises at import, and
every execute call needs a gfx950 device (RDX_E_NO_DEVICE otherwise).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # reductionist-rs_amd/
REPO_ROOT = PKG_ROOT.parent
# RDX_LIB_PATH: an alternative in-tree build of the same library (A/B tuning measurements only)
LIB_PATH = Path(os.environ.get("RDX_LIB_PATH", str(PKG_ROOT / "librdx.so")))

RDX_ABI_VERSION = 2
RDX_MAX_NDIM = 32

# rdx_status
OK, E_INVALID_ARGUMENT, E_REQUEST_VALIDATION, E_FROM_BYTES, E_SHAPE_INVALID, E_INCOMPATIBLE_MISSING, \
    E_SHUFFLE_LENGTH, E_NAN_UNORDERED, E_UNSUPPORTED, E_DEVICE, E_OUT_OF_MEMORY, E_BUFFER_TOO_SMALL, \
    E_NO_DEVICE, E_DECOMPRESSION = range(14)

# rdx_inflate_error (detail of E_DECOMPRESSION)
INFLATE_OK, INFLATE_GZIP_HEADER, INFLATE_ZLIB_METHOD, INFLATE_ZLIB_HEADER, INFLATE_TRUNCATED, \
    INFLATE_BLOCK_TYPE, INFLATE_STORED_LENGTH, INFLATE_CODE_LENGTHS, INFLATE_BAD_SYMBOL, INFLATE_DISTANCE, \
    INFLATE_CHECKSUM, INFLATE_OUTPUT_OVERFLOW, BLOSC2_INVALID, BLOSC2_FAILED, BLOSC2_SIZE, \
    BLOSC2_UNSUPPORTED = range(16)

# rdx_unsupported_reason (cause of E_UNSUPPORTED)
UNSUPPORTED_NONE, UNSUPPORTED_BLOSC2_CODEC, UNSUPPORTED_RANK, UNSUPPORTED_VIEW_SIZE, UNSUPPORTED_VIEW_DIMS, \
    UNSUPPORTED_MISSING_LIST, UNSUPPORTED_CBOR_SIZE, UNSUPPORTED_INFLATE_DECLINED = range(8)

# rdx_inflate_path (rdx_inflate_last_path)
INFLATE_PATH_NONE, INFLATE_PATH_SERIAL, INFLATE_PATH_PARALLEL, INFLATE_PATH_PARALLEL_FALLBACK, \
    INFLATE_PATH_DECLINED = range(5)

OPS = {"count": 0, "max": 1, "min": 2, "select": 3, "sum": 4}
DTYPES = {"int32": 0, "int64": 1, "uint32": 2, "uint64": 3, "float32": 4, "float64": 5}
DTYPE_SIZE = {"int32": 4, "int64": 8, "uint32": 4, "uint64": 8, "float32": 4, "float64": 8}
DTYPE_NAMES = {v: k for k, v in DTYPES.items()}
BYTE_ORDER = {None: 0, "little": 1, "big": 2}
ORDER = {None: 0, "C": 1, "F": 2}
AXES_ALL, AXES_ONE, AXES_MULTI = 0, 1, 2
CBOR_SHAPE_AS_BYTES, CBOR_COUNT_AS_BYTES = 1, 2   # rdx_cbor_* flags (RequestData.option_*_as_bytes)
FILTER_IDS = {"shuffle": 1, "shuffle_simd": 2}
COMPRESSION = {None: 0, "gzip": 1, "zlib": 2, "blosc2": 3}
MISSING_KINDS = {None: 0, "missing_value": 1, "missing_values": 2, "valid_min": 3, "valid_max": 4,
                 "valid_range": 5}


class rdx_slice(C.Structure):
    _fields_ = [("start", C.c_int64), ("end", C.c_int64), ("stride", C.c_int64)]


class rdx_filter(C.Structure):
    _fields_ = [("id", C.c_uint32), ("reserved", C.c_uint32), ("element_size", C.c_uint64)]


class rdx_missing(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("reserved", C.c_uint32), ("n_values", C.c_uint64),
                ("values", C.c_void_p)]


class rdx_request(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("op", C.c_uint32), ("dtype", C.c_uint32),
        ("byte_order", C.c_uint32), ("order", C.c_uint32), ("axes_kind", C.c_uint32),
        ("ndim", C.c_uint32), ("n_axes", C.c_uint32),
        ("shape", C.POINTER(C.c_uint64)), ("selection", C.POINTER(rdx_slice)),
        ("axes", C.POINTER(C.c_uint64)),
        ("n_filters", C.c_uint32), ("compression", C.c_uint32),
        ("filters", C.POINTER(rdx_filter)),
        ("missing", rdx_missing),
        ("has_size", C.c_uint32), ("reserved", C.c_uint32), ("size", C.c_uint64),
    ]


class rdx_response_info(C.Structure):
    _fields_ = [("dtype", C.c_uint32), ("ndim", C.c_uint32), ("shape", C.c_uint64 * RDX_MAX_NDIM),
                ("body_bytes", C.c_uint64), ("n_counts", C.c_uint64)]

    def shape_list(self):
        return [int(self.shape[i]) for i in range(self.ndim)]


class rdx_multi_item(C.Structure):
    _fields_ = [("req", C.POINTER(rdx_request)), ("d_chunk", C.c_void_p), ("chunk_len", C.c_uint64),
                ("d_body", C.c_void_p), ("d_counts", C.c_void_p), ("d_status", C.c_void_p)]


class rdx_result(C.Structure):
    _fields_ = [("info", rdx_response_info), ("body", C.c_void_p), ("counts", C.POINTER(C.c_int64)),
                ("cbor_bytes", C.c_uint64), ("reserved", C.c_uint64)]


class rdx_context_config(C.Structure):
    _fields_ = [("max_workspaces", C.c_uint32), ("coalesce", C.c_uint32), ("coalesce_lanes", C.c_uint32),
                ("inflate_fallback", C.c_uint32), ("coalesce_max_bytes", C.c_uint64),
                ("coalesce_host_max_bytes", C.c_uint64)]


class rdx_device_stats(C.Structure):
    _fields_ = [("device", C.c_int32), ("workspaces", C.c_uint32), ("workspaces_busy", C.c_uint32),
                ("max_workspaces", C.c_uint32), ("requests", C.c_uint64), ("coalesced_requests", C.c_uint64),
                ("coalesced_launches", C.c_uint64), ("outstanding_bytes", C.c_uint64), ("waits", C.c_uint64),
                ("direct_requests", C.c_uint64), ("placed_bytes", C.c_uint64),
                ("peak_outstanding_bytes", C.c_uint64), ("host_read_requests", C.c_uint64),
                ("sleeps", C.c_uint64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class CRequest:
    """Owns the ctypes arrays an rdx_request points into (keep it alive during the call)."""

    def __init__(self, op: str, dtype: str, *, shape=None, selection=None, axis=None, order=None,
                 byte_order=None, filters=None, compression=None, missing_kind=None,
                 missing_values: bytes = b"", n_missing=0, size=None):
        r = rdx_request()
        r.abi_version = RDX_ABI_VERSION
        r.op = OPS[op]
        r.dtype = DTYPES[dtype]
        r.byte_order = BYTE_ORDER[byte_order]
        r.order = ORDER[order]
        self._keep = []
        if shape is not None:
            arr = (C.c_uint64 * len(shape))(*shape)
            self._keep.append(arr)
            r.ndim = len(shape)
            r.shape = C.cast(arr, C.POINTER(C.c_uint64))
        if selection is not None:
            arr = (rdx_slice * len(selection))(*[rdx_slice(int(a), int(b), int(c)) for a, b, c in selection])
            self._keep.append(arr)
            r.selection = C.cast(arr, C.POINTER(rdx_slice))
        if axis is None:
            r.axes_kind = AXES_ALL
        else:
            axes = [axis] if isinstance(axis, int) else list(axis)
            r.axes_kind = AXES_ONE if isinstance(axis, int) else AXES_MULTI
            r.n_axes = len(axes)
            arr = (C.c_uint64 * max(1, len(axes)))(*axes)
            self._keep.append(arr)
            r.axes = C.cast(arr, C.POINTER(C.c_uint64))
        if filters:
            arr = (rdx_filter * len(filters))(*[rdx_filter(FILTER_IDS[f["id"]], 0, int(f["element_size"]))
                                                for f in filters])
            self._keep.append(arr)
            r.n_filters = len(filters)
            r.filters = C.cast(arr, C.POINTER(rdx_filter))
        r.compression = COMPRESSION[compression]
        r.missing.kind = MISSING_KINDS[missing_kind]
        if missing_kind is not None:
            buf = C.create_string_buffer(missing_values, max(1, len(missing_values)))
            self._keep.append(buf)
            r.missing.values = C.cast(buf, C.c_void_p)
            r.missing.n_values = n_missing
        if size is not None:
            r.has_size = 1
            r.size = size
        self.c = r

    @property
    def ref(self):
        return C.byref(self.c)


def _declare(lib):
    P, U64, VP = C.POINTER, C.c_uint64, C.c_void_p
    req_p, info_p = P(rdx_request), P(rdx_response_info)
    sig = {
        "rdx_abi_version": (C.c_uint32, []),
        "rdx_status_string": (C.c_char_p, [C.c_int]),
        "rdx_device_count": (C.c_int, []),
        "rdx_context_create": (C.c_int, [P(C.c_int), C.c_int, P(VP)]),
        "rdx_context_destroy": (None, [VP]),
        "rdx_validate_request": (C.c_int, [req_p]),
        "rdx_plan": (C.c_int, [req_p, U64, info_p]),
        "rdx_missing_from_i64": (C.c_int, [C.c_uint32, C.c_int64, VP]),
        "rdx_missing_from_u64": (C.c_int, [C.c_uint32, C.c_uint64, VP]),
        "rdx_missing_from_f64": (C.c_int, [C.c_uint32, C.c_double, VP]),
        "rdx_execute": (C.c_int, [VP, req_p, VP, U64, VP, U64, P(C.c_int64), U64, info_p]),
        "rdx_host_alloc": (C.c_int, [VP, U64, P(VP)]),
        "rdx_host_free": (None, [VP, VP]),
        "rdx_workspace_create": (C.c_int, [VP, C.c_int, P(VP)]),
        "rdx_workspace_destroy": (None, [VP]),
        "rdx_execute_device": (C.c_int, [VP, req_p, VP, U64, VP, VP, VP, VP, info_p]),
        "rdx_execute_batch_device": (C.c_int, [VP, req_p, U64, P(VP), U64, VP, VP, VP, VP, info_p]),
        "rdx_inflate_error_string": (C.c_char_p, [C.c_uint32]),
        "rdx_inflate_last_error": (C.c_uint32, []),
        "rdx_inflate_last_path": (C.c_uint32, []),
        "rdx_decompress_one_device": (C.c_int, [VP, C.c_uint32, VP, U64, VP, U64, P(U64), P(C.c_uint32), VP]),
        "rdx_last_unsupported_reason": (C.c_uint32, []),
        "rdx_decompress_batch_device": (C.c_int, [VP, C.c_uint32, U64, P(VP), P(U64), VP, U64, VP, VP, VP]),
        "rdx_blosc2_cbuffer_sizes": (C.c_int, [VP, U64, P(U64), P(U64), P(U64)]),
        "rdx_execute_multi_device": (C.c_int, [VP, U64, P(rdx_multi_item), VP, P(C.c_uint32), info_p]),
        "rdx_execute_owned": (C.c_int, [VP, req_p, VP, U64, P(P(rdx_result))]),
        "rdx_result_free": (None, [VP, P(rdx_result)]),
        "rdx_execute_cbor": (C.c_int, [VP, req_p, VP, U64, C.c_uint32, P(P(rdx_result))]),
        "rdx_cbor_bound": (U64, [P(rdx_response_info), C.c_uint32]),
        "rdx_cbor_encode": (C.c_int, [P(rdx_response_info), VP, VP, C.c_uint32, VP, U64, P(U64)]),
        "rdx_cbor_encode_device": (C.c_int, [VP, P(rdx_response_info), VP, VP, C.c_uint32, VP, U64, VP, VP, VP]),
        "rdx_context_configure": (C.c_int, [VP, P(rdx_context_config)]),
        "rdx_context_stats": (C.c_int, [VP, C.c_uint32, P(rdx_device_stats)]),
        "rdx_execute_resident": (C.c_int, [VP, C.c_int, req_p, VP, U64, VP, U64, P(C.c_int64), U64, info_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None
EXPORTED = ["rdx_abi_version", "rdx_status_string", "rdx_device_count", "rdx_context_create",
            "rdx_context_destroy", "rdx_validate_request", "rdx_plan", "rdx_missing_from_i64",
            "rdx_missing_from_u64", "rdx_missing_from_f64", "rdx_execute", "rdx_host_alloc", "rdx_host_free",
            "rdx_workspace_create",
            "rdx_workspace_destroy", "rdx_execute_device", "rdx_execute_batch_device", "rdx_inflate_error_string",
            "rdx_inflate_last_error", "rdx_decompress_batch_device", "rdx_execute_multi_device",
            "rdx_execute_owned", "rdx_result_free", "rdx_cbor_bound", "rdx_cbor_encode", "rdx_cbor_encode_device",
            "rdx_execute_cbor", "rdx_blosc2_cbuffer_sizes", "rdx_last_unsupported_reason",
            "rdx_context_configure", "rdx_context_stats", "rdx_execute_resident", "rdx_inflate_last_path",
            "rdx_decompress_one_device"]


def lib():
    """Load librdx.so (once).  torch is imported first when available so that the library binds
    to the same HIP runtime as torch (both carry SONAME libamdhip64.so.7)."""
    global _LIB
    if _LIB is None:
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is plumbing, not required for the ABI
            pass
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                               "(the device engine has no CPU fallback)")
        _LIB = _declare(C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | os.RTLD_LOCAL))
        if _LIB.rdx_abi_version() != RDX_ABI_VERSION:
            raise RuntimeError("librdx.so ABI version mismatch")
    return _LIB


def status_string(code: int) -> str:
    return lib().rdx_status_string(code).decode()


def inflate_error_string(code: int) -> str:
    return lib().rdx_inflate_error_string(code).decode()


def blosc2_cbuffer_sizes(data: bytes):
    """blosc2_cbuffer_sizes (compression.rs:33) through the C ABI: (nbytes, cbytes, blocksize)."""
    a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    st = lib().rdx_blosc2_cbuffer_sizes(buf, len(data), C.byref(a), C.byref(b), C.byref(c))
    assert st == OK
    return a.value, b.value, c.value
