"""Request / response model mirror of src/models.rs (RequestData :133-176, validators :179-313,
Response :316-351, CBORResponse :355-416) and the missing-data descriptor of
src/types/missing.rs + src/types/dvalue.rs.  Host logic only: the data path is the C ABI.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Union

from . import _abi
from .errors import IncompatibleMissing, RequestDataValidation

_FIELDS = {"interface_type", "url", "dtype", "byte_order", "offset", "size", "shape", "axis", "order",
           "selection", "compression", "filters", "missing", "option_disable_chunk_cache",
           "option_shape_as_bytes", "option_count_as_bytes"}


@dataclass
class RequestData:
    interface_type: str = "s3"
    url: str = "http://example.com/bucket/object"
    dtype: str = "int32"
    byte_order: Optional[str] = None
    offset: Optional[int] = None
    size: Optional[int] = None
    shape: Optional[List[int]] = None
    axis: Union[None, int, List[int]] = None        # ReductionAxes: None == All
    order: Optional[str] = None
    selection: Optional[List[List[int]]] = None
    compression: Optional[str] = None
    filters: Optional[List[dict]] = None
    missing: Optional[dict] = None                   # {"missing_value": 42}, {"valid_range": [a, b]}, ...
    option_disable_chunk_cache: Optional[bool] = None
    option_shape_as_bytes: Optional[bool] = None
    option_count_as_bytes: Optional[bool] = None

    # ---- serde: deny_unknown_fields, tagged enums (models.rs:98-127) -------------------------------
    @classmethod
    def from_json(cls, obj: dict) -> "RequestData":
        unknown = set(obj) - _FIELDS
        if unknown:
            raise RequestDataValidation(f"unknown field(s) {sorted(unknown)}")
        for req in ("interface_type", "url", "dtype"):
            if req not in obj:
                raise RequestDataValidation(f"missing field `{req}`")
        rd = cls(**obj)
        if rd.dtype not in _abi.DTYPES:
            raise RequestDataValidation(f"unknown dtype {rd.dtype}")
        if rd.byte_order not in _abi.BYTE_ORDER:
            raise RequestDataValidation(f"unknown byte_order {rd.byte_order}")
        if rd.order not in _abi.ORDER:
            raise RequestDataValidation(f"unknown order {rd.order}")
        if isinstance(rd.compression, dict):
            rd.compression = rd.compression.get("id")
        if rd.compression not in _abi.COMPRESSION:
            raise RequestDataValidation(f"unknown compression {rd.compression}")
        for f in rd.filters or []:
            if f.get("id") not in _abi.FILTER_IDS or set(f) != {"id", "element_size"}:
                raise RequestDataValidation(f"bad filter {f}")
        if rd.selection is not None:
            rd.selection = [list(s) if not isinstance(s, dict) else [s["start"], s["end"], s["stride"]]
                            for s in rd.selection]
        if rd.missing is not None and (len(rd.missing) != 1 or next(iter(rd.missing)) not in _abi.MISSING_KINDS):
            raise RequestDataValidation(f"bad missing {rd.missing}")
        return rd

    # ---- validator (models.rs:133-313, missing.rs:47-80) ----------------------------------------
    def validate(self) -> None:
        if not self.interface_type:
            raise RequestDataValidation("interface type must not be empty")
        if self.size is not None and self.size < 1:
            raise RequestDataValidation("size must be greater than 0")
        if self.shape is not None:
            if len(self.shape) < 1:
                raise RequestDataValidation("shape length must be greater than 0")
            if 0 in self.shape:
                raise RequestDataValidation("shape indices must be greater than 0")
        if self.selection is not None:
            if len(self.selection) < 1:
                raise RequestDataValidation("selection length must be greater than 0")
            for s in self.selection:
                if s[2] == 0:
                    raise RequestDataValidation("Selection stride must not be equal to zero")
        if self.size is not None and self.compression is None:
            validate_raw_size(self.size, self.dtype, self.shape)
        if self.shape is not None and self.selection is not None and len(self.shape) != len(self.selection):
            raise RequestDataValidation("Shape and selection must have the same length")
        if self.shape is None and self.selection is not None:
            raise RequestDataValidation("Selection requires shape to be specified")
        if self.axis is not None:
            if self.shape is None:
                raise RequestDataValidation("Axis requires shape to be specified")
            if isinstance(self.axis, int):
                if self.axis > len(self.shape) - 1:
                    raise RequestDataValidation("Reduction axis must be within shape")
            else:
                axes = list(self.axis)
                if len(axes) > len(self.shape):
                    raise RequestDataValidation(
                        "Number of reduction axes must be less than or equal to length of shape")
                if sorted(axes) != axes:
                    raise RequestDataValidation("Reduction axes must be provided in ascending order")
                if any(a > len(self.shape) - 1 for a in axes):
                    raise RequestDataValidation("All reduction axes must be within shape")
                if len(set(axes)) != len(axes):
                    raise RequestDataValidation("Reduction axes contains duplicates")
        if self.missing is not None:
            kind, values, n = typed_missing(self.missing, self.dtype, as_validation=True)
            if kind == "valid_range":
                lo, hi = _unpack(values, self.dtype)
                if not lo < hi:
                    raise RequestDataValidation("Missing data valid range min must be less than max")


def validate_raw_size(raw_size: int, dtype: str, shape: Optional[List[int]]) -> None:
    """src/models.rs:214-239"""
    ds = _abi.DTYPE_SIZE[dtype]
    if shape is not None:
        expected = 1
        for s in shape:
            expected *= s
        if raw_size != expected * ds:
            raise RequestDataValidation(
                "Raw data size must be equal to the product of shape indices and dtype size in bytes")
    elif raw_size % ds != 0:
        raise RequestDataValidation("Raw data size must be a multiple of dtype size in bytes")


def _unpack(values: bytes, dtype: str):
    import struct
    fmt = {"int32": "i", "int64": "q", "uint32": "I", "uint64": "Q", "float32": "f", "float64": "d"}[dtype]
    n = len(values) // _abi.DTYPE_SIZE[dtype]
    return struct.unpack(f"<{n}{fmt}", values)


def dvalue_to_bytes(value, dtype: str) -> bytes:
    """TryFromDValue (src/types/dvalue.rs:43-83) through the C ABI's rdx_missing_from_*."""
    lib = _abi.lib()
    out = (C.c_uint8 * 8)()
    code = _abi.DTYPES[dtype]
    if isinstance(value, bool) or not isinstance(value, (int, float)):
        raise IncompatibleMissing(f"Incompatible value {value!r} for missing")
    if isinstance(value, int):
        if value < -(2 ** 63) or value >= 2 ** 64:
            raise IncompatibleMissing(f"Incompatible value {value} for missing")
        st = lib.rdx_missing_from_i64(code, value, out) if value < 2 ** 63 else \
            lib.rdx_missing_from_u64(code, value, out)
    else:
        st = lib.rdx_missing_from_f64(code, value, out)
    if st != _abi.OK:
        raise IncompatibleMissing(f"Incompatible value {value} for missing", st)
    return bytes(out)[: _abi.DTYPE_SIZE[dtype]]


def typed_missing(missing: dict, dtype: str, as_validation: bool = False):
    """Missing<DValue> -> (kind, packed T values, n)   (src/types/missing.rs:85-110)."""
    (kind, raw), = missing.items()
    if kind in ("missing_value", "valid_min", "valid_max"):
        vals = [raw]
    elif kind == "missing_values":
        vals = list(raw)
    elif kind == "valid_range":
        vals = list(raw)
        if len(vals) != 2:
            raise RequestDataValidation("valid_range needs [min, max]")
    else:
        raise RequestDataValidation(f"unknown missing kind {kind}")
    try:
        packed = b"".join(dvalue_to_bytes(v, dtype) for v in vals)
    except IncompatibleMissing as e:
        if as_validation:
            raise RequestDataValidation(f"Missing data descriptor is invalid: {e}") from e
        raise
    return kind, packed, len(vals)


@dataclass
class Response:
    """src/models.rs:316-351"""
    body: bytes
    dtype: str
    shape: List[int]
    count: List[int]
    option_shape_as_bytes: bool = False
    option_count_as_bytes: bool = False

    def cbor_fields(self) -> dict:
        """The map CBORResponse::new serialises (models.rs:373-416); byte_order is the host's."""
        import struct
        count, count_bytes = (self.count, b"") if not self.option_count_as_bytes else \
            ([], struct.pack(f"<{len(self.count)}q", *self.count))
        shape, shape_bytes = (self.shape, b"") if not self.option_shape_as_bytes else \
            ([], struct.pack(f"<{len(self.shape)}Q", *self.shape))
        return {"bytes": self.body, "dtype": self.dtype, "shape": shape, "shape_as_bytes": shape_bytes,
                "count": count, "count_as_bytes": count_bytes, "byte_order": "little"}


def to_c_request(rd: RequestData, op: str) -> _abi.CRequest:
    kind, values, n = (None, b"", 0)
    if rd.missing is not None:
        kind, values, n = typed_missing(rd.missing, rd.dtype)
    return _abi.CRequest(op, rd.dtype, shape=rd.shape, selection=rd.selection, axis=rd.axis, order=rd.order,
                         byte_order=rd.byte_order, filters=rd.filters, compression=rd.compression,
                         missing_kind=kind, missing_values=values, n_missing=n, size=rd.size)
