"""ActiveStorageError mirror (src/error.rs:30-130, status mapping :242-376) for the hot path.

Each rdx_status raised by the C ABI maps onto the variant the reference would produce, with the same
HTTP status.  Where the reference PANICS (shuffle length assert, NaN in min/max) the mirror raises a
distinct exception carrying the reference's panic message; the Rust shim in INTEGRATION.md re-panics.
"""
from __future__ import annotations

from . import _abi


class ActiveStorageError(Exception):
    http_status = 500

    def __init__(self, message: str, status: int | None = None):
        super().__init__(message)
        self.status = status


class RequestDataValidation(ActiveStorageError):      # error.rs RequestDataValidation*, 400
    http_status = 400


class FromBytes(ActiveStorageError):                  # error.rs FromBytes, 500
    http_status = 500


class ShapeInvalid(ActiveStorageError):               # error.rs ShapeInvalid, 400
    http_status = 400


class IncompatibleMissing(ActiveStorageError):        # error.rs IncompatibleMissing, 400
    http_status = 400


class UnsupportedOperation(ActiveStorageError):       # error.rs UnsupportedOperation, 400
    http_status = 400


class ReferencePanic(ActiveStorageError):
    """The reference panics here (no catch_unwind): the client sees a dropped connection."""
    http_status = 500


class DeviceError(ActiveStorageError):                # new with the device engine
    http_status = 500


class Unsupported(ActiveStorageError):                # a blosc2 codec not decoded on the device: host fallback
    http_status = 500


class Decompression(ActiveStorageError):              # error.rs DecompressionFlate2 / Zune / Blosc2, 400
    http_status = 400


_MAP = {
    _abi.E_REQUEST_VALIDATION: (RequestDataValidation, "request data is not valid"),
    _abi.E_FROM_BYTES: (FromBytes, "failed to convert from bytes"),
    _abi.E_SHAPE_INVALID: (ShapeInvalid, "failed to create array from shape"),
    _abi.E_INCOMPATIBLE_MISSING: (IncompatibleMissing, "Incompatible value for missing"),
    _abi.E_SHUFFLE_LENGTH: (ReferencePanic, "assertion `left == right` failed (data.len() % element_size)"),
    _abi.E_NAN_UNORDERED: (ReferencePanic, "unexpected undefined order error for min"),
    _abi.E_UNSUPPORTED: (Unsupported, "unsupported by the device engine"),
    _abi.E_DEVICE: (DeviceError, "device error"),
    _abi.E_OUT_OF_MEMORY: (DeviceError, "out of device memory"),
    _abi.E_NO_DEVICE: (DeviceError, "no gfx950 device"),
    _abi.E_BUFFER_TOO_SMALL: (DeviceError, "output buffer too small"),
    _abi.E_INVALID_ARGUMENT: (DeviceError, "invalid argument"),
}


def check(status: int) -> None:
    if status == _abi.OK:
        return
    if status == _abi.E_DECOMPRESSION:  # the detail: compression.rs:35-53 (blosc2), :166-190 messages
        raise Decompression(_abi.inflate_error_string(_abi.lib().rdx_inflate_last_error()), status)
    cls, msg = _MAP.get(status, (DeviceError, f"rdx status {status}"))
    raise cls(msg, status)
