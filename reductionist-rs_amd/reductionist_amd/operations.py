"""The five operations behind the reference's plugin surface (src/operation.rs:53-96,
src/operations.rs Count/Max/Min/Select/Sum) and the synchronous request glue operation<T>()
(src/app.rs:163-183), executed by the MI355X engine through the C ABI.

    response = Sum.execute(request_data, data)          # like operations::Sum::execute
    response = operation(Sum, request_data, data)        # like app::operation::<Sum>

`execute` takes the RAW chunk: the filter pipeline (byte unshuffle) and the byte-order swap run
on the device inside the same call, as do validate_raw_size / from_bytes / from_shape checks.
"""
from __future__ import annotations

import threading

import dataclasses
import gzip
import zlib

from . import _abi
from .engine import Engine
from .errors import Decompression, Unsupported
from .models import RequestData, Response, to_c_request

_ENGINE = None
_LOCK = threading.Lock()


def default_engine() -> Engine:
    global _ENGINE
    with _LOCK:
        if _ENGINE is None:
            _ENGINE = Engine()
        return _ENGINE


class Operation:
    name = ""

    @classmethod
    def execute(cls, request_data: RequestData, data: bytes, engine: Engine | None = None) -> Response:
        eng = engine or default_engine()
        creq = to_c_request(request_data, cls.name)
        try:
            info, body, counts = eng.execute(creq, data)
        except Unsupported:
            # a lone gzip / zlib stream the device's parallel decoder declined (rdx.h
            # RDX_UNSUPPORTED_INFLATE_DECLINED): the host decodes it, as integration/app_gpu.rs does, and the
            # uncompressed chunk runs on the device
            if _abi.lib().rdx_last_unsupported_reason() != _abi.UNSUPPORTED_INFLATE_DECLINED:
                raise
            rd = dataclasses.replace(request_data, compression=None, size=None)
            info, body, counts = eng.execute(to_c_request(rd, cls.name), host_decompress(request_data.compression, data))
        return Response(body=body, dtype=_abi.DTYPE_NAMES[info.dtype], shape=info.shape_list(), count=counts,
                        option_shape_as_bytes=bool(request_data.option_shape_as_bytes),
                        option_count_as_bytes=bool(request_data.option_count_as_bytes))


class Count(Operation):
    name = "count"


class Max(Operation):
    name = "max"


class Min(Operation):
    name = "min"


class Select(Operation):
    name = "select"


class Sum(Operation):
    name = "sum"


OPERATIONS = {"count": Count, "max": Max, "min": Min, "select": Select, "sum": Sum}


def host_decompress(compression: str, data: bytes) -> bytes:
    """compression::decompress (src/compression.rs:60-82) on the host, for a stream the device declined:
    one gzip member (trailing bytes ignored, as flate2's GzDecoder) or one zlib stream."""
    try:
        if compression == "gzip":
            d = zlib.decompressobj(16 + zlib.MAX_WBITS)
            out = d.decompress(data)
            if not d.eof:
                raise zlib.error("unexpected end of compressed data")
            return out
        return zlib.decompress(data)
    except (zlib.error, gzip.BadGzipFile, EOFError) as e:
        raise Decompression(str(e), _abi.E_DECOMPRESSION) from None


def operation(op: type[Operation], request_data: RequestData, data: bytes, engine: Engine | None = None) -> Response:
    """src/app.rs:163-183 — validated request + raw chunk -> Response (filters, size check, op)."""
    return op.execute(request_data, data, engine)
