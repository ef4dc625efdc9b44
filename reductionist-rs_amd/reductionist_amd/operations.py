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

from . import _abi
from .engine import Engine
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
        info, body, counts = eng.execute(creq, data)
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


def operation(op: type[Operation], request_data: RequestData, data: bytes, engine: Engine | None = None) -> Response:
    """src/app.rs:163-183 — validated request + raw chunk -> Response (filters, size check, op)."""
    return op.execute(request_data, data, engine)
