"""ctypes wrapper of the ORACLE (oracle/rdx_oracle.cpp -> oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / CPU baseline — never by the product package.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"

_LIB = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        VP, U64 = C.c_void_p, C.c_uint64
        L.oracle_execute.restype = C.c_int
        L.oracle_execute.argtypes = [VP, VP, U64, VP, U64, C.POINTER(C.c_int64), U64, VP]
        L.oracle_bench.restype = C.c_int
        L.oracle_bench.argtypes = [VP, VP, U64, U64, C.c_int, C.POINTER(C.c_uint64)]
        L.oracle_validate_request.restype = C.c_int
        L.oracle_validate_request.argtypes = [VP]
        L.oracle_shuffle.restype = None
        L.oracle_shuffle.argtypes = [VP, U64, U64, VP]
        L.oracle_deshuffle.restype = C.c_int
        L.oracle_deshuffle.argtypes = [VP, U64, U64, VP]
        L.oracle_decompress.restype = C.c_uint32
        L.oracle_decompress.argtypes = [C.c_uint32, VP, U64, VP, U64, C.POINTER(C.c_uint64)]
        L.oracle_inflate_last_error.restype = C.c_uint32
        L.oracle_inflate_last_error.argtypes = []
        L.oracle_blosc2_sizes.restype = None
        L.oracle_blosc2_sizes.argtypes = [VP, U64, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]
        L.oracle_zstd_decompress.restype = C.c_int
        L.oracle_zstd_decompress.argtypes = [VP, U64, VP, U64, C.POINTER(U64)]
        L.oracle_xxh64.restype = U64
        L.oracle_xxh64.argtypes = [VP, U64]
        L.oracle_blosc2_decompress.restype = C.c_uint32
        L.oracle_blosc2_decompress.argtypes = [VP, U64, VP, U64, C.POINTER(U64)]
        L.oracle_missing_convert.restype = C.c_int
        L.oracle_missing_convert.argtypes = [C.c_uint32, C.c_uint32, C.c_int64, C.c_uint64, C.c_double, VP]
        _LIB = L
    return _LIB


def execute(creq, data: bytes, body_cap: int | None = None, counts_cap: int | None = None):
    """Run the reference path on the CPU.  creq: reductionist_amd._abi.CRequest (plain C struct of
    include/rdx.h).  Returns (status, info, body bytes, counts list)."""
    from reductionist_amd import _abi  # the interface structs only
    L = lib()
    info = _abi.rdx_response_info()
    n = len(data)
    if body_cap is None:
        body_cap = max(64, 8 * n + 64)
    if counts_cap is None:
        counts_cap = max(8, n + 8)
    body = (C.c_uint8 * body_cap)()
    counts = (C.c_int64 * counts_cap)()
    src = C.create_string_buffer(bytes(data), max(1, n))
    st = L.oracle_execute(C.addressof(creq.c), src, n, body, body_cap, counts, counts_cap, C.byref(info))
    return st, info, bytes(body)[: info.body_bytes], [int(c) for c in counts[: info.n_counts]]


def bench(creq, data: bytes, reps: int, clone: bool) -> float:
    """Seconds per execution of the reference path over one chunk on this thread (oracle_bench)."""
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    ns = C.c_uint64(0)
    st = lib().oracle_bench(C.addressof(creq.c), src, len(data), reps, 1 if clone else 0, C.byref(ns))
    if st:
        raise RuntimeError(f"oracle_bench failed: status {st}")
    return ns.value / 1e9 / max(1, reps)


def validate(creq) -> int:
    return lib().oracle_validate_request(C.addressof(creq.c))


def shuffle(data: bytes, es: int) -> bytes:
    out = (C.c_uint8 * max(1, len(data)))()
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    lib().oracle_shuffle(src, len(data), es, out)
    return bytes(out)[: len(data)]


def deshuffle(data: bytes, es: int):
    out = (C.c_uint8 * max(1, len(data)))()
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    st = lib().oracle_deshuffle(src, len(data), es, out)
    return st, bytes(out)[: len(data)]


DTYPE_CODE = {"int32": 0, "int64": 1, "uint32": 2, "uint64": 3, "float32": 4, "float64": 5}
DTYPE_SIZE = {"int32": 4, "int64": 8, "uint32": 4, "uint64": 8, "float32": 4, "float64": 8}


def convert(dtype: str, value):
    """TryFromDValue restated (dvalue.rs:43-83): returns (status, bytes)."""
    out = (C.c_uint8 * 8)()
    if isinstance(value, float):
        st = lib().oracle_missing_convert(DTYPE_CODE[dtype], 2, 0, 0, value, out)
    elif value < 0 or value < 2 ** 63:
        if value < -(2 ** 63):
            return 5, b""
        st = lib().oracle_missing_convert(DTYPE_CODE[dtype], 0, value, 0, 0.0, out)
    else:
        if value >= 2 ** 64:
            return 5, b""
        st = lib().oracle_missing_convert(DTYPE_CODE[dtype], 1, 0, value, 0.0, out)
    return st, bytes(out)[: DTYPE_SIZE[dtype]]


def decompress(compression: int, data: bytes, cap: int | None = None):
    """compression.rs:18-27 restated (oracle_inflate.cpp): returns (rdx_inflate_error, bytes)."""
    L = lib()
    if cap is None:
        cap = 4 * len(data) + 4096
    out = (C.c_uint8 * max(1, cap))()
    got = C.c_uint64(0)
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    e = L.oracle_decompress(compression, src, len(data), out, cap, C.byref(got))
    return int(e), bytes(out)[: min(got.value, cap)]


def blosc2_sizes(data: bytes):
    """blosc2_cbuffer_sizes (compression.rs:33) restated (oracle_blosc2.cpp): (nbytes, cbytes, blocksize)."""
    a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    lib().oracle_blosc2_sizes(src, len(data), C.byref(a), C.byref(b), C.byref(c))
    return a.value, b.value, c.value


def blosc2_decompress(data: bytes, cap: int | None = None):
    """decompress_blusc_blosc2 (compression.rs:29-57) restated: (rdx_inflate_error, bytes)."""
    if cap is None:
        cap = max(blosc2_sizes(data)[0], 1)
    out = (C.c_uint8 * max(1, cap))()
    got = C.c_uint64(0)
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    e = lib().oracle_blosc2_decompress(src, len(data), out, cap, C.byref(got))
    return int(e), bytes(out)[: min(got.value, cap)]



def zstd_decompress(data: bytes, cap: int):
    """ZSTD_decompressDCtx restated (oracle_zstd.cpp): (0, bytes) or (-1, b"")."""
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    out = C.create_string_buffer(max(1, cap))
    got = C.c_uint64(0)
    e = lib().oracle_zstd_decompress(src, len(data), out, cap, C.byref(got))
    return (e, out.raw[:got.value] if e == 0 else b"")


def xxh64(data: bytes) -> int:
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    return lib().oracle_xxh64(src, len(data))
