"""The real-library CPU baseline (oracle/cpu_baselines.cpp, bench.py's cpu_baseline_lz4_lib): the chunks it
decodes with the system's liblz4 (LZ4_decompress_safe) and unshuffles must be the golden chunks' bytes, so
that the time it reports is the time of the same work the device does."""
import ctypes as C
import hashlib
import json
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden" / "blosc2_chunks.json"


def _lib():
    lib = C.CDLL(str(ROOT / "oracle" / "build" / "liboracle.so"))
    lib.cpu_blosc2_lz4lib_one.restype = C.c_int
    lib.cpu_blosc2_lz4lib_one.argtypes = [C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int]
    return lib


def test_lz4lib_baseline_decodes_the_golden_lz4_chunks():
    lib = _lib()
    if not lib.cpu_lz4lib_available():
        pytest.skip("liblz4.so.1 not loadable here")
    chunks = {c["name"]: c for c in json.loads(GOLDEN.read_text())["chunks"]}
    for name in ("lz4_shuffle_ts4", "lz4_liblz4_streams"):   # LZ4 streams + byte shuffle: the bench's shape
        c = chunks[name]
        raw = bytes.fromhex(c["chunk"])
        out = C.create_string_buffer(c["nbytes"] + 64)
        assert lib.cpu_blosc2_lz4lib_one(raw, len(raw), out, c["nbytes"], 1) == 0, name
        assert hashlib.sha256(out.raw[: c["nbytes"]]).hexdigest() == c["sha256"], name
