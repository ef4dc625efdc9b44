"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's response serialisation, the checker
for rdx_cbor_encode / rdx_cbor_encode_device.  Nothing in the product path imports this.

Reference: src/app.rs:33-40 `serde_cbor::to_vec(&CBORResponse::new(&self))`, src/models.rs:355-416
`CBORResponse` (field order bytes, dtype, shape, shape_as_bytes, count, count_as_bytes, byte_order;
`option_*_as_bytes` move shape / count into native-endian u64 / i64 byte strings, models.rs:379-401),
serialised by serde_cbor 0.11.2 (Cargo.lock:3486-3488; the crate is not vendored here).  Its published
behaviour, restated: a #[derive(Serialize)] struct is a definite-length map keyed by the field names as
text strings; `Bytes` goes through serialize_bytes (major type 2); `String` / `&str` are text (major 3);
`Vec<usize>` / `Vec<i64>` definite arrays (major 4); unsigned integers major 0 and negative i64 v
major 1 with argument -1 - v, every argument in its shortest form (RFC 7049 §2.1: < 24 in the initial
byte, else 1 / 2 / 4 / 8 big-endian bytes after 24 / 25 / 26 / 27).

Pinning: the primitive encodings against RFC 7049 Appendix A (tests/golden/cbor_rfc7049.json); the
field names, order and value forms against the reference's models.rs tests (test_cbor_response*,
models.rs:1031-1110) and the response example of docs/api.md:94-130.  The exact bytes serde_cbor emits
are otherwise parity unpinned (no serde_cbor here to run).
"""
import struct

DTYPE_NAMES = ["int32", "int64", "uint32", "uint64", "float32", "float64"]


def head(major: int, arg: int) -> bytes:
    if arg < 24:
        return bytes([(major << 5) | arg])
    for n, ai in ((1, 24), (2, 25), (4, 26), (8, 27)):
        if arg < (1 << (8 * n)):
            return bytes([(major << 5) | ai]) + arg.to_bytes(n, "big")
    raise ValueError("argument out of range")


def enc_int(v: int) -> bytes:
    return head(1, -1 - v) if v < 0 else head(0, v)


def enc_text(s: str) -> bytes:
    b = s.encode()
    return head(3, len(b)) + b


def enc_bytes(b: bytes) -> bytes:
    return head(2, len(b)) + bytes(b)


def cbor_response(body: bytes, dtype: str, shape, count, shape_as_bytes=False, count_as_bytes=False) -> bytes:
    """CBORResponse::new(&Response) serialised (models.rs:374-414)."""
    if count_as_bytes:
        count_v, count_b = [], b"".join(struct.pack("<q", c) for c in count)
    else:
        count_v, count_b = list(count), b""
    if shape_as_bytes:
        shape_v, shape_b = [], b"".join(struct.pack("<Q", s) for s in shape)
    else:
        shape_v, shape_b = list(shape), b""
    out = head(5, 7)
    out += enc_text("bytes") + enc_bytes(body)
    out += enc_text("dtype") + enc_text(dtype)
    out += enc_text("shape") + head(4, len(shape_v)) + b"".join(head(0, s) for s in shape_v)
    out += enc_text("shape_as_bytes") + enc_bytes(shape_b)
    out += enc_text("count") + head(4, len(count_v)) + b"".join(enc_int(c) for c in count_v)
    out += enc_text("count_as_bytes") + enc_bytes(count_b)
    out += enc_text("byte_order") + enc_text("little")
    return out


def decode(buf: bytes):
    """A minimal CBOR decoder (definite lengths, major types 0-5, the simple values false / true / null):
    returns (value, bytes consumed); maps decode to lists of (key, value) pairs to keep their order."""
    def arg(pos):
        ib = buf[pos]
        ai = ib & 31
        if ai < 24:
            return ai, pos + 1
        n = {24: 1, 25: 2, 26: 4, 27: 8}[ai]
        return int.from_bytes(buf[pos + 1:pos + 1 + n], "big"), pos + 1 + n

    def item(pos):
        major = buf[pos] >> 5
        if major == 7:
            ai = buf[pos] & 31
            return {20: False, 21: True, 22: None}[ai], pos + 1
        a, pos = arg(pos)
        if major == 0:
            return a, pos
        if major == 1:
            return -1 - a, pos
        if major == 2:
            return bytes(buf[pos:pos + a]), pos + a
        if major == 3:
            return buf[pos:pos + a].decode(), pos + a
        if major == 4:
            out = []
            for _ in range(a):
                v, pos = item(pos)
                out.append(v)
            return out, pos
        if major == 5:
            out = []
            for _ in range(a):
                k, pos = item(pos)
                v, pos = item(pos)
                out.append((k, v))
            return out, pos
        raise ValueError(f"unsupported major type {major}")

    return item(0)
