"""Thin owner of an rdx_context / rdx_workspace (include/rdx.h).  No CPU fallback."""
from __future__ import annotations

import ctypes as C
from typing import Sequence

from . import _abi
from .errors import check


class Engine:
    """Device pool (rdx_context).  One per process; thread-safe like the C ABI."""

    def __init__(self, devices: Sequence[int] | None = None):
        self.lib = _abi.lib()
        ctx = C.c_void_p()
        if devices:
            arr = (C.c_int * len(devices))(*devices)
            check(self.lib.rdx_context_create(arr, len(devices), C.byref(ctx)))
        else:
            check(self.lib.rdx_context_create(None, 0, C.byref(ctx)))
        self.ctx = ctx

    def close(self):
        if self.ctx:
            self.lib.rdx_context_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def plan(self, creq: _abi.CRequest, chunk_len: int) -> _abi.rdx_response_info:
        info = _abi.rdx_response_info()
        check(self.lib.rdx_plan(creq.ref, chunk_len, C.byref(info)))
        return info

    def execute_raw(self, creq: _abi.CRequest, data: bytes):
        """Host chunk in, (status, info, body, counts) out — no exception on kernel-side status."""
        info = _abi.rdx_response_info()
        src = C.c_char_p(bytes(data)) if len(data) else None
        if creq.c.compression != _abi.COMPRESSION[None]:
            # the response size depends on the DECOMPRESSED length: a first call with no output
            # capacity decompresses on the device and reports it (RDX_E_BUFFER_TOO_SMALL + info)
            st = self.lib.rdx_execute(self.ctx, creq.ref, src, len(data), None, 0, None, 0, C.byref(info))
            if st not in (_abi.OK, _abi.E_BUFFER_TOO_SMALL):
                return st, info, b"", []
        else:
            st = self.lib.rdx_plan(creq.ref, len(data), C.byref(info))
            if st != _abi.OK:
                return st, info, b"", []
        body = (C.c_uint8 * max(1, info.body_bytes))()
        counts = (C.c_int64 * max(1, info.n_counts))()
        st = self.lib.rdx_execute(self.ctx, creq.ref, src, len(data), body, info.body_bytes, counts,
                                  info.n_counts, C.byref(info))
        return st, info, bytes(body)[: info.body_bytes], [int(c) for c in counts[: info.n_counts]]

    def execute_owned(self, creq: _abi.CRequest, data):
        """rdx_execute_owned: one call, engine-allocated (pooled, page-locked) response buffers, for any
        request incl. gzip / zlib chunks.  `data`: bytes, or (pointer, length) of host memory."""
        if isinstance(data, tuple):
            src, n = C.c_void_p(data[0]), data[1]
        else:
            src, n = (C.c_char_p(bytes(data)) if len(data) else None), len(data)
        res = C.POINTER(_abi.rdx_result)()
        st = self.lib.rdx_execute_owned(self.ctx, creq.ref, src, n, C.byref(res))
        if st != _abi.OK:
            return st, _abi.rdx_response_info(), b"", []
        r = res.contents
        info = _abi.rdx_response_info.from_buffer_copy(r.info)
        body = C.string_at(r.body, info.body_bytes) if info.body_bytes else b""
        counts = [int(r.counts[i]) for i in range(info.n_counts)]
        self.lib.rdx_result_free(self.ctx, res)
        return st, info, body, counts

    def execute_cbor(self, creq: _abi.CRequest, data, flags: int = 0):
        """rdx_execute_cbor: the response as the reference's HTTP body (serde_cbor CBORResponse, app.rs:33-40),
        serialised on the device.  Returns (status, info, cbor bytes)."""
        if isinstance(data, tuple):
            src, n = C.c_void_p(data[0]), data[1]
        else:
            src, n = (C.c_char_p(bytes(data)) if len(data) else None), len(data)
        res = C.POINTER(_abi.rdx_result)()
        st = self.lib.rdx_execute_cbor(self.ctx, creq.ref, src, n, flags, C.byref(res))
        if st != _abi.OK:
            return st, _abi.rdx_response_info(), b""
        r = res.contents
        info = _abi.rdx_response_info.from_buffer_copy(r.info)
        body = C.string_at(r.body, r.cbor_bytes)
        self.lib.rdx_result_free(self.ctx, res)
        return st, info, body

    def execute_resident(self, creq: _abi.CRequest, device: int, d_chunk: int, chunk_len: int):
        """rdx_execute_resident: a chunk already in HBM of `device`, the response into host buffers (small
        all-axes requests coalesce with concurrent callers').  Returns (status, info, body, counts); the
        ctypes call releases the GIL, so Python threads issue concurrent requests."""
        info = _abi.rdx_response_info()
        st = self.lib.rdx_plan(creq.ref, chunk_len, C.byref(info))
        if st != _abi.OK:
            return st, info, b"", []
        body = (C.c_uint8 * max(1, info.body_bytes))()
        counts = (C.c_int64 * max(1, info.n_counts))()
        st = self.lib.rdx_execute_resident(self.ctx, device, creq.ref, C.c_void_p(d_chunk), chunk_len, body,
                                           info.body_bytes, counts, info.n_counts, C.byref(info))
        return st, info, bytes(body)[: info.body_bytes], [int(c) for c in counts[: info.n_counts]]

    def configure(self, max_workspaces=0, coalesce=True, coalesce_lanes=0, coalesce_max_bytes=0,
                  coalesce_host_max_bytes=0, inflate_fallback=False):
        """rdx_context_configure (0 = the engine's default for that field)."""
        cfg = _abi.rdx_context_config(max_workspaces, 1 if coalesce else 0, coalesce_lanes,
                                      1 if inflate_fallback else 0, coalesce_max_bytes, coalesce_host_max_bytes)
        check(self.lib.rdx_context_configure(self.ctx, C.byref(cfg)))

    def stats(self, index: int = 0) -> dict:
        """rdx_context_stats of pool entry `index`."""
        st = _abi.rdx_device_stats()
        check(self.lib.rdx_context_stats(self.ctx, index, C.byref(st)))
        return st.as_dict()

    def host_alloc(self, nbytes: int):
        """Page-locked host buffer (rdx_host_alloc) as (pointer, numpy uint8 view); free with host_free."""
        import numpy as np
        p = C.c_void_p()
        check(self.lib.rdx_host_alloc(self.ctx, nbytes, C.byref(p)))
        return p.value, np.ctypeslib.as_array((C.c_uint8 * max(1, nbytes)).from_address(p.value))

    def host_free(self, ptr: int):
        self.lib.rdx_host_free(self.ctx, C.c_void_p(ptr))

    def execute(self, creq: _abi.CRequest, data: bytes):
        st, info, body, counts = self.execute_raw(creq, data)
        check(st)
        return info, body, counts

    def workspace(self, device: int = 0) -> "Workspace":
        return Workspace(self, device)


class Workspace:
    """Per-stream scratch for the device-resident entry points (pointers are plain ints)."""

    def __init__(self, engine: Engine, device: int = 0):
        self.engine = engine
        self.lib = engine.lib
        ws = C.c_void_p()
        check(self.lib.rdx_workspace_create(engine.ctx, device, C.byref(ws)))
        self.ws = ws

    def close(self):
        if self.ws:
            self.lib.rdx_workspace_destroy(self.ws)
            self.ws = None

    def execute_device(self, creq, d_chunk: int, chunk_len: int, d_body: int, d_counts: int,
                       d_status: int | None, stream: int | None) -> _abi.rdx_response_info:
        info = _abi.rdx_response_info()
        check(self.lib.rdx_execute_device(self.ws, creq.ref, C.c_void_p(d_chunk), chunk_len, C.c_void_p(d_body),
                                          C.c_void_p(d_counts), C.c_void_p(d_status or 0),
                                          C.c_void_p(stream or 0), C.byref(info)))
        return info

    def execute_batch_device(self, creq, d_chunks: Sequence[int], chunk_len: int, d_bodies: int, d_counts: int,
                             d_status: int | None, stream: int | None) -> _abi.rdx_response_info:
        info = _abi.rdx_response_info()
        ptrs = (C.c_void_p * len(d_chunks))(*d_chunks)
        check(self.lib.rdx_execute_batch_device(self.ws, creq.ref, len(d_chunks), ptrs, chunk_len,
                                                C.c_void_p(d_bodies), C.c_void_p(d_counts),
                                                C.c_void_p(d_status or 0), C.c_void_p(stream or 0),
                                                C.byref(info)))
        return info

    def execute_multi_device(self, items, stream: int | None):
        """Heterogeneous batch (rdx_execute_multi_device): items = [(creq, d_chunk, chunk_len, d_body,
        d_counts, d_status or None), ...].  Returns (per-request planning statuses, response infos)."""
        n = len(items)
        arr = (_abi.rdx_multi_item * max(1, n))()
        for i, (creq, d_chunk, ln, d_body, d_counts, d_status) in enumerate(items):
            arr[i] = _abi.rdx_multi_item(C.pointer(creq.c), d_chunk or None, ln, d_body or None, d_counts or None,
                                         d_status or None)
        statuses = (C.c_uint32 * max(1, n))()
        infos = (_abi.rdx_response_info * max(1, n))()
        check(self.lib.rdx_execute_multi_device(self.ws, n, arr, C.c_void_p(stream or 0), statuses, infos))
        return [int(x) for x in statuses[:n]], [infos[i] for i in range(n)]

    def decompress_one_device(self, compression: str, d_in: int, length: int, d_out: int, out_capacity: int,
                              stream: int | None = None):
        """rdx_decompress_one_device: one device-resident gzip / zlib stream decoded by the whole device
        (k_pinflate; a stream it declines: k_inflate when the context has inflate_fallback on), synchronously.
        Returns (rdx_inflate_error, decompressed size, rdx_inflate_last_path); the error is None when the
        stream was declined (RDX_UNSUPPORTED_INFLATE_DECLINED)."""
        n = C.c_uint64()
        err = C.c_uint32()
        st = self.lib.rdx_decompress_one_device(self.ws, _abi.COMPRESSION[compression], C.c_void_p(d_in), length,
                                                C.c_void_p(d_out), out_capacity, C.byref(n), C.byref(err),
                                                C.c_void_p(stream or 0))
        if st == _abi.E_UNSUPPORTED and self.lib.rdx_last_unsupported_reason() == _abi.UNSUPPORTED_INFLATE_DECLINED:
            # declined by k_pinflate (the workspace's context has inflate_fallback off): no error detail, the
            # caller's host decoder answers
            return None, 0, int(self.lib.rdx_inflate_last_path())
        check(st)
        return int(err.value), int(n.value), int(self.lib.rdx_inflate_last_path())

    def decompress_batch_device(self, compression: str, d_streams: Sequence[int], lens: Sequence[int], d_out: int,
                                out_capacity: int, d_out_lens: int, d_errors: int, stream: int | None) -> None:
        """compression::decompress (compression.rs:18-27) of device-resident gzip/zlib streams:
        stream i -> d_out + i*out_capacity, its length -> d_out_lens[i] (u64), rdx_inflate_error ->
        d_errors[i] (u32).  Asynchronous on `stream`."""
        n = len(d_streams)
        ptrs = (C.c_void_p * max(1, n))(*d_streams)
        ls = (C.c_uint64 * max(1, n))(*lens)
        check(self.lib.rdx_decompress_batch_device(self.ws, _abi.COMPRESSION[compression], n, ptrs, ls,
                                                   C.c_void_p(d_out), out_capacity, C.c_void_p(d_out_lens),
                                                   C.c_void_p(d_errors), C.c_void_p(stream or 0)))
