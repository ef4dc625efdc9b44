"""The Rust binding (integration/rdx_ffi.rs) against include/rdx.h, without a Rust toolchain:

* every #[repr(C)] struct's field layout, computed from its Rust declaration (C layout rules), equals
  the C compiler's offsetof / sizeof for the same struct of rdx.h, field by field;
* the file's own `const _: () = assert!(size_of / offset_of ...)` pins hold for rdx.h;
* every function of rdx.h is declared in the extern block with the same number of parameters, and
  nothing else is.
"""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
FFI = (ROOT / "integration" / "rdx_ffi.rs").read_text()
HDR = (ROOT / "include" / "rdx.h").read_text()

RUST_TO_C = {"RdxSlice": "rdx_slice", "RdxFilter": "rdx_filter", "RdxMissing": "rdx_missing",
             "RdxRequest": "rdx_request", "RdxResponseInfo": "rdx_response_info", "RdxMultiItem": "rdx_multi_item",
             "RdxResult": "rdx_result", "RdxContextConfig": "rdx_context_config",
             "RdxDeviceStats": "rdx_device_stats"}
PRIM = {"u32": (4, 4), "i32": (4, 4), "c_int": (4, 4), "u64": (8, 8), "i64": (8, 8), "f64": (8, 8)}


def rust_structs():
    out = {}
    for name, body in re.findall(r"pub struct (\w+) \{(.*?)\n\}", FFI, re.S):
        fields = re.findall(r"pub (\w+):\s*([^,]+),", body)
        out[name] = [(f, t.strip()) for f, t in fields]
    return out


def rust_layout(structs, name):
    """(size, align, {field: offset}) of a #[repr(C)] struct from its declaration."""
    off, align, offs = 0, 1, {}

    def size_align(t):
        t = t.strip()
        if t.startswith("*"):
            return 8, 8
        m = re.match(r"\[(\w+);\s*(\w+)\]", t)
        if m:
            s, a = size_align(m.group(1))
            n = 32 if m.group(2) == "RDX_MAX_NDIM" else int(m.group(2))
            return s * n, a
        if t in PRIM:
            return PRIM[t]
        size, al, _ = rust_layout(structs, t)
        return size, al

    for f, t in structs[name]:
        s, a = size_align(t)
        off = (off + a - 1) // a * a
        offs[f] = off
        off += s
        align = max(align, a)
    return (off + align - 1) // align * align, align, offs


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    structs = rust_structs()
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rdx.h"', "int main(void) {"]
    for rname, cname in RUST_TO_C.items():
        lines.append(f'printf("size {rname} %zu\\n", sizeof({cname}));')
        for f, _ in structs[rname]:
            lines.append(f'printf("off {rname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    d = tmp_path_factory.mktemp("layout")
    (d / "layout.c").write_text("\n".join(lines))
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", "-o", str(d / "layout"), str(d / "layout.c")],
                   check=True)
    out = subprocess.run([str(d / "layout")], check=True, capture_output=True, text=True).stdout
    sizes, offs = {}, {}
    for line in out.splitlines():
        p = line.split()
        if p[0] == "size":
            sizes[p[1]] = int(p[2])
        else:
            offs[(p[1], p[2])] = int(p[3])
    return sizes, offs


def test_every_struct_matches_rdx_h(c_layout):
    sizes, offs = c_layout
    structs = rust_structs()
    assert set(RUST_TO_C) <= set(structs)
    for rname in RUST_TO_C:
        size, _, roffs = rust_layout(structs, rname)
        assert size == sizes[rname], rname
        for f, o in roffs.items():
            assert o == offs[(rname, f)], (rname, f, o, offs[(rname, f)])


def test_const_layout_pins_hold(c_layout):
    sizes, offs = c_layout
    pins = re.findall(r"assert!\(size_of::<(\w+)>\(\) == (\d+)\)", FFI)
    opins = re.findall(r"assert!\(offset_of!\((\w+), (\w+)\) == (\d+)\)", FFI)
    assert len(pins) == len(RUST_TO_C) and len(opins) >= 15
    for name, n in pins:
        assert sizes[name] == int(n), name
    for name, f, n in opins:
        assert offs[(name, f)] == int(n), (name, f)


def _c_functions():
    body = re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)
    fns = {}
    for ret, name, args in re.findall(r"^\s*(?:const\s+)?(\w+\s*\**)\s*(rdx_\w+)\(([^)]*)\);", body, re.M | re.S):
        a = args.strip()
        fns[name] = 0 if a in ("", "void") else a.count(",") + 1
    return fns


def _rust_functions():
    block = FFI[FFI.index('extern "C" {'):]
    block = block[: block.index("\n}\n")]
    fns = {}
    for name, args in re.findall(r"pub fn (rdx_\w+)\(([^)]*)\)", block, re.S):
        a = args.strip().rstrip(",")
        fns[name] = 0 if not a else a.count(",") + 1
    return fns


def test_every_function_declared_with_its_arity():
    c, r = _c_functions(), _rust_functions()
    assert len(c) >= 23
    assert c == r


def test_plugins_cover_every_route_and_status():
    ops = (ROOT / "integration" / "operations_gpu.rs").read_text()
    for t in ("GpuCount", "GpuMax", "GpuMin", "GpuSelect", "GpuSum"):
        assert f"pub type {t}" in ops
    # every rdx_status is mapped (none falls through to an unrelated variant)
    for code in ("E_REQUEST_VALIDATION", "E_FROM_BYTES", "E_SHAPE_INVALID", "E_SHUFFLE_LENGTH", "E_NAN_UNORDERED",
                 "E_UNSUPPORTED", "E_DECOMPRESSION", "E_OUT_OF_MEMORY"):
        assert f"{code} =>" in ops, code
    assert "ChunkCacheError" not in ops
    assert "GpuEngine" in (ROOT / "integration" / "error_gpu.rs").read_text()


def test_shim_clears_size_after_host_decompression():
    """app.rs:169-172 validates the decompressed length of a compressed request; the engine does that only
    when `size` is absent, so every host-decompressed request goes in with compression AND size cleared."""
    app = (ROOT / "integration" / "app_gpu.rs").read_text()
    fn = app[app.index("fn host_decompressed"):]
    fn = fn[: fn.index("\n}\n")]
    assert "rd.compression = None;" in fn and "rd.size = None;" in fn
    # every host decompression hands its request through host_decompressed, and nothing else clears it
    assert app.count("compression::decompress(") == 3
    assert app.count("host_decompressed(") == 4          # the definition + three call sites
    assert app.count("compression = None") == 1


def test_shim_error_details_match_the_reference():
    ops = (ROOT / "integration" / "operations_gpu.rs").read_text()
    # array.rs:22-24: FromBytes carries std::any::type_name::<T>() of the element type
    assert 'type_name: "T"' not in ops
    assert "FromBytes { type_name: type_name_of(dtype) }" in ops
    for t in ("i32", "i64", "u32", "u64", "f32", "f64"):
        assert f"std::any::type_name::<{t}>()" in ops
    # RDX_E_UNSUPPORTED: only the chunk-encoding reasons (a blosc2 codec, a gzip / zlib stream k_pinflate
    # declined) become UnsupportedOperation (host decompression); the others run the reference's own
    # operation::<T> on the CPU, in both plugin entry points
    assert "unsupported::BLOSC2_CODEC | unsupported::INFLATE_DECLINED" in ops
    assert ops.count("if planned_on_cpu(st)") == 2
    for op in ("Count", "Max", "Min", "Select", "Sum"):
        assert f"crate::app::operation::<operations::{op}>(rd, data)" in ops


def test_pinned_download_path():
    """§8f row 3 (s3_client.rs:215-233, chunk_downloader_http.rs:137-146): the downloader fills a page-locked
    PinnedBuf (rdx_host_alloc / rdx_host_free) with the same one copy per body part, and operation_gpu hands
    the Bytes to the engine as a slice — no Bytes -> Vec conversion anywhere on the GPU path."""
    pin = (ROOT / "integration" / "pinned_gpu.rs").read_text()
    assert "rdx_host_alloc(" in pin and "rdx_host_free(" in pin and "Bytes::from_owner(self)" in pin
    assert "impl Drop for PinnedBuf" in pin and "impl AsRef<[u8]> for PinnedBuf" in pin
    app = (ROOT / "integration" / "app_gpu.rs").read_text()
    code = "\n".join(line for line in app.splitlines() if not line.strip().startswith("//"))
    assert ".into();" not in code and "T::execute(" not in code
    assert code.count("operations_gpu::execute_slice(&request_data, &data, T::OP)") == 2
    ops = (ROOT / "integration" / "operations_gpu.rs").read_text()
    assert "pub fn execute_slice(rd: &models::RequestData, data: &[u8], op: u32)" in ops
    assert "execute_slice(rd, &data, OP)" in ops            # the Operation trait goes through it too
    # the downloaders' patch: both bodies into a PinnedBuf, part by part, only with the engine created
    dl = (ROOT / "integration" / "download_gpu.rs").read_text()
    code = "\n".join(line for line in dl.splitlines() if not line.strip().startswith("//"))
    assert "s3_client.rs:215-233" in dl and "chunk_downloader_http.rs:137-146" in dl
    assert code.count("PinnedBuf::with_capacity(content_length)?") == 2
    assert code.count("buf.extend_from_slice(&part)?;") == 2 and code.count("Ok(buf.into_bytes())") == 2
    assert "crate::operations_gpu::initialized()" in code and "pub fn initialized() -> bool" in ops
    assert ".bytes().await" not in code                     # no whole-body intermediate copy
