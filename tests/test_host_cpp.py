"""Build and run the C++ host-mirror tests (tests/cpp/test_host.cpp) against librdx.so."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "reductionist-rs_amd"


def _binary():
    out = ROOT / "tests" / "cpp" / "build" / "test_host"   # built here, travels to the GPU box
    src = ROOT / "tests" / "cpp" / "test_host.cpp"
    hdr = PKG / "host" / "reductionist.hpp"
    lib = PKG / "librdx.so"
    if not out.exists() or out.stat().st_mtime < max(src.stat().st_mtime, hdr.stat().st_mtime, lib.stat().st_mtime):
        out.parent.mkdir(exist_ok=True)
        subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", str(src), "-o", str(out), f"-L{PKG}", "-lrdx",
                        f"-Wl,-rpath,{PKG}"], check=True)
    return out


def test_cpp_host_mirror_cpu():
    r = subprocess.run([str(_binary()), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_host_mirror_gpu():
    r = subprocess.run([str(_binary()), "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
