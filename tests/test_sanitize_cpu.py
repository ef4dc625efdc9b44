"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer: the product planner
(rdx_plan.cpp) and the oracle built with -fsanitize=address,undefined -fno-sanitize-recover=all, driven
by tests/cpp/test_sanitize.cpp (random requests planner-vs-oracle, inflate on corrupted streams, the blosc2
decoder on corrupted golden chunks); and the coalescer's job hand-off (rdx_jobsync.hpp) under
ThreadSanitizer with many short-lived stack-allocated jobs (tests/cpp/test_jobsync.cpp).  Any sanitizer
report fails the run."""
import json
import os
import struct
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SRCS = [ROOT / "tests" / "cpp" / "test_sanitize.cpp", ROOT / "reductionist-rs_amd" / "csrc" / "rdx_plan.cpp",
        ROOT / "oracle" / "rdx_oracle.cpp", ROOT / "oracle" / "oracle_inflate.cpp", ROOT / "oracle" / "oracle_blosc2.cpp",
        ROOT / "oracle" / "oracle_zstd.cpp"]
DEPS = SRCS + [ROOT / "include" / "rdx.h", ROOT / "reductionist-rs_amd" / "csrc" / "rdx_plan.hpp",
               ROOT / "reductionist-rs_amd" / "csrc" / "rdx_kdesc.h"]


def _binary():
    out = ROOT / "tests" / "cpp" / "build" / "test_sanitize"
    if not out.exists() or out.stat().st_mtime < max(p.stat().st_mtime for p in DEPS):
        out.parent.mkdir(exist_ok=True)
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-fno-omit-frame-pointer", *map(str, SRCS), "-o", str(out)], check=True)
    return out


def test_planner_and_oracle_under_asan_ubsan():
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    seeds = ROOT / "tests" / "cpp" / "build" / "blosc2_seeds.bin"
    chunks = json.loads((ROOT / "tests" / "golden" / "blosc2_chunks.json").read_text())["chunks"]
    binary = _binary()
    seeds.write_bytes(b"".join(struct.pack("<I", len(c)) + c for c in (bytes.fromhex(x["chunk"]) for x in chunks)))
    r = subprocess.run([str(binary), "4000", str(seeds)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "sanitize: ok" in r.stdout, (r.stdout + r.stderr)[-4000:]


def test_job_handoff_under_tsan():
    """the dispatcher must not touch a caller's stack-allocated Job after completing it;
    every spin / sleep interleaving of job_wait against job_finish, under -fsanitize=thread."""
    src = ROOT / "tests" / "cpp" / "test_jobsync.cpp"
    hdr = ROOT / "reductionist-rs_amd" / "csrc" / "rdx_jobsync.hpp"
    out = ROOT / "tests" / "cpp" / "build" / "test_jobsync"
    if not out.exists() or out.stat().st_mtime < max(src.stat().st_mtime, hdr.stat().st_mtime):
        out.parent.mkdir(exist_ok=True)
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", str(src), "-o", str(out)],
                       check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([str(out), "8", "3000"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "jobsync: ok" in r.stdout and "ThreadSanitizer" not in r.stderr, (r.stdout + r.stderr)[-4000:]
