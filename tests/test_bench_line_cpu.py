"""bench.py's stdout line stays small enough for the driver to parse (round 5's 21.5 KB
line came back `parsed: null`).  Built from a canned full record (round 5's `--steps 20 --warmup 5` line,
tests/golden/bench_full_r05.json); no GPU."""
import json
from pathlib import Path

import bench

GOLD = Path(__file__).resolve().parent / "golden" / "bench_full_r05.json"
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def test_compact_line_small_and_complete():
    full = json.loads(GOLD.read_text())
    s = bench.compact_line(full, "gpurun_out/bench_full.json")
    assert "\n" not in s
    assert len(s.encode()) <= bench.LINE_MAX_BYTES
    d = json.loads(s)
    for k in REQUIRED:
        assert k in d, k
    assert d["value"] == full["value"] and d["ms_per_step"] == full["ms_per_step"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    # extra is flat scalars, one or two per leg
    assert all(isinstance(v, (int, float)) for v in d["extra"].values())
    assert d["extra"]["c2_single_chunk_frac"] == full["extra"]["c2_single_chunk"]["roofline_frac"]
    assert d["extra"]["f64_64mib_frac"] == full["extra"]["f64_64mib"]["roofline_frac"]
    assert d["full_record"] == "gpurun_out/bench_full.json"


def test_compact_line_bounded_even_when_extra_explodes():
    full = json.loads(GOLD.read_text())
    full["extra"]["concurrent_native"] = full["extra"]["concurrent_native"] * 200
    for i, r in enumerate(full["extra"]["concurrent_native"]):
        r["threads"] = i
    s = bench.compact_line(full)
    assert len(s.encode()) <= bench.LINE_MAX_BYTES
    d = json.loads(s)
    for k in REQUIRED:
        assert k in d, k


def test_compact_line_minimal_record():
    line = {"metric": "m", "value": 1.0, "unit": "GiB/s", "n_gpus": 1, "steps": 1, "warmup": 0, "ms_per_step": 1.0,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "c2"}, "roofline": {"frac": 0.5}, "extra": {}}
    d = json.loads(bench.compact_line(line))
    assert d["extra"] == {} and "cpu_baseline" not in d and "full_record" not in d
