"""A hand-off record that never arrives ends the launch with RDX_E_DEVICE instead of hanging the GPU
(rdx_device.hpp: every poll of a record is bounded by kSpinLimit).  Probe build librdx_probe.so
(make -C reductionist-rs_amd probe: -DRDX_PROBES=1, spin limit 2^12 polls) with RDX_DROP_BLOCK = 1 + b:
grid block b skips publishing its record — what a faulted producer looks like to the folder — in both
hand-off forms (RDX_FOLD_LAST=1: the chunk's last block folds by polling; 0: arrival counters elect the
folder).  Each case runs in its own process (the engine reads its tuning environment once)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
PROBE = ROOT / "reductionist-rs_amd" / "librdx_probe.so"

SCRIPT = r"""
import json, sys, time
sys.path[:0] = [sys.argv[1] + "/reductionist-rs_amd", sys.argv[1]]
import numpy as np
from reductionist_amd import Engine, _abi
eng = Engine([0])
v = np.arange(1 << 20, dtype=np.float32) % 7          # C1 shape: 4 MiB, 128 workgroups
t = time.time()
st, info, body, counts = eng.execute_raw(_abi.CRequest("sum", "float32"), v.tobytes())
out = {"status": st, "seconds": time.time() - t}
if st == 0:
    out["sum"] = float(np.frombuffer(body, np.float32)[0])
    out["expect"] = float(v.astype(np.float64).sum())
print(json.dumps(out))
"""


def run(drop, fold_last):
    env = dict(os.environ, RDX_LIB_PATH=str(PROBE), RDX_DROP_BLOCK=str(drop), RDX_FOLD_LAST=str(fold_last))
    r = subprocess.run([sys.executable, "-c", SCRIPT, str(ROOT)], env=env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("fold_last", [1, 0])
def test_missing_publisher_is_a_device_error(fold_last):
    if not PROBE.exists():
        pytest.fail(f"{PROBE} missing: make -C reductionist-rs_amd probe")
    ok = run(0, fold_last)
    assert ok["status"] == 0 and ok["sum"] == ok["expect"]
    for drop in (6, 128):          # a middle block, and the chunk's last block (the folder in fold-last form)
        bad = run(drop, fold_last)
        assert bad["status"] == 9, bad      # RDX_E_DEVICE
        assert bad["seconds"] < 30, bad
