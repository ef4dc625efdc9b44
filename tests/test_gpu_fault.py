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
dt = sys.argv[2]                                      # float32 sum: records; int32 sum / float64 max: atomics
v = (np.arange((4 << 20) // np.dtype(dt).itemsize) % 7).astype(dt)   # C1's 4 MiB: 128 workgroups
op = sys.argv[3]
t = time.time()
st, info, body, counts = eng.execute_raw(_abi.CRequest(op, dt), v.tobytes())
out = {"status": st, "seconds": time.time() - t}
if st == 0:
    out["value"] = float(np.frombuffer(body, dt)[0])
    out["expect"] = float(v.astype(np.float64).sum() if op == "sum" else v.max())
    # the next request on the same engine sees clean accumulators (the folder zeroes them)
    st2, _, body2, _ = eng.execute_raw(_abi.CRequest(op, dt), v.tobytes())
    out["again"] = float(np.frombuffer(body2, dt)[0]) if st2 == 0 else None
print(json.dumps(out))
"""


def run(drop, fold_last, dt="float32", op="sum"):
    env = dict(os.environ, RDX_LIB_PATH=str(PROBE), RDX_DROP_BLOCK=str(drop), RDX_FOLD_LAST=str(fold_last))
    r = subprocess.run([sys.executable, "-c", SCRIPT, str(ROOT), dt, op], env=env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("fold_last,dt,op", [(1, "float32", "sum"), (0, "float32", "sum"), (2, "int32", "sum"),
                                             (2, "float64", "max")])
def test_missing_publisher_is_a_device_error(fold_last, dt, op):
    """fold_last 2 with an order-free op: the folder waits on the arrivals in the accumulator lines
    (rdx_device.hpp atomic_fold), and a block that never arrives ends the same way."""
    if not PROBE.exists():
        pytest.fail(f"{PROBE} missing: make -C reductionist-rs_amd probe")
    ok = run(0, fold_last, dt, op)
    assert ok["status"] == 0 and ok["value"] == ok["expect"] and ok["again"] == ok["expect"], ok
    for drop in (6, 128):         # a middle block, and the chunk's last block (the folder in fold-last form)
        bad = run(drop, fold_last, dt, op)
        assert bad["status"] == 9, bad      # RDX_E_DEVICE
        assert bad["seconds"] < 30, bad


SCRIPT_DIRTY = r"""
import json, sys
sys.path[:0] = [sys.argv[1] + "/reductionist-rs_amd", sys.argv[1]]
import numpy as np
from reductionist_amd import Engine, _abi
eng = Engine([0])
v = (np.arange(1 << 20) % 7).astype(np.int32)        # 4 MiB: 128 workgroups, an order-free fold (fold_last 2)
req = _abi.CRequest("max", "int32")
out = []
for _ in range(3):
    st, info, body, counts = eng.execute_raw(req, v.tobytes())
    out.append(st)
print(json.dumps({"statuses": out}))
"""


def test_timed_out_atomic_fold_poisons_its_slot():
    """A fold that timed out (RDX_DROP_LAUNCHES=1: only the first launch loses a publisher) zeroes its lines but
    cannot know whether the missing publisher will still add to them, so it sets the chunk slot's dirty word:
    every later order-free fold on that workspace reports RDX_E_DEVICE instead of folding over stale words
    (rdx_device.hpp atomic_fold)."""
    if not PROBE.exists():
        pytest.fail(f"{PROBE} missing: make -C reductionist-rs_amd probe")
    env = dict(os.environ, RDX_LIB_PATH=str(PROBE), RDX_DROP_BLOCK="6", RDX_DROP_LAUNCHES="1", RDX_FOLD_LAST="2")
    r = subprocess.run([sys.executable, "-c", SCRIPT_DIRTY, str(ROOT)], env=env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    st = json.loads(r.stdout.strip().splitlines()[-1])["statuses"]
    assert st == [9, 9, 9], st   # RDX_E_DEVICE: the timed-out launch, then the poisoned slot
