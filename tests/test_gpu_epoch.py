"""Result slots and hand-off records across the 16-bit tag wrap (rdx_runtime.cpp next_epoch / launch_lane):
when a workspace's epoch passes 0xffff the records and the lanes' page-locked slots are cleared so that no
granule left by a launch 65535 epochs earlier can carry a current tag.  Probe build librdx_probe.so with
RDX_EPOCH_START = 65530, so every workspace wraps after a few launches: coalesced launches (lanes on their own
streams, RDX_COALESCE_DEPTH=1, and launch-ahead pairs sharing a stream, =2) and the idle-queue fast path
cross the wrap many times over; every result must equal the exact sum (D-int data).  Each case runs in its
own process (the engine reads its tuning environment once)."""
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
import json, sys, threading
sys.path[:0] = [sys.argv[1] + "/reductionist-rs_amd", sys.argv[1]]
import numpy as np, torch
from reductionist_amd import Engine, _abi
eng = Engine([0])
rng = np.random.default_rng(99)
chunks = [rng.integers(-8, 9, n).astype(np.float32) for n in (1 << 12, 1 << 16, 1 << 20) for _ in range(4)]
expect = [float(c.astype(np.float64).sum()) for c in chunks]
dev = [torch.from_numpy(c.view(np.uint8).copy()).cuda() for c in chunks]
torch.cuda.synchronize()
creq = _abi.CRequest("sum", "float32")
bad = []
def run(t, n):
    for i in range(n):
        k = (i * 7 + t) % len(chunks)
        st, info, body, counts = eng.execute_resident(creq, 0, dev[k].data_ptr(), chunks[k].nbytes)
        got = float(np.frombuffer(body, np.float32)[0]) if st == 0 else None
        if st != 0 or got != expect[k] or counts != [chunks[k].size]:
            bad.append((t, i, k, st, got, expect[k]))
run(0, 40)                                   # one caller: the fast path across the wrap
th = [threading.Thread(target=run, args=(t, 60)) for t in range(8)]
for x in th: x.start()
for x in th: x.join()
s = eng.stats(0)
print(json.dumps({"bad": bad[:5], "n_bad": len(bad), "direct": s["direct_requests"],
                  "coalesced": s["coalesced_requests"], "launches": s["coalesced_launches"]}))
"""


@pytest.mark.parametrize("depth", [1, 2])
def test_tags_cross_the_wrap(depth):
    if not PROBE.exists():
        pytest.fail(f"{PROBE} missing: make -C reductionist-rs_amd probe")
    env = dict(os.environ, RDX_LIB_PATH=str(PROBE), RDX_EPOCH_START="65530", RDX_COALESCE_DEPTH=str(depth))
    r = subprocess.run([sys.executable, "-c", SCRIPT, str(ROOT)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_bad"] == 0, out
    assert out["direct"] >= 40 and out["coalesced"] > 0 and out["launches"] > 10, out
