"""world_size-2 gloo rehearsal of the multi-GPU path on CPU: chunk shards are disjoint and complete,
per-rank results gathered in rank order equal the single-process results, and the max-over-ranks
timing reduction works.  The per-chunk computation here is the ORACLE (no device on this host); the
device engine is exercised per rank by bench.py on the GPU box."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from reductionist_amd.sharding import device_for, max_over_ranks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _chunk(i):
    rng = np.random.default_rng(0x5EED1000 + i)
    vals = rng.integers(-8, 9, 4096).astype(np.float32)
    return vals.view(np.uint8).reshape(-1, 4).T.copy().tobytes()   # shuffle es=4


def _worker(rank, world, port, n_chunks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "reductionist-rs_amd"), str(root)]
    from oracle import py_oracle as oracle
    from reductionist_amd import _abi
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n_chunks, rank, world)
    creq = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}])
    res = [struct_sum(oracle.execute(creq, _chunk(i))) for i in range(lo, hi)]
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, res))
    t = max_over_ranks(float(rank + 1))
    if rank == 0:
        q.put((gathered, t))
    dist.barrier()
    dist.destroy_process_group()


def struct_sum(r):
    import struct
    st, info, body, counts = r
    assert st == 0
    return struct.unpack("<f", body)[0], counts[0]


@pytest.mark.parametrize("n_chunks", [7, 64])
def test_gloo_world2_sharded_chunks(n_chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_chunks, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0
    spans = [(lo, hi) for lo, hi, _ in gathered]
    assert spans[0][0] == 0 and spans[-1][1] == n_chunks and spans[0][1] == spans[1][0]
    merged = [x for _, _, res in gathered for x in res]
    from oracle import py_oracle as oracle
    from reductionist_amd import _abi
    creq = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}])
    single = [struct_sum(oracle.execute(creq, _chunk(i))) for i in range(n_chunks)]
    assert merged == single


def test_shard_range_properties():
    for n in (0, 1, 7, 1024, 1025):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    assert device_for(5, 8) == 5 and device_for(9, 8) == 1 and device_for(1, 1) == 0
