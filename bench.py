#!/usr/bin/env python3
"""bench.py — GiB/s of device-resident chunk unshuffle+reduce (f32 sum) on MI355X.

Workload (BASELINE.json configs[1], "c2"): 64 MiB chunks of 16 Mi f32 values stored big-endian and
byte-shuffled (element_size 4), each reduced with `sum` (its own result + count).  8 distinct chunks
(512 MiB > the 256 MiB Infinity Cache) are resident in HBM before timing; one step = one launch of the
fused unshuffle + byte-swap + f64-accumulated sum kernel over those 8 independent chunks through the
engine's batch entry point (rdx_execute_batch_device), so every step streams 512 MiB from HBM and the
per-launch ramp/finalisation (~6 us, profiles/) is paid once per 8 chunks.  extra.c2_single_chunk
reports the same chunks at one chunk per launch (rdx_execute_device); extra.c2_concurrent_requests
issues those single-chunk calls round-robin over 4 HIP streams (one workspace each), as concurrent
server requests would be (RDX_BENCH_STREAMS overrides the 4).
Ranks (one per GPU, torchrun) each process their own chunks: weak scaling, no data-path collective
(the control-plane barrier / max-time reduction uses gloo).

Also reported (extra.c4_batch): BASELINE configs[3] — a batch of 1024 independent 4 MiB shuffled f32
chunks summed by one launch per step, the batch split across ranks (strong scaling of that batch).
extra.f64_64mib / extra.f64_4mib: the north_star's f64 legs — 8 x 64 MiB and 128 x 4 MiB f64 chunks
per GPU (big-endian, shuffle element_size 8, sum), one batched launch per step (weak scaling).

Roofline: bytes_alg per launch = n_elements * 4 B read (unshuffle / byte swap add no algorithmic
bytes; the 16 B result is negligible) / average kernel duration from HIP events recorded on the
launch stream around every step of the timed region; peak = 8.0 TB/s HBM3E (MI355X_MICROARCH.md).
`traffic` comes from a rocprofv3 PMC pass (profiles/*_pmc.json) when one is committed.
cpu_baseline: the oracle (CPU restatement of the reference's sequential path) on 1 host core.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (str(ROOT / "reductionist-rs_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GIB = float(1 << 30)
PEAK_GBS = 8000.0          # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md "Chip-level parameters")
C2_ELEMS = 16 * 1024 * 1024
C2_BYTES = C2_ELEMS * 4
N_BUF = 8
C4_CHUNKS = 1024
C4_ELEMS = 1024 * 1024


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--c4-steps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--no-inflate", action="store_true")
    ap.add_argument("--no-f64", action="store_true")
    ap.add_argument("--primary-only", action="store_true", help="only the headline batched C2 loop (profiling)")
    return ap.parse_args()


def shuffled_be_f32(torch, vals):
    """values (…, n) f32 on device -> big-endian bytes, byte-shuffled with element_size 4
    (src/filters/shuffle.rs:124-135 encoder), laid out (…, 4*n) uint8 contiguous."""
    b = vals.contiguous().view(torch.uint8).reshape(*vals.shape, 4).flip(-1)       # big-endian
    return b.transpose(-1, -2).contiguous().reshape(*vals.shape[:-1], 4 * vals.shape[-1])


def f64_batch(torch, ws, stream, g, rank, barrier, max_over_ranks, world, elems, n_chunks, steps):
    """n_chunks independent HBM-resident f64 chunks (big-endian, shuffle element_size 8, sum) per rank,
    one rdx_execute_batch_device launch per step; results checked against an f64 sum of the values
    (f64 chunks are summed Neumaier-compensated)."""
    g.manual_seed(0x5EED2000 + rank)
    vals = torch.rand(n_chunks, elems, device="cuda", generator=g, dtype=torch.float64)
    exact = vals.sum(dim=1).cpu()
    b = vals.view(torch.uint8).reshape(n_chunks, elems, 8).flip(-1)            # big-endian
    chunks = b.transpose(-1, -2).contiguous().reshape(n_chunks, 8 * elems)     # shuffle es=8
    del vals, b
    bodies = torch.zeros(n_chunks, dtype=torch.float64, device="cuda")
    counts = torch.zeros(n_chunks, dtype=torch.int64, device="cuda")
    status = torch.zeros(n_chunks, dtype=torch.int32, device="cuda")
    from reductionist_amd import _abi
    creq = _abi.CRequest("sum", "float64", byte_order="big", filters=[{"id": "shuffle", "element_size": 8}])
    ptrs = [chunks[i].data_ptr() for i in range(n_chunks)]

    def launch():
        ws.execute_batch_device(creq, ptrs, 8 * elems, bodies.data_ptr(), counts.data_ptr(), status.data_ptr(),
                                stream.cuda_stream)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 and bool((counts.cpu() == elems).all())
    assert bool(((bodies.cpu() - exact).abs() <= exact.abs() * 2.0 ** -44).all()), (bodies.cpu(), exact)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    el = max_over_ranks(t1 - t0)
    k = e0.elapsed_time(e1) / 1e3 / steps
    step_bytes = n_chunks * 8 * elems
    return {"workload": f"{n_chunks} x {8 * elems >> 20} MiB f64 chunks per GPU, big-endian, shuffle es=8, sum; "
                        "one batched launch per step",
            "value": round(steps * step_bytes * world / el / GIB, 2), "unit": "GiB/s", "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 5), "kernel_us_avg": round(k * 1e6, 3),
            "roofline_frac": round(step_bytes / k / 1e9 / PEAK_GBS, 4)}


def traffic_from_profiles(tag):
    p = ROOT / "profiles" / f"{tag}_pmc.json"
    if p.exists():
        try:
            return json.loads(p.read_text()).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def cpu_baseline(seconds):
    """Oracle on the host: unshuffle + byte swap + sequential f32 fold of one 64 MiB chunk."""
    import numpy as np
    from oracle import py_oracle as oracle
    from reductionist_amd import _abi
    rng = np.random.default_rng(0x5EED0004)
    vals = rng.random(C2_ELEMS, dtype=np.float32)
    data = vals.astype(">f4").view(np.uint8).reshape(C2_ELEMS, 4).T.copy().tobytes()
    creq = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
    lib = oracle.lib()
    src = C.create_string_buffer(data, len(data))
    body = (C.c_uint8 * 64)()
    counts = (C.c_int64 * 8)()
    info = _abi.rdx_response_info()
    reps, t0 = 0, time.perf_counter()
    while True:
        st = lib.oracle_execute(C.addressof(creq.c), src, len(data), body, 64, counts, 8, C.byref(info))
        assert st == 0
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 1000:
            break
    return {"value": round(reps * C2_BYTES / el / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x one 64 MiB chunk (16 Mi f32, big-endian, shuffle es=4), sum, sequential "
                      f"oracle/rdx_oracle.cpp g++ -O2 on 1 host core, {el:.1f} s"}


def cpu_baseline_c4(threads, distinct=64):
    """C4 on the host the way the reference serves it: independent requests on a worker pool
    (thread_limit = num_cpus - 1, src/app_state.rs:22; capped at the box's CPU share).  1024 chunks of
    4 MiB (64 distinct, cycled), unshuffle + f32 sum each, by the oracle; ctypes releases the GIL."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from oracle import py_oracle as oracle
    from reductionist_amd import _abi
    lib = oracle.lib()
    creq = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}])
    rng = np.random.default_rng(0x5EED1000)
    srcs = []
    for _ in range(distinct):
        v = rng.random(C4_ELEMS, dtype=np.float32)
        b = v.view(np.uint8).reshape(C4_ELEMS, 4).T.copy().tobytes()
        srcs.append(C.create_string_buffer(b, len(b)))

    def one(i):
        body = (C.c_uint8 * 64)()
        counts = (C.c_int64 * 8)()
        info = _abi.rdx_response_info()
        assert lib.oracle_execute(C.addressof(creq.c), srcs[i % distinct], 4 * C4_ELEMS, body, 64, counts, 8,
                                  C.byref(info)) == 0

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(threads)))                      # warm the pool
        t0 = time.perf_counter()
        list(ex.map(one, range(C4_CHUNKS)))
        el = time.perf_counter() - t0
    return {"value": round(C4_CHUNKS * 4 * C4_ELEMS / el / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port", "sample": f"all {C4_CHUNKS} chunks ({distinct} distinct, cycled), {threads} worker "
                                      f"threads, oracle g++ -O2, {el:.2f} s"}


def inflate_batch(torch, ws, stream, rank, world, with_cpu, n_total=1024, distinct=16, reps=3):
    """BASELINE configs[3]'s batch shape with zlib on top: 1024 x 4 MiB N(0,1) f32 chunks, byte-shuffled,
    zlib level 1 (distinct chunks cycled), split over ranks; one rdx_decompress_batch_device launch per
    rep.  GB/s of decompressed output; CPU: CPython zlib (the C library) on 15 threads."""
    import zlib
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from reductionist_amd.sharding import shard_range
    lo, hi = shard_range(n_total, rank, world)
    n = hi - lo
    rng = np.random.default_rng(0x5EED2000)
    raws, streams = [], []
    for _ in range(distinct):
        v = rng.standard_normal(C4_ELEMS).astype(np.float32)
        raw = v.view(np.uint8).reshape(C4_ELEMS, 4).T.copy().tobytes()
        c = zlib.compressobj(1, zlib.DEFLATED, 15)
        raws.append(raw)
        streams.append(c.compress(raw) + c.flush())
    offs, total = [], 0
    for s in streams:
        offs.append(total)
        total += (len(s) + 255) // 256 * 256
    host = np.zeros(total, dtype=np.uint8)
    for o, s in zip(offs, streams):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    d_in = torch.from_numpy(host).cuda()
    raw_len = 4 * C4_ELEMS
    d_out = torch.empty(max(1, n) * raw_len, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(max(1, n), dtype=torch.int64, device="cuda")
    d_err = torch.zeros(max(1, n), dtype=torch.int32, device="cuda")
    ptrs = [d_in.data_ptr() + offs[(lo + i) % distinct] for i in range(n)]
    lens = [len(streams[(lo + i) % distinct]) for i in range(n)]

    def launch():
        ws.decompress_batch_device("zlib", ptrs, lens, d_out.data_ptr(), raw_len, d_len.data_ptr(),
                                   d_err.data_ptr(), stream.cuda_stream)

    launch()
    torch.cuda.synchronize()
    assert int(d_err.abs().sum()) == 0 and bool((d_len == raw_len).all())
    assert d_out[:raw_len].cpu().numpy().tobytes() == raws[lo % distinct]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    out = {"workload": "1024 x 4 MiB N(0,1) f32 chunks, shuffle es=4, zlib level 1 (ratio %.2f), batch split over "
                       "ranks; one rdx_decompress_batch_device launch" % (raw_len * distinct / sum(len(s) for s in streams)),
           "value": round(n * raw_len / t / 1e9, 2), "unit": "GB/s decompressed (this rank)", "ms_per_launch":
           round(t * 1e3, 2), "kernel": "k_inflate", "bound": "serial decode per wavefront (DESIGN.md §9), not HBM"}
    if with_cpu:
        threads = max(1, min(15, (os.cpu_count() or 2) - 1))

        def one(i):
            zlib.decompress(streams[i % distinct])

        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(threads)))
            c0 = time.perf_counter()
            list(ex.map(one, range(n_total)))
            tz = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": round(n_total * raw_len / tz / 1e9, 2), "unit": "GB/s", "cores": threads,
                               "kind": "library", "sample": f"CPython zlib.decompress of all {n_total} streams on a "
                                                            f"{threads}-thread pool, {tz:.2f} s"}
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from reductionist_amd import Engine, _abi
    from reductionist_amd.sharding import device_for, shard_range

    device = device_for(local_rank, torch.cuda.device_count())
    torch.cuda.set_device(device)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    eng = Engine([device])
    ws = eng.workspace(device)
    lib = _abi.lib()
    stream = torch.cuda.current_stream()
    sh = C.c_void_p(stream.cuda_stream)

    # ---- C2: 8 distinct 64 MiB chunks resident in HBM --------------------------------------------------
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0004 + rank)
    vals = torch.rand(N_BUF, C2_ELEMS, device="cuda", generator=g, dtype=torch.float32)
    chunks = shuffled_be_f32(torch, vals)
    exact = vals.double().sum(dim=1).cpu()
    del vals
    bodies = torch.zeros(N_BUF, dtype=torch.float32, device="cuda")
    counts = torch.zeros(N_BUF, dtype=torch.int64, device="cuda")
    status = torch.zeros(N_BUF, dtype=torch.int32, device="cuda")
    creq = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
    info = _abi.rdx_response_info()
    ptrs = (C.c_void_p * N_BUF)(*[chunks[i].data_ptr() for i in range(N_BUF)])
    batch_args = (ws.ws, creq.ref, N_BUF, ptrs, C2_BYTES, C.c_void_p(bodies.data_ptr()),
                  C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), sh, C.byref(info))
    single_args = [(ws.ws, creq.ref, C.c_void_p(chunks[i].data_ptr()), C2_BYTES, C.c_void_p(bodies[i:].data_ptr()),
                    C.c_void_p(counts[i:].data_ptr()), C.c_void_p(status[i:].data_ptr()), sh, C.byref(info))
                   for i in range(N_BUF)]

    def check_results():
        torch.cuda.synchronize()
        got = bodies.double().cpu()
        assert int(status.abs().sum()) == 0 and bool((counts.cpu() == C2_ELEMS).all()), (status.cpu(), counts.cpu())
        tol = exact.abs() * 2.0 ** -23 + 1e-3
        assert bool(((got - exact).abs() <= tol).all()), (got, exact)
        bodies.zero_()
        counts.zero_()

    def batch_step(i):
        st = lib.rdx_execute_batch_device(*batch_args)
        if st:
            raise RuntimeError(f"rdx_execute_batch_device failed: {_abi.status_string(st)}")

    def single_step(i):
        st = lib.rdx_execute_device(*single_args[i % N_BUF])
        if st:
            raise RuntimeError(f"rdx_execute_device failed: {_abi.status_string(st)}")

    def timed(step, n):
        """n back-to-back launches on one stream, bracketed by barrier + synchronize; HIP events on the
        launch stream around the same region give the average launch duration (gaps included)."""
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(n):
            step(i)
        ev1.record(stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        return max_over_ranks(t1 - t0), ev0.elapsed_time(ev1) / 1e3 / n

    for i in range(max(args.warmup, 1)):   # (at least one launch, so the check below has results)
        batch_step(i)
    check_results()                       # what we time is correct: every chunk vs an f64 sum
    elapsed, kern_avg_s = timed(batch_step, args.steps)
    check_results()
    step_bytes = N_BUF * C2_BYTES
    value = args.steps * step_bytes * world / elapsed / GIB
    achieved = step_bytes / kern_avg_s / 1e9

    extra = {}
    if args.primary_only:
        args.no_c4 = args.no_cpu_baseline = args.no_inflate = args.no_f64 = True
    else:
        for i in range(max(args.warmup, N_BUF)):   # every chunk at least once, whatever --warmup is
            single_step(i)
        check_results()
        el1, k1 = timed(single_step, args.steps)
        extra["c2_single_chunk"] = {
        "workload": "the same 64 MiB chunks, one chunk per launch (rdx_execute_device)",
        "value": round(args.steps * C2_BYTES * world / el1 / GIB, 2), "unit": "GiB/s",
        "ms_per_step": round(el1 / args.steps * 1e3, 5), "kernel_us_avg": round(k1 * 1e6, 3),
        "roofline_frac": round(C2_BYTES / k1 / 1e9 / PEAK_GBS, 4)}

        # concurrent single-chunk requests, the way a server runs them (one request per worker thread,
        # app.rs:123-153): one workspace + HIP stream per in-flight request, chunks round-robin, so one
        # launch's ramp / hand-off tail overlaps the next launch's streaming
        n_st = int(os.environ.get("RDX_BENCH_STREAMS", "4"))
        sts = [torch.cuda.Stream() for _ in range(n_st)]
        wss = [eng.workspace(device) for _ in range(n_st)]
        conc_args = [(wss[i % n_st].ws,) + single_args[i][1:-2] + (C.c_void_p(sts[i % n_st].cuda_stream),
                                                                   single_args[i][-1]) for i in range(N_BUF)]

        def conc_step(i):
            st = lib.rdx_execute_device(*conc_args[i % N_BUF])
            if st:
                raise RuntimeError(f"rdx_execute_device failed: {_abi.status_string(st)}")

        for i in range(max(args.warmup, N_BUF)):
            conc_step(i)
        check_results()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            conc_step(i)
        torch.cuda.synchronize()
        elc = max_over_ranks(time.perf_counter() - t0)
        barrier()
        check_results()
        extra["c2_concurrent_requests"] = {
            "workload": f"the same 64 MiB chunks, one chunk per rdx_execute_device call, {n_st} streams / "
                        "workspaces round-robin (concurrent requests)",
            "value": round(args.steps * C2_BYTES * world / elc / GIB, 2), "unit": "GiB/s",
            "us_per_request": round(elc / args.steps * 1e6, 3),
            "roofline_frac": round(args.steps * C2_BYTES / elc / 1e9 / PEAK_GBS, 4),
            "timing": "host wall clock around the K calls, synchronize on both sides"}
        for w in wss:
            w.close()

    # ---- C4 (extra): 1024 x 4 MiB chunks, one batched launch per step ----------------------------------
    if not args.no_c4:
        lo4, hi4 = shard_range(C4_CHUNKS, rank, world)
        n_local = hi4 - lo4
        g.manual_seed(0x5EED1000 + lo4)
        v4 = torch.rand(n_local, C4_ELEMS, device="cuda", generator=g, dtype=torch.float32)
        ex4 = v4.double().sum(dim=1).cpu()
        # native byte order, shuffle es=4
        c4 = v4.view(torch.uint8).reshape(n_local, C4_ELEMS, 4).transpose(1, 2).contiguous().reshape(n_local, -1)
        del v4
        b4 = torch.zeros(n_local, dtype=torch.float32, device="cuda")
        n4 = torch.zeros(n_local, dtype=torch.int64, device="cuda")
        s4 = torch.zeros(n_local, dtype=torch.int32, device="cuda")
        creq4 = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}])
        ptrs = [c4[i].data_ptr() for i in range(n_local)]
        for _ in range(2):
            ws.execute_batch_device(creq4, ptrs, 4 * C4_ELEMS, b4.data_ptr(), n4.data_ptr(), s4.data_ptr(),
                                    stream.cuda_stream)
        torch.cuda.synchronize()
        assert bool((n4.cpu() == C4_ELEMS).all()) and int(s4.abs().sum()) == 0
        assert bool(((b4.double().cpu() - ex4).abs() <= ex4.abs() * 2.0 ** -23 + 1e-3).all())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.c4_steps):
            ws.execute_batch_device(creq4, ptrs, 4 * C4_ELEMS, b4.data_ptr(), n4.data_ptr(), s4.data_ptr(),
                                    stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        el4 = max_over_ranks(t1 - t0)
        k4 = e0.elapsed_time(e1) / 1e3 / args.c4_steps
        extra["c4_batch"] = {
            "workload": "1024 x 4 MiB f32 chunks, shuffle es=4, native order, sum; batch split over ranks",
            "value": round(args.c4_steps * C4_CHUNKS * 4 * C4_ELEMS / el4 / GIB, 2), "unit": "GiB/s",
            "scaling": "strong", "steps": args.c4_steps, "ms_per_step": round(el4 / args.c4_steps * 1e3, 4),
            "chunks_per_rank": n_local,
            "roofline_frac": round(n_local * 4 * C4_ELEMS / k4 / 1e9 / PEAK_GBS, 4)}
        del c4
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            extra["c4_batch"]["cpu_baseline"] = cpu_baseline_c4(max(1, min(15, (os.cpu_count() or 2) - 1)))

    # ---- f64 chunks (extra): north_star's "4 MiB and 64 MiB f32/f64 chunks", f64 legs --------------------
    if not args.no_f64:
        extra["f64_64mib"] = f64_batch(torch, ws, stream, g, rank, barrier, max_over_ranks, world,
                                       elems=8 * 1024 * 1024, n_chunks=N_BUF, steps=max(10, args.steps // 4))
        extra["f64_4mib"] = f64_batch(torch, ws, stream, g, rank, barrier, max_over_ranks, world,
                                      elems=512 * 1024, n_chunks=128, steps=max(10, args.steps // 4))

    # ---- decompression (extra): the filter pipeline's first stage on the device ------------
    if not args.no_inflate:
        extra["c4z_inflate"] = inflate_batch(torch, ws, stream, rank, world, not args.no_cpu_baseline and rank == 0
                                             and world == 1)

    line = {
        "metric": "GiB/s device-resident chunk unshuffle+reduce (f32 sum), 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic U[0,1) f32, big-endian, byte-shuffled (es=4)",
        "config": {"workload": "c2: f32 sum over 64 MiB chunks (16 Mi elements each), byte shuffle es=4 + "
                               "non-native (big) byte order; one step = one launch over 8 independent "
                               "HBM-resident chunks (512 MiB) per GPU, one result per chunk",
                   "chunk_bytes": C2_BYTES, "chunks_per_step": N_BUF, "elements_per_chunk": C2_ELEMS,
                   "parallelism": f"independent chunks x{world} GPUs"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_GBS, 4), "traffic": traffic_from_profiles("c2"),
                     "kernel": "k_all_contig<float, OP_SUM, FUSED=1, MK=0>",
                     "kernel_us_avg": round(kern_avg_s * 1e6, 3), "bytes_alg_per_launch": step_bytes,
                     "timing": "HIP events on the launch stream around the K back-to-back launches / K"},
        "extra": extra,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        line["cpu_baseline"]["nproc"] = os.cpu_count()
    if rank == 0:
        print(json.dumps(line), flush=True)
    ws.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
