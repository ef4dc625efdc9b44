#!/usr/bin/env python3
"""bench.py — GiB/s of device-resident chunk unshuffle+reduce (f32 sum) on 1/2/4/8 MI355X.

Headline workload (BASELINE.json configs[1], "c2"): 64 MiB chunks of 16 Mi f32 values stored big-endian
and byte-shuffled (element_size 4), each reduced with `sum` (its own result + count).  8 distinct chunks
per GPU (512 MiB > the 256 MiB Infinity Cache) are resident in HBM before timing; one step = one launch
of the fused unshuffle + byte-swap + f64-accumulated sum kernel over those 8 independent chunks through
the engine's batch entry point (rdx_execute_batch_device).

Multi-GPU: one process per GPU, each owning its own chunks (weak scaling, no data-path
collective; the control-plane barrier and max-over-ranks timing use gloo on the host).  Under torchrun
the ranks come from the environment; `python bench.py --gpus N` outside torchrun starts N ranks itself
(a child torchrun, from this parent, which makes no GPU call) and fails loudly when fewer than N GPUs are
visible.  Every rank uses its own device (LOCAL_RANK); the line reports the distinct devices used.

extra (every number DESIGN.md quotes comes from here):
  c2_single_chunk        the same chunks, one chunk per launch (rdx_execute_device)
  c2_concurrent_requests one chunk per rdx_execute_device call over 4 HIP streams / workspaces; the
                         calls are queued behind a gate so the device time is measured (HIP events on
                         every stream), not the host's issue rate
  c4_batch               BASELINE configs[3]: 1024 x 4 MiB shuffled f32 chunks, one launch, split over
                         ranks (strong scaling of that batch)
  f64_64mib / f64_4mib   the north_star's f64 legs (shuffle es=8, big-endian, sum)
  c4z_inflate            the batch compressed with zlib, decompressed on the device
  c4b_blosc2             the batch as blosc2 chunks (LZ4 / BloscLZ + shuffle), decoded on the device
  configs                (N=1) device-resident C1, C3 (min / max / valid_range) and C5 select launches
  mixed_requests         (N=1) 20 mixed C1/C3 requests in ONE heterogeneous launch (rdx_execute_multi_device)
  concurrent_native      (N=1) C1 / C2 / C3 requests from native C++ threads (rdx_conc_bench): independent
                         launches per thread, and the context pool's coalesced path (rdx_execute_resident)
  pool                   (rank 0, all --gpus devices) ONE process, one context over every GPU, native threads
                         issuing C4 requests from pinned host memory and HBM-resident (the server's shape)
  cbor_response          (N=1) the CBOR response body of an axis = [] count over the C5 shape (32 Mi counts)
                         packed on the device (rdx_cbor_encode_device) vs the host encoder
  host_inclusive         (N=1) C2 / C3 / C5 through rdx_execute from pageable and pinned host memory,
                         next to the raw PCIe copy time of the same bytes
  cpu_baselines          (N=1) the oracle (CPU restatement of the reference path) on host cores: C1 with
                         and without the per-iteration clone of benches/operations.rs:63, C3, C5; CPU
                         model, affinity and cgroup quota

Roofline: bytes_alg per launch = n_elements * 4 B read (unshuffle / byte swap add no algorithmic bytes;
the 16 B result is negligible) / average kernel duration from HIP events recorded on the launch stream
around every step of the timed region; peak = 8.0 TB/s HBM3E (MI355X_MICROARCH.md).  `traffic` comes
from a rocprofv3 PMC pass (profiles/c2_pmc.json) when one is committed.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
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
C3_SEL = [[8, 120, 1], [0, 128, 2], [16, 112, 1]]
C3_NSEL = 112 * 64 * 96
C5_SEL = [[0, 512, 1], [64, 192, 1], [0, 256, 1]]


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
    ap.add_argument("--no-configs", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--primary-only", action="store_true", help="only the headline batched C2 loop (profiling)")
    ap.add_argument("--full-out", default="gpurun_out/bench_full.json",
                    help="where rank 0 writes the full record (every leg); '' = stderr only")
    return ap.parse_args()


# ---- N ranks without an external launcher ----------------------------------------------------------------
def spawn_ranks(args) -> int:
    """`bench.py --gpus N` outside torchrun: N per-GPU ranks as a child torchrun (this process makes no GPU
    call: torch.cuda.device_count() does not initialise HIP on this image)."""
    import torch
    n_dev = torch.cuda.device_count()
    if args.gpus > n_dev and os.environ.get("RDX_BENCH_OVERSUBSCRIBE") != "1":
        print(f"bench.py: --gpus {args.gpus} requested but only {n_dev} GPU(s) are visible; refusing to "
              "report a multi-GPU number from fewer devices (RDX_BENCH_OVERSUBSCRIBE=1 rehearses the N-rank "
              "code path on shared devices and reports the distinct devices used)", file=sys.stderr)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd)


# ---- helpers ------------------------------------------------------------------------------------------------
def shuffled_be_f32(torch, vals):
    """values (…, n) f32 on device -> big-endian bytes, byte-shuffled with element_size 4
    (src/filters/shuffle.rs:124-135 encoder), laid out (…, 4*n) uint8 contiguous."""
    b = vals.contiguous().view(torch.uint8).reshape(*vals.shape, 4).flip(-1)       # big-endian
    return b.transpose(-1, -2).contiguous().reshape(*vals.shape[:-1], 4 * vals.shape[-1])


def traffic_from_profiles(tag):
    p = ROOT / "profiles" / f"{tag}_pmc.json"
    if p.exists():
        try:
            return json.loads(p.read_text()).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def cpu_info():
    """CPU model, the threads this process may run on, and the cgroup CPU quota (the GPU box gives each
    one-GPU job a share of a large host: nproc shows the whole machine)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = round(q / per, 2) if q > 0 else None
        except (OSError, ValueError):
            pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def pool_threads():
    """Worker threads for the multi-chunk CPU baseline: the reference's default thread_limit is
    num_cpus - 1 (src/app_state.rs:22), capped by the CPUs this job may actually use (affinity, cgroup
    quota, OMP_NUM_THREADS as the box's stated share)."""
    info = cpu_info()
    n = (info["affinity_cpus"] or 2) - 1
    if info["cgroup_cpu_quota"]:
        n = min(n, max(1, int(info["cgroup_cpu_quota"]) - 1))
    if info["omp_num_threads"]:
        try:
            n = min(n, max(1, int(info["omp_num_threads"]) - 1))
        except ValueError:
            pass
    return max(1, n)


class Ctx:
    """Per-rank state shared by the legs."""

    def __init__(self, torch, dist, args, world, rank, device):
        from reductionist_amd import Engine, _abi
        self.torch, self.dist, self.args = torch, dist, args
        self.world, self.rank, self.device = world, rank, device
        self.abi = _abi
        self.eng = Engine([device])
        self.ws = self.eng.workspace(device)
        self.lib = _abi.lib()
        self.stream = torch.cuda.current_stream()
        self.sh = C.c_void_p(self.stream.cuda_stream)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def events(self):
        return (self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True))

    def timed(self, step, n):
        """n back-to-back launches on one stream, bracketed by barrier + synchronize; HIP events on the
        launch stream around the same region give the average launch duration (gaps included)."""
        torch = self.torch
        ev0, ev1 = self.events()
        self.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(self.stream)
        for i in range(n):
            step(i)
        ev1.record(self.stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        self.barrier()
        return self.max_over_ranks(t1 - t0), ev0.elapsed_time(ev1) / 1e3 / n

    def dev_time(self, step, n, warm=3):
        """Device time per launch: HIP events around n back-to-back launches on the launch stream."""
        for i in range(warm):
            step(i)
        self.torch.cuda.synchronize()
        e0, e1 = self.events()
        e0.record(self.stream)
        for i in range(n):
            step(i)
        e1.record(self.stream)
        self.torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / n

    def gate(self, streams, hold_s=0.02):
        """Hold `streams` behind a device-side sleep so that the host can queue every call before the
        device starts on them; returns the event that opens the gate (timing starts there)."""
        torch = self.torch
        gs = torch.cuda.Stream()
        with torch.cuda.stream(gs):
            torch.cuda._sleep(int(hold_s * self.sleep_rate()))
        opened = torch.cuda.Event(enable_timing=True)
        opened.record(gs)
        for s in streams:
            s.wait_event(opened)
        return opened

    _rate = None

    def sleep_rate(self):
        """torch.cuda._sleep cycles per second on this device (measured once)."""
        if Ctx._rate is None:
            torch = self.torch
            e0, e1 = self.events()
            e0.record(self.stream)
            torch.cuda._sleep(1_000_000)
            e1.record(self.stream)
            torch.cuda.synchronize()
            Ctx._rate = 1_000_000 / max(1e-6, e0.elapsed_time(e1) / 1e3)
        return Ctx._rate


# ---- legs ---------------------------------------------------------------------------------------------------
def leg_c2(cx):
    """Headline: 8 x 64 MiB HBM-resident chunks per GPU, one batched launch per step; plus the single-chunk
    and concurrent-request legs over the same chunks."""
    torch, args, lib, _abi = cx.torch, cx.args, cx.lib, cx.abi
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0004 + cx.rank)
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
    batch_args = (cx.ws.ws, creq.ref, N_BUF, ptrs, C2_BYTES, C.c_void_p(bodies.data_ptr()),
                  C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), cx.sh, C.byref(info))
    single_args = [(cx.ws.ws, creq.ref, C.c_void_p(chunks[i].data_ptr()), C2_BYTES, C.c_void_p(bodies[i:].data_ptr()),
                    C.c_void_p(counts[i:].data_ptr()), C.c_void_p(status[i:].data_ptr()), cx.sh, C.byref(info))
                   for i in range(N_BUF)]

    def check_results():
        torch.cuda.synchronize()
        got = bodies.double().cpu()
        assert int(status.abs().sum()) == 0 and bool((counts.cpu() == C2_ELEMS).all()), (status.cpu(), counts.cpu())
        tol = exact.abs() * 2.0 ** -23 + 1e-3
        assert bool(((got - exact).abs() <= tol).all()), (got, exact)
        bodies.zero_()
        counts.zero_()
        torch.cuda.synchronize()

    def batch_step(i):
        st = lib.rdx_execute_batch_device(*batch_args)
        if st:
            raise RuntimeError(f"rdx_execute_batch_device failed: {_abi.status_string(st)}")

    def single_step(i):
        st = lib.rdx_execute_device(*single_args[i % N_BUF])
        if st:
            raise RuntimeError(f"rdx_execute_device failed: {_abi.status_string(st)}")

    batch_step(0)
    check_results()                       # what we time is correct: every chunk vs an f64 sum
    for i in range(args.warmup):          # the warm-up launches directly before the timed region (no host-side
        batch_step(i)                     # check in between: an idle GPU clocks down)
    elapsed, kern_avg_s = cx.timed(batch_step, args.steps)
    check_results()                       # and what the timed region computed
    step_bytes = N_BUF * C2_BYTES
    out = {"value": args.steps * step_bytes * cx.world / elapsed / GIB, "elapsed": elapsed,
           "kern_avg_s": kern_avg_s, "step_bytes": step_bytes, "extra": {}}
    if args.primary_only:
        return out
    extra = out["extra"]
    # the same number of steps again, each launch between its own pair of HIP events: the spread of the
    # per-launch kernel time behind the timed region's average (the first steps after the warm-up, the
    # box's run-to-run variation)
    evs = [cx.events() for _ in range(args.steps)]
    cx.barrier()
    torch.cuda.synchronize()
    for i in range(args.steps):
        evs[i][0].record(cx.stream)
        batch_step(i)
        evs[i][1].record(cx.stream)
    torch.cuda.synchronize()
    per = [round(a.elapsed_time(b) * 1e3, 2) for a, b in evs]
    srt = sorted(per)
    extra["headline_per_step"] = {
        "kernel_us": per, "min_us": srt[0], "median_us": srt[len(srt) // 2], "max_us": srt[-1],
        "timed_region_avg_us": round(kern_avg_s * 1e6, 3),
        "note": "one event pair per launch over --steps launches after the timed region (same chunks, same stream)"}
    check_results()
    for i in range(N_BUF):                     # every chunk once, checked
        single_step(i)
    check_results()
    for i in range(max(args.warmup, N_BUF)):   # then the warm-up, directly before the timed region
        single_step(i)
    el1, k1 = cx.timed(single_step, args.steps)
    check_results()
    extra["c2_single_chunk"] = {
        "workload": "the same 64 MiB chunks, one chunk per launch (rdx_execute_device), one stream",
        "value": round(args.steps * C2_BYTES * cx.world / el1 / GIB, 2), "unit": "GiB/s",
        "ms_per_step": round(el1 / args.steps * 1e3, 5), "kernel_us_avg": round(k1 * 1e6, 3),
        "roofline_frac": round(C2_BYTES / k1 / 1e9 / PEAK_GBS, 4)}

    # concurrent single-chunk requests, the way a server runs them (one request per worker thread,
    # app.rs:123-153): one workspace + HIP stream per in-flight request, chunks round-robin, so one
    # launch's ramp / hand-off tail overlaps the next launch's streaming.  The calls are queued behind a
    # device-side gate and timed with events on every stream (K fixed, independent of --steps).
    n_st = int(os.environ.get("RDX_BENCH_STREAMS", "4"))
    k_conc = max(args.steps, 400)
    sts = [torch.cuda.Stream() for _ in range(n_st)]
    wss = [cx.eng.workspace(cx.device) for _ in range(n_st)]
    conc_args = [(wss[i % n_st].ws,) + single_args[i][1:-2] + (C.c_void_p(sts[i % n_st].cuda_stream),
                                                               single_args[i][-1]) for i in range(N_BUF)]

    def conc_step(i):
        st = lib.rdx_execute_device(*conc_args[i % N_BUF])
        if st:
            raise RuntimeError(f"rdx_execute_device failed: {_abi.status_string(st)}")

    for s in sts:   # the zeroing in check_results() ran on the launch stream
        s.wait_stream(cx.stream)
    for i in range(max(args.warmup, N_BUF)):
        conc_step(i)
    check_results()
    for s in sts:
        s.wait_stream(cx.stream)
    cx.barrier()
    torch.cuda.synchronize()
    opened = cx.gate(sts, hold_s=0.01 + k_conc * 15e-6)
    for i in range(k_conc):
        conc_step(i)
    ends = []
    for s in sts:
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        ends.append(e)
    torch.cuda.synchronize()
    dev_s = max(opened.elapsed_time(e) for e in ends) / 1e3
    elc = cx.max_over_ranks(dev_s)
    cx.barrier()
    check_results()
    extra["c2_concurrent_requests"] = {
        "workload": f"the same 64 MiB chunks, one chunk per rdx_execute_device call, {n_st} streams / "
                    f"workspaces round-robin (concurrent requests), {k_conc} requests",
        "value": round(k_conc * C2_BYTES * cx.world / elc / GIB, 2), "unit": "GiB/s",
        "us_per_request": round(elc / k_conc * 1e6, 3),
        "roofline_frac": round(k_conc * C2_BYTES / elc / 1e9 / PEAK_GBS, 4),
        "timing": "calls queued behind a device-side gate; HIP events: gate open -> last stream's end"}
    for w in wss:
        w.close()
    return out


def leg_c4(cx):
    """BASELINE configs[3]: 1024 x 4 MiB f32 chunks, shuffle es=4, sum; the batch is split over ranks."""
    torch, args, _abi = cx.torch, cx.args, cx.abi
    from reductionist_amd.sharding import shard_range
    lo4, hi4 = shard_range(C4_CHUNKS, cx.rank, cx.world)
    n_local = hi4 - lo4
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED1000 + lo4)
    v4 = torch.rand(n_local, C4_ELEMS, device="cuda", generator=g, dtype=torch.float32)
    ex4 = v4.double().sum(dim=1).cpu()
    c4 = v4.view(torch.uint8).reshape(n_local, C4_ELEMS, 4).transpose(1, 2).contiguous().reshape(n_local, -1)
    del v4
    b4 = torch.zeros(n_local, dtype=torch.float32, device="cuda")
    n4 = torch.zeros(n_local, dtype=torch.int64, device="cuda")
    s4 = torch.zeros(n_local, dtype=torch.int32, device="cuda")
    creq4 = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}])
    ptrs = [c4[i].data_ptr() for i in range(n_local)]

    def step(i):
        cx.ws.execute_batch_device(creq4, ptrs, 4 * C4_ELEMS, b4.data_ptr(), n4.data_ptr(), s4.data_ptr(),
                                   cx.stream.cuda_stream)

    step(0)
    torch.cuda.synchronize()
    assert bool((n4.cpu() == C4_ELEMS).all()) and int(s4.abs().sum()) == 0
    assert bool(((b4.double().cpu() - ex4).abs() <= ex4.abs() * 2.0 ** -23 + 1e-3).all())
    for i in range(2):   # warm-up directly before the timed region
        step(i)
    el4, k4 = cx.timed(step, args.c4_steps)
    out = {"workload": "1024 x 4 MiB f32 chunks, shuffle es=4, native order, sum; batch split over ranks, one "
                       "rdx_execute_batch_device launch per rank per step",
           "value": round(args.c4_steps * C4_CHUNKS * 4 * C4_ELEMS / el4 / GIB, 2), "unit": "GiB/s",
           "scaling": "strong", "steps": args.c4_steps, "ms_per_step": round(el4 / args.c4_steps * 1e3, 4),
           "chunks_per_rank": n_local, "kernel_us_avg": round(k4 * 1e6, 2),
           "roofline_frac": round(n_local * 4 * C4_ELEMS / k4 / 1e9 / PEAK_GBS, 4)}
    del c4
    return out


def leg_f64(cx, elems, n_chunks, steps):
    """n_chunks independent HBM-resident f64 chunks (big-endian, shuffle element_size 8, sum) per rank,
    one rdx_execute_batch_device launch per step; results checked against an f64 sum of the values
    (f64 chunks are summed Neumaier-compensated)."""
    torch, _abi = cx.torch, cx.abi
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED2000 + cx.rank)
    vals = torch.rand(n_chunks, elems, device="cuda", generator=g, dtype=torch.float64)
    exact = vals.sum(dim=1).cpu()
    b = vals.view(torch.uint8).reshape(n_chunks, elems, 8).flip(-1)            # big-endian
    chunks = b.transpose(-1, -2).contiguous().reshape(n_chunks, 8 * elems)     # shuffle es=8
    del vals, b
    bodies = torch.zeros(n_chunks, dtype=torch.float64, device="cuda")
    counts = torch.zeros(n_chunks, dtype=torch.int64, device="cuda")
    status = torch.zeros(n_chunks, dtype=torch.int32, device="cuda")
    creq = _abi.CRequest("sum", "float64", byte_order="big", filters=[{"id": "shuffle", "element_size": 8}])
    ptrs = [chunks[i].data_ptr() for i in range(n_chunks)]

    def step(i):
        cx.ws.execute_batch_device(creq, ptrs, 8 * elems, bodies.data_ptr(), counts.data_ptr(), status.data_ptr(),
                                   cx.stream.cuda_stream)

    step(0)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 and bool((counts.cpu() == elems).all())
    assert bool(((bodies.cpu() - exact).abs() <= exact.abs() * 2.0 ** -44).all()), (bodies.cpu(), exact)
    for i in range(3):   # warm-up directly before the timed region
        step(i)
    el, k = cx.timed(step, steps)
    step_bytes = n_chunks * 8 * elems
    return {"workload": f"{n_chunks} x {8 * elems >> 20} MiB f64 chunks per GPU, big-endian, shuffle es=8, sum; "
                        "one batched launch per step",
            "value": round(steps * step_bytes * cx.world / el / GIB, 2), "unit": "GiB/s", "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 5), "kernel_us_avg": round(k * 1e6, 3),
            "roofline_frac": round(step_bytes / k / 1e9 / PEAK_GBS, 4)}


def leg_inflate(cx, with_cpu, n_total=1024, distinct=16, reps=3):
    """BASELINE configs[3]'s batch shape with zlib on top: 1024 x 4 MiB N(0,1) f32 chunks, byte-shuffled,
    zlib level 1 (distinct chunks cycled), split over ranks; one rdx_decompress_batch_device launch per
    rep.  GB/s of decompressed output; CPU: CPython zlib (the C library) on a thread pool."""
    import zlib
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from reductionist_amd.sharding import shard_range
    torch = cx.torch
    lo, hi = shard_range(n_total, cx.rank, cx.world)
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

    def step(i):
        cx.ws.decompress_batch_device("zlib", ptrs, lens, d_out.data_ptr(), raw_len, d_len.data_ptr(),
                                      d_err.data_ptr(), cx.stream.cuda_stream)

    step(0)
    torch.cuda.synchronize()
    assert int(d_err.abs().sum()) == 0 and bool((d_len == raw_len).all())
    assert d_out[:raw_len].cpu().numpy().tobytes() == raws[lo % distinct]
    t = cx.dev_time(step, reps, warm=0)
    out = {"workload": "1024 x 4 MiB N(0,1) f32 chunks, shuffle es=4, zlib level 1 (ratio %.2f), batch split over "
                       "ranks; one rdx_decompress_batch_device launch" % (raw_len * distinct / sum(len(s) for s in streams)),
           "value": round(n * raw_len / t / 1e9, 2), "unit": "GB/s decompressed (this rank)", "ms_per_launch":
           round(t * 1e3, 2), "kernel": "k_inflate", "bound": "serial decode per wavefront (DESIGN.md §9), not HBM"}
    if with_cpu:
        threads = pool_threads()

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
    out["lone"] = leg_inflate_lone(cx, streams, raws, with_cpu)
    return out


def leg_inflate_lone(cx, streams, raws, with_cpu, reps=20):
    """ONE compressed request (compression.rs:60-82): a lone 4 MiB zlib level-1 chunk of the c4z data decoded
    by the whole device (k_pinflate: block starts found, blocks and the symbols inside them decoded in
    parallel), against one host core's zlib (the reference decodes a request on its own thread).  Device:
    rdx_decompress_one_device on the HBM-resident stream, wall clock per synchronous call (two host round
    trips included), median of `reps`.  End to end: rdx_execute_owned of the compressed chunk as the plugin
    sends it (shuffled f32 sum: H2D of the compressed bytes, device decode, unshuffle + sum, result back)
    against the former route (host zlib on the request's thread, then rdx_execute_owned of the raw chunk)."""
    import zlib
    import numpy as np
    torch, _abi = cx.torch, cx.abi
    s, raw = streams[0], raws[0]
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_out = torch.empty(len(raw) + 16, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    err, n, path = cx.ws.decompress_one_device("zlib", d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
    assert err == 0 and n == len(raw) and path == 2, (err, n, path)
    assert d_out[:n].cpu().numpy().tobytes() == raw
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        cx.ws.decompress_one_device("zlib", d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
        ts.append(time.perf_counter() - t0)
    dev = float(np.median(ts))
    out = {"workload": "one 4 MiB shuffled N(0,1) f32 chunk, zlib level 1 (ratio %.3f: 191 stored + 20 Huffman "
                       "blocks), decoded by the whole device (k_pinflate)" % (len(raw) / len(s)),
           "device_ms": round(dev * 1e3, 3), "device_GBs": round(len(raw) / dev / 1e9, 2),
           "timing": "rdx_decompress_one_device on the HBM-resident stream, wall clock per synchronous call, "
                     f"median of {reps}", "path": "k_pinflate (rdx_inflate_last_path 2)"}
    creq = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}], compression="zlib")
    creq_raw = _abi.CRequest("sum", "float32", filters=[{"id": "shuffle", "element_size": 4}])
    st, *_ = cx.eng.execute_owned(creq, s)
    assert st == 0
    te, tr = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        st, *_ = cx.eng.execute_owned(creq, s)
        te.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        st2, *_ = cx.eng.execute_owned(creq_raw, zlib.decompress(s))
        tr.append(time.perf_counter() - t0)
        assert st == st2 == 0
    out["request_device_decode_ms"] = round(1e3 * float(np.median(te)), 3)
    out["request_host_decode_ms"] = round(1e3 * float(np.median(tr)), 3)
    if with_cpu:
        hs = []
        for _ in range(reps):
            t0 = time.perf_counter()
            zlib.decompress(s)
            hs.append(time.perf_counter() - t0)
        host = float(np.median(hs))
        out["cpu_baseline"] = {"value": round(host * 1e3, 3), "unit": "ms per chunk", "cores": 1, "kind": "library",
                               "sample": f"CPython zlib.decompress (the C library) of the same stream on one thread, "
                                         f"median of {reps}", "GBs": round(len(raw) / host / 1e9, 2)}
        out["speedup_vs_one_core"] = round(host / dev, 2)
    return out


def leg_blosc2(cx, with_cpu, n_total=1024, distinct=16, reps=3):
    """The C4 batch shape as blosc2 chunks (compression.rs:29-57): 1024 x 4 MiB f32 chunks of a smooth
    field quantized to 1/64 (the low mantissa bytes repeat, as in real model output), blosc2 chunks with
    the SHUFFLE filter, typesize 4, 64 KiB blocks split into 4 streams, written by this repo's own writer
    (datagen/blosc2_chunk.py; distinct chunks cycled), split over ranks; one rdx_decompress_batch_device
    launch per rep, per codec.  Also one lone chunk per call (a single request).  GB/s of decompressed
    output; CPU: the oracle's blosc2 decoder (scalar C++, oracle/oracle_blosc2.cpp) on a thread pool."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from datagen import blosc2_chunk as B
    from reductionist_amd.sharding import shard_range
    torch = cx.torch
    lo, hi = shard_range(n_total, cx.rank, cx.world)
    n = hi - lo
    rng = np.random.default_rng(0x5EED2100)
    raw_len = 4 * C4_ELEMS
    raws = [(np.round(np.cumsum(rng.standard_normal(C4_ELEMS)) * 64) / 64).astype(np.float32).tobytes()
            for _ in range(distinct)]
    out = {"workload": "1024 x 4 MiB f32 chunks (random walk quantized to 1/64) as blosc2 chunks: SHUFFLE, "
                       "typesize 4, 64 KiB blocks x 4 streams; batch split over ranks, one "
                       "rdx_decompress_batch_device launch per codec; lone = one chunk per call",
           "kernel": "k_blosc2_decode (+ k_blosc2_zstd for zstd) + k_blosc2_filter", "unit": "GB/s decompressed (this rank)",
           "bound": "serial token chain per wavefront (one stream each), not HBM"}
    d_out = torch.empty(max(1, n) * raw_len, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(max(1, n), dtype=torch.int64, device="cuda")
    d_err = torch.zeros(max(1, n), dtype=torch.int32, device="cuda")
    chunks_by_codec = {}
    # lz4 / blosclz: this repo's writer's streams; lz4_lib / zstd: streams by the real liblz4 / libzstd
    # (pyarrow's bundled codecs; zstd level 3), decoded by k_blosc2_decode / k_blosc2_zstd
    for name, codec, enc in (("lz4", B.LZ4, "repo"), ("blosclz", B.BLOSCLZ, "repo"), ("lz4_lib", B.LZ4, "lib"),
                             ("zstd", B.ZSTD, "lib")):
        chunks = [B.build(r, 4, 1 << 16, codec, (0, 0, 0, 0, 0, B.SHUFFLE), memcpyed=False, enc=enc) for r in raws]
        chunks_by_codec[name] = chunks
        offs, total = [], 0
        for c in chunks:
            offs.append(total)
            total += (len(c) + 255) // 256 * 256
        host = np.zeros(total, dtype=np.uint8)
        for o, c in zip(offs, chunks):
            host[o:o + len(c)] = np.frombuffer(c, dtype=np.uint8)
        d_in = torch.from_numpy(host).cuda()
        ptrs = [d_in.data_ptr() + offs[(lo + i) % distinct] for i in range(n)]
        lens = [len(chunks[(lo + i) % distinct]) for i in range(n)]

        def step(i, k=n):
            cx.ws.decompress_batch_device("blosc2", ptrs[:k], lens[:k], d_out.data_ptr(), raw_len, d_len.data_ptr(),
                                          d_err.data_ptr(), cx.stream.cuda_stream)

        step(0)
        torch.cuda.synchronize()
        assert int(d_err.abs().sum()) == 0 and bool((d_len == raw_len).all())
        assert d_out[:raw_len].cpu().numpy().tobytes() == raws[lo % distinct]
        t = cx.dev_time(step, reps, warm=0)
        t1 = cx.dev_time(lambda i: step(i, 1), 20, warm=2)
        ratio = raw_len * distinct / sum(len(c) for c in chunks)
        out[name] = {"ratio": round(ratio, 3), "value": round(n * raw_len / t / 1e9, 2), "ms_per_launch": round(t * 1e3, 3),
                     "lone_chunk_us": round(t1 * 1e6, 1), "lone_chunk_GBs": round(raw_len / t1 / 1e9, 2)}
    if with_cpu:
        from oracle import py_oracle as oracle
        import ctypes as C
        threads = pool_threads()
        L = oracle.lib()
        chunks = chunks_by_codec["lz4"]
        bufs = [C.create_string_buffer(c, len(c)) for c in chunks]
        outs = [(C.c_uint8 * raw_len)() for _ in range(threads)]

        def one(i):
            got = C.c_uint64(0)
            e = L.oracle_blosc2_decompress(bufs[i % distinct], len(chunks[i % distinct]), outs[i % threads], raw_len,
                                           C.byref(got))
            assert e == 0

        with ThreadPoolExecutor(threads) as ex:   # ctypes releases the GIL during the call
            list(ex.map(one, range(threads)))
            c0 = time.perf_counter()
            list(ex.map(one, range(n_total)))
            tz = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": round(n_total * raw_len / tz / 1e9, 2), "unit": "GB/s", "cores": threads,
                               "kind": "port", "sample": f"this repo's scalar port of the blosc2 decoder "
                                                         f"(oracle_blosc2_decompress, g++ -O2; NOT c-blosc2 / blusc, "
                                                         f"whose SIMD decoders are absent from the image) over all "
                                                         f"{n_total} lz4 chunks on a {threads}-thread pool, {tz:.2f} s"}
        # zstd: the real libzstd (the reference's codec: zstd-sys 1.5.7) on the zstd streams of the chunks,
        # through pyarrow (releases the GIL): a chunk's zstd frames concatenated and decoded by one call
        # (libzstd decodes concatenated frames; raw / run streams skipped), on the same pool, 256 chunks
        import pyarrow as pa
        import struct as S
        zjobs = []
        for c in chunks_by_codec["zstd"]:
            nb, bs = S.unpack_from("<ii", c, 4)
            frames, out_n = [], 0
            for j in range((nb + bs - 1) // bs):
                pos = S.unpack_from("<i", c, 32 + 4 * j)[0]
                for _ in range(4):
                    cs = S.unpack_from("<i", c, pos)[0]
                    pos += 4
                    if 0 < cs < bs // 4:
                        frames.append(c[pos:pos + cs])
                        out_n += bs // 4
                    pos += cs if cs > 0 else (1 if cs < 0 else 0)
            zjobs.append((pa.py_buffer(b"".join(frames)), out_n))
        sample = 256

        def zone(i):
            buf, out_n = zjobs[i % distinct]
            pa.decompress(buf, decompressed_size=out_n, codec="zstd")

        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(zone, range(threads)))
            c0 = time.perf_counter()
            list(ex.map(zone, range(sample)))
            tz = time.perf_counter() - c0
        zbytes = sum(zjobs[i % distinct][1] for i in range(sample))
        # one chunk on one thread (a lone request: the reference decodes it on the request's own thread)
        t1 = time.perf_counter()
        for i in range(20):
            zone(i)
        lone_cpu = (time.perf_counter() - t1) / 20
        # LZ4: the real liblz4 (the system's liblz4.so.1: LZ4_decompress_safe, c-blosc2's LZ4 codec) on the
        # lz4_lib chunks' streams, then the block unshuffle (oracle/cpu_baselines.cpp, -O3 -mavx2), on the same
        # pool over all chunks, and one chunk on one thread
        if L.cpu_lz4lib_available():
            lchunks = chunks_by_codec["lz4_lib"]
            keep = [C.create_string_buffer(c, len(c)) for c in lchunks]
            cp = (C.c_void_p * distinct)(*[C.cast(k, C.c_void_p) for k in keep])
            cl = (C.c_uint64 * distinct)(*[len(c) for c in lchunks])
            sec, nb = C.c_double(), C.c_uint64()
            res = {}
            for mode in (1, 0):
                assert L.cpu_blosc2_lz4lib(cp, cl, C.c_uint64(distinct), C.c_uint64(n_total), C.c_uint32(threads),
                                           C.c_uint64(raw_len), mode, C.byref(sec), C.byref(nb)) == 0
                res[mode] = n_total * raw_len / sec.value / 1e9
            assert L.cpu_blosc2_lz4lib(cp, cl, C.c_uint64(distinct), C.c_uint64(20), C.c_uint32(1),
                                       C.c_uint64(raw_len), 1, C.byref(sec), C.byref(nb)) == 0
            out["cpu_baseline_lz4_lib"] = {
                "value": round(res[1], 2), "unit": "GB/s", "cores": threads, "kind": "library",
                "sample": f"the real liblz4 (liblz4.so.1 LZ4_decompress_safe) on the lz4_lib chunks' streams + the "
                          f"block unshuffle (oracle/cpu_baselines.cpp, -O3 -mavx2), all {n_total} chunks on a "
                          f"{threads}-thread pool; device leg to compare: lz4_lib",
                "lz4_streams_only_GBs": round(res[0], 2),
                "lone_chunk_one_thread_us": round(sec.value / 20 * 1e6, 1)}
        out["cpu_baseline_zstd"] = {"value": round(sample * raw_len / tz / 1e9, 2), "unit": "GB/s", "cores": threads,
                                    "kind": "library", "sample": f"the real libzstd (pyarrow's bundled codec) on "
                                                                 f"the zstd streams of {sample} chunks, each chunk's "
                                                                 f"frames in one call, {threads}-thread pool, "
                                                                 f"{tz:.2f} s; value = the chunks' whole output "
                                                                 f"({sample * raw_len >> 20} MiB, as the device leg "
                                                                 f"counts) / that time: the raw / run streams are not "
                                                                 f"copied, which favours the CPU ({zbytes >> 20} MiB "
                                                                 f"decoded by libzstd)",
                                    "zstd_stream_GBs": round(zbytes / tz / 1e9, 2),
                                    "lone_chunk_one_thread_us": round(lone_cpu * 1e6, 1)}
    return out


def _c3_host():
    import numpy as np
    rng = np.random.default_rng(0x5EED0005)
    v = rng.standard_normal(128 ** 3) * 100
    v[rng.random(v.size) < 0.05] = -9999.0
    return v


def _c3_req(_abi, op, kind="missing_value", vals=(-9999.0,)):
    import numpy as np
    mv = b"".join(np.float64(x).tobytes() for x in vals)
    return _abi.CRequest(op, "float64", shape=[128, 128, 128], selection=C3_SEL, missing_kind=kind, missing_values=mv,
                         n_missing=len(vals))


def leg_configs(cx):
    """Device-resident launches of BASELINE configs[0], [2] and [4] on rotating buffers larger than the
    Infinity Cache (HIP events on the launch stream; results checked once)."""
    import numpy as np
    torch, lib, _abi = cx.torch, cx.lib, cx.abi
    out = {}

    def single(creq, bufs, nbytes, k):
        info = _abi.rdx_response_info()
        assert lib.rdx_plan(creq.ref, nbytes, C.byref(info)) == 0
        body = torch.zeros(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(max(2, info.n_counts), dtype=torch.int64, device="cuda")
        status = torch.zeros(4, dtype=torch.int32, device="cuda")
        args = [(cx.ws.ws, creq.ref, C.c_void_p(b.data_ptr()), nbytes, C.c_void_p(body.data_ptr()),
                 C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), cx.sh, C.byref(info)) for b in bufs]

        def step(i):
            st = lib.rdx_execute_device(*args[i % len(args)])
            if st:
                raise RuntimeError(_abi.status_string(st))

        t = cx.dev_time(step, k, warm=len(bufs))
        assert int(status.abs().sum()) == 0
        return t, body, counts

    # C1: f32 4 MiB contiguous sum (D-real), 64 rotating buffers
    r1 = np.random.default_rng(0x5EED0002)
    v1 = r1.random(1 << 20, dtype=np.float32)
    c1 = [torch.from_numpy(v1).cuda() for _ in range(64)]
    t, body, _ = single(_abi.CRequest("sum", "float32"), c1, 4 << 20, 1000)
    assert abs(float(body[:4].view(torch.float32)[0]) - float(v1.astype(np.float64).sum())) < 1e-2
    out["c1_sum_4mib"] = {"us_per_launch": round(t * 1e6, 2), "bytes_alg": 4 << 20,
                          "roofline_frac": round((4 << 20) / t / 1e9 / PEAK_GBS, 4)}
    # the same 64 chunks as ONE batched launch
    bb = torch.zeros(64, dtype=torch.float32, device="cuda")
    bc = torch.zeros(64, dtype=torch.int64, device="cuda")
    bs = torch.zeros(64, dtype=torch.int32, device="cuda")
    creq1 = _abi.CRequest("sum", "float32")
    t = cx.dev_time(lambda i: cx.ws.execute_batch_device(creq1, [b.data_ptr() for b in c1], 4 << 20, bb.data_ptr(),
                                                         bc.data_ptr(), bs.data_ptr(), cx.stream.cuda_stream), 100)
    out["c1_batch64"] = {"us_per_launch": round(t * 1e6, 2), "us_per_chunk": round(t / 64 * 1e6, 3),
                         "roofline_frac": round(64 * (4 << 20) / t / 1e9 / PEAK_GBS, 4)}
    del c1
    # C3: f64 [128,128,128] hyperslab, missing_value -9999 at 5 %, min / max, and a valid_range max
    v3 = _c3_host()
    c3 = [torch.from_numpy(v3).cuda() for _ in range(20)]
    for name, creq in (("c3_min_missing_value", _c3_req(_abi, "min")), ("c3_max_missing_value", _c3_req(_abi, "max")),
                       ("c3_max_valid_range", _c3_req(_abi, "max", "valid_range", (-250.0, 250.0)))):
        t, body, _ = single(creq, c3, 16 << 20, 1000)
        out[name] = {"us_per_launch": round(t * 1e6, 2), "bytes_alg": C3_NSEL * 8 + 16,
                     "roofline_frac": round((C3_NSEL * 8 + 16) / t / 1e9 / PEAK_GBS, 4)}
    bb = torch.zeros(20, dtype=torch.float64, device="cuda")
    bc = torch.zeros(20, dtype=torch.int64, device="cuda")
    bs = torch.zeros(20, dtype=torch.int32, device="cuda")
    creq3 = _c3_req(_abi, "min")
    t = cx.dev_time(lambda i: cx.ws.execute_batch_device(creq3, [b.data_ptr() for b in c3], 16 << 20, bb.data_ptr(),
                                                         bc.data_ptr(), bs.data_ptr(), cx.stream.cuda_stream), 100)
    out["c3_min_batch20"] = {"us_per_launch": round(t * 1e6, 2), "us_per_chunk": round(t / 20 * 1e6, 3),
                             "roofline_frac": round(20 * (C3_NSEL * 8 + 16) / t / 1e9 / PEAK_GBS, 4)}
    del c3
    # C5: i64 [512,256,256] select -> 128 MiB
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0006)
    c5 = [torch.randint(-2 ** 62, 2 ** 62, (512 * 256 * 256,), dtype=torch.int64, device="cuda", generator=g)
          for _ in range(2)]
    creq5 = _abi.CRequest("select", "int64", shape=[512, 256, 256], selection=C5_SEL)
    t, body, counts = single(creq5, c5, 256 << 20, 40)
    assert torch.equal(body.view(torch.int64).view(512, 128, 256), c5[1].view(512, 256, 256)[:, 64:192, :])
    out["c5_select"] = {"us_per_launch": round(t * 1e6, 2), "bytes_alg": 2 * (128 << 20),
                        "roofline_frac": round(2 * (128 << 20) / t / 1e9 / PEAK_GBS, 4),
                        "note": "128 MiB read + 128 MiB written"}
    return out


def leg_mixed(cx, n_pairs=10, sets=2, k=30, serial=True):
    """20 mixed requests — 10 x C1 (f32 4 MiB contiguous sum) and 10 x C3 (f64 [128,128,128] hyperslab
    min / max, missing_value) — as ONE heterogeneous launch (rdx_execute_multi_device), rotating over
    `sets` distinct sets of chunks (> the Infinity Cache).  Device time: the k calls are queued behind a
    device-side gate (fewer than the engine's 32 table slots, so none waits for the host) and timed from
    the gate's opening to the last kernel's end; the host's own cost per call (planning 20 requests, the
    table) is reported beside it.  Also the same 20 requests as 20 single-request launches on one stream."""
    import numpy as np
    torch, _abi, lib = cx.torch, cx.abi, cx.lib
    v3 = _c3_host()
    v1 = np.random.default_rng(0x5EED0002).random(1 << 20, dtype=np.float32)
    n = 2 * n_pairs
    sets_c = []
    for _ in range(sets):
        arr = (_abi.rdx_multi_item * n)()
        keep = []
        for i in range(n_pairs):
            for j, (creq, data, nbytes) in enumerate(((_abi.CRequest("sum", "float32"), v1, 4 << 20),
                                                      (_c3_req(_abi, "min" if i % 2 == 0 else "max"), v3, 16 << 20))):
                d = torch.from_numpy(data).cuda()
                body = torch.zeros(2, dtype=torch.float64, device="cuda")
                counts = torch.zeros(2, dtype=torch.int64, device="cuda")
                status = torch.full((1,), 77, dtype=torch.int32, device="cuda")
                keep.append((creq, d, body, counts, status))
                arr[2 * i + j] = _abi.rdx_multi_item(C.pointer(creq.c), d.data_ptr(), nbytes, body.data_ptr(),
                                                     counts.data_ptr(), status.data_ptr())
        sets_c.append((arr, (C.c_uint32 * n)(), (_abi.rdx_response_info * n)(), keep))
    alg = n_pairs * ((4 << 20) + C3_NSEL * 8 + 32)

    def multi_step(i):
        arr, st, infos, _ = sets_c[i % sets]
        r = lib.rdx_execute_multi_device(cx.ws.ws, n, arr, cx.sh, st, infos)
        if r or any(st):
            raise RuntimeError(f"rdx_execute_multi_device: {r} {list(st)}")

    def gated(step, calls, hold_s):
        for i in range(2 * sets):
            step(i)
        torch.cuda.synchronize()
        opened = cx.gate([cx.stream], hold_s=hold_s)
        h0 = time.perf_counter()
        for i in range(calls):
            step(i)
        host = (time.perf_counter() - h0) / calls
        end = torch.cuda.Event(enable_timing=True)
        end.record(cx.stream)
        torch.cuda.synchronize()
        return opened.elapsed_time(end) / 1e3 / calls, host

    t, host = gated(multi_step, k, 0.01 + k * 300e-6)
    for _, _, _, keep in sets_c:
        assert all(int(kk[4][0]) == 0 for kk in keep)
        assert all(int(kk[3][0]) == (1 << 20) for kk in keep[0::2])
        assert all(int(kk[3][0]) > 0 for kk in keep[1::2])
    res = {"workload": f"{n} mixed requests per launch: {n_pairs} x C1 (f32 4 MiB sum) + {n_pairs} x C3 "
                       "(f64 hyperslab min/max, missing_value), each its own request; rdx_execute_multi_device",
           "us_per_launch": round(t * 1e6, 2), "us_per_request": round(t / n * 1e6, 3),
           "bytes_alg_per_launch": alg, "roofline_frac": round(alg / t / 1e9 / PEAK_GBS, 4),
           "host_us_per_call": round(host * 1e6, 1),
           "timing": f"{k} calls queued behind a device-side gate; HIP events gate open -> last kernel end / {k} "
                     "(the request descriptors travel in the kernel arguments)"}
    if not serial:
        return res
    flat = [kk for _, _, _, keep in sets_c for kk in keep]
    sargs = [(cx.ws.ws, kk[0].ref, C.c_void_p(kk[1].data_ptr()), kk[1].numel() * kk[1].element_size(),
              C.c_void_p(kk[2].data_ptr()), C.c_void_p(kk[3].data_ptr()), C.c_void_p(kk[4].data_ptr()), cx.sh,
              C.byref(_abi.rdx_response_info())) for kk in flat]

    def serial_step(i):
        r = lib.rdx_execute_device(*sargs[i % len(sargs)])
        if r:
            raise RuntimeError(f"rdx_execute_device: {r}")

    ts, _ = gated(serial_step, 4 * n, 0.01 + 4 * n * 50e-6)
    ts *= n
    res.update({"serial_single_launches_us": round(ts * 1e6, 2),
                "serial_roofline_frac": round(alg / ts / 1e9 / PEAK_GBS, 4)})
    return res


def conc_bench(cfg, threads, reqs, path="device", devices="0"):
    """One run of reductionist-rs_amd/rdx_conc_bench (native C++ threads over the C ABI, no Python on the
    path): its JSON line."""
    exe = ROOT / "reductionist-rs_amd" / "rdx_conc_bench"
    r = subprocess.run([str(exe), cfg, str(threads), str(reqs), path, devices], capture_output=True, text=True,
                       timeout=180)
    if r.returncode != 0:
        raise RuntimeError(f"rdx_conc_bench {cfg} {threads} {path} {devices}: {r.stderr[-500:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def leg_native_concurrent(cx):
    """Concurrent single-chunk requests from native C++ threads, the way Tokio/Rayon workers run them
    (app.rs:147-152): 1 thread and the worker-pool size (num_cpus - 1, capped at the box's CPU share).
      device:   each thread its own workspace + stream, rdx_execute_device + synchronize per request
                (independent launches);
      resident: rdx_execute_resident on the context's pool (c2: one 64 MiB chunk per request, the result seen
                in a page-locked host slot instead of a stream synchronize) — concurrent small all-axes requests are
                coalesced by the pool's dispatcher into shared launches (same-plan groups / k_multi), each
                caller's result written to page-locked host memory by the fold; an idle entry runs the
                request on the caller's own thread (the direct fast path, direct_requests);
      owned:    rdx_execute_owned of a page-locked host chunk (the plugin's own call): s1 1 MiB f32 sum,
                h4f32 / h4f64 one 4 MiB shuffled big-endian f32 / f64 sum (the north_star's host-inclusive
                4 MiB rows; pinned_copy_us_one is a plain pinned H2D copy of the same bytes, same run).
                Page-locked chunks up to 4 MiB are read by the kernel itself over PCIe (host_read_requests);
                every row carries the process's CPU per request and its split by thread."""
    exe = ROOT / "reductionist-rs_amd" / "rdx_conc_bench"
    if not exe.exists():
        return {"skipped": f"{exe} not built"}
    out = []
    pool = pool_threads()
    for cfg, threads, reqs, path in (("c3", 1, 2000, "device"), ("c3", pool, 2000, "device"),
                                     ("c3", 1, 2000, "resident"), ("c3", pool, 2000, "resident"),
                                     ("c1", 1, 2000, "device"), ("c1", pool, 2000, "device"),
                                     ("c1", 1, 2000, "resident"), ("c1", pool, 2000, "resident"),
                                     ("c1", 4 * pool, 1000, "resident"),
                                     ("s1", 1, 2000, "owned"), ("s1", pool, 2000, "owned"),
                                     ("h4f32", 1, 1000, "owned"), ("h4f64", 1, 1000, "owned"),
                                     ("c2", 1, 300, "device"), ("c2", 4, 300, "device"),
                                     ("c2", 1, 300, "resident"), ("c2", 4, 300, "resident")):
        out.append(conc_bench(cfg, threads, reqs, path))
    return out


def leg_pool(cx):
    """The server's real shape (app_state.rs:21-37: ONE process, every request on a worker thread): one
    rdx_context pooling all --gpus devices, T native threads issuing C4 requests (4 MiB shuffled f32 chunks,
    sum) — from page-locked host memory through rdx_execute (PCIe H2D per request), and HBM-resident
    through rdx_execute_resident — placed by least outstanding bytes.  Run by rank 0 alone while the other
    ranks wait at a barrier (their GPUs idle)."""
    exe = ROOT / "reductionist-rs_amd" / "rdx_conc_bench"
    res = None
    if cx.rank == 0 and exe.exists():
        n = cx.torch.cuda.device_count()
        devs = ",".join(str(d) for d in range(min(n, cx.world)))
        pool = pool_threads()
        res = {"devices": devs,
               "host": conc_bench("c4", max(pool, 2 * cx.world), 300, "host", devs),
               "resident": conc_bench("c4", max(pool, 4 * cx.world), 1000, "resident", devs)}
    cx.barrier()
    return res


def leg_cbor(cx, with_cpu):
    """Response serialisation of a large count vector where it was computed (rdx_cbor_encode_device):
    axis = [] count over the C5 chunk shape (i64 [512,256,256], missing_value) gives a 256 MiB i64 body and
    32 Mi counts; the CBOR body (serde_cbor CBORResponse, app.rs:33-40) is packed on the device.  Device
    time per call (HIP events, K back-to-back calls): the whole call (body copy + count array) and the
    count-array kernel alone (a body-less layout); against the engine's host encoder on one core."""
    import numpy as np
    torch, lib, _abi = cx.torch, cx.lib, cx.abi
    n = 512 * 256 * 256
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED00CB)
    d = torch.randint(0, 4, (n,), dtype=torch.int64, device="cuda", generator=g)
    creq = _abi.CRequest("count", "int64", shape=[512, 256, 256], axis=[], missing_kind="missing_value",
                         missing_values=np.int64(1).tobytes(), n_missing=1)
    pinfo = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, n * 8, C.byref(pinfo)) == 0
    body = torch.empty(pinfo.body_bytes, dtype=torch.uint8, device="cuda")
    counts = torch.empty(pinfo.n_counts, dtype=torch.int64, device="cuda")
    info = cx.ws.execute_device(creq, d.data_ptr(), n * 8, body.data_ptr(), counts.data_ptr(), None,
                                cx.stream.cuda_stream)
    bare = _abi.rdx_response_info.from_buffer_copy(info)
    bare.body_bytes = 0
    out = {}
    for name, inf, flags in (("count_array", info, 0), ("count_array_kernel_only", bare, 0),
                             ("count_as_bytes", info, _abi.CBOR_COUNT_AS_BYTES)):
        bound = lib.rdx_cbor_bound(C.byref(inf), flags)
        dst = torch.empty(bound, dtype=torch.uint8, device="cuda")
        dlen = torch.zeros(1, dtype=torch.int64, device="cuda")
        args = (cx.ws.ws, C.byref(inf), C.c_void_p(body.data_ptr()), C.c_void_p(counts.data_ptr()), flags,
                C.c_void_p(dst.data_ptr()), bound, C.c_void_p(dlen.data_ptr()), None, cx.sh)

        def step(i, args=args):
            st = lib.rdx_cbor_encode_device(*args)
            if st:
                raise RuntimeError(_abi.status_string(st))

        t = cx.dev_time(step, 20)
        enc = int(dlen[0])
        clen = enc - (lib.rdx_cbor_bound(C.byref(inf), flags) - (9 * n if flags == 0 else 0))
        moved = 2 * inf.body_bytes + 8 * n + (clen if flags == 0 else 8 * n)
        out[name] = {"us_per_call": round(t * 1e6, 2), "encoded_bytes": enc, "bytes_moved": moved,
                     "roofline_frac": round(moved / t / 1e9 / PEAK_GBS, 4)}
        del dst
    out["raw_response_bytes"] = int(info.body_bytes + 8 * n)
    out["note"] = ("bytes_moved = body read + write (device copy) + counts read + encoded count bytes written; "
                   "the packed body is what crosses PCIe instead of body + 8 B per count")
    if with_cpu:
        hb = np.empty(info.body_bytes, dtype=np.uint8)
        hc = counts.cpu().numpy()
        hb[:] = body.cpu().numpy()
        cap = lib.rdx_cbor_bound(C.byref(info), 0)
        buf = np.empty(cap, dtype=np.uint8)
        ln = C.c_uint64()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            st = lib.rdx_cbor_encode(C.byref(info), hb.ctypes.data, hc.ctypes.data, 0, buf.ctypes.data, cap,
                                     C.byref(ln))
            assert st == 0
        th = (time.perf_counter() - t0) / reps
        assert ln.value == out["count_array"]["encoded_bytes"]
        out["cpu_host_encoder"] = {"ms_per_call": round(th * 1e3, 2), "cores": 1,
                                   "note": "rdx_cbor_encode (C++, -O2) on host buffers, same response"}
    return out


def leg_host(cx):
    """Host-inclusive rates (chunk in host memory -> H2D -> kernels -> D2H through rdx_execute), pageable and
    page-locked (rdx_host_alloc) buffers, next to the raw PCIe copy of the same bytes (torch, pinned)."""
    import numpy as np
    torch, lib, _abi = cx.torch, cx.lib, cx.abi
    out = {}

    def pcie(nbytes_h2d, nbytes_d2h, reps=0):
        reps = reps or int(max(5, min(200, (256 << 20) // max(1, nbytes_h2d))))
        h = torch.empty(max(nbytes_h2d, 16), dtype=torch.uint8).pin_memory()
        d = torch.empty(max(nbytes_h2d, 16), dtype=torch.uint8, device="cuda")
        hd = torch.empty(max(nbytes_d2h, 16), dtype=torch.uint8).pin_memory()
        d.copy_(h, non_blocking=True)
        hd.copy_(d[:max(nbytes_d2h, 16)], non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
        th = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            hd.copy_(d[:max(nbytes_d2h, 16)], non_blocking=True)
            torch.cuda.synchronize()
        td = (time.perf_counter() - t0) / reps if nbytes_d2h > 64 else 0.0
        return th, td

    def host_buf(nbytes, pinned):
        if pinned:
            p = C.c_void_p()
            assert lib.rdx_host_alloc(cx.eng.ctx, nbytes, C.byref(p)) == 0
            return p, np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p.value))
        arr = np.empty(nbytes, dtype=np.uint8)
        return C.c_void_p(arr.ctypes.data), arr

    def run(name, creq, data, reps):
        info = _abi.rdx_response_info()
        assert lib.rdx_plan(creq.ref, data.nbytes, C.byref(info)) == 0
        th, td = pcie(data.nbytes, info.body_bytes)
        res = {"h2d_bytes": int(data.nbytes), "d2h_bytes": int(info.body_bytes),
               "pcie_pinned_copy_ms": round((th + td) * 1e3, 3), "pcie_h2d_GBs": round(data.nbytes / th / 1e9, 1)}
        for pinned in (False, True):
            src, arr = host_buf(data.nbytes, pinned)
            arr[:] = data.view(np.uint8).reshape(-1)
            body_p, body_arr = host_buf(max(16, info.body_bytes), pinned)   # (keep the array alive)
            counts = (C.c_int64 * max(1, info.n_counts))()
            o = _abi.rdx_response_info()
            for _ in range(2):
                st = lib.rdx_execute(cx.eng.ctx, creq.ref, src, data.nbytes, body_p, info.body_bytes, counts,
                                     info.n_counts, C.byref(o))
                assert st == 0, (name, "pinned" if pinned else "pageable", _abi.status_string(st))
            t0 = time.perf_counter()
            for _ in range(reps):
                lib.rdx_execute(cx.eng.ctx, creq.ref, src, data.nbytes, body_p, info.body_bytes, counts,
                                info.n_counts, C.byref(o))
            t = (time.perf_counter() - t0) / reps
            key = "pinned" if pinned else "pageable"
            res[f"{key}_ms"] = round(t * 1e3, 3)
            res[f"{key}_GiBs_chunk"] = round(data.nbytes / t / GIB, 2)
            res[f"{key}_over_pcie"] = round(t / (th + td), 3)
            if pinned:
                lib.rdx_host_free(cx.eng.ctx, src)
                lib.rdx_host_free(cx.eng.ctx, body_p)
        out[name] = res

    vals = np.random.default_rng(4).random(C2_ELEMS, dtype=np.float32)
    c2 = np.ascontiguousarray(vals.astype(">f4").view(np.uint8).reshape(-1, 4).T).reshape(-1)
    run("c2_sum_64mib", cx.abi.CRequest("sum", "float32", byte_order="big",
                                        filters=[{"id": "shuffle", "element_size": 4}]), c2, 20)
    run("c3_min_16mib", _c3_req(_abi, "min"), _c3_host(), 40)
    # the north_star's 4 MiB rows: one shuffled big-endian f32 / f64 chunk (page-locked chunks of this size
    # are read by the kernel over PCIe: no separate copy)
    for es, dt, name in ((4, "float32", "f32_sum_4mib_shuffled_be"), (8, "float64", "f64_sum_4mib_shuffled_be")):
        v = np.random.default_rng(40 + es).random((4 << 20) // es).astype(">f4" if es == 4 else ">f8")
        h4 = np.ascontiguousarray(v.view(np.uint8).reshape(-1, es).T).reshape(-1)
        run(name, cx.abi.CRequest("sum", dt, byte_order="big", filters=[{"id": "shuffle", "element_size": es}]), h4, 300)
    c5 = np.random.default_rng(6).integers(-2 ** 62, 2 ** 62, 512 * 256 * 256, dtype=np.int64)
    run("c5_select_256mib", _abi.CRequest("select", "int64", shape=[512, 256, 256], selection=C5_SEL), c5, 6)
    return out


def leg_cpu(cx, seconds):
    """The oracle (CPU restatement of the reference's sequential path, g++ -O2) on the GPU box's host:
    headline C2 on one core, C1 with / without the clone, C3, C5, each a bounded sample."""
    import numpy as np
    from oracle import py_oracle as oracle
    _abi = cx.abi
    res = {}

    def reps_for(creq, data, budget, clone=True):
        t1 = oracle.bench(creq, data, 1, clone)
        return max(1, int(budget / max(t1, 1e-6)))

    # headline C2: one 64 MiB shuffled big-endian chunk, sum
    vals = np.random.default_rng(0x5EED0004).random(C2_ELEMS, dtype=np.float32)
    data = vals.astype(">f4").view(np.uint8).reshape(C2_ELEMS, 4).T.copy().tobytes()
    creq = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
    n = reps_for(creq, data, seconds)
    t = oracle.bench(creq, data, n, True)
    headline = {"value": round(C2_BYTES / t / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": f"{n} x one 64 MiB chunk (16 Mi f32, big-endian, shuffle es=4), sum, sequential "
                          f"oracle/rdx_oracle.cpp g++ -O2 on 1 host core, {n * t:.1f} s"}
    # C1 (BASELINE configs[0], the reference's own CPU bench case): with and without the clone
    v1 = np.random.default_rng(0x5EED0002).random(1 << 20, dtype=np.float32).tobytes()
    creq1 = _abi.CRequest("sum", "float32")
    for clone in (True, False):
        n = reps_for(creq1, v1, 3.0, clone)
        t = oracle.bench(creq1, v1, n, clone)
        res["c1_sum_4mib_" + ("clone" if clone else "noclone")] = {
            "us_per_request": round(t * 1e6, 1), "GiBs": round((4 << 20) / t / GIB, 3), "reps": n,
            "note": "data.clone() inside the timed loop as benches/operations.rs:63" if clone else
                    "one buffer, no per-iteration copy"}
    v3 = _c3_host().tobytes()
    for name, creq3 in (("c3_min_missing_value", _c3_req(_abi, "min")), ("c3_max_missing_value", _c3_req(_abi, "max"))):
        n = reps_for(creq3, v3, 2.0)
        t = oracle.bench(creq3, v3, n, True)
        res[name] = {"us_per_request": round(t * 1e6, 1), "reps": n,
                     "GBs_alg": round((C3_NSEL * 8) / t / 1e9, 3)}
    v5 = np.random.default_rng(6).integers(-2 ** 62, 2 ** 62, 512 * 256 * 256, dtype=np.int64).tobytes()
    creq5 = _abi.CRequest("select", "int64", shape=[512, 256, 256], selection=C5_SEL)
    n = reps_for(creq5, v5, 3.0)
    t = oracle.bench(creq5, v5, n, True)
    res["c5_select"] = {"ms_per_request": round(t * 1e3, 2), "reps": n,
                        "GBs_alg": round(2 * (128 << 20) / t / 1e9, 3)}
    res["host"] = cpu_info()
    return headline, res


def cpu_baseline_c4(threads, distinct=256):
    """C4 on the host the way the reference serves it: independent requests on a worker pool
    (thread_limit = num_cpus - 1, src/app_state.rs:22; capped at the CPUs this job may use).  1024 chunks
    of 4 MiB (256 distinct = 1 GiB, cycled: four times the host's 256 MB L3, so the chunks stream from
    DRAM as a server's downloaded chunks would), unshuffle + f32 sum each, by the oracle; ctypes releases
    the GIL."""
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
            "kind": "port", "sample": f"all {C4_CHUNKS} chunks ({distinct} distinct = {distinct * 4} MiB, cycled), "
                                      f"{threads} worker threads, oracle g++ -O2, {el:.2f} s"}


def devices_used(cx):
    """(host, PCI bus / uuid) of this rank's device, gathered over ranks."""
    torch = cx.torch
    p = torch.cuda.get_device_properties(cx.device)
    ident = None
    for attr in ("uuid", "pci_bus_id"):
        v = getattr(p, attr, None)
        if v is not None:
            ident = f"{attr}={v}"
            break
    mine = f"{socket.gethostname()}:{ident or f'device{cx.device}'}"
    if cx.world == 1:
        return [mine]
    allv = [None] * cx.world
    cx.dist.all_gather_object(allv, mine)
    return allv


LINE_MAX_BYTES = 8192      # the driver did not parse round 5's 21.5 KB line


def _dig(d, *path):
    for p in path:
        if isinstance(d, dict):
            d = d.get(p)
        elif isinstance(d, list) and isinstance(p, int) and -len(d) <= p < len(d):
            d = d[p]
        else:
            return None
    return d


def compact_extra(extra):
    """One scalar per leg (µs or GiB/s, plus the roofline fraction where the leg has one) out of the full
    record's `extra`; missing legs are left out.  The full record goes to a file (main())."""
    out = {}

    def put(key, *path, nd=4):
        v = _dig(extra, *path)
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            out[key] = round(float(v), nd)

    put("c2_single_chunk_us", "c2_single_chunk", "kernel_us_avg", nd=3)
    put("c2_single_chunk_frac", "c2_single_chunk", "roofline_frac")
    put("c2_concurrent_us_per_request", "c2_concurrent_requests", "us_per_request", nd=3)
    put("c2_concurrent_frac", "c2_concurrent_requests", "roofline_frac")
    put("headline_step_median_us", "headline_per_step", "median_us", nd=2)
    put("c4_batch_GiBs", "c4_batch", "value", nd=2)
    put("c4_batch_frac", "c4_batch", "roofline_frac")
    put("c4_cpu_GiBs", "c4_batch", "cpu_baseline", "value", nd=3)
    put("c4_cpu_cores", "c4_batch", "cpu_baseline", "cores", nd=0)
    put("f64_64mib_us", "f64_64mib", "kernel_us_avg", nd=3)
    put("f64_64mib_frac", "f64_64mib", "roofline_frac")
    put("f64_4mib_us", "f64_4mib", "kernel_us_avg", nd=3)
    put("f64_4mib_frac", "f64_4mib", "roofline_frac")
    put("c4z_inflate_GBs", "c4z_inflate", "value", nd=2)
    put("c4z_inflate_cpu_GBs", "c4z_inflate", "cpu_baseline", "value", nd=2)
    put("inflate_lone_ms", "c4z_inflate", "lone", "device_ms", nd=3)
    put("inflate_lone_cpu_ms", "c4z_inflate", "lone", "cpu_baseline", "value", nd=3)
    for codec in ("lz4", "blosclz", "lz4_lib", "zstd"):
        put(f"blosc2_{codec}_GBs", "c4b_blosc2", codec, "value", nd=2)
    put("blosc2_lz4_lib_cpu_GBs", "c4b_blosc2", "cpu_baseline_lz4_lib", "value", nd=2)
    put("blosc2_zstd_cpu_GBs", "c4b_blosc2", "cpu_baseline_zstd", "value", nd=2)
    for k in ("c1_sum_4mib", "c3_min_missing_value", "c3_max_missing_value", "c3_max_valid_range", "c5_select",
              "c1_batch64", "c3_min_batch20"):
        put(f"{k}_us", "configs", k, "us_per_launch", nd=2)
        put(f"{k}_frac", "configs", k, "roofline_frac")
    put("mixed20_us", "mixed_requests", "us_per_launch", nd=2)
    put("mixed20_frac", "mixed_requests", "roofline_frac")
    native = extra.get("concurrent_native")
    for i, r in enumerate(native if isinstance(native, list) else []):
        if not isinstance(r, dict) or "config" not in r:
            continue
        tag = {"rdx_execute_device + synchronize": "device", "rdx_execute_resident (coalesced)": "resident"}.get(
            r.get("path"), "owned")
        key = f"native_{r['config']}_{tag}_t{r.get('threads')}"
        put(key + "_us", "concurrent_native", i, "us_per_request_aggregate", nd=3)
        put(key + "_frac", "concurrent_native", i, "roofline_frac")
    put("cbor_count_array_us", "cbor_response", "count_array", "us_per_call", nd=2)
    put("cbor_kernel_only_frac", "cbor_response", "count_array_kernel_only", "roofline_frac")
    for k in ("c2_sum_64mib", "c3_min_16mib", "f32_sum_4mib_shuffled_be", "f64_sum_4mib_shuffled_be",
              "c5_select_256mib"):
        put(f"host_{k}_pinned_ms", "host_inclusive", k, "pinned_ms", nd=3)
        put(f"host_{k}_pcie_copy_ms", "host_inclusive", k, "pcie_pinned_copy_ms", nd=3)
    put("pool_host_GiBs", "pool", "host", "GiBs_chunk", nd=2)
    put("pool_resident_frac", "pool", "resident", "roofline_frac")
    put("cpu_c1_clone_us", "cpu_baselines", "c1_sum_4mib_clone", "us_per_request", nd=1)
    put("cpu_c3_min_us", "cpu_baselines", "c3_min_missing_value", "us_per_request", nd=1)
    put("cpu_c5_select_ms", "cpu_baselines", "c5_select", "ms_per_request", nd=2)
    return out


def compact_line(line, full_path=None):
    """The one stdout line the driver parses: the contract's keys, `roofline`, `cpu_baseline` and a flat
    `extra` of scalars; the full record is named by `full_record`.  Asserted at most LINE_MAX_BYTES
    (tests/test_bench_line_cpu.py)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "oversubscribed")
    out = {k: line[k] for k in keep if k in line}
    cfg = dict(out.get("config") or {})
    if isinstance(cfg.get("devices"), list) and len(cfg["devices"]) > 8:
        cfg["devices"] = cfg["devices"][:8] + ["…"]
    out["config"] = cfg
    if isinstance(out.get("cpu_baseline"), dict):
        cb = dict(out["cpu_baseline"])
        if isinstance(cb.get("sample"), str) and len(cb["sample"]) > 240:
            cb["sample"] = cb["sample"][:237] + "..."
        out["cpu_baseline"] = cb
    out["extra"] = compact_extra(line.get("extra") or {})
    if full_path:
        out["full_record"] = str(full_path)
    s = json.dumps(out, separators=(",", ":"))
    if len(s.encode()) > LINE_MAX_BYTES:     # never hand the driver an unparseable line: drop extra first
        out["extra"] = {"dropped": "line over %d B" % LINE_MAX_BYTES}
        s = json.dumps(out, separators=(",", ":"))
    return s


def main():
    args = parse()
    if args.gpus > 1 and "LOCAL_RANK" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    oversub = os.environ.get("RDX_BENCH_OVERSUBSCRIBE") == "1"
    n_dev = torch.cuda.device_count()
    if local_rank >= n_dev and not oversub:
        raise SystemExit(f"bench.py: rank {rank} (local {local_rank}) has no GPU of its own ({n_dev} visible)")
    if world > 1:
        # gloo reports its connections on stdout; keep stdout for the one JSON line (rank 0)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    device = local_rank % n_dev
    torch.cuda.set_device(device)
    cx = Ctx(torch, dist, args, world, rank, device)
    devs = devices_used(cx)
    n_gpus = len(set(devs))
    if n_gpus != world and not oversub:
        raise SystemExit(f"bench.py: {world} ranks share {n_gpus} device(s): {devs}")

    c2 = leg_c2(cx)
    extra = c2["extra"]
    if args.primary_only:
        args.no_c4 = args.no_cpu_baseline = args.no_inflate = args.no_f64 = args.no_configs = args.no_host = True
    solo = rank == 0 and world == 1
    if not args.no_c4:
        extra["c4_batch"] = leg_c4(cx)
        if solo and not args.no_cpu_baseline:
            extra["c4_batch"]["cpu_baseline"] = cpu_baseline_c4(pool_threads())
            # the same with 64 distinct chunks (256 MiB: a chunk the downloader has just written is often
            # still in the host's L3); the headline ratios in DESIGN.md use the DRAM-bound value above
            extra["c4_batch"]["cpu_baseline_cache_resident"] = cpu_baseline_c4(pool_threads(), distinct=64)
    if not args.no_f64:
        steps = max(10, args.steps // 4)
        extra["f64_64mib"] = leg_f64(cx, 8 * 1024 * 1024, N_BUF, steps)
        extra["f64_4mib"] = leg_f64(cx, 512 * 1024, 128, steps)
    if not args.no_inflate:
        extra["c4z_inflate"] = leg_inflate(cx, solo and not args.no_cpu_baseline)
    if not args.no_inflate:
        extra["c4b_blosc2"] = leg_blosc2(cx, solo and not args.no_cpu_baseline)
    if world == 1 and not args.no_configs:
        extra["configs"] = leg_configs(cx)
        extra["mixed_requests"] = leg_mixed(cx)
        extra["concurrent_native"] = leg_native_concurrent(cx)
        extra["cbor_response"] = leg_cbor(cx, solo and not args.no_cpu_baseline)
    if world == 1 and not args.no_host:
        extra["host_inclusive"] = leg_host(cx)
    if not args.no_configs:
        extra["pool"] = leg_pool(cx)
    cpu_line = None
    if solo and not args.no_cpu_baseline:
        cpu_line, extra["cpu_baselines"] = leg_cpu(cx, args.cpu_seconds)

    achieved = c2["step_bytes"] / c2["kern_avg_s"] / 1e9
    line = {
        "metric": "GiB/s device-resident chunk unshuffle+reduce (f32 sum), 1/2/4/8 MI355X",
        "value": round(c2["value"], 2), "unit": "GiB/s", "n_gpus": n_gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(c2["elapsed"] / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic U[0,1) f32, big-endian, byte-shuffled (es=4)",
        "config": {"workload": "c2: f32 sum over 64 MiB chunks (16 Mi elements each), byte shuffle es=4 + "
                               "non-native (big) byte order; one step = one launch over 8 independent "
                               "HBM-resident chunks (512 MiB) per GPU, one result per chunk",
                   "chunk_bytes": C2_BYTES, "chunks_per_step": N_BUF, "elements_per_chunk": C2_ELEMS,
                   "parallelism": f"independent chunks x{n_gpus} GPUs", "ranks": world, "devices": devs},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_GBS, 4), "traffic": traffic_from_profiles("c2"),
                     "kernel": "k_all_contig<float, OP_SUM, FUSED=1, MK=0>",
                     "kernel_us_avg": round(c2["kern_avg_s"] * 1e6, 3), "bytes_alg_per_launch": c2["step_bytes"],
                     "timing": "HIP events on the launch stream around the K back-to-back launches / K"},
        "extra": extra,
    }
    if oversub and n_gpus != world:
        line["oversubscribed"] = True
    if cpu_line:
        line["cpu_baseline"] = cpu_line
    if rank == 0:
        # the full record: a file (gpurun_out/ travels back from a GPU box) and stderr, BEFORE the compact
        # stdout line, so the last line of either stream or of both merged is the parseable one
        full = json.dumps(line)
        full_path = Path(args.full_out) if args.full_out else None
        if full_path is not None:
            try:
                if not full_path.is_absolute():
                    full_path = ROOT / full_path
                full_path.parent.mkdir(parents=True, exist_ok=True)
                full_path.write_text(full + "\n")
            except OSError as e:
                print(f"bench.py: could not write {full_path}: {e}", file=sys.stderr)
                full_path = None
        print(full, file=sys.stderr, flush=True)
        print(compact_line(line, full_path.relative_to(ROOT) if full_path and full_path.is_relative_to(ROOT)
                           else full_path), flush=True)
    cx.ws.close()
    cx.eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
