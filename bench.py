#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on MI355X through the drop-in MPI API.

  N = 1 : configs[1] — MPI_Reduce_local SUM fp32 on 256 MiB device buffers
          (the op kernel against the HBM roofline); value = 3*S / t in GB/s.
  N > 1 : configs[2] — osu_allreduce -d rocm fp32 SUM 256 MiB, one rank per GPU;
          value = busbw = 2(n-1)/n * S / t (max over ranks), plus the 8-byte latency.

Launch: python bench.py [--gpus 1] [--steps K] [--warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
A step is one MPI call on resident device buffers (OSU loop: barrier, t0,
call, t1).  Kernel time comes from HIP events recorded on the library's own
stream around the kernel launch (mv2h_timing_enable / mv2h_last_kernel_ms),
in a second loop so the events never sit inside the timed value loop.
The CPU baseline (rank 0, N = 1 only) times the oracle's restatement of the
reference op loop on a bounded host sample.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

METRIC = "osu_allreduce busbw GB/s fp32 SUM 256MB at 1/2/4/8 MI355X; 8B latency us"
HBM_PEAK = 8000.0        # GB/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK = 153.0        # GB/s per link per direction (task statement)
S_BYTES = 256 * 1024 * 1024
# completion-word events (mv2h_get_info; runtime/coll.cpp wait_done), copied into both lines
WORD_KEYS = ("done_queried", "done_late", "done_missed", "done_xcd_split")
WORLD = 0x44000000        # MPI_COMM_WORLD (MPICH ABI)


def cpu_info():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline_reduce_local(seconds=10.0):
    """Oracle restatement of the reference host op loop (opsum.c via
    MPIR_OP_TYPE_REDUCE_CASE), single core, on the full 256 MiB fp32 operands
    (larger than the host L3) repeated for ~`seconds`.  Rate in the metric's
    unit: 3*S algorithmic bytes / t."""
    from oracle import oracle
    n = 64 * 1024 * 1024
    a = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    b = np.random.default_rng(2).standard_normal(n).astype(np.float32)
    L = oracle.lib()
    t1 = L.oracle_time_reduce_local(a.ctypes.data, b.ctypes.data, n, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], 1)
    reps = max(1, int(seconds / max(t1, 1e-6)))
    t = L.oracle_time_reduce_local(a.ctypes.data, b.ctypes.data, n, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], reps)
    gbs = 3.0 * n * 4 * reps / t / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"oracle reduce_local fp32 SUM, 256 MiB host operands x {reps} reps ({t:.1f} s), "
                      f"1 core of '{cpu_info()}'; reference device path adds D2H 2S + H2D S over PCIe"}


def host_allreduce_record(out):
    """Parse oracle/host_allreduce's output into bench's record: the JSONHDR placement row (the
    inherited cpuset, each rank's CPU, distinct CPUs / physical cores, oversubscription, cgroup
    quota) and the per-size JSON rows (latency, busbw, sched_yield fallbacks, CFS throttling)."""
    hdr = next((json.loads(l[8:]) for l in out.splitlines() if l.startswith("JSONHDR ")), None)
    stream = next((json.loads(l[11:]) for l in out.splitlines() if l.startswith("JSONSTREAM ")), None)
    rows = [json.loads(l[5:]) for l in out.splitlines() if l.startswith("JSON ")]
    by = {r["bytes"]: r for r in rows}
    if hdr is None or 8 not in by or (64 << 20) not in by or (1 << 20) not in by:
        return {"error": "incomplete host_allreduce output"}
    ranks = hdr["ranks"]
    if hdr["oversubscribed"]:
        placement = f"{ranks} ranks on {hdr['cpus_used']} CPUs: OVERSUBSCRIBED (cpuset holds {hdr['cpus_available']})"
    elif hdr["smt_shared"]:
        placement = f"{ranks} ranks pinned 1/CPU on {hdr['cores_used']} physical cores (SMT siblings shared)"
    else:
        placement = f"{ranks} ranks pinned 1/core"
    if hdr.get("l3_domains_used") is not None:
        placement += f" on {hdr['l3_domains_used']} L3 domain{'s' if hdr['l3_domains_used'] != 1 else ''}"
    return {"latency_8B_us": by[8]["lat_us"], "busbw_64MiB_GBps": by[64 << 20]["busbw_GBps"],
            "busbw_1MiB_GBps": by[1 << 20]["busbw_GBps"], "all_ok": all(r["ok"] for r in rows),
            "cores": hdr["cpus_used"], "cpus_available": hdr["cpus_available"], "cpus_used": hdr["cpus_used"],
            "cores_used": hdr["cores_used"], "oversubscribed": hdr["oversubscribed"], "smt_shared": hdr["smt_shared"],
            "rank_cpus": hdr["rank_cpus"], "rank_cpu_busy_pct_before": hdr.get("rank_cpu_busy_pct"),
            "placement_policy": hdr.get("placement_policy"), "cgroup_cpu_quota": hdr["cgroup_cpu_quota"],
            "rank_l3": hdr.get("rank_l3"), "l3_domains_used": hdr.get("l3_domains_used"),
            "l3_domain_cores": hdr.get("l3_domain_cores"),
            "yields_8B": by[8].get("yields"), "throttled_periods_8B": by[8].get("throttled"),
            "yields_all_sizes": sum(r.get("yields", 0) for r in rows),
            "throttled_periods_all_sizes": sum(r.get("throttled", 0) for r in rows),
            "dram_triad_GBps": stream["triad_GBps"] if stream else None,
            "dram_triad_what": "STREAM triad on the same pinned CPUs at once (24 B/element), the host memory "
                               "bound of this baseline (SURVEY.md §8(d) row 1)" if stream else None,
            "kind": "port", "cpu": cpu_info(), "placement": placement}


def cpu_baseline_host_allreduce(seconds=10.0, ranks=8):
    """The reference's host-buffer ch3 shared-memory MPI_Allreduce, fp32 SUM, `ranks` processes
    pinned one per CPU of the inherited cpuset, physical cores first (oracle/host_allreduce.c: the
    reference-algorithm host restatement, BASELINE.json configs[0]).  Bounded sample: 8 B .. 64 MiB,
    each size capped at ~seconds/12 s.  The record names the CPUs it ran on and whether ranks had
    to share one."""
    exe = os.path.join(ROOT, "oracle", "host_allreduce")
    if not os.path.exists(exe):
        return {"error": "oracle/host_allreduce not built"}
    cap = max(0.2, seconds / 12.0)
    try:
        out = subprocess.run([exe, "-n", str(ranks), "-m", "8:67108864", "-c", "-T", f"{cap:.2f}", "-B", "1.0"],
                             capture_output=True, text=True, timeout=max(60.0, 40 * cap)).stdout
    except subprocess.TimeoutExpired:
        return {"error": "host_allreduce timed out"}
    rec = host_allreduce_record(out)
    if "error" not in rec:
        rec["what"] = ("reference host path (topology-aware degree-4 shm tree <= 2 KiB, pt2pt_rs to 2 MiB, flat ring "
                       f"from 2 MiB, single-copy exchange), {rec['placement']}, CPUs {rec['rank_cpus']}, OSU loop, "
                       f"sizes 8 B..64 MiB, <= {cap:.2f} s per size")
    return rec


def cpu_baseline_nranks(seconds):
    """The N > 1 line's cpu_baseline: configs[0]'s host allreduce at the largest size it covers
    (64 MiB busbw, 8 ranks), with its 8-byte latency and placement in the sample text."""
    return cpu_baseline_nranks_from(cpu_baseline_host_allreduce(seconds))


def cpu_baseline_nranks_from(h):
    if "error" in h:
        return {"value": None, "unit": "GB/s", "cores": None, "kind": "port", "sample": h["error"]}
    return {"value": h["busbw_64MiB_GBps"], "unit": "GB/s", "cores": h["cpus_used"], "kind": "port",
            "correct": h["all_ok"], "cpus_available": h["cpus_available"], "cpus_used": h["cpus_used"],
            "oversubscribed": h["oversubscribed"], "rank_cpus": h["rank_cpus"],
            "rank_l3": h.get("rank_l3"), "l3_domains_used": h.get("l3_domains_used"),
            "placement_policy": h.get("placement_policy"),
            "sample": f"configs[0]: reference host-buffer ch3 shared-memory MPI_Allreduce fp32 SUM restated "
                      f"(oracle/host_allreduce.c), 64 MiB busbw; 8 B latency {h['latency_8B_us']} us, 1 MiB busbw "
                      f"{h['busbw_1MiB_GBps']} GB/s; {h['placement']} of '{h['cpu']}'; {h['what']}"}


def reduce_local_run(L, type_name, op_name, nbytes, steps, warmup):
    h, desc, size, ext = TYPES[type_name]
    count = nbytes // ext
    a = m.DeviceBuffer(count * ext)
    b = m.DeviceBuffer(count * ext)
    rng = np.random.default_rng(0x5EED)
    dt = m.np_dtype(type_name)
    if dt.kind == "f":
        x = rng.uniform(-1, 1, count).astype(dt)
        y = rng.uniform(-1, 1, count).astype(dt)
    else:
        x = rng.integers(-(2**31), 2**31 - 1, count, dtype=np.int64).astype(dt)
        y = rng.integers(-(2**31), 2**31 - 1, count, dtype=np.int64).astype(dt)
    a.upload(x)
    b.upload(y)
    for _ in range(warmup):
        m.check(L.MPI_Reduce_local(a.ptr, b.ptr, count, h, OPS[op_name]), "MPI_Reduce_local")
    # value: the blocking calls alone (no timing events in the stream)
    L.mv2h_device_synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.check(L.MPI_Reduce_local(a.ptr, b.ptr, count, h, OPS[op_name]), "MPI_Reduce_local")
    L.mv2h_device_synchronize()
    t = time.perf_counter() - t0
    # kernel duration: HIP events around the launch on the library's stream, separate loop
    L.mv2h_timing_enable(1)
    kms = []
    for _ in range(steps):
        m.check(L.MPI_Reduce_local(a.ptr, b.ptr, count, h, OPS[op_name]), "MPI_Reduce_local")
        kms.append(L.mv2h_last_kernel_ms())
    L.mv2h_timing_enable(0)
    # spot-check correctness of the last call on a slice (exact single-op fp/int)
    got = b.download(dt, count=4096)
    del a, b
    return t / steps, float(np.mean(kms)) / 1e3, count, got


def pack_run(L, steps):
    """configs[4]'s strided operand, device MPI_Pack / MPI_Unpack (replicas: per-GPU work).
    Algorithmic bytes = 2 x packed; the HBM floor of this layout is the whole
    strided span plus the packed bytes (1.5 x, profiles/pmc_pack_vector_r02e.json)."""
    nb = 8 << 20
    vt = ctypes.c_int()
    m.check(L.MPI_Type_vector(nb, 4, 8, TYPES["MPI_FLOAT"][0], ctypes.byref(vt)), "MPI_Type_vector")
    m.check(L.MPI_Type_commit(ctypes.byref(vt)), "MPI_Type_commit")
    span, packed = ((nb - 1) * 8 + 4) * 4, nb * 16
    src, dst = m.DeviceBuffer(span), m.DeviceBuffer(packed)
    src.upload(np.random.default_rng(7).standard_normal(span // 4).astype(np.float32))
    out = {}
    for name, fn in (("pack", lambda pos: L.MPI_Pack(src.ptr, 1, vt.value, dst.ptr, packed, ctypes.byref(pos), WORLD)),
                     ("unpack", lambda pos: L.MPI_Unpack(dst.ptr, packed, ctypes.byref(pos), src.ptr, 1, vt.value, WORLD))):
        m.check(fn(ctypes.c_int(0)), name)
        L.mv2h_device_synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m.check(fn(ctypes.c_int(0)), name)
        L.mv2h_device_synchronize()
        t = (time.perf_counter() - t0) / steps
        L.mv2h_timing_enable(1)  # kernel time (HIP events on the library stream), separate loop
        kms = []
        for _ in range(steps):
            m.check(fn(ctypes.c_int(0)), name)
            kms.append(L.mv2h_last_kernel_ms())
        L.mv2h_timing_enable(0)
        k = float(np.mean(kms))
        out[name] = {"GB/s_algorithmic": round(2 * packed / t / 1e9, 1), "GB/s_hbm_floor": round((span + packed) / t / 1e9, 1),
                     "ms": round(t * 1e3, 4), "kernel_ms": round(k, 4),
                     "kernel_GB/s_hbm_floor": round((span + packed) / (k / 1e3) / 1e9, 1)}
    m.check(L.MPI_Type_free(ctypes.byref(vt)), "MPI_Type_free")
    return out


def bench_n1(args, L):
    step_s, kern_s, count, _ = reduce_local_run(L, "MPI_FLOAT", "MPI_SUM", S_BYTES, args.steps, args.warmup)
    alg_bytes = 3 * count * 4
    value = alg_bytes / step_s / 1e9
    achieved = alg_bytes / kern_s / 1e9
    extra = {}
    for t, op in (("MPI_FLOAT", "MPI_MAX"), ("MPI_INT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX")):
        s, k, c, _ = reduce_local_run(L, t, op, S_BYTES, max(3, args.steps // 2), 2)
        extra[f"{t}:{op}"] = {"GB/s_call": round(3 * S_BYTES / s / 1e9, 1), "GB/s_kernel": round(3 * S_BYTES / k / 1e9, 1)}
    # host (pageable) operands: the library stages them to the GPU and back — the
    # PCIe-inclusive rate of the same call (never the headline value)
    hx = np.random.default_rng(3).uniform(-1, 1, count).astype(np.float32)
    hy = np.random.default_rng(4).uniform(-1, 1, count).astype(np.float32)
    m.check(L.MPI_Reduce_local(hx.ctypes.data, hy.ctypes.data, count, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]), "host")
    t0 = time.perf_counter()
    for _ in range(3):
        m.check(L.MPI_Reduce_local(hx.ctypes.data, hy.ctypes.data, count, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]), "host")
    extra["MPI_FLOAT:MPI_SUM host buffers (PCIe-inclusive)"] = {"GB/s_call": round(3 * S_BYTES * 3 / (time.perf_counter() - t0) / 1e9, 2)}
    del hx, hy
    extra["MPI_Pack/Unpack MPI_Type_vector(8Mi,4,8,MPI_FLOAT)"] = pack_run(L, max(3, args.steps // 2))
    # the metric's small-message half at one rank: an 8-byte MPI_Reduce_local per call, OSU-style
    # mean over args.lat_iters back-to-back blocking calls after 100 untimed ones.  MPI_UNSIGNED
    # (2 elements) so that its launches are a kernel instantiation of their own and the rocprof
    # average of the 256 MiB fp32 kernel stays that kernel's
    s8, r8 = m.DeviceBuffer(8), m.DeviceBuffer(8)
    s8.upload(np.ones(2, dtype=np.uint32))
    r8.upload(np.zeros(2, dtype=np.uint32))
    U32, SUM = TYPES["MPI_UNSIGNED"][0], OPS["MPI_SUM"]
    for _ in range(100):
        L.MPI_Reduce_local(s8.ptr, r8.ptr, 2, U32, SUM)
    aql0 = m.info("aql_calls")
    t0 = time.perf_counter()
    for _ in range(args.lat_iters):
        m.check(L.MPI_Reduce_local(s8.ptr, r8.ptr, 2, U32, SUM), "MPI_Reduce_local 8 B")
    lat = (time.perf_counter() - t0) / args.lat_iters
    via_queue = m.info("aql_calls") - aql0
    ok8 = bool(np.all(r8.download(np.uint32, count=2) == 100 + args.lat_iters))
    extra["reduce_local_8B_latency_us"] = {"us": round(lat * 1e6, 2), "correct": ok8,
                                           "calls_via_hsa_queue": via_queue, "calls": args.lat_iters,
                                           "what": "MPI_Reduce_local SUM on 2 MPI_UNSIGNED (8 B), device buffers, "
                                                   "blocking call incl. dispatch and completion word (one-wave "
                                                   "kernel in the library's own HSA queue, runtime/aql.cpp), "
                                                   "Python ctypes loop"}
    del s8, r8
    # the same 8-byte call from the OSU loop in C (tools/osu/libosu_coll.so -c reduce_local, MPI_FLOAT
    # SUM on 2 elements, validated), without the ctypes call in every iteration
    # it is the line's figure, as the N > 1 line's 8-byte latency is its C sweep's (OSU is a C
    # benchmark); the Python loop's figure stays beside it
    osu8 = osu_reduce_local_8b()
    if osu8 is not None:
        rl8 = extra["reduce_local_8B_latency_us"]
        rl8["python_loop_us"] = rl8["us"]
        rl8["us"] = osu8
        rl8["source"] = "tools/osu/osu_coll -c reduce_local (C OSU loop, MPI_FLOAT SUM on 2 elements, 2000 iterations)"
    # HBM traffic of this kernel from the newest committed PMC pass (rocprofv3 FETCH_SIZE x2 +
    # WRITE_SIZE in separate passes, tools/pmc_summary.py); the file is named in the line
    traffic, tsrc = None, None
    cands = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.startswith("pmc_reduce_local_"))
    if cands:
        tsrc = os.path.join("profiles", cands[-1])
        try:
            traffic = json.load(open(os.path.join(ROOT, tsrc))).get("hbm_bytes_per_launch")
        except Exception:
            traffic, tsrc = None, None
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "configs[1]: MPI_Reduce_local SUM fp32 on 256 MiB device buffers, 1 MI355X",
                   "count": count, "bytes_per_operand": S_BYTES, "algorithmic_bytes_per_call": alg_bytes,
                   "api": "MPI_Reduce_local via libmpi.so (MPICH ABI)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic, "traffic_source": tsrc,
                     "kernel": "k_reduce_local<R<SUM,F32>,2>", "kernel_ms": round(kern_s * 1e3, 4)},
        "cpu_baseline": cpu_baseline_reduce_local(args.cpu_seconds) if args.cpu_seconds > 0 else None,
        "extra": extra,
    }
    extra["mpi_init_ms"] = {"total": round(m.info("init_us") / 1e3, 1), "hip_start": round(m.info("hip_init_us") / 1e3, 1),
                            "code_objects": round(m.info("code_load_us") / 1e3, 1),
                            "what": "MPI_Init wall time on this rank; code objects = loading libmpi.so's gfx950 "
                                    "code (26 MB, one empty kernel per translation unit)"}
    # completion-word events of this run (runtime/coll.cpp wait_done): a word still unseen 200 us
    # after launch, a kernel that ended without raising it, a kernel whose block groups ran on
    # several XCDs -- a slow call in this line is explained or ruled out by these
    extra["completion_word"] = {k: m.info(k) for k in WORD_KEYS}
    if args.cpu_seconds > 0:
        extra["cpu_host_allreduce_8rank"] = cpu_baseline_host_allreduce(args.cpu_seconds)
    return line


def _timed(L, world, call, steps, warmup, step_call=None):
    """OSU loop on resident device buffers: warmup, barrier + device sync,
    `steps` calls, device sync + barrier.  Returns (s per call, mean kernel ms).
    step_call(i), when given, is the i-th timed call (each timed call its own result buffer, so
    that every one is verified afterwards); the kernel-time loop uses `call`."""
    for _ in range(warmup):
        m.check(call(), "warmup")
    L.MPI_Barrier(world)
    L.mv2h_device_synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        m.check(step_call(i) if step_call else call(), "timed call")
    L.mv2h_device_synchronize()
    L.MPI_Barrier(world)
    t = time.perf_counter() - t0
    # kernel durations (HIP events on the library's stream) in a separate loop
    L.mv2h_timing_enable(1)
    kms = []
    for _ in range(steps):
        m.check(call(), "timed call")
        kms.append(L.mv2h_last_kernel_ms())
    L.mv2h_timing_enable(0)
    return t / steps, float(np.mean(kms))


def _pattern(count, rank):
    """Exact-in-fp32 operand: x_r[i] = (7i + 13r) mod 1024 (sums of <= 8 ranks are exact)."""
    i = np.arange(count, dtype=np.int64)
    return ((7 * i + 13 * rank) % 1024).astype(np.float32)


def _expected_sum(count, size):
    i = np.arange(count, dtype=np.int64)
    acc = np.zeros(count, dtype=np.int64)
    for r in range(size):
        acc += (7 * i + 13 * r) % 1024
    return acc.astype(np.float32)


def rccl_child():
    """Child process of one bench rank: RCCL ncclAllReduce on the same 256 MiB
    fp32 SUM (torch.distributed "nccl" backend = RCCL), timed like
    osu_nccl_allreduce.c:107-131.  A comparator number only: never a code path
    of the library.  Runs in its own process group (own port) so a stuck
    comparator can be killed without losing the bench line."""
    import torch
    import torch.distributed as dist
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.ones(S_BYTES // 4, dtype=torch.float32, device=dev)
    steps = int(os.environ.get("MV2AMD_RCCL_STEPS", "10"))
    for _ in range(3):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    tt = torch.tensor([t], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt.item())
    del x
    # the same sizes as the library's OSU sweep (8 B .. 1 GiB, x4), timed as osu_nccl_allreduce.c:
    # per iteration t_start, ncclAllReduce, stream synchronise, t_stop, barrier; mean over ranks
    sweep = []
    if os.environ.get("MV2AMD_RCCL_SWEEP", "1") != "0":
        big = torch.empty(SWEEP_MAX // 4, dtype=torch.float32, device=dev)
        nb = 8
        while nb <= SWEEP_MAX:
            v = big[:max(1, nb // 4)]
            large = nb > 8192 * 4
            iters, skip = (20, 5) if large else (200, 20)
            tot = 0.0
            for i in range(iters + skip):
                t0 = time.perf_counter()
                dist.all_reduce(v)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if i >= skip:
                    tot += t1 - t0
                dist.barrier()
            lt = torch.tensor([tot / iters], dtype=torch.float64, device=dev)
            dist.all_reduce(lt)
            lat = float(lt.item()) / size
            sweep.append([nb, round(lat * 1e6, 2), round(2.0 * (size - 1) / size * nb / lat / 1e9, 3)])
            nb *= 4
        del big
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"busbw_GBps": round(2.0 * (size - 1) / size * S_BYTES / t / 1e9, 2), "ms": round(t * 1e3, 4),
                          "what": "torch.distributed all_reduce (RCCL) fp32 SUM 256 MiB, comparator only",
                          "sweep_columns": ["bytes", "lat_us", "busbw_GBps"], "sweep": sweep}), flush=True)


def rccl_comparator(L, world, rank, size, steps, timeout=150):
    """Every rank starts one rccl_child; rank 0 reads its line."""
    import socket
    port = np.zeros(1, dtype=np.int32)
    if rank == 0:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port[0] = s.getsockname()[1]
        s.close()
    m.check(L.MPI_Bcast(port.ctypes.data, 1, TYPES["MPI_INT"][0], 0, world), "MPI_Bcast(port)")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(int(port[0])), RANK=str(rank),
               WORLD_SIZE=str(size), MV2AMD_RCCL_STEPS=str(steps))
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rccl-child"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        p.communicate()
        return {"error": f"comparator timed out after {timeout} s"}
    if p.returncode != 0:
        lines = [l for l in (err or "").splitlines() if "rror" in l and "destroy_process_group" not in l]
        return {"error": (lines[-1] if lines else (err or "")[-200:])[-300:], "returncode": p.returncode}
    if rank == 0:
        try:
            return json.loads(out.strip().splitlines()[-1])
        except Exception:
            return {"error": "no comparator line"}
    return None


SWEEP_MAX = 1 << 30        # configs[2]: osu_allreduce 8 B .. 1 GiB
SWEEP_CAP = 256 << 20      # configs[3]: reduce_scatter / allgather / bcast up to 256 MiB


def osu_reduce_local_8b():
    """N = 1: the 8-byte MPI_Reduce_local latency from tools/osu's C OSU loop (osu_coll -c reduce_local,
    2000 iterations after 200 untimed, result validated); None when the harness is not built."""
    so = os.path.join(ROOT, "tools", "osu", "libosu_coll.so")
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    lib.osu_coll_main.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
    lib.osu_coll_main.restype = ctypes.c_int
    path = os.path.join("/tmp", f"mv2amd_rl8_{os.getpid()}.jsonl")
    args = ["osu_coll", "-c", "reduce_local", "-m", "8:8", "-i", "2000", "-x", "200", "-v", "-j", "-o", path]
    argv = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
    rc = lib.osu_coll_main(len(args), argv)
    try:
        rows = [json.loads(l[5:]) for l in open(path) if l.startswith("JSON ")]
        os.unlink(path)
    except OSError:
        return None
    row = next((r for r in rows if r.get("coll") == "reduce_local" and r.get("bytes") == 8), None)
    if rc != 0 or row is None or row.get("valid") is not True:
        return None
    return row["lat_us"]


def osu_sweep(L, world, rank, size):
    """configs[2] and [3] as OSU sweeps in the same run: every rank calls tools/osu/libosu_coll.so's
    osu_coll_main -- the OSU loop restated in C against include/mpi.h (osu_allreduce.c:98-163),
    here inside this job's MPI world, so on its MPI_Init tuning and with no second process per GPU
    -- with -c all: allreduce 8 B .. 1 GiB and reduce_scatter / allgather / bcast 8 B .. 256 MiB,
    sizes x4, every result validated against its closed form, then osu_latency / osu_bw between
    ranks 0 and 1 up to 16 MiB.  Rank 0's rows come back through a JSON file."""
    so = os.path.join(ROOT, "tools", "osu", "libosu_coll.so")
    if not os.path.exists(so):
        return {"error": "tools/osu/libosu_coll.so not built"}
    lib = ctypes.CDLL(so)
    lib.osu_coll_main.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
    lib.osu_coll_main.restype = ctypes.c_int
    path = os.path.join("/tmp", f"mv2amd_sweep_{os.getpid()}.jsonl")
    args = ["osu_coll", "-c", "all", "-m", f"8:{SWEEP_MAX}", "-f", "4", "-C", str(SWEEP_CAP), "-i", "200", "-I", "20",
            "-v", "-j", "-o", path]
    argv = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
    t0 = time.perf_counter()
    rc = lib.osu_coll_main(len(args), argv)
    secs = time.perf_counter() - t0
    if rank != 0:
        return None
    try:
        rows = [json.loads(l[5:]) for l in open(path) if l.startswith("JSON ")]
        os.unlink(path)
    except OSError as e:
        return {"error": f"no sweep rows: {e}", "returncode": rc}
    res = {"what": "tools/osu/osu_coll -c all (OSU loop in C through libmpi.so inside this job, device buffers, "
                   "every size validated): allreduce 8 B..1 GiB, reduce_scatter / allgather / bcast 8 B..256 MiB, "
                   "x4 sizes",
           "columns": ["bytes", "lat_us", "busbw_GBps", "valid"], "seconds": round(secs, 1), "returncode": rc,
           "all_valid": rc == 0 and bool(rows) and all(r["valid"] is True for r in rows if "valid" in r)}
    for c in ("allreduce", "reduce_scatter", "allgather", "bcast"):
        res[c] = [[r["bytes"], r["lat_us"], r["busbw_GBps"], r["valid"]] for r in rows if r["coll"] == c]
    # device point-to-point between ranks 0 and 1 (§8(f) rank 1): osu_latency (half round trip) and
    # osu_bw (a window of 64 MPI_Isend, the receiver's ack), 8 B .. 16 MiB
    res["osu_latency_us"] = [[r["bytes"], r["lat_us"]] for r in rows if r["coll"] == "osu_latency"]
    res["osu_bw_GBps"] = [[r["bytes"], r["bw_GBps"]] for r in rows if r["coll"] == "osu_bw"]
    return res


def user_op_lines(L, world, sb, rb, size):
    """configs[4]'s user-op allreduce on MPI_Type_vector(nb, 4, 8, MPI_FLOAT) operands, 16 MiB of
    payload (32 MiB span): `count` elements of nb blocks.  count >= n takes the reference's ring
    (each rank evaluates its own chunk, allreduce_osu.c:3925-3958); count = 1 leaves the ring
    nothing and runs recursive doubling (every rank its own tree).  The op is C (tools/osu/
    uop_vsum.c, as an OSU-style application's would be) or numpy through ctypes (round 2's line).
    Results are checked exactly on a slice (integer-valued operands)."""
    F32 = TYPES["MPI_FLOAT"][0]
    UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))
    clib = ctypes.CDLL(os.path.join(ROOT, "tools", "osu", "libuop_vsum.so"))
    out, ok = [], True
    for name, nb, count, kind in (("allreduce_user_op_vector", 4096, 256, "c"),
                                  ("allreduce_user_op_vector_numpy_op", 4096, 256, "py"),
                                  ("allreduce_user_op_vector_rd", 1 << 20, 1, "py")):
        ext = (nb - 1) * 8 + 4  # floats
        vt = ctypes.c_int()
        m.check(L.MPI_Type_vector(nb, 4, 8, F32, ctypes.byref(vt)), "MPI_Type_vector")
        m.check(L.MPI_Type_commit(ctypes.byref(vt)), "MPI_Type_commit")
        keep = None
        if kind == "c":
            clib.uop_vsum_blocks(ctypes.c_long(nb))
            fnp = ctypes.cast(clib.uop_vsum, ctypes.c_void_p)
        else:
            def _vsum(inp, io, ln, dt, nb=nb, ext=ext):  # io += in on the type map of ln[0] elements
                c = ln[0]
                a = np.lib.stride_tricks.as_strided(
                    np.ctypeslib.as_array((ctypes.c_float * (c * ext)).from_address(inp)), (c, nb, 4), (ext * 4, 32, 4))
                b = np.lib.stride_tricks.as_strided(
                    np.ctypeslib.as_array((ctypes.c_float * (c * ext)).from_address(io)), (c, nb, 4), (ext * 4, 32, 4))
                b += a
            keep = UF(_vsum)
            fnp = ctypes.cast(keep, ctypes.c_void_p)
        uop = ctypes.c_int()
        m.check(L.MPI_Op_create(fnp, 1, ctypes.byref(uop)), "MPI_Op_create")
        # operand: x_r[k] = (k % 61) + r over the span (exact sums in fp32)
        span = count * ext
        sb.upload(((np.arange(span, dtype=np.int64) % 61) + L.mv2h_rank()).astype(np.float32))
        call = lambda: L.MPI_Allreduce(sb.ptr, rb.ptr, count, vt.value, uop.value, world)  # noqa: E731
        phases = ("stage", "fetch", "eval", "deliver")
        ph0 = [m.info(f"uop_{p}_us") for p in phases]
        s_, _ = _timed(L, world, call, 3, 1)  # 1 + 3 + 3 calls (warmup, timed, kernel-timing loop)
        ph = {p: round((m.info(f"uop_{p}_us") - a) / 7 / 1e3, 3) for p, a in zip(phases, ph0)}
        got = rb.download(np.float32, count=min(span, 1 << 20))
        k = np.arange(len(got), dtype=np.int64)
        onmap = (k % ext) % 8 < 4
        want = (size * (k % 61) + size * (size - 1) // 2).astype(np.float32)
        ok = ok and bool(np.array_equal(got[onmap], want[onmap]))
        L.MPI_Op_free(ctypes.byref(uop))
        L.MPI_Type_free(ctypes.byref(vt))
        del keep
        algo = "ring (own chunk per rank)" if count >= size else "recursive doubling (every rank its own tree)"
        out.append({"name": name, "s": s_, "payload": count * nb * 16, "phases_ms_rank0": ph,
                    "what": f"configs[4]: commutative user op ({'C' if kind == 'c' else 'numpy via ctypes'}) on "
                            f"{count} x MPI_Type_vector({nb},4,8,MPI_FLOAT), {count * nb * 16 >> 20} MiB payload, {algo}"})
    return {"ok": ok, "lines": out}


def pipe_traffic_for(size, nshare, alg):
    """(traffic bytes, source file, note) for k_pipe PIPE_AR at this run's configuration: the
    newest profiles/pmc_pipe_allreduce_*.json whose recorded configuration (ranks, ranks per GPU,
    tiling knobs, remote-store flavour) equals this run's; else (None, None, why)."""
    here = {"ranks": size, "nshare": nshare, "pipe_grid": m.info("pipe_grid"), "pipe_sub": m.info("pipe_sub"),
            "pipe_rnt": m.info("pipe_rnt")}
    best = None
    for f in sorted(os.listdir(os.path.join(ROOT, "profiles"))):
        if not f.startswith("pmc_pipe_allreduce_"):
            continue
        try:
            d = json.load(open(os.path.join(ROOT, "profiles", f)))
        except Exception:
            continue
        cfg = d.get("config") or {}
        if all(cfg.get(k) == v for k, v in here.items()) and d.get("traffic_over_algorithmic"):
            best = (round(d["traffic_over_algorithmic"] * alg), os.path.join("profiles", f), None)
    if best:
        return best
    return None, None, f"no committed PMC pass at this configuration {here}"


def bench_nranks(args, L, rank, size):
    world = 0x44000000
    F32, F64, DINT = TYPES["MPI_FLOAT"][0], TYPES["MPI_DOUBLE"][0], TYPES["MPI_DOUBLE_INT"][0]
    CHAR = TYPES["MPI_CHAR"][0]
    SUM, MAX, MAXLOC = OPS["MPI_SUM"], OPS["MPI_MAX"], OPS["MPI_MAXLOC"]
    count = S_BYTES // 4
    sb = m.DeviceBuffer(S_BYTES)
    rb = m.DeviceBuffer(S_BYTES)
    sb.upload(_pattern(count, rank))

    # headline: allreduce fp32 SUM 256 MiB, validated over the whole buffer -- every timed call writes
    # its own result buffer (steps x 256 MiB of HBM) and each is checked after the timed region
    ar = lambda: L.MPI_Allreduce(sb.ptr, rb.ptr, count, F32, SUM, world)  # noqa: E731
    rb.upload(np.zeros(count, dtype=np.float32))
    m.check(ar(), "MPI_Allreduce")
    want = _expected_sum(count, size)
    ok = bool(np.array_equal(rb.download(np.float32, count=count), want))
    rbs = [m.DeviceBuffer(S_BYTES) for _ in range(args.steps)]
    step_s, kms = _timed(L, world, ar, args.steps, args.warmup,
                         step_call=lambda i: L.MPI_Allreduce(sb.ptr, rbs[i].ptr, count, F32, SUM, world))
    verified = sum(bool(np.array_equal(b.download(np.float32, count=count), want)) for b in rbs)
    del rbs
    ok = ok and verified == args.steps and bool(np.array_equal(rb.download(np.float32, count=count), want))
    del want

    # config 4 / config 5 lines at 256 MiB (fewer steps)
    ks = max(3, args.steps // 2)
    rcnt = count // size
    rsb = m.DeviceBuffer(rcnt * 4)
    rcounts = (ctypes.c_int * size)(*([rcnt] * size))
    rs_s, rs_k = _timed(L, world, lambda: L.MPI_Reduce_scatter(sb.ptr, rsb.ptr, rcounts, F32, SUM, world), ks, 2)
    agb = S_BYTES // size
    ag_s, ag_k = _timed(L, world, lambda: L.MPI_Allgather(sb.ptr, agb, CHAR, rb.ptr, agb, CHAR, world), ks, 2)
    bc_s, bc_k = _timed(L, world, lambda: L.MPI_Bcast(rb.ptr, S_BYTES, CHAR, 0, world), ks, 2)
    nrec = S_BYTES // 16
    rec = np.zeros(nrec, dtype=[("v", "<f8"), ("i", "<i4"), ("pad", "<i4")])
    rng = np.random.default_rng(1000 + rank)
    rec["v"] = np.floor(rng.random(nrec) * 1000.0)
    rec["i"] = rank
    sb.upload(rec.view(np.uint8))
    ml = lambda: L.MPI_Allreduce(sb.ptr, rb.ptr, nrec, DINT, MAXLOC, world)  # noqa: E731
    ml_s, ml_k = _timed(L, world, ml, ks, 2)

    # configs[4]: a commutative user op on MPI_Type_vector(nb, 4, 8, MPI_FLOAT) operands (the
    # reference rejects predefined ops on derived types); the op runs on the host in the selected
    # algorithm's order (mpi/user_coll.cpp: packed operands, each ring chunk evaluated by its owner)
    uops = user_op_lines(L, world, sb, rb, size)

    # 8-byte latency (OSU: small-message iterations, skip 100)
    s8 = m.DeviceBuffer(8)
    r8 = m.DeviceBuffer(8)
    s8.upload(np.ones(2, dtype=np.float32))
    for _ in range(100):
        L.MPI_Allreduce(s8.ptr, r8.ptr, 2, F32, SUM, world)
    # osu_allreduce.c:106-136: Barrier once; per iteration t_start, Allreduce, t_stop, Barrier;
    # latency = mean over iterations, reported as the mean over ranks (OSU's avg_time column);
    # no timing events in this loop (they add an event synchronisation to every call)
    lat = 0.0
    L.MPI_Barrier(world)
    for _ in range(args.lat_iters):
        t0 = time.perf_counter()
        L.MPI_Allreduce(s8.ptr, r8.ptr, 2, F32, SUM, world)
        lat += time.perf_counter() - t0
        L.MPI_Barrier(world)
    # kernel time of the same call (HIP events on the library stream), separate loop
    lat_k = []
    L.mv2h_timing_enable(1)
    for _ in range(max(50, args.lat_iters // 4)):
        L.MPI_Barrier(world)
        L.MPI_Allreduce(s8.ptr, r8.ptr, 2, F32, SUM, world)
        lat_k.append(L.mv2h_last_kernel_ms())
    L.mv2h_timing_enable(0)
    lat_ok = bool(np.all(r8.download(np.float32, count=2) == size))
    lav = m.DeviceBuffer(8)
    lav.upload(np.array([lat / args.lat_iters], dtype=np.float64))
    lsum = m.DeviceBuffer(8)
    m.check(L.MPI_Allreduce(lav.ptr, lsum.ptr, 1, TYPES["MPI_DOUBLE"][0], SUM, world), "avg latency")
    lat_avg = float(lsum.download(np.float64, count=1)[0]) / size
    # the same 8-byte allreduce stream-ordered (MPIX_Allreduce_enqueue): calls queued back to
    # back on one HIP stream, one synchronisation — the host round trip per call is gone
    hip = ctypes.CDLL("libamdhip64.so")
    hst = ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(hst))
    sq_iters = args.lat_iters
    L.MPI_Barrier(world)
    t0 = time.perf_counter()
    for _ in range(sq_iters):
        m.check(L.MPIX_Allreduce_enqueue(s8.ptr, r8.ptr, 2, F32, SUM, world, hst), "MPIX_Allreduce_enqueue")
    hip.hipStreamSynchronize(hst)
    sq_s = (time.perf_counter() - t0) / sq_iters
    m.check(L.MPIX_Enqueue_check(world), "MPIX_Enqueue_check")
    lat_ok = lat_ok and bool(np.all(r8.download(np.float32, count=2) == size))
    hip.hipStreamDestroy(hst)

    # device point-to-point bandwidth, rank 0 -> rank 1 (osu_bw pattern: a window of
    # Isends, one Waitall; the receiver posts the matching Irecvs)
    nshare = m.info("nshare")  # ranks sharing one GPU (test rehearsals): no xGMI byte moves then
    pbytes, win = 16 << 20, 8
    BYTE = TYPES["MPI_BYTE"][0]
    pb = m.DeviceBuffer(pbytes * win)
    p2p_s = 0.0
    for it in range(1 + max(2, ks)):
        L.MPI_Barrier(world)
        t0 = time.perf_counter()
        if rank in (0, 1):
            reqs = (ctypes.c_int * win)()
            for w_ in range(win):
                q = ctypes.c_int()
                if rank == 0:
                    m.check(L.MPI_Isend(pb.ptr + w_ * pbytes, pbytes, BYTE, 1, 50, world, ctypes.byref(q)), "Isend")
                else:
                    m.check(L.MPI_Irecv(pb.ptr + w_ * pbytes, pbytes, BYTE, 0, 50, world, ctypes.byref(q)), "Irecv")
                reqs[w_] = q.value
            m.check(L.MPI_Waitall(win, reqs, None), "Waitall")
            if rank == 1:  # osu_bw: the receiver's ack closes the window
                m.check(L.MPI_Send(pb.ptr, 4, BYTE, 0, 51, world), "ack")
            else:
                m.check(L.MPI_Recv(pb.ptr, 4, BYTE, 1, 51, world, None), "ack")
        if it:
            p2p_s += time.perf_counter() - t0
    p2p_s /= max(2, ks)
    del pb

    # max over ranks through the library itself (device allreduce MAX)
    vals = np.array([step_s, kms, rs_s, rs_k, ag_s, ag_k, bc_s, bc_k, ml_s, ml_k, lat / args.lat_iters,
                     float(np.median(lat_k)), 0.0 if (ok and lat_ok and uops["ok"]) else 1.0, p2p_s, sq_s,
                     float(args.steps - verified)]
                    + [u["s"] for u in uops["lines"]], dtype=np.float64)
    dm = m.DeviceBuffer(vals.nbytes)
    dm.upload(vals)
    dr = m.DeviceBuffer(vals.nbytes)
    m.check(L.MPI_Allreduce(dm.ptr, dr.ptr, len(vals), F64, MAX, world), "max")
    got = dr.download(np.float64)
    keys = ("step_s", "kms", "rs_s", "rs_k", "ag_s", "ag_k", "bc_s", "bc_k", "ml_s", "ml_k", "lat_s", "lat_k_ms", "bad",
            "p2p_s", "sq_s", "unverified")
    t = {k: float(v) for k, v in zip(keys, got[:len(keys)])}
    for u, tu in zip(uops["lines"], got[len(keys):]):
        u["s"] = float(tu)
    # completion-word events summed over ranks (runtime/coll.cpp wait_done: late words, words the
    # kernel never raised, words of kernels whose block groups ran on several XCDs)
    word = np.array([m.info(k) for k in WORD_KEYS], dtype=np.int64)
    dw = m.DeviceBuffer(word.nbytes)
    dw.upload(word)
    dws = m.DeviceBuffer(word.nbytes)
    m.check(L.MPI_Allreduce(dw.ptr, dws.ptr, len(WORD_KEYS), TYPES["MPI_LONG"][0], SUM, world), "word counts")
    checks = {"timed_calls_verified": args.steps - int(t["unverified"]), "timed_calls": args.steps,
              "completion_word_sum_over_ranks": dict(zip(WORD_KEYS, (int(v) for v in dws.download(np.int64)))),
              "release_protocol": "light" if m.info("light_release") else "full",
              "shared_gpu_constants": {"MV2AMD_AR_SCALAR_MAX": m.info("ar_scalar_max"),
                                       "MV2AMD_RS_SCALAR_MAX": m.info("rs_scalar_max"),
                                       "p2p_copy_kernels": bool(m.info("p2p_kernel_copy"))}}
    # HBM traffic of k_pipe (PIPE_AR) per launch on one rank: the PMC ratio (rocprofv3 FETCH_SIZE x2 +
    # WRITE_SIZE in separate passes, tools/pmc_summary.py) of a committed pass taken at THIS rank
    # count, ranks per GPU and tiling knobs, times this call's per-rank algorithmic HBM bytes
    # 2S(1 + 2(n-1)/n): reads of the operand, the RS and the AG slots; writes of the peers' RS
    # pushes, the own segment, the peers' AG pushes and the gathered segments.  No matching pass:
    # traffic is null and the nearest pass's configuration is named instead.
    traffic = pipe_traffic_for(size, nshare, pipe_alg_bytes(size))
    tiling = {"grid": m.info("pipe_grid"), "bytes_per_workgroup_round": m.info("pipe_sub"),
              "remote_stores": "non-temporal" if m.info("pipe_rnt") else "plain",
              "autotuned_at_init": bool(m.info("pipe_tuned")),
              "candidates_max_over_ranks_us": [
                  {"grid": m.info(f"tune_grid_{k}"), "sub": m.info(f"tune_sub_{k}"),
                   "nt": m.info(f"tune_rnt_{k}"), "us": m.info(f"tune_us_{k}")}
                  for k in range(m.info("tune_n"))],
              "oneshot_max_bytes": m.info("oneshot_max"),
              "mpi_init_ms_rank0": round(m.info("init_us") / 1e3, 1),
              "mpi_init_hip_start_ms": round(m.info("hip_init_us") / 1e3, 1),
              "mpi_init_code_objects_ms": round(m.info("code_load_us") / 1e3, 1),
              "mpi_init_selftest_ms": round(m.info("selftest_us") / 1e3, 1),
              "mpi_init_selftest_calls": m.info("selftest_calls"),
              "mpi_init_autotune_ms": round(m.info("autotune_us") / 1e3, 1),
              "oneshot_vs_pipe_us": [{"bytes": (32 << 10) << i, "oneshot": m.info(f"os_tune_one_{i}"),
                                      "pipe": m.info(f"os_tune_pipe_{i}")} for i in range(m.info("os_tune_n"))]}
    del sb, rb, rsb
    sweep = None
    if args.sweep:
        try:
            sweep = osu_sweep(L, world, rank, size)
        except Exception as e:  # a sweep problem never loses the headline line
            sweep = {"error": f"{type(e).__name__}: {e}"[:200]}
    if args.rccl and m.info("nshare") > 1:
        rccl = {"skipped": "ranks share one GPU: RCCL refuses several ranks on one device"}
    elif args.rccl:
        try:
            rccl = rccl_comparator(L, world, rank, size, max(5, args.steps // 2))
        except Exception as e:  # comparator only: never fail the bench line on it
            rccl = {"error": f"{type(e).__name__}: {e}"[:200]}
    else:
        rccl = None
    line = assemble_nranks_line(size, nshare, args.steps, args.warmup, t, lat_avg, uops["lines"], nrec, pbytes * win,
                                tiling, traffic, rccl, checks=checks)
    if sweep is not None:
        line["extra"]["osu_sweep"] = sweep
        # the metric's 8-byte latency as OSU measures it (the C loop, no ctypes call overhead); the
        # Python loop's figure stays beside it
        ar8 = [r for r in sweep.get("allreduce", []) if r[0] == 8 and r[3] is True]
        if ar8:
            cfg = line["config"]
            cfg["latency_8B_us_python_loop"] = cfg["latency_8B_us"]
            cfg["latency_8B_us"] = ar8[0][1]
            cfg["latency_8B_source"] = "osu_sweep (tools/osu/osu_coll, C OSU loop, mean over ranks)"
        rs = {r[0]: r[2] for r in (rccl or {}).get("sweep", [])}
        if rs and isinstance(sweep.get("allreduce"), list):
            line["extra"]["allreduce_busbw_vs_rccl_by_size"] = {
                "columns": ["bytes", "ours_GBps", "rccl_GBps", "ours_over_rccl"],
                "rows": [[b, bw, rs[b], round(bw / rs[b], 3) if rs[b] else None]
                         for b, _, bw, _ in sweep["allreduce"] if b in rs]}
    return line


def pipe_alg_bytes(size):
    """Per-rank algorithmic HBM bytes of one PIPE_AR call on S bytes: 2S(1 + 2(n-1)/n)."""
    return 2.0 * S_BYTES * (1.0 + 2.0 * (size - 1) / size)


def assemble_nranks_line(size, nshare, steps, warmup, t, lat_avg, uop_lines, nrec, p2p_bytes, tiling, traffic, rccl,
                         cpu_baseline=None, checks=None):
    """The N > 1 bench line from max-over-ranks measurements (pure: no GPU, no library calls, so the
    branches the 1-GPU box never takes -- nshare == 1, a successful or failed RCCL comparator -- are
    CPU-tested: tests/test_bench_line.py).  `t` holds seconds per call (`*_s`) and HIP-event kernel
    milliseconds (`kms`, `*_k`, `lat_k_ms`); `traffic` = pipe_traffic_for(...)."""
    f = (size - 1) / size
    busbw = 2.0 * f * S_BYTES / t["step_s"] / 1e9
    kbus = 2.0 * f * S_BYTES / (t["kms"] / 1e3) / 1e9
    peak_all = (size - 1) * XGMI_LINK
    pipe_alg = pipe_alg_bytes(size)
    pipe_traffic, pipe_tsrc, pipe_tnote = traffic

    def line4(ts, k, bytes_bus):
        return {"busbw_GBps": round(bytes_bus / ts / 1e9, 2), "kernel_busbw_GBps": round(bytes_bus / (k / 1e3) / 1e9, 2),
                "ms": round(ts * 1e3, 4)}

    extra = {
        "reduce_scatter_f32_sum": line4(t["rs_s"], t["rs_k"], f * S_BYTES),
        "allgather_char": line4(t["ag_s"], t["ag_k"], f * S_BYTES),
        "bcast_char": line4(t["bc_s"], t["bc_k"], S_BYTES),
        "allreduce_maxloc_double_int": line4(t["ml_s"], t["ml_k"], 2.0 * f * nrec * 12),
        **{u["name"]: {"payload_busbw_GBps": round(2.0 * f * u["payload"] / u["s"] / 1e9, 2), "ms": round(u["s"] * 1e3, 3),
                       "phases_ms_rank0": u["phases_ms_rank0"], "what": u["what"]} for u in uop_lines},
        "pt2pt_bw_16MiB_x8": {"GBps": round(p2p_bytes / t["p2p_s"] / 1e9, 2), "ms_per_window": round(t["p2p_s"] * 1e3, 3),
                              "what": "osu_bw pattern rank 0 -> 1: 8 x 16 MiB MPI_Isend / MPI_Irecv device buffers"},
    }
    checks = checks or {}
    if "completion_word_sum_over_ranks" in checks:
        extra["completion_word"] = dict(checks["completion_word_sum_over_ranks"])
    if "shared_gpu_constants" in checks:
        # chosen on one shared GPU and not probed at MPI_Init: a one-rank-per-GPU run ships them unmeasured
        extra["constants_tuned_on_shared_gpu"] = dict(
            checks["shared_gpu_constants"],
            note=("tuned on one shared GPU (profiles/r05y, r05ba, r05l), not probed at MPI_Init: "
                  "unmeasured over xGMI" if nshare == 1 else f"{nshare} ranks share this GPU, as when they were tuned"))
    if rccl is not None:
        extra["rccl_comparator"] = rccl
        if "busbw_GBps" in rccl:
            extra["rccl_comparator"]["ours_over_rccl"] = round(busbw / rccl["busbw_GBps"], 3)
    kernel = "k_pipe<R<SUM,F32>> (PIPE_AR)"
    if nshare == 1:
        roof = {"bound": "xgmi", "achieved": round(kbus, 1), "peak": peak_all, "unit": "GB/s",
                "frac": round(kbus / peak_all, 4), "traffic": pipe_traffic, "traffic_source": pipe_tsrc,
                "traffic_note": pipe_tnote, "traffic_algorithmic_hbm_bytes_per_rank": round(pipe_alg),
                "frac_vs_single_ring": round(kbus / XGMI_LINK, 3), "kernel": kernel, "kernel_ms": round(t["kms"], 4),
                "peak_note": f"direct RS+AG over the {size - 1} xGMI links each rank has to its peers: "
                             f"busbw peak = (n-1) x {XGMI_LINK} GB/s per link per direction"}
    else:
        roof = {"bound": "shared-gpu", "achieved": round(kbus, 1), "peak": None, "unit": "GB/s", "frac": None,
                "traffic": pipe_traffic, "traffic_source": pipe_tsrc, "traffic_note": pipe_tnote,
                "traffic_algorithmic_hbm_bytes_per_rank": round(pipe_alg), "kernel": kernel,
                "kernel_ms": round(t["kms"], 4),
                "note": f"{nshare} ranks share one GPU: every 'remote' store lands in the same HBM, no xGMI "
                        "link is used, so no xGMI roofline fraction applies"}
    line = {
        "metric": METRIC, "value": round(busbw, 2), "unit": "GB/s", "n_gpus": size, "steps": steps,
        "warmup": warmup, "ms_per_step": round(t["step_s"] * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "configs[2]: osu_allreduce -d rocm fp32 SUM 256 MiB, 1 rank per GPU over xGMI",
                   "count": S_BYTES // 4, "bytes": S_BYTES,
                   "algorithm": "pipelined direct RS+AG (pushes into peer arenas over xGMI)",
                   "latency_8B_us": round(lat_avg * 1e6, 2), "latency_8B_max_over_ranks_us": round(t["lat_s"] * 1e6, 2),
                   "latency_8B_kernel_us": round(t["lat_k_ms"] * 1e3, 2),
                   "allreduce_8B_stream_ordered_us_per_call": round(t["sq_s"] * 1e6, 2),
                   **({"stream_ordered_note": "ranks share one GPU: each rank's queued kernels spin until the other "
                       "processes' queues are scheduled (DESIGN.md §4 Stream order); not a one-GPU-per-rank figure"}
                      if nshare > 1 else {}),
                   "correct": not bool(t["bad"]),
                   "validation": "whole 256 MiB result vs exact expected sum: a call before timing, every timed "
                                 "call (each into its own result buffer), the buffer after the kernel-time loop",
                   **({"timed_calls_verified": checks["timed_calls_verified"], "timed_calls": checks["timed_calls"]}
                      if "timed_calls_verified" in checks else {}),
                   "pipe_tiling": dict(tiling, **({"release_protocol": checks["release_protocol"]}
                                                  if "release_protocol" in checks else {}))},
        "roofline": roof,
        "cpu_baseline": cpu_baseline,
        "extra": extra,
    }
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--lat-iters", type=int, default=1000)
    ap.add_argument("--rccl", type=int, default=1, help="N > 1: also time RCCL all_reduce as a comparator")
    ap.add_argument("--sweep", type=int, default=1, help="N > 1: OSU sweeps of configs[2] / [3] (tools/osu/osu_coll)")
    ap.add_argument("--rccl-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.rccl_child:
        rccl_child()
        return
    L = m.lib()
    size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if size != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={size}", file=sys.stderr)
    m.check(L.MPI_Init(None, None), "MPI_Init")
    if size == 1:
        line = bench_n1(args, L)
    else:
        line = bench_nranks(args, L, rank, size)
    L.MPI_Finalize()
    if rank == 0 and size > 1 and args.cpu_seconds > 0:
        # configs[0], the reference's host-buffer shared-memory MPI_Allreduce with 8 ranks on this
        # box's cores, in the same run (north_star): rank 0 after MPI_Finalize, when the GPU ranks
        # have stopped spinning on the host, as a fresh child process with a time limit
        line["cpu_baseline"] = cpu_baseline_nranks(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
