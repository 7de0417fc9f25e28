"""bench.py's line assembly and its CPU baseline, on the CPU.

The N > 1 line is assembled by a pure function (bench.assemble_nranks_line) so that the branches
the 1-GPU box never takes -- one rank per GPU (nshare == 1: the xGMI roofline), an RCCL comparator
that succeeds or fails -- run here before the driver's first 8-GPU run.
configs[0]'s host allreduce (oracle/host_allreduce) must name the CPUs it ran on and flag
oversubscription instead of wrapping silently.
"""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

HOST_AR = os.path.join(ROOT, "oracle", "host_allreduce")


def _t(step_ms=1.0):
    s = step_ms / 1e3
    return {"step_s": s, "kms": step_ms * 0.98, "rs_s": s / 2, "rs_k": step_ms / 2, "ag_s": s / 2, "ag_k": step_ms / 2,
            "bc_s": s / 2, "bc_k": step_ms / 2, "ml_s": s, "ml_k": step_ms, "lat_s": 11e-6, "lat_k_ms": 0.004,
            "bad": 0.0, "p2p_s": 0.01, "sq_s": 6e-6}


UOPS = [{"name": "allreduce_user_op_vector", "s": 0.004, "payload": 16 << 20, "phases_ms_rank0": {"eval": 1.0},
         "what": "x"}]
TILING = {"grid": 256, "bytes_per_workgroup_round": 131072}


@pytest.mark.parametrize("n", [2, 4, 8])
def test_one_rank_per_gpu_roofline(n):
    line = bench.assemble_nranks_line(n, 1, 20, 5, _t(), 9e-6, [dict(u) for u in UOPS], 1 << 24, 128 << 20, TILING,
                                      (None, None, "no committed PMC pass at this configuration {...}"),
                                      {"busbw_GBps": 300.0, "ms": 1.5, "what": "rccl"},
                                      cpu_baseline=bench.cpu_baseline_nranks_from(_fake_host_record()))
    busbw = 2.0 * (n - 1) / n * bench.S_BYTES / 1e-3 / 1e9
    kbus = 2.0 * (n - 1) / n * bench.S_BYTES / (0.98e-3) / 1e9
    assert line["value"] == round(busbw, 2) and line["n_gpus"] == n and line["scaling"] == "weak"
    r = line["roofline"]
    assert r["bound"] == "xgmi" and r["peak"] == (n - 1) * bench.XGMI_LINK
    assert r["frac"] == round(kbus / ((n - 1) * bench.XGMI_LINK), 4)
    assert r["frac_vs_single_ring"] == round(kbus / bench.XGMI_LINK, 3)
    assert r["traffic"] is None and "no committed PMC pass" in r["traffic_note"]
    assert r["traffic_algorithmic_hbm_bytes_per_rank"] == round(2.0 * bench.S_BYTES * (1 + 2.0 * (n - 1) / n))
    cb = line["cpu_baseline"]
    assert isinstance(cb["value"], float) and cb["cores"] == 8 and cb["oversubscribed"] is False
    assert line["extra"]["rccl_comparator"]["ours_over_rccl"] == round(busbw / 300.0, 3)
    assert "stream_ordered_note" not in line["config"]
    json.dumps(line)  # the line must serialise


CHECKS = {"timed_calls_verified": 20, "timed_calls": 20,
          "completion_word_sum_over_ranks": {"done_queried": 3, "done_late": 0, "done_missed": 0, "done_xcd_split": 0},
          "release_protocol": "light",
          "shared_gpu_constants": {"MV2AMD_AR_SCALAR_MAX": 1024, "MV2AMD_RS_SCALAR_MAX": 4096, "p2p_copy_kernels": True}}


@pytest.mark.parametrize("nshare", [1, 2])
def test_line_carries_the_checks(nshare):
    """every timed 256 MiB call verified (count in the line), the completion-word
    events summed over ranks, the release protocol MPI_Init adopted, and the constants tuned on a
    shared GPU named -- flagged as unmeasured over xGMI when each rank has a GPU to itself."""
    line = bench.assemble_nranks_line(8, nshare, 20, 5, _t(), 9e-6, [], 1 << 24, 128 << 20, TILING, (None, None, "n"),
                                      None, checks=dict(CHECKS))
    cfg = line["config"]
    assert cfg["timed_calls_verified"] == 20 and cfg["timed_calls"] == 20
    assert cfg["pipe_tiling"]["release_protocol"] == "light" and cfg["pipe_tiling"]["grid"] == 256
    assert line["extra"]["completion_word"] == {"done_queried": 3, "done_late": 0, "done_missed": 0, "done_xcd_split": 0}
    sg = line["extra"]["constants_tuned_on_shared_gpu"]
    assert sg["MV2AMD_AR_SCALAR_MAX"] == 1024 and sg["p2p_copy_kernels"] is True
    assert ("unmeasured over xGMI" in sg["note"]) == (nshare == 1)
    assert "every timed call" in cfg["validation"]
    json.dumps(line)


def test_shared_gpu_line_has_no_fraction():
    line = bench.assemble_nranks_line(2, 2, 20, 5, _t(), 9e-6, [dict(u) for u in UOPS], 1 << 24, 128 << 20, TILING,
                                      (123, "profiles/x.json", None),
                                      {"skipped": "ranks share one GPU"})
    assert line["roofline"]["bound"] == "shared-gpu" and line["roofline"]["frac"] is None
    assert line["roofline"]["traffic"] == 123 and "stream_ordered_note" in line["config"]


def test_comparator_failure_keeps_the_line():
    line = bench.assemble_nranks_line(8, 1, 20, 5, _t(), 9e-6, [], 1 << 24, 128 << 20, TILING, (None, None, "n"),
                                      {"error": "RuntimeError: boom", "returncode": 1})
    assert line["value"] > 0 and line["extra"]["rccl_comparator"]["error"].startswith("RuntimeError")
    json.dumps(line)


class _FakeLib:
    """Stands in for libmpi.so in rccl_comparator: MPI_Bcast of the port is a no-op at one rank."""

    def MPI_Bcast(self, *a):
        return 0


def test_comparator_child_failure_is_reported_not_raised():
    """The real child process, on a host without a GPU: it fails, and rccl_comparator turns that into
    an error record (the bench line keeps its value)."""
    env_keep = dict(os.environ)
    try:
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
        os.environ["HIP_VISIBLE_DEVICES"] = ""
        rec = bench.rccl_comparator(_FakeLib(), 0x44000000, 0, 1, 2, timeout=120)
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    assert "error" in rec, rec


def _fake_host_record():
    hdr = {"ranks": 8, "cpus_available": 16, "cpus_used": 8, "cores_used": 8, "oversubscribed": False,
           "smt_shared": False, "first_cpu_index": 0, "rank_cpus": list(range(8)), "cgroup_cpu_quota": None}
    rows = [{"bytes": b, "lat_us": 0.3 * (1 + b / 1e4), "busbw_GBps": 5.0, "ok": True, "iters": 10, "yields": 0,
             "throttled": 0, "throttled_us": 0} for b in (8, 1 << 20, 64 << 20)]
    out = ("JSONHDR " + json.dumps(hdr) + "\n" + 'JSONSTREAM {"triad_GBps": 123.4, "ranks": 8}\n' +
           "".join("JSON " + json.dumps(r) + "\n" for r in rows))
    rec = bench.host_allreduce_record(out)
    rec["what"] = "w"
    return rec


def test_host_record_parsing():
    rec = _fake_host_record()
    assert rec["cores"] == 8 and rec["cpus_available"] == 16 and rec["placement"] == "8 ranks pinned 1/core"
    assert rec["dram_triad_GBps"] == 123.4
    assert bench.host_allreduce_record("JSON {}\n".replace("{}", '{"bytes": 8}'))["error"]


def _run_host(args, cpus=None):
    cmd = ([shutil.which("taskset"), "-c", cpus] if cpus else []) + [HOST_AR] + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    hdr = next(json.loads(l[8:]) for l in out.stdout.splitlines() if l.startswith("JSONHDR "))
    rows = [json.loads(l[5:]) for l in out.stdout.splitlines() if l.startswith("JSON ")]
    return hdr, rows, out.stderr


needs_host = pytest.mark.skipif(not os.path.exists(HOST_AR) or shutil.which("taskset") is None,
                                reason="oracle/host_allreduce not built or no taskset")


@needs_host
def test_host_allreduce_flags_oversubscription():
    """`taskset -c 0-3 host_allreduce -n 8`: 4 distinct CPUs, oversubscribed, a warning on stderr."""
    if len(os.sched_getaffinity(0)) < 4 or not {0, 1, 2, 3} <= os.sched_getaffinity(0):
        pytest.skip("needs CPUs 0-3 in this process's mask")
    hdr, rows, err = _run_host(["-n", "8", "-m", "8:64", "-c", "-i", "20", "-T", "0.2"], cpus="0-3")
    assert hdr["cpus_available"] == 4 and hdr["cpus_used"] == 4 and hdr["oversubscribed"] is True
    assert sorted(set(hdr["rank_cpus"])) == [0, 1, 2, 3] and len(hdr["rank_cpus"]) == 8
    assert "oversubscribed" in err
    assert all(r["ok"] for r in rows) and all("yields" in r for r in rows)


@needs_host
def test_host_allreduce_distinct_cpus_when_they_fit():
    avail = sorted(os.sched_getaffinity(0))
    n = min(4, len(avail))
    hdr, rows, _ = _run_host(["-n", str(n), "-m", "8:4096", "-c", "-i", "20", "-T", "0.2", "-B", "0.2"])
    assert hdr["cpus_used"] == n and hdr["oversubscribed"] is False
    assert set(hdr["rank_cpus"]) <= set(avail) and len(set(hdr["rank_cpus"])) == n
    assert all(r["ok"] for r in rows)


def _fake_sysfs(root, l3_of, core_of=None):
    """A sysfs CPU tree describing CPU c as core core_of[c] (default c) in L3 domain l3_of[c]."""
    for c, l3 in enumerate(l3_of):
        d = root / f"cpu{c}"
        (d / "topology").mkdir(parents=True)
        (d / "cache" / "index3").mkdir(parents=True)
        (d / "topology" / "core_id").write_text(str(core_of[c] if core_of else c))
        (d / "topology" / "physical_package_id").write_text("0")
        (d / "cache" / "index3" / "id").write_text(str(l3))
    return str(root)


def _run_host_env(args, env):
    out = subprocess.run([HOST_AR] + args, capture_output=True, text=True, timeout=120, env=dict(os.environ, **env))
    assert out.returncode == 0, out.stderr
    return next(json.loads(l[8:]) for l in out.stdout.splitlines() if l.startswith("JSONHDR "))


@needs_host
@pytest.mark.parametrize("l3_of,n,want_dom,want_cpus", [
    ([0, 0, 0, 0, 1, 1, 1, 1], 4, 1, [0, 1, 2, 3]),     # both domains hold 4 cores: one of them, consecutive
    ([0, 0, 0, 1, 1, 1, 1, 1], 4, 1, [3, 4, 5, 6]),     # domain 0 has 3 cores: the 5-core domain
    ([0, 0, 0, 0, 1, 1, 1, 1], 8, 2, list(range(8))),   # 8 ranks need both domains
])
def test_host_allreduce_bunches_ranks_on_one_l3_domain(tmp_path, l3_of, n, want_dom, want_cpus):
    """configs[0]'s ranks on consecutive physical cores of one L3 domain
    (MVAPICH2's default hybrid-bunch binding, hwloc_bind.c:3541-3543) whenever the mask allows
    it; the row names each rank's L3 domain and how many domains were used."""
    if sorted(os.sched_getaffinity(0))[:8] != list(range(8)):
        pytest.skip("needs CPUs 0-7 in this process's mask")
    hdr = _run_host_env(["-n", str(n), "-m", "8:64", "-i", "5", "-T", "0.1"],
                        {"HOST_AR_SYSFS": _fake_sysfs(tmp_path, l3_of)})
    assert hdr["placement_policy"] == "l3-bunch" and hdr["l3_domains_used"] == want_dom
    assert len(set(hdr["rank_l3"])) == want_dom
    if l3_of.count(0) == 4 and n == 4:  # two eligible domains: the idler one (this host's load decides)
        assert hdr["rank_cpus"] in ([0, 1, 2, 3], [4, 5, 6, 7])
    else:
        assert hdr["rank_cpus"] == want_cpus


@needs_host
def test_host_allreduce_l3_bunch_puts_smt_siblings_last(tmp_path):
    """4 cores x 2 threads in one domain (CPU c and c + 4 are siblings): 4 ranks take 4 cores."""
    if sorted(os.sched_getaffinity(0))[:8] != list(range(8)):
        pytest.skip("needs CPUs 0-7 in this process's mask")
    hdr = _run_host_env(["-n", "4", "-m", "8:64", "-i", "5", "-T", "0.1"],
                        {"HOST_AR_SYSFS": _fake_sysfs(tmp_path, [0] * 8, [0, 1, 2, 3, 0, 1, 2, 3])})
    assert hdr["cores_used"] == 4 and hdr["smt_shared"] is False and hdr["l3_domains_used"] == 1


@needs_host
def test_host_allreduce_real_topology_uses_one_domain_when_it_fits():
    """On this machine's own sysfs: when one L3 domain of the mask holds >= 8 physical cores,
    8 ranks use exactly one domain."""
    mask = sorted(os.sched_getaffinity(0))
    cores = {}
    for c in mask:
        try:
            l3 = open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/id").read().strip()
            core = open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id").read().strip()
        except OSError:
            pytest.skip("no L3 ids in sysfs")
        cores.setdefault(l3, set()).add(core)
    hdr = _run_host_env(["-n", "8", "-m", "8:64", "-i", "5", "-T", "0.1"], {})
    if max(len(v) for v in cores.values()) >= 8:
        assert hdr["l3_domains_used"] == 1
    assert len(hdr["rank_l3"]) == 8


def test_osu_sweep_library_exports_its_entry():
    """bench.py's N > 1 sweep loads tools/osu/libosu_coll.so into its ranks (no second process per
    GPU) and calls osu_coll_main; the library must exist after build() and export it."""
    import ctypes
    so = os.path.join(ROOT, "tools", "osu", "libosu_coll.so")
    if not os.path.exists(so):
        pytest.skip("tools/osu not built")
    assert hasattr(ctypes.CDLL(so), "osu_coll_main")


def test_sweep_without_library_reports_instead_of_raising(monkeypatch):
    monkeypatch.setattr(bench, "ROOT", "/nonexistent")
    assert "error" in bench.osu_sweep(None, 0x44000000, 0, 2)
