"""The reference's own collective tests (MPICH test/mpi/coll shipped with MVAPICH2 2.3.7:
allred2-6, allredmany, uoplong, redscat2/3, red_scat_block2, redscatblk3, reduce, allgather2/3,
bcasttest, bcastzerotype, op_commutative, red3/4, longuser, coll8-10, coll12, iallred and the
nonblocking2 calls this library provides), restated as one C program
(tests/mpich_coll/coll_suite.c) that links the drop-in libmpi.so like an application and checks
each test's own closed-form answers.  Run with device-memory operands (the accelerated path)
and with host-memory operands, at several rank counts sharing the one GPU, on one node and on
emulated nodes (mv2run --nodes)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITE = os.path.join(ROOT, "tests", "mpich_coll")
EXE = os.path.join(SUITE, "coll_suite")
CASES = ["allred2", "allred3", "allred4", "allred5", "allred6", "allredmany", "uoplong", "redscat2",
         "red_scat_block2", "redscat3", "redscatblk3", "reduce", "allgather2", "allgather3", "bcasttest",
         "bcastzerotype", "op_commutative", "red3", "red4", "longuser", "coll8", "coll9", "coll10", "coll12", "iallred",
         "nonblocking2"]


def _exe():
    src = os.path.join(SUITE, "coll_suite.c")
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(src):
        subprocess.run(["make", "-C", SUITE], check=True, capture_output=True)
    return EXE


def run_suite(n, mem, cases=(), timeout=300, nodes=1):
    cmd = [sys.executable, "-m", "mvapich2_amd.mv2run", "-n", str(n), "--nodes", str(nodes), "--share-gpu",
           "--timeout", str(timeout - 10), _exe(), mem, *cases]
    env = dict(os.environ, MV2AMD_TIMEOUT_S="30", PYTHONPATH=ROOT)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout, p.stderr


def test_suite_lists_every_case():
    """the Python list and the C program's case table agree (CPU: reads the source)"""
    src = open(os.path.join(SUITE, "coll_suite.c")).read()
    table = src[src.index("kCases[] = {"):]
    for c in CASES:
        assert f'{{"{c}", t_{c}}}' in table, c


@pytest.mark.gpu
@pytest.mark.parametrize("mem,n,nodes", [("device", 2, 1), ("device", 3, 1), ("device", 4, 1), ("device", 8, 1),
                                         ("host", 2, 1), ("host", 5, 1),
                                         # emulated nodes: the multi-node schedules under the same tests
                                         ("device", 4, 2), ("device", 6, 3), ("device", 8, 2), ("host", 4, 2)])
def test_reference_coll_suite(mem, n, nodes):
    rc, out, err = run_suite(n, mem, nodes=nodes)
    lines = [ln.split() for ln in out.splitlines() if ln.startswith(mem + " ")]
    per_case = {ln[1]: int(ln[2]) for ln in lines if ln[1] != "TOTAL"}
    assert rc == 0 and set(per_case) == set(CASES) and not any(per_case.values()), (rc, out, err[-3000:])
