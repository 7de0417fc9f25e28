"""The reference's MPI_Pack / MPI_Unpack tests (MPICH test/mpi/datatype shipped with MVAPICH2
2.3.7: simple-pack, transpose-pack, triangular-pack, slice-pack, vecblklen, hvecblklen,
zeroblks, zero-blklen-vector, unpack, structpack2, localpack, pairtype-pack and the zero-count
type tests), restated as one C program (tests/mpich_datatype/dt_suite.c) over the drop-in
libmpi.so and checked against each test's own expected layout — with the operands and pack
buffer in device memory (the device pack kernels) and in host memory."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITE = os.path.join(ROOT, "tests", "mpich_datatype")
EXE = os.path.join(SUITE, "dt_suite")
CASES = ["simple_pack_nested", "simple_pack_contig_vector", "transpose_pack", "triangular_pack", "slice_pack",
         "vecblklen", "hvecblklen", "zeroblks", "zero_blklen_vector", "unpack_nested_indexed", "structpack2",
         "localpack", "pairtype_pack", "zero_count_types"]


def _exe():
    src = os.path.join(SUITE, "dt_suite.c")
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(src):
        subprocess.run(["make", "-C", SUITE], check=True, capture_output=True)
    return EXE


def test_suite_lists_every_case():
    src = open(os.path.join(SUITE, "dt_suite.c")).read()
    table = src[src.index("kCases[] = {"):]
    for c in CASES:
        assert f'{{"{c}", t_{c}}}' in table, c


@pytest.mark.gpu
@pytest.mark.parametrize("mem", ["device", "host"])
def test_reference_datatype_suite(mem):
    cmd = [sys.executable, "-m", "mvapich2_amd.mv2run", "-n", "1", "--share-gpu", "--timeout", "100", _exe(), mem]
    p = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True,
                       timeout=120)
    rows = [ln.split() for ln in p.stdout.splitlines() if ln.startswith(mem + " ")]
    per_case = {r[1]: int(r[2]) for r in rows if r[1] != "TOTAL"}
    assert p.returncode == 0 and set(per_case) == set(CASES) and not any(per_case.values()), \
        (p.returncode, p.stdout, p.stderr[-3000:])
