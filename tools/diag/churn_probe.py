"""Diagnosis (not a test): does uploading freshly allocated pageable host memory between collective
calls stall a device wait on a slot its peer has long overwritten (profiles/r06/r06u, r06al, r06am)?
Runs tests/mp_gpu_worker.py's upload_churn case: n ranks on the one GPU, small allreduces, `bytes` of
fresh pageable memory uploaded (hipMemcpy) and freed between calls ("fresh") or one array kept
("kept").  usage: churn_probe.py n calls bytes mode [churn ranks, comma-separated | all]"""
import json
import os
import re
import sys
import tempfile
import pathlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from tests.test_gpu_collectives_mp import run_workers  # noqa: E402


def main():
    n, calls, nbytes, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    ranks = list(range(n)) if len(sys.argv) < 6 or sys.argv[5] == "all" else [int(v) for v in sys.argv[5].split(",")]
    case = {"id": "churn", "kind": "upload_churn", "calls": calls, "churn_bytes": nbytes, "mode": mode,
            "churn_ranks": ranks}
    with tempfile.TemporaryDirectory() as d:
        got = run_workers(n, [case], pathlib.Path(d), timeout=400, extra_env={"MV2AMD_TIMEOUT_S": "5"}, expect_fail=True)
        res = []
        for r in range(n):
            f = pathlib.Path(d) / "out" / f"churn_r{r}.npy"
            res.append(np.load(f).tolist() if f.exists() else None)
    out = {"n": n, "calls": calls, "bytes": nbytes, "mode": mode, "churn_ranks": ranks,
           "rc": [rc for rc, _ in got], "result": res,
           "timeouts": [bool(re.search("timed out waiting for a peer", log)) for _, log in got]}
    stale = []
    for _, log in got:
        for mm in re.finditer(r"waited for epoch (\d+) from ranks 0x[0-9a-f]+; flags seen:([^;]*);", log):
            ep = int(mm.group(1))
            seen = dict(re.findall(r"r(\d+)=(\d+)", mm.group(2)))
            now = re.search(r"the waited slot now \(host copy\):(.*)", log[mm.end():])
            nowd = dict(re.findall(r"r(\d+)=(\d+)", now.group(1))) if now else {}
            stale += [{"epoch": ep, "rank": k, "seen": int(v), "now": int(nowd.get(k, -1))}
                      for k, v in seen.items() if int(v) < ep]
    out["late_slots"] = stale[:16]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
