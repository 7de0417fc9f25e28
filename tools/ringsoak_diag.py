# one-off diagnosis driver (not a test; tools/runs/run_r05ab.sh ... run_r05ak.sh): the multi-node
# flat-ring allreduce (>= 2 MiB over emulated nodes) many times through mp_gpu_worker's soak, every
# result checked; the workers' logs go to <out>/rank<r>.log
import json, os, socket, subprocess, sys, tempfile, uuid, pathlib
import numpy as np
ROOT = os.getcwd()
n, ppn, calls, seed = (int(a) for a in sys.argv[1:5])
case = {"id": "rs", "kind": "soak", "calls": calls, "seed": seed, "kinds": ["allreduce"],
        "sizes": [524288 + 3, 700003, 1 << 20], "detail": int(os.environ.get("DIAG_DETAIL", "1")),
        "sync_upload": int(os.environ.get("DIAG_SYNC_UPLOAD", "0")), "check_sb": int(os.environ.get("DIAG_CHECK_SB", "0"))}
d = pathlib.Path(tempfile.mkdtemp())
(d / "spec.json").write_text(json.dumps({"cases": [case]}))
(d / "out").mkdir()
so = socket.socket(); so.bind(("127.0.0.1", 0)); port = so.getsockname()[1]; so.close()
jobid = "d" + uuid.uuid4().hex[:12]
procs = []
for r in range(n):
    env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r % ppn), LOCAL_WORLD_SIZE=str(ppn),
               MV2AMD_JOBID=jobid, MV2AMD_TIMEOUT_S="30", MV2AMD_BOOT_ADDR="127.0.0.1", MV2AMD_BOOT_PORT=str(port),
               MV2AMD_NSHARE=str(n))
    env.pop("MV2AMD_DEVICE", None)
    log = open(d / f"rank{r}.log", "w")
    procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_gpu_worker.py"), str(d / "spec.json"),
                                   str(d / "out")], env=env, stdout=log, stderr=subprocess.STDOUT))
rcs = [p.wait(timeout=380) for p in procs]
out = sys.argv[5] if len(sys.argv) > 5 else None
logs = {r: open(d / f"rank{r}.log").read() for r in range(n)}
if out:
    for r in range(n):
        open(f"{out}_rank{r}.log", "w").write(logs[r])
res = [np.load(d / "out" / f"rs_r{r}.npy").tolist() if rcs[r] == 0 else [] for r in range(n)]
# ranks whose MPI_Init refused the job (more than 8 processes on one GPU, runtime/world.cpp)
refused = [r for r in range(n) if rcs[r] != 0 and "processes share one GPU, more than the 8" in logs[r]]
print(json.dumps({"n": n, "ppn": ppn, "rcs": rcs, "refused": refused, "env_p2p": os.environ.get("MV2AMD_P2P_KERNEL_COPY"),
                  "sync_upload": os.environ.get("DIAG_SYNC_UPLOAD"), "per_rank": res}), flush=True)
