"""mv2run — single-node launcher for programs linked against mvapich2_amd's
libmpi.so (the role of the reference's mpirun_rsh / mpiexec.hydra for one
node, src/pm/mpirun/mpirun_rsh.c).  Starts N ranks as child processes with
MV2_COMM_WORLD_{RANK,SIZE,LOCAL_RANK,LOCAL_SIZE} and a per-launch job id (the
key of the /dev/shm control segment), waits for all of them and exits with
the first non-zero status.  Ranks are never exec'd over an existing process.

    python -m mvapich2_amd.mv2run -n 8 ./tools/osu/osu_coll -c allreduce -m 8:1073741824
    python -m mvapich2_amd.mv2run -n 2 --share-gpu python bench.py --gpus 2
    python -m mvapich2_amd.mv2run -n 4 --nodes 2 --share-gpu ...   # two emulated nodes

--nodes K splits the ranks node-major into K groups that behave as separate nodes (own control
segment and IPC world each; the node leaders link over TCP on 127.0.0.1, runtime/internode.cpp),
which rehearses a multi-node job on one host.
"""
import argparse
import os
import socket
import subprocess
import sys
import time
import uuid


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mv2run")
    ap.add_argument("-n", "--np", type=int, required=True, help="number of ranks")
    ap.add_argument("--share-gpu", action="store_true", help="every rank uses GPU 0 (tests / protocol runs)")
    ap.add_argument("--timeout", type=float, default=0, help="kill the job after this many seconds")
    ap.add_argument("--nodes", type=int, default=1, help="emulate this many nodes (ranks split node-major)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if not a.cmd:
        ap.error("missing command")
    job = "r" + uuid.uuid4().hex[:12]
    if a.nodes < 1 or a.np % a.nodes:
        ap.error("--nodes must divide -n")
    ppn = a.np // a.nodes
    extra = {}
    if a.nodes > 1:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        extra = {"MV2AMD_BOOT_ADDR": "127.0.0.1", "MV2AMD_BOOT_PORT": str(s.getsockname()[1])}
        if a.share_gpu:
            extra["MV2AMD_NSHARE"] = str(a.np)  # the nodes' ranks all share GPU 0
        s.close()
    procs = []
    for r in range(a.np):
        lr = r % ppn
        env = dict(os.environ, MV2_COMM_WORLD_RANK=str(r), MV2_COMM_WORLD_SIZE=str(a.np),
                   MV2_COMM_WORLD_LOCAL_RANK=str(lr), MV2_COMM_WORLD_LOCAL_SIZE=str(ppn), MV2AMD_JOBID=job,
                   RANK=str(r), WORLD_SIZE=str(a.np), LOCAL_RANK=str(lr), LOCAL_WORLD_SIZE=str(ppn), **extra)
        if a.share_gpu:
            env["MV2AMD_DEVICE"] = "0"
        procs.append(subprocess.Popen(a.cmd, env=env))
    t0 = time.time()
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            for p in procs:
                if p.poll() not in (None, 0) and rc == 0:
                    rc = p.returncode
            if rc or (a.timeout and time.time() - t0 > a.timeout):
                rc = rc or 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    for p in procs:
        if p.returncode and not rc:
            rc = p.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
