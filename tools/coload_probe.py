"""Code-object load time of a libmpi.so build (the 68 MB fatbin).

HIP_ENABLE_DEFERRED_LOADING=0 makes the HIP runtime start when the library's code objects are
registered (at dlopen) and load every one of them then; with deferred loading (the default) the
runtime starts at the first HIP call (mv2h_device_count) and loads nothing.  dlopen + first call
therefore costs runtime start + code-object load in the first mode and runtime start in the second.  Each configuration runs in a
fresh process, `reps` times; the load time is the difference of the medians.  Works the same for
builds that predate the library's own MPI_Init timing.
Usage: python tools/coload_probe.py LIB [LIB ...]  -> one JSON line per library"""
import json
import os
import statistics
import subprocess
import sys

CHILD = r'''
import ctypes, sys, time
t0 = time.perf_counter()
L = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
t1 = time.perf_counter()
n = L.mv2h_device_count()
t2 = time.perf_counter()
print((t1 - t0) * 1e3, (t2 - t1) * 1e3, n)
'''


def one(lib, deferred):
    env = dict(os.environ, HIP_ENABLE_DEFERRED_LOADING=str(deferred))
    out = subprocess.run([sys.executable, "-c", CHILD, lib], env=env, capture_output=True, text=True, timeout=120)
    dl, first, n = out.stdout.split()
    assert int(n) > 0, out.stderr
    return float(dl), float(first)


def main():
    reps = 5
    for lib in sys.argv[1:]:
        fat = None
        try:
            r = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", "--wide", lib], capture_output=True, text=True)
            for line in r.stdout.splitlines():
                if ".hip_fatbin" in line:
                    f = line.split()
                    fat = int(f[f.index("PROGBITS") + 3], 16)
        except Exception:
            pass
        res = {}
        for d in (1, 0):
            xs = [one(lib, d) for _ in range(reps)]
            res[d] = (statistics.median(x[0] for x in xs), statistics.median(x[1] for x in xs))
        lazy, eager = res[1][0] + res[1][1], res[0][0] + res[0][1]
        print(json.dumps({"lib": lib, "hip_fatbin_bytes": fat,
                          "dlopen_plus_first_call_ms_deferred": round(lazy, 2),
                          "dlopen_plus_first_call_ms_eager": round(eager, 2),
                          "code_object_load_ms": round(eager - lazy, 2), "reps": reps}), flush=True)


if __name__ == "__main__":
    main()
