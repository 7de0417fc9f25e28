#!/usr/bin/env python3
"""Split the 8-byte allreduce latency from per-rank rocprofv3 kernel traces
(same GPU clock for every rank when the ranks share one GPU):
  kernel duration        = one-shot kernel begin -> end on a rank
  start skew             = max - min of the ranks' begin times for the same call
  host gap               = end of call k's kernel -> begin of call k+1's kernel on a rank
                           (return from the completion word, Python loop, plan, launch)
Usage: lat_breakdown.py OUT.json trace_rank0.csv trace_rank1.csv ..."""
import csv
import json
import sys

import numpy as np


def load(path):
    rows = [r for r in csv.DictReader(open(path)) if "k_oneshot" in r["Kernel_Name"]]
    return np.array([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows], dtype=np.int64)


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    tr = [load(p) for p in paths]
    k = min(len(t) for t in tr)
    tr = [t[-k:] for t in tr]  # the timed loop is the tail; self-test / warmup launches drop out
    tr = [t[-min(k, 2000):] for t in tr]
    st = np.stack([t[:, 0] for t in tr])
    en = np.stack([t[:, 1] for t in tr])
    dur = (en - st) / 1e3
    skew = (st.max(0) - st.min(0)) / 1e3
    gap = (st[:, 1:] - en[:, :-1]) / 1e3
    period = (st[:, 1:] - st[:, :-1]) / 1e3
    # work after the last rank arrived: end - (last start)
    after_last = (en - st.max(0)) / 1e3
    res = {"ranks": len(tr), "calls": int(st.shape[1]),
           "kernel_us_p50": float(np.median(dur)), "start_skew_us_p50": float(np.median(skew)),
           "kernel_after_last_start_us_p50": float(np.median(after_last)),
           "host_gap_us_p50": float(np.median(gap)), "period_us_p50": float(np.median(period)),
           "kernel_us_mean": float(dur.mean()), "host_gap_us_mean": float(gap.mean()),
           "period_us_mean": float(period.mean())}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
