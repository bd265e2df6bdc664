"""Device timeline of KGEModel.rank_queries_both on the bench's config-3
workload (run under rocprofv3 --kernel-trace --memory-copy-trace; the last
call's kernels and copies are then listed by tools/dbg/rank_timeline.py --csv DIR)."""
import argparse
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run():
    import numpy as np
    import torch
    from knowledgegraphembedding_amd import KGEModel, synth
    from knowledgegraphembedding_amd.filters import FilterIndex
    dev = torch.device("cuda", 0)
    Ew, Rw, ntrue, ntest, d = 40943, 11, 93003, 3134, 500
    h, r, t = synth.randint(901, (ntrue,), Ew), synth.randint(902, (ntrue,), Rw), synth.randint(903, (ntrue,), Ew)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(904, (ntest,), len(true))]
    index = FilterIndex(true, Ew, Rw)
    torch.manual_seed(0)
    m = KGEModel("DistMult", Ew, Rw, d, 12.0, False, False).to(dev)
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.rank_queries_both(test, index)
        torch.cuda.synchronize()
        print("call", i, round((time.perf_counter() - t0) * 1e3, 3), "ms", flush=True)
        time.sleep(0.05)  # separates the calls in the trace


def show(d):
    rows = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    for f in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
    rows.sort()
    # last call = after the last gap > 20 ms
    start = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > 20_000_000:
            start = i
    last = rows[start:]
    t0 = last[0][0]
    prev = t0
    for s, e, n in last:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {(s - prev) / 1e3:7.1f}  {n}")
        prev = max(prev, e)
    print("span", (last[-1][1] - t0) / 1e3, "us; busy", sum(e - s for s, e, _ in last) / 1e3, "us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    show(a.csv) if a.csv else run()
