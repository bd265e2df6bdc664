#!/usr/bin/env python3
"""Per-launch HBM-side traffic of a kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py gpurun_out/prof [--kernel k_row] [-o out.json]

Reads <dir>/pmc_FETCH_SIZE/*counter_collection.csv and
<dir>/pmc_WRITE_SIZE/*counter_collection.csv (one counter per pass — they do
not fit one pass on gfx950) and applies MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced stream, so it is doubled; WRITE_SIZE is
exact for 16-B stores.  Infinity-Cache hits are counted (not excluded), so
this is fabric-side traffic.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def per_kernel(path: str, counter: str):
    files = glob.glob(os.path.join(path, f"pmc_{counter}", "*counter_collection.csv"))
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_row")
    ap.add_argument("-o", "--out", default=None)
    a = ap.parse_args()
    fetch = per_kernel(a.dir, "FETCH_SIZE")
    write = per_kernel(a.dir, "WRITE_SIZE")
    summary = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        summary[name] = {"launches": max(len(f), len(w)), "fetch_kib_raw": fk, "write_kib": wk,
                         "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0}
    # exact kernel name (template arguments aside): "k_row" must not pick up "k_row_epi"
    sel = {k: v for k, v in summary.items() if re.search(r"(^|[:\s])" + re.escape(a.kernel) + r"[<(]", k)}
    tot_l = sum(v["launches"] for v in sel.values())
    main_bytes = (sum(v["hbm_bytes_per_launch"] * v["launches"] for v in sel.values()) / tot_l) if tot_l else None
    out = {"kernel": a.kernel, "hbm_bytes_per_launch": main_bytes,
           "method": "(2*FETCH_SIZE + WRITE_SIZE) KiB * 1024, separate --pmc passes (MI355X_MICROARCH.md HBM)",
           "kernels": sel}
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s)
    print(s)


if __name__ == "__main__":
    main()
