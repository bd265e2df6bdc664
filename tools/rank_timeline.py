#!/usr/bin/env python3
"""The config-3 ranking pass exactly as bench.py's `ranking` block runs it
(KGEModel.rank_queries_both: both directions queued, one read-back; wn18rr
shape, synthetic filter graph), repeated, for a rocprofv3 kernel trace of
where the non-tile time goes.

    rocprofv3 --kernel-trace ... -- python3 tools/rank_timeline.py [--model DistMult] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEModel, synth  # noqa: E402
from knowledgegraphembedding_amd.filters import FilterIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="DistMult", choices=("DistMult", "ComplEx", "RotatE", "TransE"))
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    Ew, Rw, ntrue, ntest, d = 40943, 11, 93003, 3134, 500
    h, r, t = synth.randint(901, (ntrue,), Ew), synth.randint(902, (ntrue,), Rw), synth.randint(903, (ntrue,), Ew)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(904, (ntest,), len(true))]
    index = FilterIndex(true, Ew, Rw)
    cplx = a.model == "ComplEx"
    torch.manual_seed(0)
    m = KGEModel(a.model, Ew, Rw, d, 12.0, cplx or a.model == "RotatE", cplx).to(dev)
    times = []
    for _ in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.rank_queries_both(test, index)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    print(json.dumps({"model": a.model, "ms": [round(x * 1e3, 3) for x in times]}), flush=True)


if __name__ == "__main__":
    main()
