#!/usr/bin/env python3
"""Host-side split of one config-3 ranking pass (`rank_queries_both`, wn18rr
shape, DistMult): time before the C call (Python preparation), the C call
itself (kge_rank_filtered_both: host work + launches) and after it (copy
queueing, the wait, read-back) — wall medians over --passes after a warm-up.

    python3 tools/rank_host_split.py [--model DistMult] [--passes 30]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEModel, ops, synth  # noqa: E402
from knowledgegraphembedding_amd.filters import FilterIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="DistMult", choices=("DistMult", "ComplEx"))
    ap.add_argument("--passes", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    Ew, Rw, ntrue, ntest, d = 40943, 11, 93003, 3134, 500
    h, r, t = synth.randint(901, (ntrue,), Ew), synth.randint(902, (ntrue,), Rw), synth.randint(903, (ntrue,), Ew)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(904, (ntest,), len(true))]
    index = FilterIndex(true, Ew, Rw)
    cplx = a.model == "ComplEx"
    torch.manual_seed(0)
    m = KGEModel(a.model, Ew, Rw, d, 12.0, cplx, cplx).to(dev)
    marks = {}
    orig = ops.rank_filtered_both

    def timed(*args, **kw):
        marks["in"] = time.perf_counter()
        out = orig(*args, **kw)
        marks["out"] = time.perf_counter()
        return out

    ops.rank_filtered_both = timed
    for _ in range(3):
        m.rank_queries_both(test, index)
    torch.cuda.synchronize()
    pre, call, post, wall = [], [], [], []
    for _ in range(a.passes):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.rank_queries_both(test, index)
        t3 = time.perf_counter()
        pre.append(marks["in"] - t0)
        call.append(marks["out"] - marks["in"])
        post.append(t3 - marks["out"])
        wall.append(t3 - t0)
    med = lambda x: float(np.median(x)) * 1e3  # noqa: E731
    print(json.dumps({"model": a.model, "wall_ms": med(wall), "python_before_call_ms": med(pre),
                      "c_call_ms": med(call), "after_call_ms": med(post)}), flush=True)


if __name__ == "__main__":
    main()
