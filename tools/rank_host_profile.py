#!/usr/bin/env python3
"""Where the host time of one config-3 ranking pass goes: the wn18rr-shape
`KGEModel.rank_queries_both` (as bench.py's `ranking` block runs it) under
cProfile, after a warm-up, plus the device span of each pass from HIP events
around it — wall − device span is what the host adds.

    python3 tools/rank_host_profile.py [--model DistMult] [--passes 20]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEModel, synth  # noqa: E402
from knowledgegraphembedding_amd.filters import FilterIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="DistMult", choices=("DistMult", "ComplEx"))
    ap.add_argument("--passes", type=int, default=20)
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
    for _ in range(3):
        m.rank_queries_both(test, index)
    torch.cuda.synchronize()
    walls, spans = [], []
    for _ in range(a.passes):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        m.rank_queries_both(test, index)
        e1.record()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        spans.append(e0.elapsed_time(e1))
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(a.passes):
        m.rank_queries_both(test, index)
    prof.disable()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(25)
    print(json.dumps({"model": a.model, "wall_ms_median": float(np.median(walls)),
                      "event_span_ms_median": float(np.median(spans)),
                      "host_ms_median": float(np.median(np.array(walls) - np.array(spans)))}), flush=True)
    print(s.getvalue())


if __name__ == "__main__":
    main()
