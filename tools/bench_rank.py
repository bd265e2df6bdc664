#!/usr/bin/env python3
"""Filtered-ranking benchmark — BASELINE config 3: DistMult + ComplEx on the
wn18rr shape (E=40943, R=11) d=500, all 3134 test triples × both directions
(6268 queries) through KGEModel.rank_queries (kge_rank_filtered).

Synthetic graph: 93,003 true triples (wn18rr's train+valid+test count) drawn
uniformly; tables U(-range, range).  `--shape fb15k`: the FB15k entity /
relation counts (E=14951, R=1345) with 592,213 true triples and 4096 test
triples, the shape best_config.sh:3 evaluates RotatE / TransE on.  Reports
queries/s and the wall time of the whole pass; for the split-bf16 MFMA path
the roofline is the bf16 flops the matrix cores issue (three bf16 products
per fp32 product, tile padding included) over the pass's wall time against
the 2.5 PF bf16 dense spec — as bench.py's `ranking` block.
--path tile times the register-tiled VALU kernel instead of the MFMA tile for
DistMult/ComplEx, --path scan the per-pair wave-reduction scan.

    python tools/bench_rank.py [--models DistMult ComplEx RotatE] [--reps 3] [--cpu-sample 8]
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

SHAPES = {"wn18rr": (40943, 11, 93003, 3134, (901, 902, 903, 904)),
          "fb15k": (14951, 1345, 592213, 4096, (911, 912, 913, 914))}
BF16_PEAK_TF = 2500.0
DIMS = {"DistMult": (False, False), "ComplEx": (True, True), "RotatE": (True, False), "TransE": (False, False),
        "pRotatE": (False, False)}


def rank_path(name, K, path="auto"):
    """Which fast pass kge_rank_filtered_ex runs (kge_capi.hip rank_path)."""
    red = K // 2 if name in ("RotatE", "ComplEx") else K
    mfma_ok = name in ("DistMult", "ComplEx") and K % 4 == 0
    if path == "mfma" or (path == "auto" and name in ("DistMult", "ComplEx")):
        return "mfma-split-bf16"
    if path == "mfma32" or (path == "auto" and mfma_ok):
        return "mfma"
    if path in ("auto", "tile") and red % 4 == 0:
        return "valu-tile"
    return "valu-scan"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["DistMult", "ComplEx"])
    ap.add_argument("-d", "--hidden_dim", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--path", default="auto", choices=("auto", "mfma", "mfma32", "tile", "scan"))
    ap.add_argument("--cpu-sample", type=int, default=0, help="queries timed through the CPU oracle (0: skip)")
    ap.add_argument("--shape", default="wn18rr", choices=sorted(SHAPES))
    ap.add_argument("--gamma", type=float, default=12.0)
    ap.add_argument("--rank-trig", default="reference", choices=("reference", "device"),
                    help="RotatE / pRotatE: the reference's host trig (exact ranks) or device trig")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    E, R, NTRUE, NTEST, seeds = SHAPES[a.shape]
    h = synth.randint(seeds[0], (NTRUE,), E)
    r = synth.randint(seeds[1], (NTRUE,), R)
    t = synth.randint(seeds[2], (NTRUE,), E)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(seeds[3], (NTEST,), len(true))]
    index = FilterIndex(true, E, R)
    out = []
    for name in a.models:
        de, dr = DIMS[name]
        torch.manual_seed(0)
        m = KGEModel(name, E, R, a.hidden_dim, a.gamma, de, dr).to(dev)
        m.rank_trig = a.rank_trig
        K = m.entity_dim
        times = []
        ranks = None
        for rep in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rh, _, lh = m.rank_queries(test, index, "head-batch", path=a.path, listed=True)
            rt, _, lt = m.rank_queries(test, index, "tail-batch", path=a.path, listed=True)
            torch.cuda.synchronize()
            if rep:
                times.append(time.perf_counter() - t0)
            ranks = np.concatenate([rh, rt])
        dt = min(times)
        nq = 2 * NTEST
        flops = 2.0 * nq * E * K
        res = {"model": name, "shape": a.shape, "entities": E, "hidden_dim": a.hidden_dim, "entity_dim": K, "queries": nq,
               "seconds": dt, "queries_per_s": nq / dt, "candidate_scores_per_s": nq * E / dt,
               "tflops": flops / dt / 1e12,
               "path": rank_path(name, K, a.path), "rank_trig": a.rank_trig,
               "pair_terms_per_s": nq * E * (K // 2 if name in ("RotatE", "ComplEx") else K) / dt,
               "mrr": float(np.mean(1.0 / ranks)),
               "listed_per_query": float(np.mean(np.concatenate([lh, lt])))}
        if res["path"].startswith("mfma-split-bf16"):
            pad = lambda x, m: -(-x // m) * m  # noqa: E731
            kp = pad(K, 16)
            issued = 2.0 * 3 * 2 * pad(NTEST, 128) * pad(E, 128) * kp  # three bf16 products per fp32 one
            res["roofline"] = {"bound": "mfma", "achieved": issued / dt / 1e12, "peak": BF16_PEAK_TF,
                               "unit": "TFLOP/s", "frac": issued / dt / 1e12 / BF16_PEAK_TF,
                               "what": "issued bf16 MFMA flops / whole-pass wall time / 2.5 PF bf16 dense spec"}
        if a.cpu_sample:
            from oracle import kge_oracle as O
            ent = m.entity_embedding.detach().cpu()
            rel = m.relation_embedding.detach().cpu()
            mod = m.modulus.detach().cpu() if name == "pRotatE" else None
            g, rng = m._host_scalars()
            t0 = time.perf_counter()
            orc = O.filtered_ranks(name, ent, rel, mod, test[:a.cpu_sample], true, "tail-batch", g, rng)
            cdt = time.perf_counter() - t0
            res["cpu_oracle_queries_per_s"] = a.cpu_sample / cdt
            res["cpu_rank_match"] = int((orc["rank_argsort"] == ranks[NTEST:NTEST + a.cpu_sample]).sum())
        out.append(res)
        print(json.dumps(res), flush=True)
    return out


if __name__ == "__main__":
    main()
