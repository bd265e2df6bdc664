#!/usr/bin/env python3
"""Cross-check the three filtered-ranking paths on the config-3 shape.

Runs kge_rank_filtered through the MFMA tile, the register tile and the wave
scan (KGE_RANK_MFMA / KGE_RANK_TILE switches, read per call) on the same
synthetic wn18rr-shaped graph, repeats the MFMA path for determinism, and for
every query where two paths disagree reports the fp64 gap between the true
entity's score and the nearest competitor (a rank may legitimately differ
only where that gap is below fp32 rounding of the scores).

    python tools/rank_consistency.py [--models DistMult ComplEx] [--queries 1024]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEModel, synth  # noqa: E402
from knowledgegraphembedding_amd.filters import FilterIndex  # noqa: E402

E, R, NTRUE = 40943, 11, 93003
PATHS = {"mfma": {"KGE_RANK_MFMA": "1", "KGE_RANK_TILE": "1"}, "tile": {"KGE_RANK_MFMA": "0", "KGE_RANK_TILE": "1"},
         "scan": {"KGE_RANK_MFMA": "0", "KGE_RANK_TILE": "0"}}


def scores64(m, q, mode):
    """fp64 scores of every candidate for the queries q (DistMult / ComplEx)."""
    ent = m.entity_embedding.detach().double().cpu().numpy()
    rel = m.relation_embedding.detach().double().cpu().numpy()
    h, r, t = q[:, 0], q[:, 1], q[:, 2]
    if m.model_name == "DistMult":
        qv = rel[r] * (ent[t] if mode == "head-batch" else ent[h])
        return qv @ ent.T
    d = ent.shape[1] // 2
    re_r, im_r = rel[r][:, :d], rel[r][:, d:]
    x = ent[t] if mode == "head-batch" else ent[h]
    re_x, im_x = x[:, :d], x[:, d:]
    if mode == "head-batch":
        qa, qb = re_r * re_x + im_r * im_x, re_r * im_x - im_r * re_x
    else:
        qa, qb = re_x * re_r - im_x * im_r, re_x * im_r + im_x * re_r
    return qa @ ent[:, :d].T + qb @ ent[:, d:].T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["DistMult", "ComplEx"])
    ap.add_argument("--queries", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    tr = np.unique(np.stack([synth.randint(901, (NTRUE,), E), synth.randint(902, (NTRUE,), R),
                             synth.randint(903, (NTRUE,), E)], 1), axis=0)
    test = tr[synth.randint(904, (a.queries,), len(tr))]
    index = FilterIndex(tr, E, R)
    true_set = {tuple(x) for x in tr.tolist()}
    for name in a.models:
        torch.manual_seed(0)
        de = dr = name == "ComplEx"
        m = KGEModel(name, E, R, 500, 12.0, de, dr).to(dev)
        for mode in ("head-batch", "tail-batch"):
            ranks = {}
            for path, env in PATHS.items():
                os.environ.update(env)
                ranks[path] = m.rank_queries(test, index, mode)[0]
            os.environ.update(PATHS["mfma"])
            again = m.rank_queries(test, index, mode)[0]
            diff = np.nonzero((ranks["mfma"] != ranks["tile"]) | (ranks["mfma"] != ranks["scan"]))[0]
            gaps = []
            if len(diff):
                s = scores64(m, test[diff], mode)
                for k, qi in enumerate(diff):
                    h, r, t = test[qi].tolist()
                    tid = h if mode == "head-batch" else t
                    row = s[k]
                    keep = np.array([not ((e, r, t) if mode == "head-batch" else (h, r, e)) in true_set
                                     for e in range(E)])
                    keep[tid] = False
                    gaps.append(float(np.min(np.abs(row[keep] - row[tid])) / max(abs(row[tid]), 1e-30)))
            print(json.dumps({"model": name, "mode": mode, "queries": int(len(test)),
                              "mfma_deterministic": bool(np.array_equal(again, ranks["mfma"])),
                              "mfma_vs_tile_diff": int((ranks["mfma"] != ranks["tile"]).sum()),
                              "mfma_vs_scan_diff": int((ranks["mfma"] != ranks["scan"]).sum()),
                              "tile_vs_scan_diff": int((ranks["tile"] != ranks["scan"]).sum()),
                              "max_rank_delta": int(max((np.abs(ranks["mfma"] - ranks[p]).max() for p in PATHS),
                                                        default=0)),
                              "max_rel_gap_where_differ": max(gaps) if gaps else None}), flush=True)


if __name__ == "__main__":
    main()
