#!/usr/bin/env python3
"""Why the entity pass's gradient part (no Adam) runs 0.044 ms when launched
back to back but 0.147 ms inside the training step (r05 kernel traces): the
ENTITY phase timed (a) repeated on one batch, (b) each time right after the
ROWS phase of the same batch, (c) after an unrelated 1 GB stream that
flushes the caches, with HIP events around the ENTITY launch alone.

    python tools/entity_gather_probe.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEModel, _lib, ops, synth  # noqa: E402

E, R, D, B, N = 14951, 1345, 1000, 1024, 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = KGEModel("RotatE", E, R, D, 24.0, True, False).to(dev)
    desc = model.desc()
    pos, neg, w = synth.kge_batch(5, B, N, E, R)
    pos, neg, w = torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev)
    ge = torch.zeros_like(model.entity_embedding)
    gr = torch.zeros_like(model.relation_embedding)
    losses = torch.zeros(5, device=dev)
    kw = dict(adversarial=True, temperature=1.0, uni_weight=False, regularization=0.0, grad_entity=ge,
              grad_relation=gr, grad_modulus=None, losses=losses)
    flush = torch.empty(256 * 1024 * 1024, device=dev)

    def rows():
        ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ROWS, **kw)

    def ent():
        ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ENTITY, **kw)

    def run(before):
        rows()
        ent()
        torch.cuda.synchronize()
        tot = 0.0
        for _ in range(a.reps):
            if before:
                before()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ent()
            e1.record()
            e1.synchronize()
            tot += e0.elapsed_time(e1)
        return tot / a.reps

    out = {}
    ref = None
    for name, before in (("repeated", None), ("after_rows", rows), ("after_flush", lambda: flush.add_(1.0)),
                         ("repeated_again", None), ("after_rows_again", rows)):
        out[name + "_ms"] = run(before)
        g = ge.clone()
        if ref is None:
            ref = g
        out[name + "_same_grad"] = bool(torch.equal(g, ref))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
