"""Smoke case under the current env: max |Δ| of the entity/relation grads and losses vs the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from argparse import Namespace
import numpy as np, torch
from knowledgegraphembedding_amd import KGEModel, synth
from oracle import kge_oracle as O
dev = torch.device("cuda", 0)
for (E, R, d, B, n) in ((300, 11, 64, 8, 32), (300, 11, 200, 24, 40), (2000, 30, 100, 64, 32)):
    for mode in ("tail-batch", "head-batch"):
        torch.manual_seed(0)
        m = KGEModel("RotatE", E, R, d, 24.0, True, False)
        ent = m.entity_embedding.detach().clone(); rel = m.relation_embedding.detach().clone()
        erange = m.embedding_range.item(); m = m.to(dev)
        pos, neg, w = synth.kge_batch(3, B, n, E, R)
        args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False, regularization=0.0)
        losses = m.compute_train_grads(torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode, args).cpu().numpy()
        log, ge, gr, _ = O.train_grads("RotatE", ent, rel, None, torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w), mode,
                                       adversarial=True, temperature=1.0, uni_weight=False, regularization=0.0, gamma=24.0, erange=erange)
        gd = m.entity_embedding.grad.cpu().numpy(); g0 = ge.numpy()
        rd = m.relation_embedding.grad.cpu().numpy(); r0 = gr.numpy()
        bad = np.abs(gd - g0) > 1e-4 * np.abs(g0).max() + 1e-7
        rows = np.unique(np.nonzero(bad)[0])
        print(os.environ.get("VARIANT", ""), (E, d, B, n), mode, "ent max|d|/max", float(np.abs(gd - g0).max() / np.abs(g0).max()),
              "rel", float(np.abs(rd - r0).max() / np.abs(r0).max()), "bad rows", rows[:10].tolist(), len(rows),
              "loss", losses[:3].tolist(), [log["positive_sample_loss"], log["negative_sample_loss"]], flush=True)
        if len(rows):
            r = rows[0]; cols = np.nonzero(bad[r])[0]
            print("   row", r, "cols", cols[:12].tolist(), "dev", gd[r, cols[:4]].tolist(), "ref", g0[r, cols[:4]].tolist(), flush=True)
