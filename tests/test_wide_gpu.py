"""Rows wider than the register-tiled kernels hold — more than 2048 floats per
(half-)row (VERDICT r04 missing #4: the reference accepts any hidden_dim,
model.py:42-45).  These dims run through kge_wide.inc (check_model's ns = 0:
run-time-looped single-float kernels) — scores, the fused training step, the
autograd backward of forward(), the fused Adam and the filtered ranks, all
against the CPU oracle (tolerances as in test_gpu_parity.py; ranks exact)."""
from argparse import Namespace

import numpy as np
import pytest
import torch

from conftest import score_tol
from knowledgegraphembedding_amd import KGEAdam, ops, synth
from oracle import kge_oracle as O
from test_gpu_parity import DEV, assert_close_grad, build_model

pytestmark = pytest.mark.gpu

# (model, hidden_dim): aligned and odd spans past 2048, complex and real rows,
# every fast ranking pass (register tile, wave scan, split-bf16 MFMA tile)
WIDE = [("RotatE", 2100), ("TransE", 2051), ("DistMult", 4099), ("ComplEx", 2100), ("pRotatE", 2049)]


@pytest.mark.parametrize("name,d", WIDE)
def test_wide_rows_vs_oracle(name, d):
    E, R, B, n, gamma = 120, 5, 6, 10, 9.0
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, 41)
    pos, neg, w = synth.kge_batch(42, B, n, E, R)
    P, N = torch.from_numpy(pos), torch.from_numpy(neg)
    g = torch.Tensor([gamma]).item()
    modt = None if mod is None else torch.from_numpy(mod)
    E_, R_ = torch.from_numpy(ent), torch.from_numpy(rel)
    with torch.no_grad():
        for mode in ("single", "head-batch", "tail-batch"):
            ref = O.forward(name, E_, R_, modt, P if mode == "single" else (P, N), mode, g, rng).numpy()
            s = (m(P.to(DEV)) if mode == "single" else m((P.to(DEV), N.to(DEV)), mode)).cpu().numpy()
            assert np.all(np.abs(s - ref) <= score_tol(ref)), f"{name} d={d} {mode} scores"
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=1e-4 if name in ("DistMult", "ComplEx") else 0.0)
    for mode in ("head-batch", "tail-batch"):
        losses = m.compute_train_grads(P.to(DEV), N.to(DEV), torch.from_numpy(w).to(DEV), mode, args).cpu().numpy()
        ops.raise_on_device_error(DEV)
        log, ge, gr, gm = O.train_grads(name, E_, R_, modt, P, N, torch.from_numpy(w), mode, adversarial=True,
                                        temperature=1.0, uni_weight=False, regularization=args.regularization,
                                        gamma=g, erange=rng)
        ref = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"]])
        assert np.all(np.abs(losses[:3] - ref) <= score_tol(ref)), f"{name} d={d} {mode} losses"
        assert_close_grad(m.entity_embedding.grad.cpu().numpy(), ge.numpy(), f"{name} d={d} {mode} ent")
        assert_close_grad(m.relation_embedding.grad.cpu().numpy(), gr.numpy(), f"{name} d={d} {mode} rel")
        if gm is not None:
            assert_close_grad(m.modulus.grad.cpu().numpy(), gm.numpy(), f"{name} d={d} {mode} modulus")
    # the backward of forward() for a given dL/dscore (kge_score_backward)
    m.zero_grad(set_to_none=True)
    gout = synth.uniform(43, (B, n), -1.0, 1.0)
    s = m((P.to(DEV), N.to(DEV)), "head-batch")
    s.backward(torch.from_numpy(gout).to(DEV))
    E2 = torch.from_numpy(ent).requires_grad_(True)
    R2 = torch.from_numpy(rel).requires_grad_(True)
    M2 = torch.from_numpy(mod).requires_grad_(True) if mod is not None else None
    ref = O.forward(name, E2, R2, M2, (P, N), "head-batch", g, rng)
    ref.backward(torch.from_numpy(gout))
    assert_close_grad(m.entity_embedding.grad.cpu().numpy(), E2.grad.numpy(), f"{name} d={d} backward ent")
    assert_close_grad(m.relation_embedding.grad.cpu().numpy(), R2.grad.numpy(), f"{name} d={d} backward rel")
    if name != "pRotatE":  # (its exact ranks need the reference's sin: test_rank_parity_gpu)
        triples = pos.tolist()
        for mode in ("head-batch", "tail-batch"):
            ranks, _ = m.rank_queries(triples, triples, mode)
            oref = O.filtered_ranks(name, E_, R_, modt, triples, triples, mode, g, rng)
            assert np.array_equal(ranks, oref["rank_count"]), (name, d, mode, ranks, oref["rank_count"])


@pytest.mark.parametrize("name,d", [("RotatE", 2100), ("TransE", 2051), ("ComplEx", 2100)])
def test_wide_rows_fused_adam_equals_unfused(name, d):
    """The wide entity pass's fused Adam (k_entity_w) against KGEAdam.step()
    on the same deterministic gradients: parameters, moments and gradients
    bit-identical over three steps."""
    E, R, B, n = 300, 7, 12, 16
    runs = []
    for fused in (True, False):
        m, *_ = build_model(name, E, R, d, 12.0, 44)
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=3e-3)
        args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=0.5, uni_weight=False,
                         regularization=1e-4 if name == "ComplEx" else 0.0)
        for step in range(3):
            pos, neg, w = synth.kge_batch(45 + step, B, n, E, R)
            mode = "tail-batch" if step % 2 == 0 else "head-batch"
            m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                  torch.from_numpy(w).to(DEV), mode, args, optimizer=opt if fused else None)
            opt.step()
        st = opt.state[m.entity_embedding]
        runs.append([t.detach().cpu().clone() for t in (m.entity_embedding, m.relation_embedding,
                                                        st["exp_avg"], st["exp_avg_sq"], m.entity_embedding.grad)])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_wide_rows_rank_refinement_reads_rows_in_place():
    """RotatE d = 3700 (entity rows of 7400 floats): the query and one row no
    longer fit the refinement's LDS with its score buffers, so k_rank_refine
    reads both in place (ref_global); ranks and ties against the oracle."""
    E, R, d, gamma = 90, 4, 3700, 12.0
    m, ent, rel, mod, rng = build_model("RotatE", E, R, d, gamma, 46)
    g = np.random.default_rng(47)
    triples = np.stack([g.integers(0, E, 24), g.integers(0, R, 24), g.integers(0, E, 24)], 1).tolist()
    E_, R_ = torch.from_numpy(ent), torch.from_numpy(rel)
    for mode in ("head-batch", "tail-batch"):
        ranks, _, listed = m.rank_queries(triples, triples, mode, listed=True)
        oref = O.filtered_ranks("RotatE", E_, R_, None, triples, triples, mode, torch.Tensor([gamma]).item(), rng)
        assert np.array_equal(ranks, oref["rank_count"]), (mode, ranks, oref["rank_count"])
