"""HIP path vs the reference's golden vectors and vs the CPU oracle (GPU box).

Tolerances (north star):
  scores / losses:  |Δ| ≤ 1e-4 · max(|s_ref|, 1)
  gradients:        |Δ| ≤ 1e-4 · max|g_ref| + 1e-4 · |g_ref|  (fp32 sums in another order)
  ranks:            tests/test_rank_parity_gpu.py
"""
from argparse import Namespace

import numpy as np
import pytest
import torch

from conftest import dims, score_tol, synth_tables
from knowledgegraphembedding_amd import KGEAdam, KGEModel, synth
from knowledgegraphembedding_amd import ops
from oracle import kge_oracle as O

pytestmark = pytest.mark.gpu
NAMES = ["TransE", "DistMult", "ComplEx", "RotatE", "pRotatE"]
DEV = torch.device("cuda", 0)


def build_model(name, E, R, d, gamma, seed):
    de, dr = {"TransE": (0, 0), "DistMult": (0, 0), "ComplEx": (1, 1), "RotatE": (1, 0), "pRotatE": (0, 0)}[name]
    m = KGEModel(name, E, R, d, gamma, bool(de), bool(dr))
    ent, rel, mod, rng = synth_tables(name, E, R, d, gamma, seed)
    with torch.no_grad():
        m.entity_embedding.copy_(torch.from_numpy(ent))
        m.relation_embedding.copy_(torch.from_numpy(rel))
    return m.to(DEV), ent, rel, mod, rng


def assert_close_grad(got, ref, msg=""):
    tol = 1e-4 * np.abs(ref).max() + 1e-4 * np.abs(ref) + 1e-12
    bad = np.abs(got - ref) > tol
    assert not bad.any(), f"{msg}: {bad.sum()} elements off, max |Δ| {np.abs(got - ref).max():.3e}"


# ------------------------------------------------------------------ scores
@pytest.mark.parametrize("tag,E,R,d,B,n,gamma,seed", [("small", 64, 8, 16, 4, 8, 12.0, 11),
                                                       ("d1000", 128, 16, 1000, 8, 16, 24.0, 12)])
@pytest.mark.parametrize("name", NAMES)
def test_scores_vs_golden(g_scores, tag, E, R, d, B, n, gamma, seed, name):
    m, *_ = build_model(name, E, R, d, gamma, seed)
    pos, neg, _ = synth.kge_batch(seed, B, n, E, R)
    P, N = torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV)
    with torch.no_grad():
        for mode in ("single", "head-batch", "tail-batch"):
            s = (m(P) if mode == "single" else m((P, N), mode)).cpu().numpy()
            ref = g_scores[f"{tag}/{name}/{mode}"]
            assert s.shape == ref.shape
            assert np.all(np.abs(s - ref) <= score_tol(ref)), f"{name} {mode} max|Δ| {np.abs(s - ref).max()}"


@pytest.mark.parametrize("name", NAMES)
def test_scores_vs_oracle_odd_dims(name):
    # d not a multiple of 4 → scalar-slot kernels (VEC=1); n not a multiple of the unroll
    E, R, d, B, n, gamma = 97, 7, 13 if name not in ("ComplEx", "RotatE") else 14, 5, 7, 6.0
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, 3)
    pos, neg, _ = synth.kge_batch(5, B, n, E, R)
    P, N = torch.from_numpy(pos), torch.from_numpy(neg)
    g = torch.Tensor([gamma]).item()
    modt = None if mod is None else torch.from_numpy(mod)
    with torch.no_grad():
        for mode in ("single", "head-batch", "tail-batch"):
            ref = O.forward(name, torch.from_numpy(ent), torch.from_numpy(rel), modt,
                            P if mode == "single" else (P, N), mode, g, rng).numpy()
            s = (m(P.to(DEV)) if mode == "single" else m((P.to(DEV), N.to(DEV)), mode)).cpu().numpy()
            assert np.all(np.abs(s - ref) <= score_tol(ref)), f"{name} {mode}"


# ------------------------------------------------------------------ training
def _train_case(g_train, golden_info, ci):
    ti = golden_info["train"]
    case = ti["cases"][ci]
    name = case["model"]
    m, ent, rel, mod, rng = build_model(name, ti["E"], ti["R"], ti["d"], ti["gamma"], ti["seed"])
    pos, neg, w = synth.kge_batch(ti["seed"] + ci, ti["B"], ti["n"], ti["E"], ti["R"])
    args = Namespace(cuda=True, negative_adversarial_sampling=case["adversarial"],
                     adversarial_temperature=ti["adversarial_temperature"], uni_weight=case["uni_weight"],
                     regularization=case["regularization"])
    batch = (torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w), case["mode"])
    return m, args, batch, case, ti


def test_train_step_vs_golden(g_train, golden_info):
    for ci in range(len(golden_info["train"]["cases"])):
        m, args, batch, case, ti = _train_case(g_train, golden_info, ci)
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=ti["lr"])
        grads = {}

        class Rec:
            def zero_grad(self):
                opt.zero_grad()

            def step(self):
                if not grads:
                    grads["e"] = m.entity_embedding.grad.detach().cpu().numpy().copy()
                    grads["r"] = m.relation_embedding.grad.detach().cpu().numpy().copy()
                    if case["model"] == "pRotatE":
                        grads["m"] = m.modulus.grad.detach().cpu().numpy().copy()
                opt.step()

        log = KGEModel.train_step(m, Rec(), iter([batch]), args)
        log2 = KGEModel.train_step(m, Rec(), iter([batch]), args)
        ref = g_train[f"{ci}/log"]
        got = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"],
                        log.get("regularization", 0.0)])
        assert np.all(np.abs(got - ref) <= score_tol(ref)), f"{case} log {got} vs {ref}"
        assert ("regularization" in log) == (case["regularization"] != 0.0)
        assert_close_grad(grads["e"], g_train[f"{ci}/grad_entity"], f"{case} grad_entity")
        assert_close_grad(grads["r"], g_train[f"{ci}/grad_relation"], f"{case} grad_relation")
        if case["model"] == "pRotatE":
            assert_close_grad(grads["m"], g_train[f"{ci}/grad_modulus"], f"{case} grad_modulus")
        ref2 = g_train[f"{ci}/log2"]
        got2 = np.array([log2["positive_sample_loss"], log2["negative_sample_loss"], log2["loss"],
                         log2.get("regularization", 0.0)])
        assert np.all(np.abs(got2 - ref2) <= score_tol(ref2)), f"{case} step-2 log"
        p2 = m.entity_embedding.detach().cpu().numpy()
        r2 = g_train[f"{ci}/param2_entity"]
        # two Adam steps of lr 0.01 on |p| ~ 1: tolerance scaled to the update size
        assert np.abs(p2 - r2).max() <= 2e-4 * 0.01 * 2 + 1e-6, f"{case} params after 2 steps"


@pytest.mark.parametrize("name,d", [("DistMult", 2000), ("TransE", 1001), ("RotatE", 1001), ("ComplEx", 2047),
                                    ("pRotatE", 1999), ("DistMult", 2048), ("RotatE", 2000)])
def test_wide_and_odd_dims_vs_oracle(name, d):
    """Any hidden_dim up to 2048 floats per (half-)row: best_config.sh:44-50's
    DistMult d = 2000, odd / unaligned d (the single-float slot kernels with 16
    or 32 slots per lane) — scores, the fused train step's losses and
    gradients in both modes, and filtered ranks against the oracle."""
    E, R, B, n, gamma = 150, 5, 6, 12, 9.0
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, 17)
    pos, neg, w = synth.kge_batch(18, B, n, E, R)
    P, N = torch.from_numpy(pos), torch.from_numpy(neg)
    g = torch.Tensor([gamma]).item()
    modt = None if mod is None else torch.from_numpy(mod)
    E_, R_ = torch.from_numpy(ent), torch.from_numpy(rel)
    with torch.no_grad():
        for mode in ("single", "head-batch", "tail-batch"):
            ref = O.forward(name, E_, R_, modt, P if mode == "single" else (P, N), mode, g, rng).numpy()
            s = (m(P.to(DEV)) if mode == "single" else m((P.to(DEV), N.to(DEV)), mode)).cpu().numpy()
            assert np.all(np.abs(s - ref) <= score_tol(ref)), f"{name} d={d} {mode}"
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
    if name != "pRotatE":  # (pRotatE's sin is correctly rounded here: ranks are checked in test_rank_parity_gpu)
        triples = pos.tolist()
        for mode in ("head-batch", "tail-batch"):
            ranks, _ = m.rank_queries(triples, triples, mode)
            oref = O.filtered_ranks(name, E_, R_, modt, triples, triples, mode, g, rng)
            assert np.array_equal(ranks, oref["rank_count"]), (name, d, mode, ranks, oref["rank_count"])


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_train_grads_vs_oracle_realistic(name, mode):
    """d=1000-class rows, n=64: fused kernel vs the oracle's autograd."""
    E, R, d, B, n, gamma = 600, 20, 200 if name != "DistMult" else 400, 16, 64, 24.0
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, 8)
    pos, neg, w = synth.kge_batch(9, B, n, E, R)
    g = torch.Tensor([gamma]).item()
    for adv in (True, False):
        args = Namespace(negative_adversarial_sampling=adv, adversarial_temperature=1.0, uni_weight=False,
                         regularization=0.0)
        losses = m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                       torch.from_numpy(w).to(DEV), mode, args).cpu().numpy()
        ops.raise_on_device_error(DEV)
        log, ge, gr, gm = O.train_grads(name, torch.from_numpy(ent), torch.from_numpy(rel),
                                        None if mod is None else torch.from_numpy(mod), torch.from_numpy(pos),
                                        torch.from_numpy(neg), torch.from_numpy(w), mode, adversarial=adv,
                                        temperature=1.0, uni_weight=False, regularization=0.0, gamma=g, erange=rng)
        ref = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"]])
        assert np.all(np.abs(losses[:3] - ref) <= score_tol(ref))
        assert_close_grad(m.entity_embedding.grad.cpu().numpy(), ge.numpy(), f"{name} {mode} adv={adv} ent")
        assert_close_grad(m.relation_embedding.grad.cpu().numpy(), gr.numpy(), f"{name} {mode} adv={adv} rel")
        if gm is not None:
            assert_close_grad(m.modulus.grad.cpu().numpy(), gm.numpy(), f"{name} modulus")


def test_train_grads_deterministic():
    m, *_ = build_model("RotatE", 3000, 50, 250, 24.0, 4)
    pos, neg, w = synth.kge_batch(4, 64, 128, 3000, 50)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    outs = []
    for _ in range(2):
        losses = m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                       torch.from_numpy(w).to(DEV), "tail-batch", args)
        outs.append((losses.cpu().clone(), m.entity_embedding.grad.cpu().clone(),
                     m.relation_embedding.grad.cpu().clone()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_fused_adam_train_step_vs_golden(g_train, golden_info):
    """KGEModel.train_step with KGEAdam (Adam fused into the gradient passes)
    against the reference's params after two steps."""
    for ci in range(0, len(golden_info["train"]["cases"]), 3):
        m, args, batch, case, ti = _train_case(g_train, golden_info, ci)
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=ti["lr"])
        log = KGEModel.train_step(m, opt, iter([batch]), args)
        KGEModel.train_step(m, opt, iter([batch]), args)
        ref = g_train[f"{ci}/log"]
        got = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"],
                        log.get("regularization", 0.0)])
        assert np.all(np.abs(got - ref) <= score_tol(ref)), f"{case} log"
        p2 = m.entity_embedding.detach().cpu().numpy()
        assert np.abs(p2 - g_train[f"{ci}/param2_entity"]).max() <= 2e-4 * 0.01 * 2 + 1e-6, f"{case} entity"
        r2 = m.relation_embedding.detach().cpu().numpy()
        assert np.abs(r2 - g_train[f"{ci}/param2_relation"]).max() <= 2e-4 * 0.01 * 2 + 1e-6, f"{case} relation"
        if case["model"] == "pRotatE":
            mo = m.modulus.detach().cpu().numpy()
            assert np.abs(mo - g_train[f"{ci}/param2_modulus"]).max() <= 1e-5, f"{case} modulus"
        assert opt.state[m.entity_embedding]["step"].item() == 2


@pytest.mark.parametrize("name", NAMES)
def test_fused_adam_bitwise_equals_unfused(name):
    """The fused optimizer step applies the same per-element Adam to the same
    deterministic gradients as KGEAdam.step(): parameters, moments and grads
    must agree bit for bit over several steps."""
    E, R, d, B, n = 700, 9, 64, 32, 48
    runs = []
    for fused in (True, False):
        m, *_ = build_model(name, E, R, d, 12.0, 31)
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=3e-3)
        args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=0.5, uni_weight=False,
                         regularization=1e-4 if name in ("DistMult", "ComplEx") else 0.0)
        for step in range(3):
            pos, neg, w = synth.kge_batch(40 + step, B, n, E, R)
            mode = "tail-batch" if step % 2 == 0 else "head-batch"
            m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                  torch.from_numpy(w).to(DEV), mode, args, optimizer=opt if fused else None)
            opt.step()
        st = opt.state[m.entity_embedding]
        runs.append([t.detach().cpu().clone() for t in (m.entity_embedding, m.relation_embedding,
                                                        st["exp_avg"], st["exp_avg_sq"], m.entity_embedding.grad)])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name,uni,B", [("RotatE", False, 1500), ("RotatE", True, 300), ("TransE", False, 64),
                                         ("pRotatE", False, 200), ("ComplEx", True, 1100)])
def test_fused_finalize_bitwise_equals_separate(name, uni, B, monkeypatch):
    """The loss finalisation in the entity launch's last block (256 threads)
    folds its sums in k_finalize's 1024-thread order: losses, modulus gradient
    and the fused Adam state are bit-identical with KGE_FIN_SEPARATE=1 (the
    separate k_finalize launch), for batches below, between and above the
    workgroup widths."""
    E, R, d, n = 900, 9, 64, 24
    pos, neg, w = synth.kge_batch(5, B, n, E, R)
    P, N, W = torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV), torch.from_numpy(w).to(DEV)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=0.7, uni_weight=uni,
                     regularization=0.0)
    runs = []
    for sep in ("0", "1"):
        monkeypatch.setenv("KGE_FIN_SEPARATE", sep)
        m, *_ = build_model(name, E, R, d, 12.0, 17)
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=3e-3)
        out = []
        for step, mode in enumerate(("tail-batch", "head-batch", "tail-batch")):
            fused_opt = opt if step > 0 else None  # one plain step (grads + k_finalize's twin), then fused Adam
            out.append(m.compute_train_grads(P, N, W, mode, args, optimizer=fused_opt).cpu().clone())
            if fused_opt is None:
                opt.step()
        out += [t.detach().cpu().clone() for t in m.parameters()]
        runs.append(out)
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", NAMES)
def test_phased_step_bitwise_equals_single_call(name):
    """kge_train_step_grads_phased (rows, entity-row chunks in any order,
    finalize) — the data-parallel overlap path — gives the single call's
    gradients and losses bit for bit, and the chunk hook sees every row once."""
    E, R, d, B, n = 701, 9, 64, 32, 48
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=0.5, uni_weight=False,
                     regularization=1e-4 if name in ("DistMult", "ComplEx") else 0.0)
    pos, neg, w = synth.kge_batch(77, B, n, E, R)
    P, N, W = torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV), torch.from_numpy(w).to(DEV)
    out = []
    for chunks in (None, [(500, 701), (0, 233), (233, 500)]):
        m, *_ = build_model(name, E, R, d, 12.0, 31)
        seen = []
        for mode in ("tail-batch", "head-batch"):
            losses = m.compute_train_grads(P, N, W, mode, args, entity_chunks=chunks,
                                           on_entity_chunk=lambda e0, e1, g: seen.append((e0, e1)))
            out.append([t.detach().cpu().clone() for t in (losses, m.entity_embedding.grad,
                                                           m.relation_embedding.grad)])
        if chunks:
            assert sorted(seen) == sorted(chunks * 2)
    for a, b in zip(out[:2], out[2:]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


# ------------------------------------------------------------ forward autograd
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("mode", ["single", "head-batch", "tail-batch"])
def test_forward_backward_vs_oracle(name, mode):
    E, R, d, B, n, gamma = 80, 6, 24, 6, 10, 9.0
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, 13)
    pos, neg, _ = synth.kge_batch(14, B, n, E, R)
    n_eff = 1 if mode == "single" else n
    gout = synth.uniform(15, (B, n_eff), -1.0, 1.0)
    P, N = torch.from_numpy(pos), torch.from_numpy(neg)
    s = m(P.to(DEV)) if mode == "single" else m((P.to(DEV), N.to(DEV)), mode)
    s.backward(torch.from_numpy(gout).to(DEV))
    E_ = torch.from_numpy(ent).requires_grad_(True)
    R_ = torch.from_numpy(rel).requires_grad_(True)
    M_ = torch.from_numpy(mod).requires_grad_(True) if mod is not None else None
    ref = O.forward(name, E_, R_, M_, P if mode == "single" else (P, N), mode, torch.Tensor([gamma]).item(), rng)
    ref.backward(torch.from_numpy(gout))
    assert np.all(np.abs(s.detach().cpu().numpy() - ref.detach().numpy()) <= score_tol(ref.detach().numpy()))
    assert_close_grad(m.entity_embedding.grad.cpu().numpy(), E_.grad.numpy(), f"{name} {mode} ent")
    assert_close_grad(m.relation_embedding.grad.cpu().numpy(), R_.grad.numpy(), f"{name} {mode} rel")
    if M_ is not None:
        assert_close_grad(m.modulus.grad.cpu().numpy(), M_.grad.numpy(), f"{name} {mode} modulus")


@pytest.mark.parametrize("name", NAMES)
def test_plugin_methods(name):
    """model.TransE(head, relation, tail, mode) on gathered rows == forward()."""
    E, R, d, B, n = 50, 5, 16, 3, 7
    m, ent, rel, mod, rng = build_model(name, E, R, d, 12.0, 21)
    pos, neg, _ = synth.kge_batch(22, B, n, E, R)
    P, N = torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV)
    with torch.no_grad():
        for mode in ("single", "head-batch", "tail-batch"):
            h, r, t = O.gather(m.entity_embedding, m.relation_embedding, P if mode == "single" else (P, N), mode)
            a = getattr(m, name)(h, r, t, mode)
            b = m(P) if mode == "single" else m((P, N), mode)
            torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_index_error():
    m, *_ = build_model("RotatE", 30, 4, 8, 12.0, 1)
    bad = torch.tensor([[0, 1, 99]], device=DEV)
    with pytest.raises(IndexError):
        m(bad)
        ops.raise_on_device_error(DEV)


def test_deferred_step_log():
    """train_step's StepLog: same floats as the synchronous read-back, a bad
    index raises IndexError when the log is read, or within two further steps
    when it is never read (the ring bounds the run-ahead)."""
    import json
    import pickle
    E, R, d, B, n = 40, 4, 8, 6, 5
    pos, neg, w = synth.kge_batch(61, B, n, E, R)
    batch = (torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV), torch.from_numpy(w).to(DEV), "tail-batch")
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=1e-3, dp_group=None)
    logs = {}
    for defer in (True, False):
        m, *_ = build_model("DistMult", E, R, d, 12.0, 5)
        m.defer_log = defer
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)
        logs[defer] = [KGEModel.train_step(m, opt, iter([batch]), args) for _ in range(3)]
    for a, b in zip(logs[True], logs[False]):
        assert dict(a.items()) == dict(b.items())
        assert set(a) == {"regularization", "positive_sample_loss", "negative_sample_loss", "loss"}
        assert json.loads(json.dumps(a)) == b and pickle.loads(pickle.dumps(a)) == b
    bad_neg = neg.copy()
    bad_neg[2, 3] = E + 7
    bad = (batch[0], torch.from_numpy(bad_neg).to(DEV), batch[2], "tail-batch")
    m, *_ = build_model("DistMult", E, R, d, 12.0, 5)
    opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)
    log = KGEModel.train_step(m, opt, iter([bad]), args)
    with pytest.raises(IndexError):
        log["loss"]
    KGEModel.train_step(m, opt, iter([bad]), args)  # unread
    with pytest.raises(IndexError):
        for _ in range(2):
            KGEModel.train_step(m, opt, iter([batch]), args)


# ------------------------------------------------------------------ Adam
def test_kge_adam_matches_torch_adam():
    torch.manual_seed(0)
    p0 = torch.randn(1001, 37)
    grads = [torch.randn(1001, 37) for _ in range(3)]
    a = p0.clone().to(DEV).requires_grad_(True)
    b = p0.clone().to(DEV).requires_grad_(True)
    oa, ob = KGEAdam([a], lr=1e-3), torch.optim.Adam([b], lr=1e-3)
    for g in grads:
        a.grad, b.grad = g.to(DEV), g.to(DEV).clone()
        oa.step()
        ob.step()
    torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-7)
    sd = oa.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


# ------------------------------------------------------------------ ranking
# rank parity with the reference: tests/test_rank_parity_gpu.py


def test_test_step_metrics_vs_golden(g_ranks, golden_info):
    kg = golden_info["ranks"][0]
    tag, E, R, d, seed = kg["tag"], kg["E"], kg["R"], kg["d"], kg["seed"]
    all_true = [tuple(x) for x in g_ranks[f"{tag}/all_true"].tolist()]
    test = [tuple(x) for x in g_ranks[f"{tag}/test"].tolist()]
    for name in kg["models"]:
        m, *_ = build_model(name, E, R, d, kg["gamma"], seed)
        args = Namespace(countries=False, nentity=E, nrelation=R, test_batch_size=4, cpu_num=2, test_log_steps=1000,
                         cuda=True)
        met = KGEModel.test_step(m, test, all_true, args)
        got = np.array([met[k] for k in golden_info["metric_order"]])
        ref = g_ranks[f"{tag}/{name}/metrics"]
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12, err_msg=name)


def test_countries_auc_pr(g_countries, golden_info):
    ci = golden_info["countries"]
    m, *_ = build_model("TransE", ci["nentity"], ci["nrelation"], ci["d"], ci["gamma"], ci["seed"])
    args = Namespace(countries=True, regions=g_countries["regions"].tolist(), cuda=True)
    test = [tuple(x) for x in g_countries["test"].tolist()]
    met = KGEModel.test_step(m, test, [], args)
    assert abs(met["auc_pr"] - g_countries["auc_pr"][0]) < 1e-6


# ------------------------------------------------------------- full size
@pytest.mark.parametrize("mode", ["tail-batch", "head-batch"])
def test_config2_full_shape_grads_vs_oracle(mode):
    """The benchmarked launch shapes (RotatE FB15k, B = 1024, n = 256, d = 1000
    -adv, Σw subsampling: the 4-slice entity pass with its LDS budget, 1024
    row blocks) against the oracle's autograd of the reference's op chain:
    the three losses, every relation-gradient row and 512 sampled entity-
    gradient rows (all rows each sampled entity occurs in are included — the
    oracle runs the whole batch, in 128-row chunks whose gradients are
    re-weighted by Σw_chunk / Σw, the reference's loss being linear in them)."""
    E, R, d, B, n, gamma = 14951, 1345, 1000, 1024, 256, 24.0
    m, ent, rel, mod, rng = build_model("RotatE", E, R, d, gamma, 0)
    pos, neg, w = synth.kge_batch(2, B, n, E, R)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    losses = m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                   torch.from_numpy(w).to(DEV), mode, args).cpu().numpy()
    ge = m.entity_embedding.grad.cpu().numpy()
    gr = m.relation_embedding.grad.cpu().numpy()
    ops.raise_on_device_error(DEV)
    torch.set_num_threads(max(1, min(16, len(__import__("os").sched_getaffinity(0)))))
    E_, R_ = torch.from_numpy(ent), torch.from_numpy(rel)
    wsum = float(np.float64(w.astype(np.float64).sum()))
    ref_l = np.zeros(3)
    ref_ge = np.zeros_like(ent, dtype=np.float64)
    ref_gr = np.zeros_like(rel, dtype=np.float64)
    for c0 in range(0, B, 128):
        sl = slice(c0, c0 + 128)
        log, cge, cgr, _ = O.train_grads("RotatE", E_, R_, None, torch.from_numpy(pos[sl]), torch.from_numpy(neg[sl]),
                                         torch.from_numpy(w[sl]), mode, adversarial=True, temperature=1.0,
                                         uni_weight=False, regularization=0.0, gamma=gamma, erange=rng)
        f = float(w[sl].astype(np.float64).sum()) / wsum
        ref_l += f * np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"]])
        ref_ge += f * cge.numpy()
        ref_gr += f * cgr.numpy()
    assert np.all(np.abs(losses[:3] - ref_l) <= 1e-4 * np.maximum(1, np.abs(ref_l))), (losses[:3], ref_l)
    rows = np.unique(np.concatenate([synth.randint(5, (384,), E), pos[:64, 0], pos[:64, 2]]))
    assert_close_grad(ge[rows], ref_ge[rows].astype(np.float32), f"entity rows ({mode})")
    assert_close_grad(gr, ref_gr.astype(np.float32), f"relation rows ({mode})")


def test_config2_full_size_properties():
    """BASELINE config 2 shape (RotatE FB15k d=1000 b=1024 n=256 -adv): finite,
    deterministic, and sampled rows equal to the oracle."""
    E, R, d, B, n, gamma = 14951, 1345, 1000, 1024, 256, 24.0
    m, ent, rel, mod, rng = build_model("RotatE", E, R, d, gamma, 0)
    pos, neg, w = synth.kge_batch(1, B, n, E, R)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    res = []
    for _ in range(2):
        losses = m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                       torch.from_numpy(w).to(DEV), "tail-batch", args)
        res.append((losses.cpu().clone(), m.entity_embedding.grad.clone()))
    ops.raise_on_device_error(DEV)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert torch.isfinite(res[0][1]).all()
    # scores of 8 sampled rows vs the oracle
    rows = [0, 1, 100, 511, 512, 777, 1000, 1023]
    P = torch.from_numpy(pos[rows])
    N = torch.from_numpy(neg[rows])
    with torch.no_grad():
        s = m((P.to(DEV), N.to(DEV)), "tail-batch").cpu().numpy()
    ref = O.forward("RotatE", torch.from_numpy(ent), torch.from_numpy(rel), None, (P, N), "tail-batch",
                    torch.Tensor([gamma]).item(), rng).numpy()
    assert np.all(np.abs(s - ref) <= score_tol(ref))
    # gradient of the full batch equals the sum of per-half-batch gradients (linearity), both normalised by Σw
    wsum = torch.tensor([float(w.sum(dtype=np.float32))], device=DEV)
    acc = None
    for lo, hi in ((0, 512), (512, 1024)):
        m.compute_train_grads(torch.from_numpy(pos[lo:hi]).to(DEV), torch.from_numpy(neg[lo:hi]).to(DEV),
                              torch.from_numpy(w[lo:hi]).to(DEV), "tail-batch", args, weight_sum=wsum)
        g = m.entity_embedding.grad.clone()
        acc = g if acc is None else acc + g
    full = res[0][1]
    tol = 1e-4 * full.abs().max() + 1e-4 * full.abs()
    assert ((acc - full).abs() <= tol).all()


@pytest.mark.parametrize("name,d,B", [("RotatE", 200, 24), ("ComplEx", 200, 24), ("TransE", 200, 24),
                                      ("pRotatE", 200, 24), ("DistMult", 200, 24), ("RotatE", 104, 1100),
                                      ("DistMult", 52, 700), ("RotatE", 1000, 24), ("DistMult", 1000, 24),
                                      ("ComplEx", 1000, 24)])
def test_entity_pass_column_slices_bitwise(name, d, B, monkeypatch):
    """The column-sliced entity pass (k_entity_sl with nsl = 1, 2, 4, 8
    slices — the count is picked per shape — reading k_row's slice-major q
    copy in the single-call step) and the row-per-wave pass (k_entity, the
    path for rows that are not float4-aligned; KGE_ENT_SLICES=0 forces it
    here) apply the same per-element arithmetic in the same occurrence order:
    identical gradients and fused Adam updates, bit for bit (the regulariser's
    partial sums only regroup).  The row-major q / line-aligned slices of the
    phased and exchanged steps: test_phased_step_bitwise_equals_single_call,
    test_dp_factors_gpu, test_dp_owner_gpu."""
    E, R, n = 300, 7, 40   # d = 200: 50 slots per (half) row: 1..8 slices all fit
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=1e-4 if name in ("ComplEx", "DistMult") else 0.0)
    pos, neg, w = synth.kge_batch(88, B, n, E, R)
    P, N, W = torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV), torch.from_numpy(w).to(DEV)
    out = {}
    variants = {200: ("0", "1", "2", "4", "8"), 1000: ("0", "4")}.get(d, ("0", "-1"))
    for nsl in variants:
        monkeypatch.setenv("KGE_ENT_SLICES", nsl)
        m, *_ = build_model(name, E, R, d, 12.0, 5)
        opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)
        res = []
        for mode in ("tail-batch", "head-batch"):
            losses = m.compute_train_grads(P, N, W, mode, args, optimizer=opt)
            opt.step()
            res.append((losses.cpu().clone(), m.entity_embedding.grad.cpu().clone(),
                        m.entity_embedding.detach().cpu().clone()))
        out[nsl] = res
    for nsl in variants[1:]:
        for (l0, g0, p0), (l1, g1, p1) in zip(out["0"], out[nsl]):
            assert torch.equal(g0, g1) and torch.equal(p0, p1), nsl
            torch.testing.assert_close(l0[:4], l1[:4], rtol=1e-6, atol=0)


@pytest.mark.parametrize("name,E,d,B,n", [(nm, 400, 120, 24, 40) for nm in NAMES] +
                         [("RotatE", 300, 64, 8, 32), ("RotatE", 2000, 100, 64, 32), ("DistMult", 500, 16, 300, 8)])
def test_fused_epilogue_bitwise(name, E, d, B, n):
    """k_row with the epilogue in its tail (the single-call step) and the
    separate k_row_epi launch (the phased step the data-parallel overlap uses)
    give the same losses and gradients bit for bit: same per-element
    arithmetic, same fixed-order Σw reduction, same epilogue function.  Many
    blocks per launch (B = 64, 300) exercise the fused tail's c_i, which must
    not read the Σw that block 0 publishes in the same launch; d = 16 with
    B = 300 needs the Σw tree's 256 floats of LDS beyond the 2·Le merge buffer."""
    R = 9
    pos, neg, w = synth.kge_batch(91, B, n, E, R)
    P, N, W = torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV), torch.from_numpy(w).to(DEV)
    res = {}
    for phased in (False, True):
        out = []
        chunks = [(0, E)] if phased else None
        for adv, uni in ((True, False), (False, True)):
            m, *_ = build_model(name, E, R, d, 12.0, 7)
            args = Namespace(negative_adversarial_sampling=adv, adversarial_temperature=0.7, uni_weight=uni,
                             regularization=0.0)
            for mode in ("tail-batch", "head-batch"):
                losses = m.compute_train_grads(P, N, W, mode, args, entity_chunks=chunks)
                out.append([t.detach().cpu().clone() for t in (losses, m.entity_embedding.grad,
                                                               m.relation_embedding.grad)])
            # Σw supplied by the caller (the data-parallel path)
            losses = m.compute_train_grads(P, N, W, "tail-batch", args, weight_sum=W.sum().reshape(1),
                                           entity_chunks=chunks)
            out.append([losses.detach().cpu().clone(), m.entity_embedding.grad.cpu().clone()])
        res[phased] = out
    for a, b in zip(res[False], res[True]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
