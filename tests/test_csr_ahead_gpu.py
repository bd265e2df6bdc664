"""train_step's CSR look-ahead (KGEModel.csr_ahead → kge_train_step_ahead):
the next batch is drawn one step early and its occurrence CSR built beside the
current step's entity pass.  Batches are used in the iterator's order and the
arithmetic is the one-call step's, so tables, Adam state and losses must be
bit-identical to training with the look-ahead off — over alternating head /
tail batches, with the fused KGEAdam and with torch's own Adam (gradient-only
step), when the iterator ends, when the caller switches iterators, and with
two models interleaving their steps on one device (the library keeps one
look-ahead CSR per device)."""
from argparse import Namespace

import pytest
import torch

from knowledgegraphembedding_amd import KGEAdam, KGEModel, _lib, ops, synth
from test_gpu_parity import DEV, build_model

pytestmark = pytest.mark.gpu

E, R, D, B, N = 700, 9, 48, 64, 32


def _batches(seed, k, mode0=0):
    out = []
    for i in range(k):
        pos, neg, w = synth.kge_batch(seed + i, B, N, E, R)
        out.append((torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w),
                    ("head-batch", "tail-batch")[(i + mode0) % 2]))
    return out


def _args():
    return Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)


def _train(name, ahead, fused, plan):
    """plan: list of iterator indices, one per step (switching iterators midway)."""
    m, *_ = build_model(name, E, R, D, 9.0, 5)
    m.csr_ahead = ahead
    params = [p for p in m.parameters() if p.requires_grad]
    opt = KGEAdam(params, lr=1e-2) if fused else torch.optim.Adam(params, lr=1e-2)
    its = [iter(_batches(100, 5)), iter(_batches(300, 5, 1))]
    logs = []
    for k in plan:
        logs.append(dict(KGEModel.train_step(m, opt, its[k], _args())))
    torch.cuda.synchronize()
    return m, logs


@pytest.mark.parametrize("name,fused", [("RotatE", True), ("ComplEx", True), ("pRotatE", False), ("TransE", False)])
def test_csr_ahead_bitwise(name, fused):
    plan = [0, 0, 0, 1, 1, 0, 0, 1]  # iterator 0 runs out after its 5th batch; switches in between
    ref, lref = _train(name, False, fused, plan)
    got, lgot = _train(name, True, fused, plan)
    assert torch.equal(got.entity_embedding, ref.entity_embedding)
    assert torch.equal(got.relation_embedding, ref.relation_embedding)
    for a, b in zip(lgot, lref):
        assert a == b, (a, b)


def test_csr_ahead_two_models_interleaved():
    """Two models alternate steps on one device: each one's look-ahead CSR is
    replaced by the other's in the library's single slot, so each rebuilds its
    own (the owner token) — the results equal training each alone."""
    def run(interleave):
        ms = []
        for seed in (5, 6):
            m, *_ = build_model("RotatE", E, R, D, 9.0, seed)
            m.csr_ahead = True
            ms.append((m, KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-2), iter(_batches(seed, 6))))
        order = [0, 1] * 4 if interleave else [0] * 4 + [1] * 4
        for k in order:
            m, opt, it = ms[k]
            KGEModel.train_step(m, opt, it, _args())
        torch.cuda.synchronize()
        return [m.entity_embedding.detach().clone() for m, _, _ in ms]

    a, b = run(True), run(False)
    assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_csr_ahead_capi_rejects_a_foreign_batch():
    """csr_ready = 1 with a batch / workspace the previous call did not build a
    CSR for is refused (KGE_ERR_ARG), never a silent read of a stale CSR."""
    m, *_ = build_model("RotatE", E, R, D, 9.0, 5)
    (p0, n0, w0, _), (p1, n1, _, _) = _batches(7, 2)
    p0, n0, w0, p1, n1 = (t.to(DEV) for t in (p0, n0, w0, p1, n1))
    ws = ops.ahead_workspaces(m.desc(), B, N, DEV)
    ge, gr, gm, losses = m._grad_buffers()
    kw = dict(adversarial=True, temperature=1.0, uni_weight=False, regularization=0.0, grad_entity=ge,
              grad_relation=gr, grad_modulus=gm, losses=losses)
    ops.train_step_ahead(m.desc(), "tail-batch", p0, n0, w0, DEV, workspace=ws[0], csr_ready=False,
                         next_batch=(p1, n1), next_workspace=ws[1], **kw)
    with pytest.raises(_lib.KGEHipError):  # KGE_ERR_ARG: the look-ahead was built for (p1, n1) in ws[1]
        ops.train_step_ahead(m.desc(), "head-batch", p0, n0, w0, DEV, workspace=ws[1], csr_ready=True, **kw)
    torch.cuda.synchronize()
    assert _lib.load().kge_version()
