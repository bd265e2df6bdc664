"""Edge shapes through the HIP path, against the CPU oracle (GPU box):
one positive with one negative, a "hot" entity that takes every negative of
the batch (one occurrence bucket of 1600 ids: the entity pass's 64-id chunks
and the CSR's long bucket), many negatives per row (n = 2000: the row pass's
LDS score buffer), a two-entity graph, an empty scoring batch, and filtered
ranking where the filter removes every candidate (rank 1).  Tolerances as in
test_gpu_parity.py."""
from argparse import Namespace

import numpy as np
import pytest
import torch

from conftest import score_tol
from knowledgegraphembedding_amd import KGEModel, synth
from knowledgegraphembedding_amd import ops
from oracle import kge_oracle as O
from test_gpu_parity import DEV, NAMES, assert_close_grad, build_model

pytestmark = pytest.mark.gpu


def _check_train(name, E, R, d, pos, neg, w, mode, adv=True, gamma=12.0, seed=3):
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, seed)
    args = Namespace(negative_adversarial_sampling=adv, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    losses = m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                   torch.from_numpy(w).to(DEV), mode, args).cpu().numpy()
    ops.raise_on_device_error(DEV)
    log, ge, gr, gm = O.train_grads(name, torch.from_numpy(ent), torch.from_numpy(rel),
                                    None if mod is None else torch.from_numpy(mod), torch.from_numpy(pos),
                                    torch.from_numpy(neg), torch.from_numpy(w), mode, adversarial=adv,
                                    temperature=1.0, uni_weight=False, regularization=0.0,
                                    gamma=torch.Tensor([gamma]).item(), erange=rng)
    ref = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"]])
    assert np.all(np.abs(losses[:3] - ref) <= score_tol(ref)), (losses[:3], ref)
    assert_close_grad(m.entity_embedding.grad.cpu().numpy(), ge.numpy(), f"{name} ent")
    assert_close_grad(m.relation_embedding.grad.cpu().numpy(), gr.numpy(), f"{name} rel")
    if gm is not None:
        assert_close_grad(m.modulus.grad.cpu().numpy(), gm.numpy(), f"{name} modulus")


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_one_positive_one_negative(name, mode):
    E, R, d = 50, 3, 40
    pos, neg, w = synth.kge_batch(21, 1, 1, E, R)
    _check_train(name, E, R, d, pos, neg, w, mode)


@pytest.mark.parametrize("name", ["RotatE", "DistMult", "pRotatE"])
def test_hot_entity_bucket(name):
    """Every negative of the batch is entity 7 (1600 occurrences in one bucket)."""
    E, R, d, B, n = 120, 5, 48, 8, 200
    pos, _, w = synth.kge_batch(22, B, n, E, R)
    neg = np.full((B, n), 7, dtype=np.int64)
    _check_train(name, E, R, d, pos, neg, w, "tail-batch")


@pytest.mark.parametrize("name", ["RotatE", "TransE"])
def test_many_negatives_per_row(name):
    E, R, d, B, n = 3000, 4, 24, 4, 2000
    pos, neg, w = synth.kge_batch(23, B, n, E, R)
    _check_train(name, E, R, d, pos, neg, w, "head-batch", adv=True)


@pytest.mark.parametrize("name", NAMES)
def test_two_entity_graph(name):
    E, R, d, B, n = 2, 1, 16, 6, 5
    pos, neg, w = synth.kge_batch(24, B, n, E, R)
    _check_train(name, E, R, d, pos, neg, w, "tail-batch")


def test_empty_scoring_batch():
    m, *_ = build_model("RotatE", 30, 3, 16, 12.0, 1)
    with torch.no_grad():
        out = m((torch.zeros(0, 3, dtype=torch.int64, device=DEV), torch.zeros(0, 4, dtype=torch.int64, device=DEV)),
                "tail-batch")
    assert tuple(out.shape) == (0, 4)


@pytest.mark.parametrize("name", NAMES)
def test_everything_filtered_ranks_first(name):
    """With every entity a true tail of (h, r), each query's rank is 1 (the
    reference's filter_bias leaves only the true entity unfiltered)."""
    E, R, d = 40, 2, 32
    m, *_ = build_model(name, E, R, d, 12.0, 2)
    true = np.array([[0, 1, t] for t in range(E)], dtype=np.int64)
    ranks, ties = m.rank_queries(true[:10], true, "tail-batch")
    assert np.array_equal(ranks, np.ones(10, dtype=np.int64)) and not ties.any()


@pytest.mark.parametrize("name", ["DistMult", "RotatE"])
def test_rank_queries_both_directions_pipelined(name):
    """rank_queries_both (both directions queued, one read-back — what bench.py's
    ranking section and test_step do) returns exactly rank_queries' per-direction
    ranks and ties."""
    E, R, d = 300, 5, 32
    m, *_ = build_model(name, E, R, d, 12.0, 7)
    rng = np.random.default_rng(3)
    true = np.unique(np.stack([rng.integers(0, E, 2000), rng.integers(0, R, 2000), rng.integers(0, E, 2000)], 1),
                     axis=0)
    q = true[:257]
    (rh, th), (rt, tt) = m.rank_queries_both(q, true)
    rh1, th1 = m.rank_queries(q, true, "head-batch")
    rt1, tt1 = m.rank_queries(q, true, "tail-batch")
    assert np.array_equal(rh, rh1) and np.array_equal(th, th1)
    assert np.array_equal(rt, rt1) and np.array_equal(tt, tt1)


@pytest.mark.parametrize("name", ["DistMult", "ComplEx"])
def test_test_step_query_blocks_reuse_the_table(name):
    """test_step ranks in query blocks of at most 16384 and, from the second
    block (and direction) on, reuses the table statistics and split operands
    the first call left in the workspace (KGE_RANK_REUSE_TABLE); its ranks
    must equal one unblocked rank_queries call per direction without reuse.
    A training step between two evaluations must drop the reuse (the step
    writes the shared workspace and the table)."""
    E, R, d = 300, 7, 24
    m, *_ = build_model(name, E, R, d, 12.0, 9)
    g = np.random.default_rng(4)
    test = np.stack([g.integers(0, E, 20000), g.integers(0, R, 20000), g.integers(0, E, 20000)], 1).astype(np.int64)
    true = np.unique(test, axis=0)
    args = Namespace(countries=False, nentity=E, nrelation=R, test_batch_size=16, cpu_num=2, test_log_steps=10 ** 9,
                     cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)

    def expected():
        ranks = np.concatenate([m.rank_queries(test, true, mode)[0] for mode in ("head-batch", "tail-batch")])
        return float(np.mean(1.0 / ranks)), float(np.mean(ranks))

    for rnd in range(2):
        met = KGEModel.test_step(m, [tuple(x) for x in test.tolist()], [tuple(x) for x in true.tolist()], args)
        mrr, mr = expected()
        assert abs(met["MRR"] - mrr) < 1e-9 and abs(met["MR"] - mr) < 1e-6, (rnd, met, mrr, mr)
        # one training step changes the table before the next evaluation
        pos, neg, w = synth.kge_batch(50 + rnd, 32, 16, E, R)
        m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                              torch.from_numpy(w).to(DEV), "tail-batch", args)
        with torch.no_grad():
            m.entity_embedding.add_(m.entity_embedding.grad, alpha=-100.0)
