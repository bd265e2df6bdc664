"""Data-parallel training logic (knowledgegraphembedding_amd.distributed) with
world_size 2 over gloo on CPU: two ranks, each with half of a global batch,
must reproduce the single-process loss and gradients of the whole batch
(model.py:268-301 semantics: the subsampling normaliser Σw is global).

On CPU the per-rank fused kernel is replaced by the oracle's autograd of the
same per-rank objective (this file is test infrastructure); everything the DP
layer itself does — Σw all-reduce, gradient + loss all-reduce, loss
recomposition, regularisation counted once — runs for real.
"""
import os
import socket
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from knowledgegraphembedding_amd import KGEModel, synth
from knowledgegraphembedding_amd import distributed as kdist
from oracle import kge_oracle as O

E, R, D, B, N, GAMMA = 60, 5, 8, 8, 6, 12.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_model(name):
    torch.manual_seed(0)
    de, dr = {"RotatE": (True, False), "ComplEx": (True, True), "TransE": (False, False),
              "DistMult": (False, False), "pRotatE": (False, False)}[name]
    return KGEModel(name, E, R, D, GAMMA, de, dr)


def oracle_rank_grads(model, pos, neg, w, mode, args, weight_sum=None, uni_batch=0, optimizer=None,
                      entity_chunks=None, on_entity_chunk=None):
    """Per-rank objective: the rank's share of the global loss.  Honours the
    chunk hook of KGEModel.compute_train_grads (called after the gradient is
    complete, chunk by chunk, as the kernels would)."""
    name = model.model_name
    ent = model.entity_embedding.detach().clone().requires_grad_(True)
    rel = model.relation_embedding.detach().clone().requires_grad_(True)
    mod = model.modulus.detach().clone().requires_grad_(True) if name == "pRotatE" else None
    g, rng = model.gamma.item(), model.embedding_range.item()
    s_neg = O.forward(name, ent, rel, mod, (pos, neg), mode, g, rng)
    if args.negative_adversarial_sampling:
        neg_term = (torch.softmax(s_neg * args.adversarial_temperature, 1).detach()
                    * torch.nn.functional.logsigmoid(-s_neg)).sum(1)
    else:
        neg_term = torch.nn.functional.logsigmoid(-s_neg).mean(1)
    pos_term = torch.nn.functional.logsigmoid(O.forward(name, ent, rel, mod, pos, "single", g, rng)).squeeze(1)
    if args.uni_weight:
        pl, nl = -pos_term.sum() / uni_batch, -neg_term.sum() / uni_batch
    else:
        pl, nl = -(w * pos_term).sum() / weight_sum[0], -(w * neg_term).sum() / weight_sum[0]
    loss = (pl + nl) / 2
    reg = torch.zeros(())
    if args.regularization != 0.0:
        reg = args.regularization * (ent.norm(p=3) ** 3 + rel.norm(p=3).norm(p=3) ** 3)
        loss = loss + reg
    loss.backward()
    model.entity_embedding.grad = ent.grad
    model.relation_embedding.grad = rel.grad
    if mod is not None:
        model.modulus.grad = mod.grad
    for e0, e1 in (entity_chunks or []):
        if on_entity_chunk is not None:
            on_entity_chunk(e0, e1, model.entity_embedding.grad)
    return torch.stack([pl.detach(), nl.detach(), loss.detach(), reg.detach(), torch.zeros(())]).float()


def _worker(rank, world, port, name, adv, uni, reg, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _make_model(name)
    model.compute_train_grads = lambda *a, **k: oracle_rank_grads(model, *a, **k)
    pos, neg, w = synth.kge_batch(3, B, N, E, R)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    args = Namespace(negative_adversarial_sampling=adv, adversarial_temperature=0.8, uni_weight=uni,
                     regularization=reg, dp_group=dist.group.WORLD)
    losses = kdist.dp_train_grads(model, torch.from_numpy(pos[sl]), torch.from_numpy(neg[sl]),
                                  torch.from_numpy(w[sl]), "tail-batch", args)
    res = [losses.numpy(), model.entity_embedding.grad.numpy(), model.relation_embedding.grad.numpy()]
    if name == "pRotatE":
        res.append(model.modulus.grad.numpy())
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("name,adv,uni,reg,world", [("RotatE", True, False, 0.0, 2), ("ComplEx", False, True, 1e-3, 2),
                                                    ("pRotatE", True, False, 0.0, 2), ("DistMult", True, False, 1e-3, 2),
                                                    ("RotatE", True, False, 0.0, 4), ("TransE", False, True, 1e-3, 4),
                                                    ("DistMult", True, False, 1e-3, 8)])
def test_dp_ranks_match_global_batch(name, adv, uni, reg, world):
    """world 2, 4 and 8 (the driver's 4- and 8-GPU runs use this "grads" exchange;
    at 8 ranks each holds one positive of the global batch)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), name, adv, uni, reg, out), nprocs=world, join=True)
    model = _make_model(name)
    pos, neg, w = synth.kge_batch(3, B, N, E, R)
    log, ge, gr, gm = O.train_grads(name, model.entity_embedding.detach(), model.relation_embedding.detach(),
                                    model.modulus.detach() if name == "pRotatE" else None, torch.from_numpy(pos),
                                    torch.from_numpy(neg), torch.from_numpy(w), "tail-batch", adversarial=adv,
                                    temperature=0.8, uni_weight=uni, regularization=reg,
                                    gamma=model.gamma.item(), erange=model.embedding_range.item())
    ref_losses = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"],
                           log.get("regularization", 0.0)])
    for rank in range(world):
        losses, g_e, g_r = out[rank][:3]
        np.testing.assert_allclose(losses[:4], ref_losses, rtol=1e-5, atol=1e-6)
        assert losses[4] == 0.0  # error flag
        np.testing.assert_allclose(g_e, ge.numpy(), rtol=1e-4, atol=1e-6 * np.abs(ge.numpy()).max())
        np.testing.assert_allclose(g_r, gr.numpy(), rtol=1e-4, atol=1e-6 * np.abs(gr.numpy()).max())
        if name == "pRotatE":
            np.testing.assert_allclose(out[rank][3], gm.numpy(), rtol=1e-4)


# ---------------------------------------------------------------- factor exchange
# The exchange's data movement (distributed.dp_train_step_factors) with world
# size 2 over gloo on CPU.  The two HIP entry points are replaced by stand-ins
# that write a known function of the rank's own rows and record what the
# global step receives (test infrastructure); the parity of the real kernels
# is tests/test_dp_factors_gpu.py (bit-identical to one process).
LE = 2 * D


def _fx_rows(pos, neg, w, g_out, dq_out, stats_out):
    g_out.copy_(neg.float() * w[:, None])
    dq_out.copy_(pos.float().sum(1, keepdim=True) + torch.arange(LE, dtype=torch.float32))
    stats_out.zero_()
    stats_out[:, 1] = 2 * w
    stats_out[:, 2] = 3 * w


def _fx_worker(rank, world, port, uni, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd import ops
    seen = {}

    def rows_slice(desc, mode, pos, neg, w, wsum, dev, *, adversarial, temperature, uni_weight, uni_batch, g_out,
                   dq_out, stats_out):
        seen["slice"] = (uni_batch, None if wsum is None else float(wsum[0]))
        _fx_rows(pos, neg, w, g_out, dq_out, stats_out)

    def csr(desc, mode, pos, neg, dev, workspace=None, entity_range=None):
        seen["csr"] = [t.clone() for t in (pos, neg)]
        seen["csr_range"] = entity_range

    def from_rows(desc, mode, pos, neg, w, wsum, dev, *, uni_weight, uni_batch, regularization, g_in, dq_in, stats,
                  grad_entity, grad_relation, grad_modulus, losses, adam=None, csr_ready=False, workspace=None):
        seen["csr_ready"] = csr_ready
        seen["global"] = [t.clone() for t in (pos, neg, w, g_in, dq_in, stats)]
        seen["global_scalars"] = (uni_batch, regularization, None if wsum is None else float(wsum[0]))
        losses.copy_(torch.tensor([float(w.sum()), float(g_in.sum()), float(dq_in.sum()), float(stats.sum()), 0.]))

    ops.train_rows_slice, ops.train_step_from_rows, ops.train_csr = rows_slice, from_rows, csr
    ops.weight_sum = lambda w, o: o.copy_(w.sum().reshape(1))
    model = _make_model("RotatE")
    pos, neg, w = synth.kge_batch(5, B, N, E, R)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=uni,
                     regularization=1e-3, dp_group=dist.group.WORLD)
    losses = kdist.dp_train_step_factors(model, torch.from_numpy(pos[sl]), torch.from_numpy(neg[sl]),
                                         torch.from_numpy(w[sl]), "tail-batch", args)
    out[rank] = {"losses": losses.clone(), "seen": seen}
    dist.destroy_process_group()


@pytest.mark.parametrize("uni,world", [(False, 2), (True, 2), (False, 4)])
def test_factor_exchange_gathers_global_batch(uni, world):
    out = mp.Manager().dict()
    mp.spawn(_fx_worker, args=(world, _free_port(), uni, out), nprocs=world, join=True)
    pos, neg, w = (torch.from_numpy(x) for x in synth.kge_batch(5, B, N, E, R))
    g = torch.empty(B, N)
    dq = torch.empty(B, LE)
    st = torch.empty(B, 4)
    _fx_rows(pos, neg, w, g, dq, st)  # the stand-in over the whole batch = the two slices concatenated
    assert kdist.dp_exchange_mode(2) == "factors" and kdist.dp_exchange_mode(8) == "owner"
    for rank in range(world):
        s = out[rank]["seen"]
        for got, want in zip(s["global"], (pos, neg, w, g, dq, st)):
            assert torch.equal(got, want.to(got.dtype))
        assert s["slice"][0] == B and s["global_scalars"][:2] == (B, 1e-3)
        # the CSR built ahead saw the same global ids the rest of the step sees
        assert s["csr_ready"] and all(torch.equal(a, b) for a, b in zip(s["csr"], s["global"][:2]))
        assert s["csr_range"] is None  # every rank runs the whole global step: every entity's bucket
        if uni:
            assert s["slice"][1] is None and s["global_scalars"][2] is None
        else:  # Σw of the GLOBAL weights, on both sides of the exchange
            assert s["slice"][1] == pytest.approx(float(w.sum())) and s["global_scalars"][2] == s["slice"][1]
    for rank in range(1, world):
        assert torch.equal(out[0]["losses"], out[rank]["losses"])


def _shard_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd.dataloader import RankShardSampler
    from knowledgegraphembedding_amd.run import shared_seed
    torch.manual_seed(1000 + 17 * rank)  # every rank's own torch seed differs
    seed = shared_seed(dist.group.WORLD)
    sampler = RankShardSampler(103, rank, world, seed)
    out[rank] = (seed, list(sampler), list(sampler))  # two epochs
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank_shards_disjoint_with_per_rank_torch_seeds(world):
    """the sampler seed is rank 0's, broadcast, so even with
    different torch seeds per rank one epoch's shards are disjoint, equally
    long and cover world·⌊n/world⌋ positives; the next epoch reshuffles."""
    out = mp.Manager().dict()
    mp.spawn(_shard_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    seeds = {out[r][0] for r in range(world)}
    assert len(seeds) == 1
    for ep in (1, 2):
        shards = [out[r][ep] for r in range(world)]
        assert all(len(s) == 103 // world for s in shards)
        union = set().union(*map(set, shards))
        assert len(union) == world * (103 // world)
    assert out[0][1] != out[0][2]


def _fp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(5)
    ent, rel = torch.randn(37, 6), torch.randn(4, 3)
    same = kdist.replicas_disagree(kdist.table_fingerprint(ent, rel))
    if rank == 2:  # one rank's replica diverges: one row zeroed, then one bit of the relation table
        ent[11, :2] = 0.0
    after_row = kdist.replicas_disagree(kdist.table_fingerprint(ent, rel))
    if rank == 2:
        ent[11, :2] = torch.randn(37, 6, generator=torch.Generator().manual_seed(5))[11, :2]
        rel.view(-1).view(torch.int32)[5] ^= 1
    after_bit = kdist.replicas_disagree(kdist.table_fingerprint(ent, rel))
    out[rank] = (same, after_row, after_bit)
    dist.destroy_process_group()


def test_replica_fingerprint_names_diverged_rank():
    """bench.py's multi-GPU replica check (distributed.replicas_disagree):
    identical replicas agree; a leading part of one rank's row zeroed, or one
    flipped bit of its relation table, names exactly that rank on every rank."""
    world = 3
    out = mp.Manager().dict()
    mp.spawn(_fp_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        assert out[r] == ([], [2], [2]), (r, out[r])
