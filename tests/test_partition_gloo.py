"""Row-partitioned entity table (knowledgegraphembedding_amd.partition, BASELINE
config 5) with world_size 2 over gloo on CPU.

Two ranks, each owning half of the entity rows and training on half of a
global batch through KGEModel.train_step, must reproduce single-process
training on the whole batch: the tables after two Adam steps (tail-batch,
then head-batch), the losses, and the Adam state gathered back to the full
table layout.  The entity count is odd, so the last shard carries a padding
row.

As in test_dp_gloo.py the per-rank fused kernel is replaced on CPU by the
oracle's autograd of the rank's share of the objective (test infrastructure),
written into the model's gradient buffers as the kernel would; everything
partition.py does — Σw all-reduce, reduce-scatter of the dense entity
gradient to the owners, relation/loss all-reduce, shard Adam, all-gather of
the updated rows — runs for real.
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
from knowledgegraphembedding_amd.partition import EntityRowPartition
from test_dp_gloo import oracle_rank_grads

E, R, D, B, N, GAMMA, LR = 61, 5, 8, 8, 6, 12.0, 1e-2
DIMS = {"RotatE": (True, False), "ComplEx": (True, True), "TransE": (False, False), "DistMult": (False, False),
        "pRotatE": (False, False)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_model(name):
    torch.manual_seed(0)
    de, dr = DIMS[name]
    return KGEModel(name, E, R, D, GAMMA, de, dr)


def _batches():
    out = []
    for k, mode in enumerate(("tail-batch", "head-batch")):
        pos, neg, w = synth.kge_batch(10 + k, B, N, E, R)
        out.append((torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w), mode))
    return out


def _kernel_standin(model):
    """The oracle gradients, delivered into the model's gradient buffers (where the kernel writes)."""
    def run(*a, **k):
        losses = oracle_rank_grads(model, *a, **k)
        ge, gr, gm, _ = model._grad_bufs
        ge.copy_(model.entity_embedding.grad)
        gr.copy_(model.relation_embedding.grad)
        model.entity_embedding.grad, model.relation_embedding.grad = ge, gr
        if gm is not None:
            gm.copy_(model.modulus.grad)
            model.modulus.grad = gm
        return losses
    return run


def _args(adv, uni, reg, group):
    return Namespace(negative_adversarial_sampling=adv, adversarial_temperature=0.8, uni_weight=uni,
                     regularization=reg, dp_group=group)


def _worker(rank, world, port, name, adv, uni, reg, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _make_model(name)
    part = EntityRowPartition(model)
    model.compute_train_grads = _kernel_standin(model)
    opt = torch.optim.Adam(part.parameters(), lr=LR)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _batches()])
    args = _args(adv, uni, reg, dist.group.WORLD)
    logs = [KGEModel.train_step(model, opt, it, args) for _ in range(2)]
    sd = part.gathered_optimizer_state_dict(opt)
    # round trip: a full-table optimizer state loads back into the shard optimizer
    opt2 = torch.optim.Adam(part.parameters(), lr=LR)
    part.load_optimizer_state_dict(opt2, sd)
    same = all(torch.equal(opt2.state[part.shard][k], opt.state[part.shard][k]) for k in ("exp_avg", "exp_avg_sq"))
    res = {"logs": logs, "ent": model.entity_embedding.detach().numpy().copy(),
           "rel": model.relation_embedding.detach().numpy().copy(),
           "m": sd["state"][0]["exp_avg"].numpy(), "v": sd["state"][0]["exp_avg_sq"].numpy(),
           "shape": tuple(part.shard.shape), "roundtrip": same}
    if name == "pRotatE":
        res["mod"] = model.modulus.detach().numpy().copy()
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("name,adv,uni,reg,world", [("RotatE", True, False, 0.0, 2), ("DistMult", False, True, 1e-3, 2),
                                                    ("pRotatE", True, False, 0.0, 2), ("RotatE", True, False, 0.0, 3),
                                                    ("ComplEx", False, False, 1e-3, 4)])
def test_row_partition_matches_single_process(name, adv, uni, reg, world):
    """world 2, 3 (E not a multiple of the world: a padded last shard) and 4."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), name, adv, uni, reg, out), nprocs=world, join=True)

    # single process, whole batch, replicated Adam over (entity, relation[, modulus])
    model = _make_model(name)
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.Adam(params, lr=LR)
    ref_logs = []
    for pos, neg, w, mode in _batches():
        opt.zero_grad()
        losses = oracle_rank_grads(model, pos, neg, w, mode, _args(adv, uni, reg, None),
                                   weight_sum=w.sum().reshape(1), uni_batch=B)
        opt.step()
        ref_logs.append(losses.numpy())
    ent = model.entity_embedding.detach().numpy()
    st = opt.state[model.entity_embedding]
    for rank in range(world):
        r = out[rank]
        assert r["shape"] == (-(-E // world), model.entity_embedding.shape[1])
        np.testing.assert_allclose(r["ent"], ent, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(r["rel"], model.relation_embedding.detach().numpy(), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(r["m"], st["exp_avg"].numpy(), rtol=1e-4, atol=1e-9)
        np.testing.assert_allclose(r["v"], st["exp_avg_sq"].numpy(), rtol=1e-4, atol=1e-12)
        assert r["roundtrip"]
        if name == "pRotatE":
            np.testing.assert_allclose(r["mod"], model.modulus.detach().numpy(), rtol=1e-5)
        for got, ref in zip(r["logs"], ref_logs):
            np.testing.assert_allclose(got["positive_sample_loss"], ref[0], rtol=1e-5)
            np.testing.assert_allclose(got["negative_sample_loss"], ref[1], rtol=1e-5)
            np.testing.assert_allclose(got["loss"], ref[2], rtol=1e-5)


def _ship_host_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _make_model("RotatE")
    full = model.entity_embedding.detach().clone()
    part = EntityRowPartition(model, exchange="queries")
    res = {"placeholder": tuple(model.entity_embedding.shape), "shard": tuple(part.shard.shape),
           "rows": (part.lo, part.lo + part.nown),
           "shard_ok": bool(torch.equal(part.shard[:part.nown].detach(), full[part.lo:part.lo + part.nown]))}
    with torch.no_grad():  # a step's worth of change on this rank's rows only
        part.shard[:part.nown] += 1.0 + rank
    table = part.materialize()
    want = full.clone()
    for r in range(world):
        lo = r * part.rows
        want[lo:min(E, lo + part.rows)] += 1.0 + r
    res["gathered_ok"] = bool(torch.equal(table.detach(), want))
    # a checkpoint written into the gathered table comes back to the shard
    with torch.no_grad():
        model.entity_embedding.mul_(2.0)
    part.reload_from_replica()
    res["reload_ok"] = bool(torch.equal(part.shard[:part.nown].detach(), 2.0 * want[part.lo:part.lo + part.nown]))
    part.release()
    res["released"] = tuple(model.entity_embedding.shape)
    # optimizer state: shard moments gather to the full-table layout and slice back
    opt = torch.optim.Adam(part.parameters(), lr=LR)
    part.shard.grad = torch.ones_like(part.shard)
    model.relation_embedding.grad = torch.zeros_like(model.relation_embedding)
    opt.step()
    sd = part.gathered_optimizer_state_dict(opt)
    res["state_shape"] = tuple(sd["state"][0]["exp_avg"].shape)
    opt2 = torch.optim.Adam(part.parameters(), lr=LR)
    part.load_optimizer_state_dict(opt2, sd)
    res["state_roundtrip"] = bool(torch.equal(opt2.state[part.shard]["exp_avg"][:part.nown],
                                              opt.state[part.shard]["exp_avg"][:part.nown]))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_query_shipping_shards_host(world):
    """Query shipping's host side (partition.py exchange "queries") over gloo
    on CPU: each rank keeps only its shard (the model's table becomes an
    empty placeholder), materialize() gathers every rank's rows in order and
    release() drops them, a checkpoint loaded into the gathered table reaches
    the shard, and the shard's Adam state gathers to the reference's
    full-table layout and slices back.  (The step itself runs only through
    the HIP kernels: tests/test_ship_gpu.py.)"""
    out = mp.Manager().dict()
    mp.spawn(_ship_host_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rows = -(-E // world)
    for rank in range(world):
        r = out[rank]
        assert r["placeholder"] == (0, 2 * D) and r["released"] == (0, 2 * D)
        assert r["shard"] == (rows, 2 * D)
        assert r["rows"] == (rank * rows, min(E, (rank + 1) * rows))
        assert r["shard_ok"] and r["gathered_ok"] and r["reload_ok"] and r["state_roundtrip"], r
        assert r["state_shape"] == (E, 2 * D)
