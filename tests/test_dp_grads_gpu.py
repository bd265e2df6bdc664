"""Data-parallel GRADIENT exchange through the HIP kernels (distributed.py,
exchange "grads" — what `auto` picks above 2 ranks, i.e. the 8-GPU config-4
path): 2 or 4 ranks (gloo, all on cuda:0 — the one-GPU rehearsal of a node)
each run the fused step on their shard of a global batch with the global Σw,
then the chunked async all-reduce of the dense entity gradient (overlapped
with the entity pass, row chunk by row chunk), the packed all-reduce of the
relation / modulus gradients and loss partials, and the replicated Adam.
Against one process training on the whole batch: the sums over ranks are
taken in another order than the single entity pass's, so gradients, losses
and parameters agree to fp32 rounding, not bit for bit (tolerances below)."""
import os
import socket
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import spawn_ranks
from knowledgegraphembedding_amd import KGEAdam, KGEModel, synth

pytestmark = pytest.mark.gpu

E, R, D, B, N, GAMMA, LR = 301, 7, 40, 16, 24, 12.0, 1e-2
DIMS = {"RotatE": (True, False), "pRotatE": (False, False), "ComplEx": (True, True), "TransE": (False, False),
        "DistMult": (False, False)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(name):
    torch.manual_seed(0)
    de, dr = DIMS[name]
    return KGEModel(name, E, R, D, GAMMA, de, dr).to("cuda:0")


def _batches(dev):
    out = []
    for k, mode in enumerate(("tail-batch", "head-batch")):
        pos, neg, w = synth.kge_batch(70 + k, B, N, E, R)
        out.append((torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode))
    return out


def _args(group, reg, uni):
    return Namespace(cuda=True, negative_adversarial_sampling=not uni, adversarial_temperature=0.8, uni_weight=uni,
                     regularization=reg, dp_group=group, dp_exchange="grads")


def _snapshot(model, logs):
    return {"logs": [dict(l) for l in logs], "ent": model.entity_embedding.detach().cpu().numpy(),
            "rel": model.relation_embedding.detach().cpu().numpy(),
            "gent": model.entity_embedding.grad.cpu().numpy(), "grel": model.relation_embedding.grad.cpu().numpy(),
            "mod": model.modulus.detach().cpu().numpy() if model.model_name == "pRotatE" else None}


def _worker(rank, world, port, name, reg, uni, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _model(name)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _batches("cuda:0")])
    logs = [KGEModel.train_step(model, opt, it, _args(dist.group.WORLD, reg, uni)) for _ in range(2)]
    torch.cuda.synchronize()
    out[rank] = _snapshot(model, logs)
    dist.destroy_process_group()


@pytest.mark.parametrize("name,reg,uni,world", [("RotatE", 0.0, False, 2), ("RotatE", 0.0, False, 4),
                                                ("ComplEx", 1e-4, False, 4), ("pRotatE", 0.0, True, 2),
                                                ("TransE", 0.0, False, 4), ("DistMult", 1e-4, True, 2)])
def test_grads_exchange_matches_one_process(name, reg, uni, world):
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), name, reg, uni, out), world)
    model = _model(name)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    it = iter(_batches("cuda:0"))
    ref = _snapshot(model, [KGEModel.train_step(model, opt, it, _args(None, reg, uni)) for _ in range(2)])
    for rank in range(world):
        r = out[rank]
        # replicas stay identical: every rank applied the same reduced gradient
        assert np.array_equal(r["ent"], out[0]["ent"]) and np.array_equal(r["rel"], out[0]["rel"])
        for k in ("gent", "grel"):
            tol = 1e-5 * np.abs(ref[k]).max() + 1e-5 * np.abs(ref[k])
            assert np.all(np.abs(r[k] - ref[k]) <= tol), (rank, k, float(np.abs(r[k] - ref[k]).max()))
        for k in ("ent", "rel"):
            np.testing.assert_allclose(r[k], ref[k], rtol=1e-4, atol=2e-6, err_msg=f"rank {rank} {k}")
        if ref["mod"] is not None:
            np.testing.assert_allclose(r["mod"], ref["mod"], rtol=1e-5)
        for lg, lr_ in zip(r["logs"], ref["logs"]):
            assert set(lg) == set(lr_)
            for key in lr_:
                assert abs(lg[key] - lr_[key]) <= 1e-5 * max(1.0, abs(lr_[key])), (key, lg[key], lr_[key])
