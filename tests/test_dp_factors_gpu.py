"""Data-parallel FACTOR EXCHANGE through the HIP kernels (distributed.py,
exchange "factors"): two ranks (gloo, both on cuda:0 — the one-GPU rehearsal
of a 2-GPU node) each run the row pass on half of a global batch, all-gather
the per-row factors and run the rest of the step for the global batch.  The
tables after two fused KGEAdam steps, the gradients and the losses must be
BIT-identical to one process training on the whole batch: every per-row
quantity is computed by the same kernel from the same inputs (Σw included,
kge_weight_sum uses the in-kernel order), and the global pass sees the same
batch."""
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
        pos, neg, w = synth.kge_batch(60 + k, B, N, E, R)
        out.append((torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode))
    return out


def _args(group, reg, uni):
    return Namespace(cuda=True, negative_adversarial_sampling=not uni, adversarial_temperature=0.8, uni_weight=uni,
                     regularization=reg, dp_group=group, dp_exchange="factors")


def _snapshot(model, logs):
    return {"logs": [dict(l) for l in logs], "ent": model.entity_embedding.detach().cpu().numpy(),
            "rel": model.relation_embedding.detach().cpu().numpy(),
            "gent": model.entity_embedding.grad.cpu().numpy(),
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


@pytest.mark.parametrize("name,reg,uni", [("RotatE", 0.0, False), ("pRotatE", 0.0, True), ("ComplEx", 1e-4, False),
                                          ("TransE", 0.0, False), ("DistMult", 1e-4, True)])
def test_factor_exchange_two_ranks_bitwise(name, reg, uni):
    world = 2
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), name, reg, uni, out), world)
    model = _model(name)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    it = iter(_batches("cuda:0"))
    ref = _snapshot(model, [KGEModel.train_step(model, opt, it, _args(None, reg, uni)) for _ in range(2)])
    for rank in range(world):
        r = out[rank]
        for k in ("ent", "rel", "gent"):
            assert np.array_equal(r[k], ref[k]), (rank, k, float(np.abs(r[k] - ref[k]).max()))
        if ref["mod"] is not None:
            assert np.array_equal(r["mod"], ref["mod"])
        assert r["logs"] == ref["logs"], (r["logs"], ref["logs"])
