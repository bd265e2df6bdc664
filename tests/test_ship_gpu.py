"""QUERY SHIPPING through the HIP kernels (partition.py exchange "queries",
kge_ship_step): 2-4 ranks (gloo, all on cuda:0) each hold ONLY their shard
of the entity table; the global batch's q vectors travel instead of rows.
Against one process training on the whole batch the gradients, losses and
tables agree to fp32 rounding (the softmax normaliser, dL/dq and the
relation gradient are summed over the shards in shard order, so not bit
for bit)."""
import faulthandler
import os
import socket
import sys
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import spawn_ranks
from knowledgegraphembedding_amd import KGEAdam, KGEModel, synth

pytestmark = pytest.mark.gpu

E, R, D, B, N, GAMMA, LR = 301, 7, 40, 16, 24, 12.0, 1e-3
DIMS = {"RotatE": (True, False), "pRotatE": (False, False), "ComplEx": (True, True), "TransE": (False, False),
        "DistMult": (False, False)}
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(name, e=E, d=D):
    torch.manual_seed(0)
    de, dr = DIMS[name]
    return KGEModel(name, e, R, d, GAMMA, de, dr).to("cuda:0")


def _batches(dev, e=E):
    out = []
    for k, mode in enumerate(("tail-batch", "head-batch", "tail-batch")):
        pos, neg, w = synth.kge_batch(80 + k, B, N, e, R)
        out.append((torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode))
    return out


def _args(group, reg, uni):
    return Namespace(cuda=True, negative_adversarial_sampling=not uni, adversarial_temperature=0.8, uni_weight=uni,
                     regularization=reg, dp_group=group)


def _worker(rank, world, port, name, reg, uni, e, d, env, out):
    faulthandler.dump_traceback_later(45, repeat=True, file=sys.stderr)  # a slow rank shows where it waits
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd.partition import EntityRowPartition
    model = _model(name, e, d)
    part = EntityRowPartition(model, dist.group.WORLD, exchange="queries")
    assert model.entity_embedding.shape[0] == 0  # no replica while training
    opt = KGEAdam(part.parameters(), lr=LR)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _batches("cuda:0", e)])
    logs, grads = [], []
    for _ in range(STEPS):
        logs.append(dict(KGEModel.train_step(model, opt, it, _args(dist.group.WORLD, reg, uni))))
        grads.append((part.shard.grad[:part.nown].cpu().numpy().copy(), model.relation_embedding.grad.cpu().numpy()))
    torch.cuda.synchronize()
    ent = part.materialize().detach().cpu().numpy()
    out[rank] = {"logs": logs, "grads": grads, "ent": ent, "rel": model.relation_embedding.detach().cpu().numpy(),
                 "lo": part.lo, "hi": part.lo + part.nown,
                 "mod": model.modulus.detach().cpu().numpy() if name == "pRotatE" else None}
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def _close(got, want, what, rtol=2e-4):
    if want.size == 0:
        return
    scale = max(1e-30, float(np.abs(want).max()))
    err = float(np.abs(got - want).max())
    assert err <= rtol * scale, (what, err, scale)


@pytest.mark.parametrize("name,reg,uni,world,e,d,env", [
    ("RotatE", 0.0, False, 2, E, D, {}), ("RotatE", 0.0, False, 4, 6, D, {}),
    ("ComplEx", 1e-4, False, 4, E, D, {"KGE_ENT_SLICES": "0"}), ("pRotatE", 0.0, True, 2, E, D, {}),
    ("TransE", 0.0, False, 4, E, 30, {}), ("DistMult", 1e-4, True, 2, E, D, {})])
def test_query_shipping_matches_one_process(name, reg, uni, world, e, d, env):
    """e = 6 at world 4: shards of 2 rows, the last one empty; d = 30: rows
    that are not float4-aligned (scalar-slot kernels, row-per-wave entity
    pass); KGE_ENT_SLICES=0: the row-per-wave entity pass on float4 rows."""
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), name, reg, uni, e, d, env, out), world)
    model = _model(name, e, d)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    it = iter(_batches("cuda:0", e))
    ref, ref_grads = [], []
    for _ in range(STEPS):
        ref.append(dict(KGEModel.train_step(model, opt, it, _args(None, reg, uni))))
        ref_grads.append((model.entity_embedding.grad.cpu().numpy().copy(), model.relation_embedding.grad.cpu().numpy()))
    ent = model.entity_embedding.detach().cpu().numpy()
    rel = model.relation_embedding.detach().cpu().numpy()
    for rank in range(world):
        r = out[rank]
        lo, hi = r["lo"], r["hi"]
        for s, ((ge, gr), (ge_ref, gr_ref)) in enumerate(zip(r["grads"], ref_grads)):
            _close(ge, ge_ref[lo:hi], ("entity grad", rank, s))
            _close(gr, gr_ref, ("relation grad", rank, s))
        _close(r["ent"], ent, ("entity table", rank), rtol=1e-4)
        _close(r["rel"], rel, ("relation table", rank), rtol=1e-4)
        if r["mod"] is not None:
            _close(r["mod"], model.modulus.detach().cpu().numpy(), "modulus", rtol=1e-5)
        for got, want in zip(r["logs"], ref):
            for k in ("positive_sample_loss", "negative_sample_loss", "loss") + (("regularization",) if reg else ()):
                assert abs(got[k] - want[k]) <= 1e-5 * max(1.0, abs(want[k])), (k, got[k], want[k])
