"""OWNER-COMPUTES exchange through the HIP kernels (partition.py exchange
"factors" = distributed.py "owner", what `auto` picks above 2 ranks): 2 or 4
ranks (gloo, all on cuda:0) exchange the row pass's factors, each runs the
entity-major pass with fused Adam for the rows it owns over the global batch
(kge_train_step_from_rows_range), and the updated rows are all-gathered.
Against one process training on the whole batch the tables, the Adam moments
of each owner's rows and the losses are BIT-identical (every row sees the
same occurrences in the same order, with the same gathered factors); only
the regularisation loss is summed over the owners in another order."""
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


def _worker(rank, world, port, name, reg, uni, chunks, e, d, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd import partition
    from knowledgegraphembedding_amd.partition import EntityRowPartition
    partition.OWNER_CHUNKS = chunks
    model = _model(name, e, d)
    part = EntityRowPartition(model, dist.group.WORLD, exchange="factors")
    opt = KGEAdam(part.parameters(), lr=LR)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _batches("cuda:0", e)])
    logs = [dict(KGEModel.train_step(model, opt, it, _args(dist.group.WORLD, reg, uni))) for _ in range(3)]
    torch.cuda.synchronize()
    st = opt.state[part.shard]
    out[rank] = {"logs": logs, "ent": model.entity_embedding.detach().cpu().numpy(),
                 "rel": model.relation_embedding.detach().cpu().numpy(), "lo": part.e0, "hi": part.e1,
                 "m": st["exp_avg"][:part.nown].cpu().numpy(),
                 "v": st["exp_avg_sq"][:part.nown].cpu().numpy(),
                 "mod": model.modulus.detach().cpu().numpy() if name == "pRotatE" else None}
    dist.destroy_process_group()


@pytest.mark.parametrize("name,reg,uni,world,chunks,e,d", [("RotatE", 0.0, False, 2, 4, E, D), ("RotatE", 0.0, False, 4, 4, E, D),
                                                           ("RotatE", 0.0, False, 2, 1, E, D), ("ComplEx", 1e-4, False, 4, 4, E, D),
                                                           ("pRotatE", 0.0, True, 2, 4, E, D), ("TransE", 0.0, False, 4, 1, E, D),
                                                           ("DistMult", 1e-4, True, 2, 3, E, D), ("RotatE", 1e-4, False, 4, 4, 5, D),
                                                           ("RotatE", 0.0, False, 2, 4, E, 2100), ("TransE", 1e-4, False, 2, 1, E, 2051)])
def test_owner_exchange_bitwise(name, reg, uni, world, chunks, e, d):
    """chunks > 1: the owned rows' pass in chunks (kge_train_step_from_rows_phased),
    each chunk's all-gather issued before the next chunk runs (151 owned rows
    at world 2 give 4 chunks, 76 at world 4 give 2); 1: one call and one
    all-gather.  Both bit-identical to one process.  e = 5 at world 4: shards
    of 2 rows, rank 2 owns one row and rank 3 starts past the table (lo = 6),
    so its range is empty (the owner step clamps it).  d = 2100 /
    2051: rows over 2048 floats (kge_wide.inc) through the same exchange."""
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), name, reg, uni, chunks, e, d, out), world)
    model = _model(name, e, d)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    it = iter(_batches("cuda:0", e))
    ref = [dict(KGEModel.train_step(model, opt, it, _args(None, reg, uni))) for _ in range(3)]
    ent = model.entity_embedding.detach().cpu().numpy()
    rel = model.relation_embedding.detach().cpu().numpy()
    st = opt.state[model.entity_embedding]
    m_ref, v_ref = st["exp_avg"].cpu().numpy(), st["exp_avg_sq"].cpu().numpy()
    for rank in range(world):
        r = out[rank]
        assert np.array_equal(r["ent"], ent), (rank, float(np.abs(r["ent"] - ent).max()))
        assert np.array_equal(r["rel"], rel), rank
        lo, hi = r["lo"], r["hi"]
        assert np.array_equal(r["m"], m_ref[lo:hi]) and np.array_equal(r["v"], v_ref[lo:hi]), rank
        if r["mod"] is not None:
            assert np.array_equal(r["mod"], model.modulus.detach().cpu().numpy())
        for got, want in zip(r["logs"], ref):
            for k in ("positive_sample_loss", "negative_sample_loss"):
                assert got[k] == want[k], (k, got[k], want[k])
            for k in ("loss",) + (("regularization",) if reg else ()):
                assert abs(got[k] - want[k]) <= 1e-6 * max(1.0, abs(want[k])), (k, got[k], want[k])
