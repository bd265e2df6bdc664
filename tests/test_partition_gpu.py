"""Row-partitioned entity table through the HIP kernels: two ranks (gloo, both
on cuda:0 — the one-GPU box rehearsal of BASELINE config 5), each owning half
of the entity rows and training on half of a global batch, against
single-process training of the whole batch on the same GPU.  Tables after two
KGEAdam steps and the losses must agree to fp32 rounding (the two paths sum
the per-rank dense gradients in a different order)."""
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

E, R, D, B, N, GAMMA, LR = 301, 7, 32, 16, 8, 12.0, 1e-2
DIMS = {"RotatE": (True, False), "pRotatE": (False, False), "ComplEx": (True, True)}


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
        pos, neg, w = synth.kge_batch(40 + k, B, N, E, R)
        out.append((torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode))
    return out


def _args(group, reg=0.0):
    return Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=reg, dp_group=group)


def _worker(rank, world, port, name, reg, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd.partition import EntityRowPartition
    model = _model(name)
    part = EntityRowPartition(model)
    opt = KGEAdam(part.parameters(), lr=LR)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _batches("cuda:0")])
    logs = [KGEModel.train_step(model, opt, it, _args(dist.group.WORLD, reg)) for _ in range(2)]
    torch.cuda.synchronize()
    out[rank] = {"logs": logs, "ent": model.entity_embedding.detach().cpu().numpy(),
                 "rel": model.relation_embedding.detach().cpu().numpy()}
    dist.destroy_process_group()


@pytest.mark.parametrize("name,reg", [("RotatE", 0.0), ("pRotatE", 0.0), ("ComplEx", 1e-4)])
def test_row_partition_two_ranks_on_gpu(name, reg):
    world = 2
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), name, reg, out), world)
    model = _model(name)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    it = iter(_batches("cuda:0"))
    ref = [KGEModel.train_step(model, opt, it, _args(None, reg)) for _ in range(2)]
    ent = model.entity_embedding.detach().cpu().numpy()
    rel = model.relation_embedding.detach().cpu().numpy()
    for rank in range(world):
        r = out[rank]
        np.testing.assert_allclose(r["ent"], ent, rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(r["rel"], rel, rtol=1e-5, atol=2e-6)
        for got, want in zip(r["logs"], ref):
            for k in ("positive_sample_loss", "negative_sample_loss", "loss") + (("regularization",) if reg else ()):
                np.testing.assert_allclose(got[k], want[k], rtol=2e-5)


# ---------------------------------------------------------- config 5 shape
YE, YR, YD, YB, YN = 123182, 37, 1000, 1024, 1024
SAMPLE_ROWS = np.unique(synth.randint(93, (4096,), YE))


def _yago_model():
    torch.manual_seed(3)
    return KGEModel("RotatE", YE, YR, YD, 24.0, True, False).to("cuda:0")


def _yago_batches(dev, world=1):
    """The global batches of the two steps: world × 1024 rows (rank order)."""
    out = []
    for k, mode in enumerate(("tail-batch", "head-batch")):
        pos, neg, w = synth.kge_batch(95 + k, world * YB, YN, YE, YR)
        out.append((torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode))
    return out


ROWS8 = [0, 1, 100, 511, 512, 700, 900, 1023]


def _yago_worker(rank, world, port, exchange, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd.partition import EntityRowPartition
    model = _yago_model()
    part = EntityRowPartition(model, dist.group.WORLD, exchange=exchange)
    opt = KGEAdam(part.parameters(), lr=1e-4)
    sl = slice(rank * YB, (rank + 1) * YB)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _yago_batches("cuda:0", world)])
    logs, fps = [], []
    for _ in range(2):
        logs.append(dict(KGEModel.train_step(model, opt, it, _args(dist.group.WORLD))))
        fps.append(part.replica_checksums().cpu().numpy())  # per step: which step a replica diverged in
    torch.cuda.synchronize()
    ent = part.materialize()  # query shipping: the shards gathered (collective); otherwise the replica
    res = {"logs": logs, "ent": ent.detach()[torch.from_numpy(SAMPLE_ROWS).cuda()].cpu().numpy(),
           "rel": model.relation_embedding.detach().cpu().numpy(), "fps": fps}
    if rank == 0:
        # 8 rows' scores of the trained (gathered) table against the oracle's op chain on the same table
        from oracle import kge_oracle as O
        pos, neg, _, _ = _yago_batches("cpu", world)[0]
        P, N = pos[ROWS8], neg[ROWS8]
        with torch.no_grad():
            s = model((P.cuda(), N.cuda()), "tail-batch").cpu().numpy()
        sref = O.forward("RotatE", ent.detach().cpu(), model.relation_embedding.detach().cpu(), None, (P, N),
                         "tail-batch", 24.0, model.embedding_range.item()).numpy()
        res["score_err"] = float(np.max(np.abs(s - sref) / np.maximum(np.abs(sref), 1.0)))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange", [(2, "grads"), (2, "factors"), (2, "queries"), (4, "queries"),
                                            (4, "factors"), (8, "factors"), (8, "queries")])
def test_row_partition_yago3_10_shape(world, exchange):
    """BASELINE config 5's shape (RotatE, E = 123182, d = 1000 -de, n = 1024;
    985 MB entity table) at its own 1024 positives per rank (VERDICT r03 #7,
    r04 #2: up to its own 8 ranks): `world` ranks each owning 1/world of the
    rows — 15,398 at world 8 — with the reduce-scatter ("grads"),
    owner-computes ("factors", run.py's --row_partition default) and
    query-shipping ("queries": no rank holds the table; q vectors travel, the
    softmax merged over `world` shards) exchanges, for two KGEAdam steps,
    against one process training the world × 1024-row global batch (8192
    rows at world 8).  Owner-computes is bit-identical to the one process
    (every per-row quantity comes from the same kernels on the same inputs);
    the others agree on sampled entity rows, the relation table and the
    losses to fp32 rounding.  Then rank 0's trained (gathered) table scores 8
    rows against the CPU oracle's op chain on that same table (north-star
    tolerance)."""
    out = mp.Manager().dict()
    spawn_ranks(_yago_worker, (world, _free_port(), exchange, out), world)
    model = _yago_model()
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    it = iter(_yago_batches("cuda:0", world))
    ref = [dict(KGEModel.train_step(model, opt, it, _args(None))) for _ in range(2)]
    ent = model.entity_embedding.detach()[torch.from_numpy(SAMPLE_ROWS).cuda()].cpu().numpy()
    rel = model.relation_embedding.detach().cpu().numpy()

    def close(got, want, what):
        # an element whose gradient sums to ~0 can take Adam's ±lr step with
        # the other sign when the two paths round the sum differently (world
        # 8's query shipping sums the relation gradient over 8 shards: one such
        # element of the 37,000 relation entries, r05d): allow such elements
        # (≤ 1e-5 of them, at least 2), never a step larger than 2 lr
        bad = np.abs(got - want) > 1e-5 * np.abs(want) + 2e-7
        assert bad.sum() <= max(2, 1e-5 * got.size), (what, int(bad.sum()))
        assert np.abs(got - want).max() <= 2 * 2 * 1e-4 + 1e-6, what

    # every rank's replica (query shipping: relation table) fingerprint, per step, equals rank 0's
    fps = [out[r]["fps"] for r in range(world)]
    for step in range(2):
        diverged = [r for r in range(world) if not np.array_equal(fps[r][step], fps[0][step])]
        assert not diverged, ("replica fingerprints differ from rank 0's after step", step + 1, diverged)
    for rank in range(world):
        r = out[rank]
        if exchange == "factors":
            if not np.array_equal(r["ent"], ent):
                # which rows (by owner) and columns differ, for the record
                S = -(-YE // world)
                badr = np.nonzero((r["ent"] != ent).any(1))[0]
                owners = np.bincount(SAMPLE_ROWS[badr] // S, minlength=world).tolist()
                cols = np.nonzero((r["ent"] != ent).any(0))[0]
                zero = int((r["ent"][badr] == 0).all(1).sum())
                raise AssertionError(("entity rows", rank, float(np.abs(r["ent"] - ent).max()), "bad rows", len(badr),
                                      "by owner", owners, "all-zero", zero, "cols", int(cols.min()), int(cols.max()),
                                      len(cols)))
            assert np.array_equal(r["rel"], rel), ("relation table", rank)
            for got, want in zip(r["logs"], ref):
                for k in ("positive_sample_loss", "negative_sample_loss", "loss"):
                    assert got[k] == want[k], (k, rank, got[k], want[k])
            continue
        close(r["ent"], ent, ("entity rows", rank))
        close(r["rel"], rel, ("relation table", rank))
        for got, want in zip(r["logs"], ref):
            for k in ("positive_sample_loss", "negative_sample_loss", "loss"):
                np.testing.assert_allclose(got[k], want[k], rtol=2e-5)
    assert out[0]["score_err"] <= 1e-4, out[0]["score_err"]
