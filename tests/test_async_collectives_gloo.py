"""The data-parallel exchanges under RCCL-like asynchrony, on CPU (gloo).

Gloo on CPU completes a collective inside the call, so it cannot show a
buffer that is read before its collective has landed or overwritten while a
collective may still read it — exactly what RCCL's semantics allow to go
wrong (an async collective runs on its own stream; `wait()` orders the
caller's stream behind it, it does not block the host).  Here every
`async_op=True` collective is DEFERRED: nothing moves until its `wait()` (or
never, if nobody waits), so its input is read at the latest moment and its
output written at the latest moment RCCL could.  Each exchange then runs two
consecutive steps with different data and no extra host synchronisation:

  * "grads" (distributed.dp_train_grads): per-chunk async all-reduces of the
    entity gradient, Adam per chunk behind its wait, the packed relation /
    loss all-reduce — losses and gradients of both steps against the oracle;
  * "factors" (distributed.dp_train_step_factors): the pieces' async
    all-gathers into the reused staging buffers (_FX_BUFS) and the ids'
    all-gathers — the global step of each step must see exactly that step's
    global batch;
  * "owner" (partition.EntityRowPartition put_chunk / gather): per-chunk async
    row all-gathers into the reused per-chunk staging buffers — every rank's
    replica must hold every rank's rows of THAT step.

The C-ABI's own side stream (CSR, relation pass) is joined by events inside
each call (kge_capi.hip run_grad), so no collective ever sees it."""
import os
import socket
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from knowledgegraphembedding_amd import KGEModel, partition, synth
from knowledgegraphembedding_amd import distributed as kdist
from oracle import kge_oracle as O

E, R, D, B, N, GAMMA = 60, 5, 8, 8, 6, 12.0
ASYNC = ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "all_gather", "broadcast")


class _DeferredWork:
    def __init__(self, fn):
        self._fn = fn

    def wait(self, timeout=None):
        if self._fn is not None:
            fn, self._fn = self._fn, None
            fn()
        return True

    def is_completed(self):
        return self._fn is None


def install_deferred_collectives():
    """Make every async collective of torch.distributed run at its wait()."""
    for name in ASYNC:
        orig = getattr(dist, name)

        def wrapper(*a, _orig=orig, async_op=False, **k):
            if not async_op:
                return _orig(*a, **k)
            return _DeferredWork(lambda: _orig(*a, **k))
        setattr(dist, name, wrapper)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    install_deferred_collectives()


def _model(name="RotatE"):
    torch.manual_seed(0)
    de, dr = {"RotatE": (True, False), "DistMult": (False, False)}[name]
    return KGEModel(name, E, R, D, GAMMA, de, dr)


# ------------------------------------------------------------------- grads
def _grads_worker(rank, world, port, out):
    _init(rank, world, port)
    from test_dp_gloo import oracle_rank_grads
    model = _model()
    model.compute_train_grads = lambda *a, **k: oracle_rank_grads(model, *a, **k)
    res = []
    for step, mode in enumerate(("tail-batch", "head-batch")):
        pos, neg, w = synth.kge_batch(30 + step, B, N, E, R)
        sl = slice(rank * B // world, (rank + 1) * B // world)
        args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=0.8, uni_weight=False,
                         regularization=1e-3, dp_group=dist.group.WORLD)
        losses = kdist.dp_train_grads(model, torch.from_numpy(pos[sl]), torch.from_numpy(neg[sl]),
                                      torch.from_numpy(w[sl]), mode, args)
        res.append((losses.clone().numpy(), model.entity_embedding.grad.clone().numpy(),
                    model.relation_embedding.grad.clone().numpy()))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_grads_exchange_two_steps_deferred(world):
    out = mp.Manager().dict()
    mp.spawn(_grads_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    model = _model()
    for step, mode in enumerate(("tail-batch", "head-batch")):
        pos, neg, w = synth.kge_batch(30 + step, B, N, E, R)
        log, ge, gr, _ = O.train_grads("RotatE", model.entity_embedding.detach(), model.relation_embedding.detach(),
                                       None, torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w), mode,
                                       adversarial=True, temperature=0.8, uni_weight=False, regularization=1e-3,
                                       gamma=model.gamma.item(), erange=model.embedding_range.item())
        ref = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"], log["regularization"]])
        for rank in range(world):
            losses, g_e, g_r = out[rank][step]
            np.testing.assert_allclose(losses[:4], ref, rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(g_e, ge.numpy(), rtol=1e-4, atol=1e-6 * np.abs(ge.numpy()).max())
            np.testing.assert_allclose(g_r, gr.numpy(), rtol=1e-4, atol=1e-6 * np.abs(gr.numpy()).max())


# ----------------------------------------------------------------- factors
def _factors_worker(rank, world, port, pieces, out):
    _init(rank, world, port)
    kdist.FX_CHUNKS = pieces
    from knowledgegraphembedding_amd import ops
    from test_dp_gloo import _fx_rows
    seen = []

    def rows_slice(desc, mode, pos, neg, w, wsum, dev, *, adversarial, temperature, uni_weight, uni_batch, g_out,
                   dq_out, stats_out):
        _fx_rows(pos, neg, w, g_out, dq_out, stats_out)

    def from_rows(desc, mode, pos, neg, w, wsum, dev, *, uni_weight, uni_batch, regularization, g_in, dq_in, stats,
                  grad_entity, grad_relation, grad_modulus, losses, adam=None, csr_ready=False, workspace=None):
        seen.append([t.clone() for t in (pos, neg, w, g_in, dq_in, stats)])
        losses.zero_()

    ops.train_rows_slice, ops.train_step_from_rows = rows_slice, from_rows
    ops.train_csr = lambda *a, **k: None
    ops.weight_sum = lambda w, o: o.copy_(w.sum().reshape(1))
    model = _model()
    for step in range(2):
        pos, neg, w = synth.kge_batch(40 + step, B, N, E, R)
        sl = slice(rank * B // world, (rank + 1) * B // world)
        args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                         regularization=0.0, dp_group=dist.group.WORLD)
        kdist.dp_train_step_factors(model, torch.from_numpy(pos[sl]), torch.from_numpy(neg[sl]),
                                    torch.from_numpy(w[sl]), "tail-batch", args)
    out[rank] = seen
    dist.destroy_process_group()


@pytest.mark.parametrize("world,pieces", [(2, 2), (4, 2), (2, 1)])
def test_factor_exchange_two_steps_deferred(world, pieces):
    out = mp.Manager().dict()
    mp.spawn(_factors_worker, args=(world, _free_port(), pieces, out), nprocs=world, join=True)
    from test_dp_gloo import _fx_rows
    for step in range(2):
        pos, neg, w = (torch.from_numpy(x) for x in synth.kge_batch(40 + step, B, N, E, R))
        g, dq, st = torch.empty(B, N), torch.empty(B, 2 * D), torch.empty(B, 4)
        _fx_rows(pos, neg, w, g, dq, st)
        for rank in range(world):
            for got, want in zip(out[rank][step], (pos, neg, w, g, dq, st)):
                assert torch.equal(got, want.to(got.dtype)), (rank, step)


# ------------------------------------------------------------------- owner
def _owner_worker(rank, world, port, chunks, out):
    _init(rank, world, port)
    model = _model()
    partition.OWNER_CHUNKS = chunks
    part = partition.EntityRowPartition(model, dist.group.WORLD, exchange="factors")
    res = []
    for step in range(2):
        vals = 1000.0 * (rank + 1) + 100.0 * step + torch.arange(part.rows * part.dim, dtype=torch.float32).view(
            part.rows, part.dim) * 0.25
        for c0, c1 in part._owner_chunks():
            with torch.no_grad():
                part.full[part.lo + c0:part.lo + c1].copy_(vals[c0:c1])  # chunk c's update, then its gather
            part.put_chunk(c0, c1)
        part.gather()
        res.append(part.full.clone())
    out[rank] = (res, part.rows, part.dim)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 1)])
def test_owner_row_exchange_two_steps_deferred(world, chunks):
    """(E = 60 gives 30 / 20 rows per shard: one chunk; the multi-chunk form
    is tests/test_owner_chunks_gloo.py with the same put_chunk / gather)."""
    out = mp.Manager().dict()
    mp.spawn(_owner_worker, args=(world, _free_port(), chunks, out), nprocs=world, join=True)
    rows, dim = out[0][1], out[0][2]
    for step in range(2):
        want = torch.cat([1000.0 * (r + 1) + 100.0 * step + torch.arange(rows * dim, dtype=torch.float32).view(
            rows, dim) * 0.25 for r in range(world)])
        for rank in range(world):
            assert torch.equal(out[rank][0][step], want), (rank, step)


def test_deferred_collective_catches_a_missing_wait():
    """The harness itself: an async all-reduce nobody waits for never lands."""
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_missing_wait_worker, args=(2, port, out), nprocs=2, join=True)
    assert out[0] == (1.0, 3.0) and out[1] == (2.0, 3.0)


def _missing_wait_worker(rank, world, port, out):
    _init(rank, world, port)
    t = torch.tensor([float(rank + 1)])
    w = dist.all_reduce(t, async_op=True)
    before = float(t[0])  # RCCL: undefined here; deferred: still this rank's own value
    w.wait()
    out[rank] = (before, float(t[0]))
    dist.destroy_process_group()
