"""Data-parallel training over one process per GPU (torch.distributed; the
"nccl" backend is RCCL on ROCm, gloo on CPU for tests).

The reference is single-device.  Sharding the positive
batch across ranks changes nothing in the maths as long as the loss
normaliser is global: every rank

  1. all-reduces Σw (one scalar) so c_i = w_i / Σw_global (model.py:285-286),
     or uses 1 / (B * world) under --uni_weight;
  2. runs the fused kernel on its shard → dense partial gradients;
  3. all-reduces (SUM) the entity/relation(/modulus) gradients and the four
     loss partials — the entity gradient in row chunks, each chunk's
     all-reduce issued (async, RCCL's own stream) as soon as the entity pass
     has queued it, so the reduction of chunk k overlaps the computation of
     chunk k+1 (bucket entity-row ranges as the entity-major
     backward finishes them);
  4. steps the (replicated) optimizer identically.

The regularisation term reads the full tables, so only rank 0 adds it before
the sum (it would otherwise be counted world_size times).
"""
from __future__ import annotations

import copy
import os

import torch
import torch.distributed as dist

DP_CHUNKS = int(os.environ.get("KGE_DP_CHUNKS", "4"))


def entity_chunks(nentity: int, chunks: int = DP_CHUNKS):
    """Contiguous entity-row ranges for the overlapped gradient all-reduce."""
    chunks = max(1, min(chunks, nentity))
    step = -(-nentity // chunks)
    return [(e0, min(nentity, e0 + step)) for e0 in range(0, nentity, step)]


def dp_allreduce_(tensors, group=None) -> None:
    """In-place SUM all-reduce of a list of tensors (one collective per tensor;
    RCCL runs them on its own stream in issue order)."""
    for t in tensors:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


def dp_weight_sum(subsampling_weight: torch.Tensor, group=None) -> torch.Tensor:
    ws = subsampling_weight.float().sum().reshape(1)
    dist.all_reduce(ws, op=dist.ReduceOp.SUM, group=group)
    return ws


def dp_train_grads(model, positive_sample, negative_sample, subsampling_weight, mode, args, optimizer=None):
    """Fused per-rank gradients + global reduction; returns the global [5] loss vector.
    With a KGEAdam `optimizer` the entity table's update runs chunk by chunk as
    each chunk's all-reduce lands (the next train_step optimizer.step() skips it)."""
    group = args.dp_group
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    B = positive_sample.shape[0]
    wsum = None if args.uni_weight else dp_weight_sum(subsampling_weight, group)
    local_args = args
    if rank != 0 and args.regularization != 0.0:
        local_args = copy.copy(args)
        local_args.regularization = 0.0
    pending = []

    def reduce_chunk(e0, e1, grad_entity):
        pending.append(dist.all_reduce(grad_entity[e0:e1], op=dist.ReduceOp.SUM, group=group, async_op=True))

    chunks = entity_chunks(model.entity_embedding.shape[0])
    losses = model.compute_train_grads(positive_sample, negative_sample, subsampling_weight, mode, local_args,
                                       weight_sum=wsum, uni_batch=B * world, entity_chunks=chunks,
                                       on_entity_chunk=reduce_chunk)
    rest = [model.relation_embedding.grad]
    if model.model_name == 'pRotatE' and model.modulus.grad is not None:
        rest.append(model.modulus.grad)
    for t in rest + [losses]:
        pending.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True))
    if optimizer is not None and hasattr(optimizer, 'step_param') and model.entity_embedding.requires_grad:
        # Adam on each entity-row chunk as soon as its reduction lands, while
        # the later chunks are still on the wire
        optimizer.step_param(model.entity_embedding, chunks, before_chunk=lambda k: pending[k].wait())
    for work in pending:  # (waiting twice on a chunk is a no-op)
        work.wait()
    # loss = (pos + neg) / 2 + reg must be recomputed from the summed parts
    losses[2] = (losses[0] + losses[1]) / 2 + losses[3]
    return losses
