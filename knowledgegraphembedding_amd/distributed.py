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
the sum (it would otherwise be counted world_size times).  Every rank must
feed the same local batch size: the --uni_weight normaliser is taken as
1 / (B_local * world) without a host round trip (the factor exchange's
all-gathers require equal sizes anyway).

Two exchanges implement step 3 (`dp_exchange_mode`):

* "grads" — the all-reduce above: 2·(N-1)/N × the dense entity gradient
  (120 MB for RotatE FB15k) per rank and step, bandwidth-optimal for many ranks.
* "factors" — the ranks all-gather the row pass's per-row factors instead
  (dL/ds [B, n], dL/dq [B, Le], row statistics: ≈9 MB per rank) and every rank
  runs the entity-major pass, Adam included, for the GLOBAL batch
  (kge_train_step_from_rows).  On xGMI, where two GPUs share a single link,
  that is ~13× fewer bytes than the all-reduce, paid for with N× the
  occurrence work of the entity pass; the result is bit-identical to one
  process training on the whole batch.  "auto" picks it for N <= 2.
* "owner" — the factors as above, but each rank runs the entity-major pass
  (gradient + fused Adam) only for the 1/N of the entity rows it owns, over
  the global batch's occurrences, and the updated rows are all-gathered
  (partition.EntityRowPartition, exchange "factors"): per rank ≈ 9 MB·(N−1) of
  factors plus (N−1)/N of the table inbound, the occurrence work of one
  single-GPU entity pass and 1/N of the Adam stream.  "auto" picks it above
  2 ranks.
"""
from __future__ import annotations

import copy
import os

import torch
import torch.distributed as dist

DP_CHUNKS = int(os.environ.get("KGE_DP_CHUNKS", "4"))
# factor exchange: the rank's rows go through the row pass in this many pieces,
# each piece's all-gather issued as soon as it is queued (overlaps the next piece)
FX_CHUNKS = int(os.environ.get("KGE_FX_CHUNKS", "2"))
# ... and the global batch's occurrence CSR is built on a side stream as soon as its ids arrive
FX_CSR_AHEAD = os.environ.get("KGE_FX_CSR_AHEAD", "1") == "1"


def entity_chunks(nentity: int, chunks: int = DP_CHUNKS):
    """Contiguous entity-row ranges for the overlapped gradient all-reduce."""
    chunks = max(1, min(chunks, nentity))
    step = -(-nentity // chunks)
    return [(e0, min(nentity, e0 + step)) for e0 in range(0, nentity, step)]


def dp_allreduce_(tensors, group=None) -> None:
    """In-place SUM all-reduce of a list of tensors as ONE collective over
    their concatenation (the small relation/modulus gradients and the loss
    partials would otherwise each pay a collective's fixed latency)."""
    finish = dp_allreduce_packed_async(tensors, group)
    finish()


def dp_allreduce_packed_async(tensors, group=None):
    """Issue one async SUM all-reduce over the concatenation of `tensors`;
    returns a callable that waits for it and copies the sums back in place.
    The copy-back is elementwise, so the sums are those of separate
    all-reduces."""
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return lambda: None
    flat = torch.cat([t.reshape(-1).float() for t in tensors])
    work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=True)

    def finish():
        work.wait()
        off = 0
        for t in tensors:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n
    return finish


def dp_exchange_mode(world: int, override: str | None = None) -> str:
    """"grads" (overlapped all-reduce of the dense gradient), "factors"
    (all-gather of the per-row factors, global entity pass on every rank) or
    "owner" (the factors all-gathered, each rank's entity pass and Adam on the
    1/N of the rows it owns, the updated rows all-gathered: partition.py);
    KGE_DP_EXCHANGE=auto|grads|factors|owner, auto = factors for up to 2
    ranks, owner above (DESIGN.md §9 byte model)."""
    mode = override or os.environ.get("KGE_DP_EXCHANGE", "auto")
    if mode == "auto":
        return "factors" if world <= 2 else "owner"
    if mode not in ("grads", "factors", "owner"):
        raise ValueError(f"KGE_DP_EXCHANGE must be auto, grads, factors or owner, not {mode!r}")
    return mode


_OWNER_WARNED = [False]


def warn_owner_without_partition() -> None:
    """The "owner" exchange runs through a partition.EntityRowPartition(model,
    group, exchange="factors") attached to the model (run.py builds one); a
    KGEModel trained with a dp_group and no partition falls back to the "grads"
    exchange — said once, so the exchange in use is never misreported."""
    if not _OWNER_WARNED[0]:
        _OWNER_WARNED[0] = True
        import logging
        logging.warning('data-parallel exchange "owner" needs EntityRowPartition(model, group, exchange="factors") '
                        'attached to the model; no partition is attached, so this run uses the "grads" exchange '
                        '(set KGE_DP_EXCHANGE=grads|factors to choose explicitly)')


_FX_BUFS: dict = {}


def _fx_buffers(dev, Bg: int, n: int, Le: int, tag: str = "global"):
    key = (dev, Bg, n, Le, tag)
    b = _FX_BUFS.get(key)
    if b is None:
        b = _FX_BUFS[key] = (torch.empty(Bg, n, device=dev), torch.empty(Bg, Le, device=dev),
                             torch.empty(Bg, 4, device=dev))
    return b


_CSR_STREAMS: dict = {}


def _csr_stream(dev):
    """A side stream per device for the factor exchange's CSR (None on CPU)."""
    if dev.type != "cuda":
        return None
    st = _CSR_STREAMS.get(dev)
    if st is None:
        st = _CSR_STREAMS[dev] = torch.cuda.Stream(dev)
    return st


def fx_pieces(B: int, chunks: int = FX_CHUNKS):
    """Row ranges [r0, r1) of a rank's B rows for the overlapped factor gather
    (equal pieces; one piece when B does not split evenly)."""
    k = chunks if chunks > 1 and B % chunks == 0 else 1
    step = B // k
    return [(c * step, (c + 1) * step) for c in range(k)]


class RowFactors:
    """The gathered inputs of the global step (see _exchange_row_factors)."""
    __slots__ = ("pos", "neg", "w", "wsum", "g", "dq", "stats", "workspace", "B", "uni")


def _exchange_row_factors(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                          csr_range=None) -> RowFactors:
    """Everything the factor-exchanging steps share: the global batch's ids and
    weights all-gathered, Σw over them, this rank's row pass into its place in
    the gather buffers (in FX_CHUNKS pieces, each piece's all-gather overlapping
    the next piece's row pass), the gathered dL/ds, dL/dq and row statistics,
    and the global batch's occurrence CSR built on a side stream as soon as the
    ids arrive (FX_CSR_AHEAD, into `workspace`; with `csr_range` (e0, e1)
    only those entities' buckets — an owner's rows)."""
    from . import ops
    group = args.dp_group
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = model.entity_embedding.device
    pos = positive_sample.to(dev).long().contiguous()
    neg = negative_sample.to(dev).long().contiguous()
    B, n = neg.shape
    Bg, r0 = B * world, rank * B
    uni = bool(args.uni_weight)
    w_l = subsampling_weight.to(dev, dtype=torch.float32).contiguous().view(-1)
    w_g = torch.empty(Bg, device=dev)
    dist.all_gather_into_tensor(w_g, w_l, group=group)
    pos_g = torch.empty(Bg, 3, dtype=torch.int64, device=dev)
    neg_g = torch.empty(Bg, n, dtype=torch.int64, device=dev)
    ids = [dist.all_gather_into_tensor(pos_g, pos, group=group, async_op=True),
           dist.all_gather_into_tensor(neg_g, neg, group=group, async_op=True)]
    wsum = None
    if not uni:
        wsum = torch.empty(1, device=dev)
        ops.weight_sum(w_g, wsum)  # the single-process Σw: same fixed order as the in-kernel sum
    desc = model.desc()
    # the global batch's occurrence CSR needs only the ids: built on a side
    # stream as soon as they arrive, beside this rank's row pass (as the
    # single-process step builds it beside k_row)
    side = _csr_stream(dev) if FX_CSR_AHEAD else None
    gws = None  # the global step's own workspace (the row pass below uses the shared one meanwhile)
    if FX_CSR_AHEAD:
        gws = ops.exchange_workspace(desc, Bg, n, dev) if dev.type == "cuda" else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(dev))  # the previous step's use of that workspace
            with torch.cuda.stream(side):
                for h in ids:
                    h.wait()
                ops.train_csr(desc, mode, pos_g, neg_g, dev, workspace=gws, entity_range=csr_range)
        else:
            for h in ids:
                h.wait()
            ops.train_csr(desc, mode, pos_g, neg_g, dev, workspace=gws, entity_range=csr_range)
    Le = model.entity_dim
    g_g, dq_g, st_g = _fx_buffers(dev, Bg, n, Le)
    pieces = fx_pieces(B)
    if len(pieces) == 1:
        sl = slice(r0, r0 + B)
        ops.train_rows_slice(desc, mode, pos, neg, w_g[sl], wsum, dev,
                             adversarial=bool(args.negative_adversarial_sampling),
                             temperature=float(getattr(args, 'adversarial_temperature', 1.0)), uni_weight=uni,
                             uni_batch=Bg, g_out=g_g[sl], dq_out=dq_g[sl], stats_out=st_g[sl])
        for t in (g_g, dq_g, st_g):  # in place: this rank's rows are already at its slot
            dist.all_gather_into_tensor(t, t[sl], group=group)
    else:
        # piece c of every rank is gathered into a [world, P, ...] staging slot
        # while piece c+1 is computed, then scattered to rows r·B + c·P .. of
        # the global buffers: same rows, same bits, the gather overlapped
        P = pieces[0][1]
        k = len(pieces)
        stage = _fx_buffers(dev, Bg, n, Le, "stage")  # row c·world·P + r·P + j ↔ global row r·B + c·P + j
        pending = []
        for c, (a0, a1) in enumerate(pieces):
            sg = slice(c * world * P, (c + 1) * world * P)
            mine = slice(c * world * P + rank * P, c * world * P + (rank + 1) * P)
            ops.train_rows_slice(desc, mode, pos[a0:a1], neg[a0:a1], w_g[r0 + a0:r0 + a1], wsum, dev,
                                 adversarial=bool(args.negative_adversarial_sampling),
                                 temperature=float(getattr(args, 'adversarial_temperature', 1.0)), uni_weight=uni,
                                 uni_batch=Bg, g_out=stage[0][mine], dq_out=stage[1][mine], stats_out=stage[2][mine])
            for t in stage:
                pending.append(dist.all_gather_into_tensor(t[sg], t[mine], group=group, async_op=True))
        for h in pending:
            h.wait()
        for t, dst in zip(stage, (g_g, dq_g, st_g)):
            rest = t.shape[1:]
            dst.view(world, k, P, *rest).copy_(t.view(k, world, P, *rest).transpose(0, 1))
    for h in ids:
        h.wait()
    if side is not None:
        torch.cuda.current_stream(dev).wait_stream(side)
    fx = RowFactors()
    fx.pos, fx.neg, fx.w, fx.wsum, fx.g, fx.dq, fx.stats, fx.workspace, fx.B, fx.uni = (
        pos_g, neg_g, w_g, wsum, g_g, dq_g, st_g, gws, Bg, uni)
    return fx


def dp_train_step_factors(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                          optimizer=None):
    """One data-parallel step by factor exchange (module docstring): the row
    factors exchanged (_exchange_row_factors), then the rest of the step for
    the global batch on every rank (the fused Adam update included when the
    optimizer is a KGEAdam).  Returns the global [5] loss vector (the same on
    every rank, nothing left to reduce)."""
    from . import ops
    dev = model.entity_embedding.device
    fx = _exchange_row_factors(model, positive_sample, negative_sample, subsampling_weight, mode, args)
    adam = None
    if optimizer is not None and model.fuse_optimizer and hasattr(optimizer, 'prepare_fused'):
        adam = optimizer.prepare_fused(model.entity_embedding, model.relation_embedding, model._modulus(),
                                       write_grad=model.keep_grads)
    ge, gr, gm, losses = model._grad_buffers()
    ops.train_step_from_rows(model.desc(), mode, fx.pos, fx.neg, fx.w, fx.wsum, dev, uni_weight=fx.uni,
                             uni_batch=fx.B, regularization=float(args.regularization), g_in=fx.g, dq_in=fx.dq,
                             stats=fx.stats, grad_entity=ge, grad_relation=gr, grad_modulus=gm, losses=losses,
                             adam=adam, csr_ready=FX_CSR_AHEAD, workspace=fx.workspace)
    if model.entity_embedding.requires_grad:
        model.entity_embedding.grad = ge
    if model.relation_embedding.requires_grad:
        model.relation_embedding.grad = gr
    if gm is not None and model.modulus.requires_grad:
        model.modulus.grad = gm
    return losses


def table_fingerprint(*tables) -> torch.Tensor:
    """[len(tables)] int64: each fp32 table's bit patterns summed as integers
    (any changed bit of any element changes it, bar exact cancellations)."""
    return torch.stack([torch.sum(t.detach().reshape(-1).view(torch.int32), dtype=torch.int64) for t in tables])


def replicas_disagree(fingerprint: torch.Tensor, group=None) -> list:
    """Collective: the ranks whose replica fingerprint differs from rank 0's
    (empty when every rank holds the same bits).  The exchanges that keep a
    replicated table — factors, owner-computes, the row partition's
    reduce-scatter — leave it bit-identical on every rank after each step;
    bench.py checks that after its timed steps at N > 1, so a replica that
    diverged on one rank shows in the driver's line instead of staying silent."""
    world = dist.get_world_size(group)
    allfp = torch.empty(world * fingerprint.numel(), dtype=fingerprint.dtype, device=fingerprint.device)
    dist.all_gather_into_tensor(allfp, fingerprint.contiguous(), group=group)
    allfp = allfp.view(world, -1).cpu()
    return [r for r in range(world) if not torch.equal(allfp[r], allfp[0])]


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
    # relation (+ modulus) gradient and the loss partials: one packed collective
    finish_rest = dp_allreduce_packed_async(rest + [losses], group)
    if optimizer is not None and hasattr(optimizer, 'step_param') and model.entity_embedding.requires_grad:
        # Adam on each entity-row chunk as soon as its reduction lands, while
        # the later chunks are still on the wire
        optimizer.step_param(model.entity_embedding, chunks, before_chunk=lambda k: pending[k].wait())
    for work in pending:  # (waiting twice on a chunk is a no-op)
        work.wait()
    finish_rest()
    # loss = (pos + neg) / 2 + reg must be recomputed from the summed parts
    losses[2] = (losses[0] + losses[1]) / 2 + losses[3]
    return losses
