"""Row-partitioned entity table for YAGO3-10-scale entity counts (BASELINE
config 5: RotatE YAGO3-10 d=1000 n=1024 over 8 ranks).

The reference is single-device and keeps the whole table in one
``nn.Embedding``-like parameter (model.py:45-53).  Here each rank OWNS a
contiguous row range ("shard") of the entity table together with its Adam
moments, so the optimizer reads and writes 1/world of the table per rank:

  rank r owns rows [r·S, (r+1)·S), S = ceil(E / world) (the last shard padded)

One training step (same maths as the single-device step on the global batch):

  1. the fused kernel runs on the rank's own positives and negatives against
     a gathered replica of the whole table (the negative rows the rank
     sampled; with 1024×1024 draws per rank over 123 k rows every row is hit
     with probability 1 − e^-8.5, so the sampled-row gather IS a full-table
     all-gather);
  2. the dense entity gradient is REDUCE-SCATTERED (SUM) to the owners — each
     rank receives only its shard's summed gradient;
  3. relation/modulus gradients and the loss partials are all-reduced, Σw is
     all-reduced before the kernel (global loss normaliser, model.py:285-286);
  4. each rank steps Adam on its shard (and on the replicated relation table);
  5. the updated shards are ALL-GATHERED into the replica for the next step,
     so after ``train_step`` returns the replica (``model.entity_embedding``)
     is current and test_step / save_model read it unchanged.

Collective volume per rank and step: one reduce-scatter and one all-gather of
the (E_pad × d_e) fp32 table, each moving (world−1)/world of it over xGMI.
The regularisation term reads the full replica, so only rank 0 adds it.

Exchange "factors" (owner-computes; distributed.py "owner"): instead of
steps 1-2, the ranks all-gather the row pass's per-row factors (dL/ds, dL/dq,
row statistics: ≈ 9 MB per rank for b = 1024 on FB15k, 12 MB on YAGO3-10)
and each rank runs the entity-major pass for the GLOBAL batch's occurrences
of the rows it owns, its Adam fused into that pass on its shard
(kge_train_step_from_rows_range); the shard is a view of the replica, so the
updated rows go straight into the all-gather of step 5.  Per rank and step:
(N−1)·9-12 MB of factors plus (N−1)/N of the table inbound — about half of the
reduce-scatter + all-gather — and the occurrence work of one single-GPU
entity pass; the rows' gradients, the Adam update and the relation pass are
bit-identical to one process training on the global batch.

Exchange "queries" (query shipping): no replica at all — each
rank holds only its shard (and its Adam moments), so the table's memory is
split world ways.  The ranks ship the global batch's ids and q vectors
instead of rows (kge_ship_step; the stages and collectives in _ship_step):

  all-gather ids/weights → q from the owner of its row, all-reduce(q)
  → every shard scores the negatives it owns for every row (partial softmax
  state, V) → all-gather the per-row states (16 B per row and shard)
  → merge in shard order; dL/dq shares, dL/ds, the positive on the owner of t
  → all-reduce(dL/dq) → chain rule on the owners of h / t; the relation
  gradient all-reduced → entity pass + fused Adam of the owned rows.

Per rank and step that is ≈ 2·B·d_e·4 bytes (q out, dL/dq back) plus the
ids instead of (N−1)/N of the table (see DESIGN §9 for the byte model).  The
cross-shard sums (softmax normaliser, dL/dq, relation gradient) run in
shard order, so the result matches one process to fp32 rounding, not bit
for bit.  ``model.entity_embedding`` is an empty placeholder while training;
``materialize()`` (collective) gathers the table for test_step / save_model
and ``release()`` drops it again.

Checkpoints stay in the reference layout: ``gathered_optimizer_state_dict``
rebuilds the Adam state of the full table, ``load_optimizer_state_dict``
slices a full-table state back to the shard.
"""
from __future__ import annotations

import copy
import os
from argparse import Namespace

import torch
import torch.distributed as dist
from torch import nn

from . import _lib
from . import distributed as _dist
from .distributed import dp_allreduce_, dp_weight_sum

# owner-computes step: the owned rows' entity pass + Adam in this many chunks,
# each chunk's all-gather overlapping the next chunk's pass (1 = one all-gather
# after the whole step)
OWNER_CHUNKS = int(os.environ.get("KGE_OWNER_CHUNKS", "4"))


def _lib_phase(name: str) -> int:
    return getattr(_lib, "PHASE_" + name)


class EntityRowPartition:
    """Attach to a (replicated-initialised) KGEModel: ``EntityRowPartition(model, group)``.

    After construction ``model.entity_embedding`` is a Parameter viewing the
    gathered replica; the trainable tensor is ``self.shard``.  Build the
    optimizer over ``self.parameters()``.
    """

    def __init__(self, model, group=None, exchange: str = "grads"):
        if exchange not in ("grads", "factors", "queries"):
            raise ValueError(f"row-partition exchange must be grads, factors or queries, not {exchange!r}")
        self.exchange = exchange
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        ent = model.entity_embedding
        E, d = ent.shape
        self.nentity, self.dim = E, d
        self.rows = -(-E // self.world)
        self.lo = self.rank * self.rows
        self.hi = min(E, self.lo + self.rows)
        self.nown = max(0, self.hi - self.lo)  # the last shards may be short (or empty)
        # the owned entity rows as a valid range of [0, E): a trailing rank of a
        # small table can start past E (E = 5, world 4: lo = 6), its range is then empty
        self.e0 = min(self.lo, E)
        self.e1 = self.e0 + self.nown
        dev = ent.device
        self._pending = []  # (all-gather work, staging buffer, shard rows c0, c1) of the owner step's chunks
        self._stage = {}
        self.model = model
        model.row_partition = self
        if exchange == "queries":
            self.shard = nn.Parameter(torch.zeros(self.rows, d, device=dev), requires_grad=ent.requires_grad)
            with torch.no_grad():
                self.shard[:self.nown].copy_(ent.detach()[self.lo:self.lo + self.nown])
            self.full = self.grad_full = None
            self.grad_shard = torch.zeros(self.rows, d, device=dev)
            self._ship = None
            self._placeholder = nn.Parameter(torch.empty(0, d, device=dev), requires_grad=ent.requires_grad)
            model.entity_embedding = self._placeholder  # the whole table is never held during training
            rel = model.relation_embedding
            gm = torch.empty(1, 1, device=dev) if model.model_name == 'pRotatE' else None
            model._grad_bufs = (torch.empty(0, d, device=dev),  # the placeholder's shape; the shard's is grad_shard
                                torch.empty_like(rel, memory_format=torch.contiguous_format), gm,
                                torch.empty(5, device=dev))
            return
        self.full = torch.zeros(self.world * self.rows, d, device=dev)
        self.full[:E].copy_(ent.detach())
        if exchange == "factors":  # the owner updates its rows of the replica in place
            self.shard = nn.Parameter(self.full[self.lo:self.lo + self.rows])
        else:
            self.shard = nn.Parameter(self.full[self.lo:self.lo + self.rows].clone())
        self.grad_full = torch.zeros(self.world * self.rows, d, device=dev)
        # the kernels read the replica and write the dense gradient straight
        # into the reduce-scatter input (its padding rows stay zero)
        model.entity_embedding = nn.Parameter(self.full[:E], requires_grad=ent.requires_grad)
        rel = model.relation_embedding
        gm = torch.empty(1, 1, device=dev) if model.model_name == 'pRotatE' else None
        model._grad_bufs = (self.grad_full[:E], torch.empty_like(rel, memory_format=torch.contiguous_format), gm,
                            torch.empty(5, device=dev))
        if exchange == "grads":
            model.fuse_optimizer = False  # Adam runs on the shard, not on the replica the kernel reads

    # ------------------------------------------------------------ parameters
    def parameters(self):
        """Trainable tensors in the reference's order (entity, relation[, modulus])."""
        m = self.model
        out = [self.shard, m.relation_embedding]
        if m.model_name == 'pRotatE':
            out.append(m.modulus)
        return [p for p in out if p.requires_grad]

    def gather(self) -> None:
        """Refresh the replica from every rank's shard (all-gather).  After an
        owner step whose chunks were already put on the wire
        (_owner_step), wait for those and place them instead.  Query
        shipping keeps no replica: nothing to do."""
        if self.exchange == "queries":
            return
        if self._pending:
            for work, stage, c0, c1 in self._pending:
                work.wait()  # the caller's stream now waits for the gather's output (RCCL and gloo alike)
                # stage row r·(c1-c0) + j = rank r's shard row c0 + j
                self.full.view(self.world, self.rows, self.dim)[:, c0:c1].copy_(
                    stage.view(self.world, c1 - c0, self.dim))
            self._pending = []
            return
        src = self.shard.detach()
        if self.exchange == "factors":
            src = src.clone()  # the shard views the output: gather from a copy, never in place
        dist.all_gather_into_tensor(self.full, src, group=self.group)

    def reload_from_replica(self) -> None:
        """After writing the replica (load_state_dict), take this rank's rows back."""
        with torch.no_grad():
            if self.exchange == "queries":
                self.shard[:self.nown].copy_(self.model.entity_embedding.detach()[self.lo:self.lo + self.nown])
                return
            self.shard.copy_(self.full[self.lo:self.lo + self.rows])

    def materialize(self) -> torch.Tensor:
        """Query shipping: gather every rank's shard into a full table and make
        it ``model.entity_embedding`` (for test_step / save_model / loading a
        checkpoint; collective).  Other exchanges: the replica, as is."""
        if self.exchange != "queries":
            return self.model.entity_embedding
        full = torch.empty(self.world * self.rows, self.dim, device=self.shard.device)
        dist.all_gather_into_tensor(full, self.shard.detach(), group=self.group)
        self.model.entity_embedding = nn.Parameter(full[:self.nentity], requires_grad=self._placeholder.requires_grad)
        return self.model.entity_embedding

    def release(self) -> None:
        """Query shipping: drop the gathered table again (training needs only the shard)."""
        if self.exchange == "queries":
            self.model.entity_embedding = self._placeholder

    # -------------------------------------------------------------- training
    def train_grads(self, model, positive_sample, negative_sample, subsampling_weight, mode, args, optimizer=None):
        """This rank's part of one step; returns the global [5] loss vector.
        "grads": fused per-rank gradients, reduce-scatter to the owners.
        "factors": the row factors exchanged, the owned rows' pass (+ fused Adam)."""
        if self.exchange == "factors":
            return self._owner_step(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                                    optimizer)
        if self.exchange == "queries":
            return self._ship_step(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                                   optimizer)
        group = self.group
        B = positive_sample.shape[0]
        wsum = None if args.uni_weight else dp_weight_sum(subsampling_weight, group)
        local_args = args
        if self.rank != 0 and args.regularization != 0.0:
            local_args = copy.copy(args)
            local_args.regularization = 0.0
        losses = model.compute_train_grads(positive_sample, negative_sample, subsampling_weight, mode, local_args,
                                           weight_sum=wsum, uni_batch=B * self.world)
        if self.shard.grad is None or self.shard.grad.shape != self.shard.shape:
            self.shard.grad = torch.empty_like(self.shard)
        dist.reduce_scatter_tensor(self.shard.grad, self.grad_full, op=dist.ReduceOp.SUM, group=group)
        model.entity_embedding.grad = None  # the replica is not optimised; its gradient went to the owners
        rest = [model.relation_embedding.grad]
        if model.model_name == 'pRotatE' and model.modulus.grad is not None:
            rest.append(model.modulus.grad)
        dp_allreduce_(rest + [losses], group)
        losses[2] = (losses[0] + losses[1]) / 2 + losses[3]
        return losses

    def _owner_step(self, model, positive_sample, negative_sample, subsampling_weight, mode, args, optimizer):
        from . import ops
        dev = model.entity_embedding.device
        fx = _dist._exchange_row_factors(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                                         csr_range=(self.e0, self.e1))
        adam = None
        if optimizer is not None and model.fuse_optimizer and hasattr(optimizer, 'prepare_fused_rows'):
            adam = optimizer.prepare_fused_rows(self.shard, model.entity_embedding, self.lo,
                                                model.relation_embedding, model._modulus(),
                                                write_grad=model.keep_grads)
        ge, gr, gm, losses = model._grad_buffers()  # ge = grad_full[:E]; rows [lo, hi) are written
        kw = dict(uni_weight=fx.uni, uni_batch=fx.B, regularization=float(args.regularization), g_in=fx.g,
                  dq_in=fx.dq, stats=fx.stats, grad_entity=ge, grad_relation=gr, grad_modulus=gm, losses=losses,
                  adam=adam, csr_ready=_dist.FX_CSR_AHEAD, workspace=fx.workspace, reg_relations=self.rank == 0)
        desc = model.desc()
        chunks = self._owner_chunks() if adam is not None else []
        own = (self.e0, self.e1)
        if len(chunks) <= 1:
            ops.train_step_from_rows(desc, mode, fx.pos, fx.neg, fx.w, fx.wsum, dev, entity_range=own, **kw)
        else:
            # the entity pass + fused Adam of the owned rows in chunks; chunk
            # c's all-gather (every rank's rows c0..c1 of its shard) is on the
            # wire while chunk c+1 is computed; gather() places them
            ops.train_step_from_rows(desc, mode, fx.pos, fx.neg, fx.w, fx.wsum, dev, entity_range=own,
                                     phases=_lib_phase("ROWS"), **kw)
            for c0, c1 in chunks:
                e0, e1 = min(self.e1, self.e0 + c0), min(self.e1, self.e0 + c1)
                if e1 > e0:
                    ops.train_step_from_rows(desc, mode, fx.pos, fx.neg, fx.w, fx.wsum, dev, entity_range=(e0, e1),
                                             phases=_lib_phase("ENTITY"), **kw)
                self.put_chunk(c0, c1)
            ops.train_step_from_rows(desc, mode, fx.pos, fx.neg, fx.w, fx.wsum, dev, entity_range=own,
                                     phases=_lib_phase("FINALIZE"), **kw)
        # the owner's rows of the gradient; the replica itself is not optimised
        self.shard.grad = self.grad_full[self.lo:self.lo + self.rows] if adam is None or model.keep_grads else None
        model.entity_embedding.grad = None
        if model.relation_embedding.requires_grad:
            model.relation_embedding.grad = gr  # the global batch's: the same on every rank
        if gm is not None and model.modulus.requires_grad:
            model.modulus.grad = gm
        if args.regularization != 0.0:  # each rank summed |x|^3 over its rows only
            dist.all_reduce(losses[3:4], op=dist.ReduceOp.SUM, group=self.group)
            losses[2] = (losses[0] + losses[1]) / 2 + losses[3]
        return losses

    def _ship_buffers(self, model, Bg: int, n: int):
        """Per-step buffers of the query-shipping step, reused while the shape holds."""
        key = (Bg, n)
        if self._ship is not None and self._ship[0] == key:
            return self._ship[1]
        dev, Le, Lr = self.shard.device, self.dim, model.relation_embedding.shape[1]
        f32 = dict(device=dev, dtype=torch.float32)
        b = Namespace(
            pos=torch.empty(Bg, 3, dtype=torch.int64, device=dev), neg=torch.empty(Bg, n, dtype=torch.int64, device=dev),
            w=torch.empty(Bg, **f32),
            qq=torch.empty(2 * Bg * Le, **f32),                # q | qp (head-batch)
            part=torch.empty(Bg, 4, **f32), parts=torch.empty(self.world * Bg, 4, **f32),
            scores=torch.empty(Bg, n, **f32), g=torch.empty(Bg, n, **f32),
            flat=torch.empty(Bg * Le + 4 * Bg + Bg * Le, **f32),  # dq | pstats | pq (head-batch)
            ent_contrib=torch.empty(2 * Bg, Le, **f32), rel_contrib=torch.empty(Bg, Lr, **f32),
            row_stats=torch.empty(Bg, 4, **f32))
        self._ship = (key, b)
        return b

    def _ship_model_desc(self, model):
        """The model descriptor for the shard: entity rows addressed by global id."""
        from . import ops
        g, rng = model._host_scalars()
        d = ops.make_desc(model.model_name, self.shard.detach(), model.relation_embedding.detach(), g, rng,
                          None if model._modulus() is None else model._modulus().detach())
        d.entity_embedding = self.shard.data_ptr() - self.lo * self.dim * 4
        d.nentity = self.nentity
        return d

    def _ship_step(self, model, positive_sample, negative_sample, subsampling_weight, mode, args, optimizer):
        from . import ops
        group, dev = self.group, self.shard.device
        B, n = negative_sample.shape
        Bg, Le = B * self.world, self.dim
        head = mode == 'head-batch'
        b = self._ship_buffers(model, Bg, n)
        # the global batch, rank order (what one process would train on)
        dist.all_gather_into_tensor(b.pos, positive_sample.to(dev, torch.int64).contiguous(), group=group)
        dist.all_gather_into_tensor(b.neg, negative_sample.to(dev, torch.int64).contiguous(), group=group)
        uni = bool(args.uni_weight)
        wsum = None
        if not uni:
            dist.all_gather_into_tensor(b.w, subsampling_weight.to(dev, torch.float32).contiguous().view(-1),
                                        group=group)
            wsum = dp_weight_sum(subsampling_weight, group)
        row_bytes = self.dim * 4
        adam = None
        if optimizer is not None and model.fuse_optimizer and hasattr(optimizer, 'prepare_fused'):
            adam = optimizer.prepare_fused(self.shard, model.relation_embedding, model._modulus(),
                                           write_grad=model.keep_grads)
            if adam is not None:  # entity pointers by global row id, like the descriptor's
                off = self.lo * row_bytes
                adam.entity.param -= off
                adam.entity.exp_avg -= off
                adam.entity.exp_avg_sq -= off
        _, gr, gm, losses = model._grad_buffers()
        sd = _lib.ShipDesc()
        sd.world, sd.rank = self.world, self.rank
        sd.own_begin = min(self.lo, self.nentity)
        sd.own_end = sd.own_begin + self.nown
        sd.pos, sd.neg, sd.batch, sd.nneg = b.pos.data_ptr(), b.neg.data_ptr(), Bg, n
        sd.subsampling_weight = b.w.data_ptr()
        sd.weight_sum = wsum.data_ptr() if wsum is not None else None
        sd.uni_weight, sd.adversarial, sd.uni_batch = int(uni), int(bool(args.negative_adversarial_sampling)), Bg
        sd.adversarial_temperature = float(getattr(args, 'adversarial_temperature', 1.0))
        sd.regularization = float(args.regularization)
        q_n = Bg * Le
        sd.q, sd.qp = b.qq.data_ptr(), b.qq[q_n:].data_ptr()
        sd.part, sd.parts = b.part.data_ptr(), b.parts.data_ptr()
        sd.scores, sd.g = b.scores.data_ptr(), b.g.data_ptr()
        sd.dq, sd.pstats, sd.pq = b.flat.data_ptr(), b.flat[q_n:].data_ptr(), b.flat[q_n + 4 * Bg:].data_ptr()
        sd.ent_contrib, sd.rel_contrib, sd.row_stats = (b.ent_contrib.data_ptr(), b.rel_contrib.data_ptr(),
                                                        b.row_stats.data_ptr())
        desc = self._ship_model_desc(model)
        ws = ops._train_ws(desc, Bg, n, dev)

        def run(stage, **kw):
            ops.ship_step(desc, mode, stage, sd, dev, workspace=ws, **kw)

        run(_lib.SHIP_Q)
        dist.all_reduce(b.qq[:(2 if head else 1) * q_n], op=dist.ReduceOp.SUM, group=group)
        run(_lib.SHIP_ROWS)
        dist.all_gather_into_tensor(b.parts, b.part, group=group)
        run(_lib.SHIP_MERGE)
        dist.all_reduce(b.flat[:q_n + 4 * Bg + (q_n if head else 0)], op=dist.ReduceOp.SUM, group=group)
        run(_lib.SHIP_CHAIN, grad_relation=gr)
        dist.all_reduce(gr, op=dist.ReduceOp.SUM, group=group)
        rel = model.relation_embedding
        if adam is not None:  # the relation rows' Adam (marked fused by prepare_fused), on the summed gradient
            st = optimizer.state[rel]
            _lib.check(_lib.load().kge_adam_step(rel.data_ptr(), gr.data_ptr(), st['exp_avg'].data_ptr(),
                                                 st['exp_avg_sq'].data_ptr(), rel.numel(), adam.beta1, adam.beta2,
                                                 adam.eps, adam.relation.step_size,
                                                 adam.relation.bias_correction2_sqrt, ops._stream(dev)),
                       "kge_adam_step")
        run(_lib.SHIP_ENTITY, adam=adam, grad_entity_ptr=self.grad_shard.data_ptr() - self.lo * row_bytes,
            grad_relation=gr, grad_modulus=gm, losses=losses)
        self.shard.grad = self.grad_shard if adam is None or model.keep_grads else None
        if rel.requires_grad:
            rel.grad = gr
        if gm is not None and model.modulus.requires_grad:
            model.modulus.grad = gm
        if args.regularization != 0.0:  # each rank summed |x|^3 over its rows (relations: rank 0)
            dist.all_reduce(losses[3:4], op=dist.ReduceOp.SUM, group=group)
            losses[2] = (losses[0] + losses[1]) / 2 + losses[3]
        return losses

    def put_chunk(self, c0: int, c1: int) -> None:
        """Start the all-gather of every rank's shard rows [c0, c1) (collective,
        async): rank r's rows land at stage rows r·(c1−c0) …, gather() waits and
        places them at replica rows r·S + c0 ….  One staging buffer per chunk,
        so the gathers of consecutive chunks can be on the wire together."""
        stage = self._stage_buf(c0, c1 - c0, self.full.device)
        # the collective's input is ordered after the chunk's entity pass (the
        # caller's stream at issue); its output after gather()'s copy of the
        # previous step ("the owner step's hand-offs")
        work = dist.all_gather_into_tensor(stage, self.full[self.lo + c0:self.lo + c1], group=self.group,
                                           async_op=True)
        self._pending.append((work, stage, c0, c1))

    def replica_checksums(self) -> torch.Tensor:
        """This rank's [2] int64 fingerprint of its replica (the bit patterns of
        the entity rows, then of the relation table, summed as integers): equal
        on every rank exactly when the replicas agree bit for bit, as the
        owner-computes and reduce-scatter exchanges guarantee.  Query
        shipping keeps no replica: [1], the relation table alone."""
        if self.full is None:
            return _dist.table_fingerprint(self.model.relation_embedding)
        return _dist.table_fingerprint(self.full, self.model.relation_embedding)

    def _owner_chunks(self):
        """Shard row ranges [c0, c1) of the chunked owner step (OWNER_CHUNKS
        equal pieces of the padded shard; one piece when the shard is small)."""
        k = max(1, min(OWNER_CHUNKS, self.rows // 32))
        step = -(-self.rows // k)
        return [(c0, min(self.rows, c0 + step)) for c0 in range(0, self.rows, step)]

    def _stage_buf(self, c0: int, nrows: int, dev) -> torch.Tensor:
        key = (c0, nrows, dev)
        b = self._stage.get(key)
        if b is None:
            b = self._stage[key] = torch.empty(self.world * nrows, self.dim, device=dev)
        return b

    # ------------------------------------------------------------ checkpoints
    def _gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty(self.world * self.rows, self.dim, device=t.device, dtype=t.dtype)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out[:self.nentity]

    def gathered_optimizer_state_dict(self, optimizer) -> dict:
        """The optimizer's state_dict with the shard's Adam moments gathered to
        full-table tensors — the layout a replicated Adam over
        (entity, relation[, modulus]) would save (run.py:93-120).  Collective."""
        sd = optimizer.state_dict()
        st = sd['state'].get(0)
        if st is not None:
            st = dict(st)
            for k in ('exp_avg', 'exp_avg_sq'):
                st[k] = self._gather_rows(st[k])
            sd['state'] = dict(sd['state'])
            sd['state'][0] = st
        return sd

    def load_optimizer_state_dict(self, optimizer, sd: dict) -> None:
        """Load a full-table optimizer state (reference layout) into the shard optimizer."""
        sd = copy.deepcopy(sd)
        st = sd['state'].get(0)
        if st is not None:
            for k in ('exp_avg', 'exp_avg_sq'):
                full = st[k]
                part = torch.zeros(self.rows, self.dim, dtype=full.dtype)
                part[:self.nown] = full[self.e0:self.e1]
                st[k] = part
        optimizer.load_state_dict(sd)
