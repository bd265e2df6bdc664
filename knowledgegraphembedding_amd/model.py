"""KGEModel — drop-in for codes/model.py:KGEModel, computing on MI355X.

Public surface kept from the reference:
  KGEModel(model_name, nentity, nrelation, hidden_dim, gamma,
           double_entity_embedding=False, double_relation_embedding=False)   model.py:22-70
  KGEModel.forward(sample, mode='single') -> [B, n] scores                    model.py:72-164
  KGEModel.TransE/DistMult/ComplEx/RotatE/pRotatE(head, relation, tail, mode)  model.py:166-249
  KGEModel.train_step(model, optimizer, train_iterator, args) -> log dict      model.py:252-312
  KGEModel.test_step(model, test_triples, all_true_triples, args) -> metrics   model.py:315-429

Parameters, their names, shapes, init and state_dict keys are the
reference's (gamma, embedding_range, entity_embedding, relation_embedding,
modulus), so reference checkpoints load unchanged.  All scoring, loss,
gradient and ranking arithmetic runs in libkge_hip.so (see ops.py); CPU
tensors are rejected instead of silently falling back.
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops, torch_ops  # noqa: F401  (torch_ops registers torch.ops.kge.*)
from .filters import FilterIndex, triples_array

_MODELS = ['TransE', 'DistMult', 'ComplEx', 'RotatE', 'pRotatE']


class StepLog(dict):
    """train_step's log — the reference's {name: float} dict (model.py:305-312)
    — filled from the device on first read.

    The step's four losses and the device error flag land in a pinned host
    slot — written there by the single-device step's k_finalize itself, or
    copied behind an event by the multi-GPU steps; reading any key (or
    iterating, printing, json dumping) waits for them and raises the deferred
    error if the step saw an out-of-range index.  Until then the host is free
    to enqueue the next step, so the GPU does not idle while Python prepares
    it.  A slot the kernel writes directly is pre-filled with NaN and polled
    (no event: a marker after every step cost ~6 µs of device time); after
    POLL_SPIN_S without all five values the read falls back to a device
    synchronize, so a NaN loss is still reported correctly."""

    __slots__ = ('_src',)

    def __init__(self, src):
        super().__init__()
        self._src = src  # (host [5] tensor, event, has_regularization, device); None once filled

    def _fill(self):
        src = self._src
        if src is None:
            return self
        self._src = None
        host, event, has_reg, dev = src
        if event is not None:
            event.synchronize()
        elif host.is_pinned():
            _poll_slot(host, dev)
        vals = host.tolist()
        if vals[4] != 0.0:  # device error flag (out-of-range index), copied by the kernels
            ops.raise_on_device_error(dev)
        if has_reg:
            dict.__setitem__(self, 'regularization', vals[3])
        dict.__setitem__(self, 'positive_sample_loss', vals[0])
        dict.__setitem__(self, 'negative_sample_loss', vals[1])
        dict.__setitem__(self, 'loss', vals[2])
        return self

    def __getitem__(self, k):
        return dict.__getitem__(self._fill(), k)

    def __setitem__(self, k, v):
        dict.__setitem__(self._fill(), k, v)

    def __delitem__(self, k):
        dict.__delitem__(self._fill(), k)

    def __contains__(self, k):
        return dict.__contains__(self._fill(), k)

    def __iter__(self):
        return dict.__iter__(self._fill())

    def __len__(self):
        return dict.__len__(self._fill())

    def __repr__(self):
        return dict.__repr__(self._fill())

    def __eq__(self, other):
        return dict.__eq__(self._fill(), other)

    __hash__ = None

    def get(self, k, default=None):
        return dict.get(self._fill(), k, default)

    def keys(self):
        return dict.keys(self._fill())

    def values(self):
        return dict.values(self._fill())

    def items(self):
        return dict.items(self._fill())

    def copy(self):
        return dict(self.items())

    def update(self, *a, **k):
        dict.update(self._fill(), *a, **k)

    def __reduce__(self):
        return (dict, (dict(self.items()),))


POLL_SPIN_S = 0.05


def _poll_slot(host: torch.Tensor, dev) -> None:
    """Wait until k_finalize's five floats replaced the NaN sentinel in the
    pinned slot (each is written once, so five non-NaN values are final), or
    synchronize the device after POLL_SPIN_S (a NaN loss, a slow step — a
    read issued long before its step finishes, e.g. queued behind an
    evaluation, pays that synchronize).  The first ~64 checks spin (a step's
    tail is tens of µs); after that the loop yields the GIL between checks."""
    arr = host.numpy()
    if not np.isnan(arr).any():
        return
    t0 = time.perf_counter()
    spins = 0
    while np.isnan(arr).any():
        el = time.perf_counter() - t0
        if el > POLL_SPIN_S:
            torch.cuda.synchronize(dev)
            return
        spins += 1
        if spins > 64:
            time.sleep(0 if el < 1e-3 else 5e-5)


class _LogRing:
    """Pinned host slots for the per-step loss read-back.  Reusing a slot first
    completes the log that occupied it, so the host runs at most len(slots)
    steps ahead of the device and a deferred device error surfaces within
    that many steps even if no log is read."""

    def __init__(self, dev, depth: int = 2):
        self.dev = dev
        cuda = dev.type == 'cuda'  # (CPU only under the gloo tests' stand-in kernels)
        self.slots = [[torch.empty(5, dtype=torch.float32, pin_memory=cuda), torch.cuda.Event() if cuda else None,
                       None] for _ in range(depth)]
        self.k = 0

    def reserve(self) -> torch.Tensor:
        """The next slot's pinned [5] buffer (its previous log completed first):
        the single-device step's k_finalize writes the losses straight into it."""
        slot = self.slots[self.k]
        if slot[2] is not None:
            slot[2]._fill()
            slot[2] = None
        slot[0].fill_(float('nan'))  # the sentinel the log polls for (a host write: the slot is pinned memory)
        return slot[0]

    def push(self, losses: torch.Tensor, has_reg: bool) -> StepLog:
        """Log of the step whose losses are in `losses` (copied unless it is the
        reserved slot itself); the event marks when the slot holds them."""
        slot = self.slots[self.k]
        self.k = (self.k + 1) % len(self.slots)
        if slot[2] is not None:
            slot[2]._fill()
        direct = losses.data_ptr() == slot[0].data_ptr()  # k_finalize wrote the reserved slot itself
        if not direct:
            slot[0].copy_(losses, non_blocking=True)
        event = None
        if slot[1] is not None and not direct:
            slot[1].record()
            event = slot[1]
        log = StepLog((slot[0], event, has_reg, self.dev))
        slot[2] = log
        return log


class KGEModel(nn.Module):
    def __init__(self, model_name, nentity, nrelation, hidden_dim, gamma,
                 double_entity_embedding=False, double_relation_embedding=False):
        super(KGEModel, self).__init__()
        self.model_name = model_name
        self.nentity = nentity
        self.nrelation = nrelation
        self.hidden_dim = hidden_dim
        self.epsilon = 2.0

        # model.py:32-40 — fp32 scalars; .item() of them is what the reference's math reads
        self.gamma = nn.Parameter(torch.Tensor([gamma]), requires_grad=False)
        self.embedding_range = nn.Parameter(
            torch.Tensor([(self.gamma.item() + self.epsilon) / hidden_dim]), requires_grad=False)

        self.entity_dim = hidden_dim * 2 if double_entity_embedding else hidden_dim
        self.relation_dim = hidden_dim * 2 if double_relation_embedding else hidden_dim

        # model.py:45-57 — same draws from torch's CPU generator as the reference
        r = self.embedding_range.item()
        self.entity_embedding = nn.Parameter(torch.zeros(nentity, self.entity_dim))
        nn.init.uniform_(tensor=self.entity_embedding, a=-r, b=r)
        self.relation_embedding = nn.Parameter(torch.zeros(nrelation, self.relation_dim))
        nn.init.uniform_(tensor=self.relation_embedding, a=-r, b=r)

        if model_name == 'pRotatE':
            self.modulus = nn.Parameter(torch.Tensor([[0.5 * r]]))

        if model_name not in _MODELS:
            raise ValueError('model %s not supported' % model_name)
        if model_name == 'RotatE' and (not double_entity_embedding or double_relation_embedding):
            raise ValueError('RotatE should use --double_entity_embedding')
        if model_name == 'ComplEx' and (not double_entity_embedding or not double_relation_embedding):
            raise ValueError('ComplEx should use --double_entity_embedding and --double_relation_embedding')

        self._scalars = None
        self._grad_bufs = None
        # train_step returns a StepLog filled on first read instead of waiting
        # for the step's losses (False: wait inside train_step, as the reference)
        self.defer_log = True
        # leave the dense gradients in .grad after a fused train_step, as
        # loss.backward() does in the reference; False skips those writes
        self.keep_grads = True
        # apply a KGEAdam update inside the gradient passes (kge_train_step)
        self.fuse_optimizer = True
        # RotatE / pRotatE ranking: the reference's own CPU trig ("reference":
        # RotatE's queries rotated by its cos / sin of the relation phases,
        # ops.reference_rotation; pRotatE's near-ties re-scored from its sin
        # of their phase sums, ops.reference_sin — ranks bit-exact to the
        # reference's), or correctly rounded values evaluated on the device
        # ("device": no host work, last-bit trig differences can move a
        # near-tied rank)
        self.rank_trig = "reference"

    # ------------------------------------------------------------------ helpers
    def _host_scalars(self):
        """(gamma, embedding_range) as Python floats, cached (they never train)."""
        if self._scalars is None:
            self._scalars = (float(self.gamma.detach().cpu().item()),
                             float(self.embedding_range.detach().cpu().item()))
        return self._scalars

    def _load_from_state_dict(self, *args, **kwargs):
        self._scalars = None
        return super()._load_from_state_dict(*args, **kwargs)

    def _modulus(self):
        return self.modulus if self.model_name == 'pRotatE' else None

    def _rank_rotation(self, dev, relation_trig=None):
        """The RotatE rotation table a ranking call uses (kge_model_desc.relation_trig):
        `relation_trig` if given, else per `rank_trig` the reference's CPU cos / sin of
        the current relation table (evaluated once per call) or None (device trig)."""
        if self.model_name != 'RotatE':
            return None
        if relation_trig is None:
            if self.rank_trig == "device":
                return None
            if self.rank_trig != "reference":
                raise ValueError("rank_trig %s not supported" % self.rank_trig)
            relation_trig = ops.reference_rotation(self.relation_embedding, self._host_scalars()[1])
        return relation_trig.to(dev, torch.float32).contiguous()

    def _rank_library_sin(self):
        """pRotatE: re-score the ranking's near-ties with the reference's own
        host sin (ops.reference_sin), per `rank_trig`."""
        if self.model_name != 'pRotatE':
            return False
        if self.rank_trig not in ("reference", "device"):
            raise ValueError("rank_trig %s not supported" % self.rank_trig)
        return self.rank_trig == "reference"

    def desc(self):
        """The C-ABI model descriptor, rebuilt only when a table moves or is replaced."""
        g, rng = self._host_scalars()
        mod = self._modulus()
        ent, rel = self.entity_embedding, self.relation_embedding
        key = (ent.data_ptr(), rel.data_ptr(), None if mod is None else mod.data_ptr(), tuple(ent.shape),
               tuple(rel.shape), g, rng)
        cached = getattr(self, '_desc_cache', None)
        if cached is None or cached[0] != key:
            d = ops.make_desc(self.model_name, ent.detach(), rel.detach(), g, rng,
                              None if mod is None else mod.detach())
            self._desc_cache = cached = (key, d)
        return cached[1]

    # ------------------------------------------------------------------ forward
    def forward(self, sample, mode='single'):
        '''Scores of a batch (model.py:72-164).

        'single': sample = triples [B, 3] -> [B, 1]
        'head-batch': sample = (tail_part [B, 3], head_part [B, n]) -> [B, n]
        'tail-batch': sample = (head_part [B, 3], tail_part [B, n]) -> [B, n]
        '''
        if mode == 'single':
            pos, neg = sample, None
        elif mode == 'head-batch':
            pos, neg = sample
        elif mode == 'tail-batch':
            pos, neg = sample
        else:
            raise ValueError('mode %s not supported' % mode)
        dev = self.entity_embedding.device
        pos = pos.to(dev)
        neg = None if neg is None else neg.to(dev)
        g, rng = self._host_scalars()
        torch_ops.load()
        return torch.ops.kge.score(self.entity_embedding, self.relation_embedding, pos, neg, _lib.MODE_IDS[mode],
                                   _lib.MODEL_IDS[self.model_name], g, rng, self._modulus())

    # ------------------------------------------------------- score plug-ins
    def _plugin(self, name, head, relation, tail, mode):
        """Plug-in call on gathered rows (model.py:151-160): the rows become
        small tables and go through the same HIP score kernel (with autograd)."""
        B = relation.shape[0]
        if mode == 'head-batch':
            n = head.shape[1]
            ent = torch.cat([head.reshape(B * n, -1), tail.reshape(B, -1)], 0)
            neg = torch.arange(B * n, device=ent.device).view(B, n)
            tid = torch.arange(B, device=ent.device) + B * n
            pos = torch.stack([tid, torch.arange(B, device=ent.device), tid], 1)
        elif mode == 'tail-batch':
            n = tail.shape[1]
            ent = torch.cat([tail.reshape(B * n, -1), head.reshape(B, -1)], 0)
            neg = torch.arange(B * n, device=ent.device).view(B, n)
            hid = torch.arange(B, device=ent.device) + B * n
            pos = torch.stack([hid, torch.arange(B, device=ent.device), hid], 1)
        elif mode == 'single':
            ent = torch.cat([head.reshape(B, -1), tail.reshape(B, -1)], 0)
            neg = None
            ar = torch.arange(B, device=ent.device)
            pos = torch.stack([ar, ar, ar + B], 1)
        else:
            raise ValueError('mode %s not supported' % mode)
        g, rng = self._host_scalars()
        torch_ops.load()
        return torch.ops.kge.score(ent.contiguous(), relation.reshape(B, -1).contiguous(), pos, neg,
                                   _lib.MODE_IDS[mode], _lib.MODEL_IDS[name], g, rng, self._modulus())

    def TransE(self, head, relation, tail, mode):
        return self._plugin('TransE', head, relation, tail, mode)

    def DistMult(self, head, relation, tail, mode):
        return self._plugin('DistMult', head, relation, tail, mode)

    def ComplEx(self, head, relation, tail, mode):
        return self._plugin('ComplEx', head, relation, tail, mode)

    def RotatE(self, head, relation, tail, mode):
        return self._plugin('RotatE', head, relation, tail, mode)

    def pRotatE(self, head, relation, tail, mode):
        return self._plugin('pRotatE', head, relation, tail, mode)

    # --------------------------------------------------------------- training
    def _grad_buffers(self):
        dev = self.entity_embedding.device
        bufs = self._grad_bufs
        if bufs is None or bufs[0].device != dev or bufs[0].shape != self.entity_embedding.shape:
            ge = torch.empty_like(self.entity_embedding, memory_format=torch.contiguous_format)
            gr = torch.empty_like(self.relation_embedding, memory_format=torch.contiguous_format)
            gm = torch.empty(1, 1, device=dev) if self.model_name == 'pRotatE' else None
            losses = torch.empty(5, device=dev)  # 4 losses + the device error flag
            self._grad_bufs = bufs = (ge, gr, gm, losses)
        return bufs

    def _log_ring_for(self, dev):
        ring = self.__dict__.get('_log_ring')
        if ring is None or ring.dev != dev:
            ring = self.__dict__['_log_ring'] = _LogRing(dev)
        return ring

    def _log_slot(self, dev):
        """Pinned host buffer the next step's losses are written to (None off-GPU)."""
        if dev.type != 'cuda' or not self.defer_log:
            return None
        return self._log_ring_for(dev).reserve()

    def compute_train_grads(self, positive_sample, negative_sample, subsampling_weight, mode, args,
                            weight_sum=None, uni_batch=0, optimizer=None, entity_chunks=None, on_entity_chunk=None,
                            losses_out=None):
        """Fused forward + self-adversarial loss + backward (model.py:268-301).
        Writes dense .grad tensors; returns the device [5] vector
        (positive_sample_loss, negative_sample_loss, loss, regularization, error flag).
        With a KGEAdam `optimizer` the Adam update is applied inside the same
        gradient passes (the optimizer's next step() then skips these tables).
        With `entity_chunks` [(e0, e1), ...] the entity-gradient pass runs one
        row range at a time and `on_entity_chunk(e0, e1, grad_entity)` is called
        as soon as each range is queued (the data-parallel path starts that
        range's all-reduce there, overlapping the next range's computation)."""
        dev = ops._require_device(self.entity_embedding)
        g, rng = self._host_scalars()
        ge, gr, gm, losses = self._grad_buffers()
        if losses_out is not None:  # e.g. a pinned host slot the kernels write directly
            losses = losses_out
        adam = None
        if optimizer is not None and self.fuse_optimizer and hasattr(optimizer, 'prepare_fused'):
            adam = optimizer.prepare_fused(self.entity_embedding, self.relation_embedding, self._modulus(),
                                           write_grad=self.keep_grads)
        kw = dict(adversarial=bool(args.negative_adversarial_sampling),
                  temperature=float(getattr(args, 'adversarial_temperature', 1.0)),
                  uni_weight=bool(args.uni_weight), regularization=float(args.regularization),
                  grad_entity=ge, grad_relation=gr, grad_modulus=gm, losses=losses,
                  weight_sum_dev=weight_sum, uni_batch=uni_batch)
        desc = self.desc()
        if entity_chunks is None:
            ops.train_step_grads(desc, mode, positive_sample, negative_sample, subsampling_weight, dev, adam=adam,
                                 **kw)
        else:
            run = lambda **x: ops.train_step_grads(desc, mode, positive_sample, negative_sample,  # noqa: E731
                                                   subsampling_weight, dev, **kw, **x)
            run(phases=_lib.PHASE_ROWS)
            for e0, e1 in entity_chunks:
                run(phases=_lib.PHASE_ENTITY, entity_range=(e0, e1))
                if on_entity_chunk is not None:
                    on_entity_chunk(e0, e1, ge)
            run(phases=_lib.PHASE_FINALIZE)
        if self.entity_embedding.requires_grad:
            self.entity_embedding.grad = ge
        if self.relation_embedding.requires_grad:
            self.relation_embedding.grad = gr
        if gm is not None and self.modulus.requires_grad:
            self.modulus.grad = gm
        return losses

    @staticmethod
    def train_step(model, optimizer, train_iterator, args):
        '''
        A single train step. Apply back-propation and return the loss
        (model.py:252-312).  One fused HIP pass replaces the two forward
        calls, the loss and loss.backward(); one 5-float D2H copy replaces
        the three .item() syncs, and nothing waits for it: the returned log
        (StepLog) is filled on first read, so the host enqueues the next
        step while this one runs (at most two steps ahead; model.defer_log =
        False restores the reference's read-back inside the step).
        '''
        model.train()
        optimizer.zero_grad()
        positive_sample, negative_sample, subsampling_weight, mode = next(train_iterator)
        dev = model.entity_embedding.device
        positive_sample = positive_sample.to(dev, non_blocking=True)
        negative_sample = negative_sample.to(dev, non_blocking=True)
        subsampling_weight = subsampling_weight.to(dev, non_blocking=True)

        part = getattr(model, 'row_partition', None)
        dp = getattr(args, 'dp_group', None)
        if part is not None:
            # row-partitioned entity table (partition.py): reduce-scatter to the owners
            losses = part.train_grads(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                                      optimizer=optimizer)
        elif dp is not None:
            import torch.distributed as dist
            from .distributed import dp_exchange_mode, dp_train_grads, dp_train_step_factors, warn_owner_without_partition
            exchange = dp_exchange_mode(dist.get_world_size(dp), getattr(args, 'dp_exchange', None))
            if exchange == "factors":
                losses = dp_train_step_factors(model, positive_sample, negative_sample, subsampling_weight, mode,
                                               args, optimizer=optimizer)
            else:
                if exchange == "owner":  # needs the row partition attached (run.py builds it); without one: grads
                    warn_owner_without_partition()
                losses = dp_train_grads(model, positive_sample, negative_sample, subsampling_weight, mode, args,
                                        optimizer=optimizer)
        else:
            # a KGEAdam optimizer is stepped inside the gradient passes; any
            # other optimizer sees ordinary dense .grad tensors.  The loss
            # vector goes straight into the next pinned log slot (no D2H copy)
            losses = model.compute_train_grads(positive_sample, negative_sample, subsampling_weight, mode, args,
                                               optimizer=optimizer, losses_out=model._log_slot(dev))

        optimizer.step()
        if part is not None:
            part.gather()  # owners' updated rows → every replica

        # the step's only device→host transfer: 4 losses + the error flag in a
        # pinned slot; the log reads it on first access (StepLog)
        log = model._log_ring_for(dev).push(losses, args.regularization != 0.0)
        if not model.defer_log:
            log._fill()
        return log

    # ------------------------------------------------------------- evaluation
    @staticmethod
    def test_step(model, test_triples, all_true_triples, args):
        '''
        Evaluate the model on test or valid datasets (model.py:315-429).
        '''
        model.eval()
        dev = ops._require_device(model.entity_embedding)

        if args.countries:
            from sklearn.metrics import average_precision_score
            # AUC-PR over every (test triple, region) pair, model.py:322-344
            sample = []
            y_true = []
            for head, relation, tail in test_triples:
                for candidate_region in args.regions:
                    y_true.append(1 if candidate_region == tail else 0)
                    sample.append((head, relation, candidate_region))
            sample = torch.LongTensor(sample).to(dev)
            with torch.no_grad():
                y_score = model(sample).squeeze(1).cpu().numpy()
            y_true = np.array(y_true)
            auc_pr = average_precision_score(y_true, y_score)
            return {'auc_pr': auc_pr}

        # Filtered MRR / MR / HITS@{1,3,10}: head-batch queries, then tail-batch
        # (model.py:349-418); the filter is dataloader.py:134-154's.
        index = FilterIndex(all_true_triples, args.nentity, args.nrelation, device=dev)  # built on the GPU
        triples = triples_array(test_triples)
        desc = model.desc()
        ranks_seq = []  # head-batch queries, then tail-batch, as the reference's logs list
        test_batch_size = max(1, int(args.test_batch_size))
        total_steps = 2 * ((len(triples) + test_batch_size - 1) // test_batch_size)
        test_log_steps = max(1, int(getattr(args, 'test_log_steps', 1000)))
        # queries per kernel launch (results do not depend on it): as many as
        # keep the per-launch q buffer and filter bitmap within 128 MB each
        row_bytes = max(4 * int(model.entity_dim), 4 * ((int(args.nentity) + 31) // 32))
        block = max(test_batch_size, min(16384, max(256, (128 << 20) // row_bytes)))
        step = 0
        per_mode = []  # device rank tensors; read back once, after both directions are queued
        with torch.no_grad():
            trig = model._rank_rotation(dev)
            lsin = model._rank_library_sin()
            both = not lsin and os.environ.get("KGE_RANK_BOTH", "1") != "0"
            if both:
                # both directions of a block in one pass (kge_rank_filtered_both;
                # its workspace holds 2 × the block); the filter as the dense
                # device table when the index has one, else per-query lists
                tabs = None
                if os.environ.get("KGE_RANK_FILTER_TABLE", "1") != "0":
                    tabs = (index.device_table('head-batch', dev), index.device_table('tail-batch', dev))
                    tabs = None if tabs[0] is None or tabs[1] is None else tabs
                heads, tails = [], []
                bb = max(1, block // 2)
                for b0 in range(0, len(triples), bb):
                    q = triples[b0:b0 + bb]
                    if tabs is not None:
                        fh, ft = tabs
                    else:
                        fh, ft = (tuple(torch.from_numpy(x) for x in index.filter_csr(q, m))
                                  for m in ('head-batch', 'tail-batch'))
                    ranks, _ = ops.rank_filtered_both(desc, torch.from_numpy(q), fh, ft, dev, relation_trig=trig,
                                                      reuse_table=b0 > 0, filter_table=tabs is not None)
                    heads.append(ranks[:len(q)])
                    tails.append(ranks[len(q):])
                per_mode = [heads, tails]
                # progress messages on the reference's batch cadence (head-batch batches, then tail-batch)
                for step in range(total_steps):
                    if step % test_log_steps == 0:
                        logging.info('Evaluating the model... (%d/%d)' % (step, total_steps))
            for mode in (() if both else ('head-batch', 'tail-batch')):
                ranks_all = []
                per_mode.append(ranks_all)
                for b0 in range(0, len(triples), block):
                    q = triples[b0:b0 + block]
                    off, ids = index.filter_csr(q, mode)
                    ranks, _ = ops.rank_filtered(desc, mode, torch.from_numpy(q), torch.from_numpy(off),
                                                 torch.from_numpy(ids), dev, relation_trig=trig,
                                                 reuse_table=step > 0, library_sin=lsin)
                    ranks_all.append(ranks)
                    # progress messages on the reference's batch cadence
                    nb = (len(q) + test_batch_size - 1) // test_batch_size
                    for _ in range(nb):
                        if step % test_log_steps == 0:
                            logging.info('Evaluating the model... (%d/%d)' % (step, total_steps))
                        step += 1
            for ranks_all in per_mode:  # head-batch, then tail-batch
                ranks_np = torch.cat(ranks_all).cpu().numpy() if ranks_all else np.zeros(0, np.int64)
                ranks_seq.extend(ranks_np.tolist())
            ops.raise_on_device_error(dev)
        # model.py:405-427: per-query log entries averaged in order — the same
        # left-to-right float sums, without materialising a dict per query
        n = len(ranks_seq)
        return {
            'MRR': sum(1.0 / r for r in ranks_seq) / n,
            'MR': sum(float(r) for r in ranks_seq) / n,
            'HITS@1': sum(1.0 if r <= 1 else 0.0 for r in ranks_seq) / n,
            'HITS@3': sum(1.0 if r <= 3 else 0.0 for r in ranks_seq) / n,
            'HITS@10': sum(1.0 if r <= 10 else 0.0 for r in ranks_seq) / n,
        }

    def rank_queries_both(self, triples, all_true_triples, path="auto", relation_trig=None):
        """rank_queries for head-batch and tail-batch, both queued before the
        one read-back (the tail direction's host filter CSR overlaps the head
        direction's kernels, as in test_step).  Returns ((ranks, ties) head,
        (ranks, ties) tail)."""
        dev = ops._require_device(self.entity_embedding)
        index = all_true_triples if isinstance(all_true_triples, FilterIndex) else \
            FilterIndex(all_true_triples, self.nentity, self.nrelation, device=dev)
        q = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        nq = len(q)
        outs = []
        with torch.no_grad():
            trig = self._rank_rotation(dev, relation_trig)
            qd = None
            use_table = os.environ.get("KGE_RANK_FILTER_TABLE", "1") != "0"
            if not self._rank_library_sin() and os.environ.get("KGE_RANK_BOTH", "1") != "0":
                # both directions in one pass (kge_rank_filtered_both): one
                # MFMA counting launch over 2·nq queries, the table's statistics
                # and split operands once, half the small launches
                fh = index.device_table('head-batch', dev) if use_table else None
                ft = index.device_table('tail-batch', dev) if fh is not None else None
                tab_mode = ft is not None  # else per-query lists (fh / ft rebound to them below)
                if tab_mode:
                    qd = torch.from_numpy(np.ascontiguousarray(q)).pin_memory()  # copied right before the launch
                else:
                    (oh, ih), (ot, it) = index.filter_csr(q, 'head-batch'), index.filter_csr(q, 'tail-batch')
                    parts = [q.reshape(-1), oh, ih if len(ih) else np.zeros(1, np.int64), ot,
                             it if len(it) else np.zeros(1, np.int64)]
                    flat = torch.from_numpy(np.concatenate(parts).astype(np.int64, copy=False)).pin_memory()
                    flat = flat.to(dev, non_blocking=True)
                    o = [3 * nq, 3 * nq + nq + 1]
                    o += [o[1] + max(1, len(ih)), o[1] + max(1, len(ih)) + nq + 1]
                    qd = flat[:3 * nq].view(nq, 3)
                    fh, ft = (flat[o[0]:o[1]], flat[o[1]:o[2]]), (flat[o[2]:o[3]], flat[o[3]:])
                # ranks and ties straight into one buffer, read back with the
                # error flag in two copies (no packing kernel)
                buf = torch.empty(6 * nq, dtype=torch.int32, device=dev)
                ops.rank_filtered_both(self.desc(), qd, fh, ft, dev, path=path, relation_trig=trig,
                                       filter_table=tab_mode, out=buf)
                host = torch.empty(6 * nq + 1, dtype=torch.int32, pin_memory=True)
                host[:6 * nq].copy_(buf, non_blocking=True)
                host[6 * nq:].copy_(ops.state(dev).err, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                h = host.numpy()
                ops.raise_device_error_value(dev, int(h[-1]))
                r = h[:4 * nq].view(np.int64)
                t = h[4 * nq:6 * nq]
                return (r[:nq].copy(), t[:nq].copy()), (r[nq:].copy(), t[nq:].copy())
            for mode in ('head-batch', 'tail-batch'):
                # a dense filter index is looked up on the device
                # (KGE_RANK_FILTER_TABLE, uploaded once per index)
                table = index.device_table(mode, dev) if use_table else None
                if table is not None:
                    if qd is None:
                        qd = torch.from_numpy(np.ascontiguousarray(q)).pin_memory().to(dev, non_blocking=True)
                    outs.append(ops.rank_filtered(self.desc(), mode, qd, table[0], table[1], dev, path=path,
                                                  relation_trig=trig, reuse_table=bool(outs),
                                                  library_sin=self._rank_library_sin(), filter_table=True))
                    continue
                # the direction's inputs in one pinned host buffer, copied
                # asynchronously: the tail's filter CSR is built on the host
                # while the head direction's kernels run, and its copy queues
                # behind them without blocking the host
                off, ids = index.filter_csr(q, mode)
                parts = ([q.reshape(-1)] if qd is None else []) + [off, ids if len(ids) else np.zeros(1, np.int64)]
                flat = torch.from_numpy(np.concatenate(parts).astype(np.int64, copy=False)).pin_memory()
                flat = flat.to(dev, non_blocking=True)
                if qd is None:
                    qd, flat = flat[:3 * nq].view(nq, 3), flat[3 * nq:]
                outs.append(ops.rank_filtered(self.desc(), mode, qd, flat[:nq + 1], flat[nq + 1:], dev, path=path,
                                              relation_trig=trig, reuse_table=bool(outs),
                                              library_sin=self._rank_library_sin()))
            # one device → host copy (pinned): both directions' ranks (int64 as
            # int32 pairs) and ties, and the error flag
            packed = torch.cat([outs[0][0].view(torch.int32), outs[1][0].view(torch.int32), outs[0][1], outs[1][1],
                                ops.state(dev).err])
            host = torch.empty(packed.shape, dtype=torch.int32, pin_memory=True)
            host.copy_(packed, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
        h = host.numpy()
        ops.raise_device_error_value(dev, int(h[-1]))
        rh, rt = h[:2 * nq].view(np.int64).copy(), h[2 * nq:4 * nq].view(np.int64).copy()
        th, tt = h[4 * nq:5 * nq].copy(), h[5 * nq:6 * nq].copy()
        return (rh, th), (rt, tt)

    def rank_queries(self, triples, all_true_triples, mode, path="auto", listed=False, relation_trig=None):
        """Per-query filtered ranks and tie counts (numpy int64, int32) — the
        quantity test_step averages; exposed for parity tests and tools.
        `path` / `listed` / `relation_trig`: see ops.rank_filtered (RotatE:
        default per `rank_trig`, see _rank_rotation)."""
        dev = ops._require_device(self.entity_embedding)
        index = all_true_triples if isinstance(all_true_triples, FilterIndex) else \
            FilterIndex(all_true_triples, self.nentity, self.nrelation, device=dev)
        q = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        off, ids = index.filter_csr(q, mode)
        with torch.no_grad():
            out = ops.rank_filtered(self.desc(), mode, torch.from_numpy(q), torch.from_numpy(off),
                                    torch.from_numpy(ids), dev, path=path, listed=listed,
                                    relation_trig=self._rank_rotation(dev, relation_trig),
                                    library_sin=self._rank_library_sin())
        res = tuple(t.cpu().numpy() for t in out)
        ops.raise_on_device_error(dev)
        return res
