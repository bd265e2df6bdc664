"""KGEAdam — torch.optim.Adam's update as one fused HIP kernel per tensor.

The reference optimises with a plain torch.optim.Adam(lr) (run.py:266-269,
re-created on every learning-rate decay, run.py:315-322).  KGEAdam keeps that
optimizer's hyper-parameters, per-parameter state keys ('step', 'exp_avg',
'exp_avg_sq') and state_dict layout, so checkpoints move between the two in
either direction; the dense update (every row, zero-grad rows included —
SURVEY §7 hard part vii) runs in kge_adam_step.
"""
from __future__ import annotations

import math

import torch

from . import ops


class KGEAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise ValueError("KGEAdam implements the reference's Adam configuration only "
                             "(weight_decay=0, amsgrad=False)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)

        self._fused_done = set()

    def _group_of(self, p):
        for g in self.param_groups:
            for q in g['params']:
                if q is p:
                    return g
        return None

    def _advance(self, p, group):
        state = self.state[p]
        if len(state) == 0:
            state['step'] = torch.tensor(0.0)
            state['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            state['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
        state['step'] += 1
        return state, int(state['step'].item())

    def prepare_fused(self, entity, relation, modulus=None, write_grad=True):
        """Adam descriptor for kge_train_step, which applies this optimizer's
        update to the tables inside the gradient passes.  Advances the step
        counters now and marks the tensors so the following step() skips them.
        Returns None (use the unfused path) if the configuration does not fit."""
        from . import _lib
        tensors = [entity, relation] + ([modulus] if modulus is not None else [])
        groups = [self._group_of(p) for p in tensors]
        if any(g is None for g in groups) or any(not p.requires_grad for p in tensors):
            return None
        if len({(g['betas'], g['eps']) for g in groups}) != 1:
            return None
        if any(not p.is_contiguous() for p in tensors):
            return None
        desc = _lib.AdamDesc()
        beta1, beta2 = groups[0]['betas']
        desc.beta1, desc.beta2, desc.eps = beta1, beta2, groups[0]['eps']
        desc.write_grad = 1 if write_grad else 0
        for p, g, field in zip(tensors, groups, ('entity', 'relation', 'modulus')):
            state, step = self._advance(p, g)
            t = getattr(desc, field)
            t.param = p.data_ptr()
            t.exp_avg = state['exp_avg'].data_ptr()
            t.exp_avg_sq = state['exp_avg_sq'].data_ptr()
            t.step_size = g['lr'] / (1 - beta1 ** step)
            t.bias_correction2_sqrt = math.sqrt(1 - beta2 ** step)
            self._fused_done.add(id(p))
        return desc

    def prepare_fused_rows(self, shard, table, row0, relation, modulus=None, write_grad=True):
        """prepare_fused for an owner of entity rows [row0, row0 + len(shard)):
        `shard` is the optimizer's parameter (a view of those rows of `table`,
        whose moments are shard-sized); the descriptor points the entity
        update at `table` and its moments `row0` rows before the shard's, so
        the kernels index them by global row (kge_train_step_from_rows_range
        touches only the owned rows).  None if the configuration does not fit."""
        from . import _lib
        if shard.data_ptr() != table.data_ptr() + row0 * table.stride(0) * table.element_size():
            return None
        desc = self.prepare_fused(shard, relation, modulus, write_grad)
        if desc is None:
            return None
        off = row0 * table.stride(0) * table.element_size()
        st = self.state[shard]
        desc.entity.param = table.data_ptr()
        desc.entity.exp_avg = st['exp_avg'].data_ptr() - off
        desc.entity.exp_avg_sq = st['exp_avg_sq'].data_ptr() - off
        return desc

    @torch.no_grad()
    def step_param(self, p, chunks=None, before_chunk=None) -> bool:
        """Apply this step's update to ONE parameter now — row range by row
        range, calling before_chunk(k) before range k (the data-parallel path
        waits there for that range's all-reduce) — and skip it in the next
        step().  Same per-element arithmetic as step()."""
        group = self._group_of(p)
        if group is None or p.grad is None or id(p) in self._fused_done:
            return False
        beta1, beta2 = group['betas']
        state, step = self._advance(p, group)
        row_bytes = p[0].numel() * p.element_size() if p.dim() > 1 else 0
        if chunks is not None and (p.dim() < 2 or row_bytes % 16 != 0 or not p.grad.is_contiguous()):
            # row ranges would break kge_adam_step's 16-byte alignment: wait for
            # every range first, then update the whole tensor at once
            if before_chunk is not None:
                for k in range(len(chunks)):
                    before_chunk(k)
            chunks, before_chunk = None, None
        if chunks is None:
            chunks = [(0, p.shape[0] if p.dim() else 1)]
        for k, (r0, r1) in enumerate(chunks):
            if before_chunk is not None:
                before_chunk(k)
            sl = (slice(r0, r1),) if p.dim() else ()
            ops.adam_step(p.data[sl], p.grad[sl], state['exp_avg'][sl], state['exp_avg_sq'][sl], step=step,
                          lr=group['lr'], beta1=beta1, beta2=beta2, eps=group['eps'])
        self._fused_done.add(id(p))
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        done, self._fused_done = self._fused_done, set()
        for group in self.param_groups:
            beta1, beta2 = group['betas']
            for p in group['params']:
                if p.grad is None or id(p) in done:
                    continue
                state, step = self._advance(p, group)
                grad = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                ops.adam_step(p.data, grad, state['exp_avg'], state['exp_avg_sq'], step=step,
                              lr=group['lr'], beta1=beta1, beta2=beta2, eps=group['eps'])
        return loss
