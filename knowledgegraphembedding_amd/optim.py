"""KGEAdam — torch.optim.Adam's update as one fused HIP kernel per tensor.

The reference optimises with a plain torch.optim.Adam(lr) (run.py:266-269,
re-created on every learning-rate decay, run.py:315-322).  KGEAdam keeps that
optimizer's hyper-parameters, per-parameter state keys ('step', 'exp_avg',
'exp_avg_sq') and state_dict layout, so checkpoints move between the two in
either direction; the dense update (every row, zero-grad rows included —
SURVEY §7 hard part vii) runs in kge_adam_step.
"""
from __future__ import annotations

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

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group['betas']
            for p in group['params']:
                if p.grad is None:
                    continue
                state = self.state[p]
                if len(state) == 0:
                    state['step'] = torch.tensor(0.0)
                    state['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state['step'] += 1
                grad = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                ops.adam_step(p.data, grad, state['exp_avg'], state['exp_avg_sq'], step=int(state['step'].item()),
                              lr=group['lr'], beta1=beta1, beta2=beta2, eps=group['eps'])
        return loss
