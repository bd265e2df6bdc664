#!/usr/bin/env python3
"""Where the host time of one KGEModel.train_step goes (diagnostic).

Replays bench.py's configuration and times, per step, the Python/ctypes work
from entry to the kernel launches being queued, and the wait for the result.
"""
import os
import sys
import time
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from knowledgegraphembedding_amd import KGEAdam, KGEModel, ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    m = KGEModel("RotatE", bench.E, bench.R, bench.D, bench.GAMMA, True, False).to(dev)
    args = Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0, dp_group=None)
    opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-4)
    it = bench.DeviceBatches(dev, 5)
    for _ in range(5):
        KGEModel.train_step(m, opt, it, args)
    torch.cuda.synchronize()
    acc = {"prologue": 0.0, "prepare_fused": 0.0, "desc": 0.0, "ctypes_call": 0.0, "opt_step": 0.0, "sync_d2h": 0.0}
    N = 50
    t_all = time.perf_counter()
    for _ in range(N):
        t0 = time.perf_counter()
        m.train()
        opt.zero_grad()
        pos, neg, w, mode = next(it)
        pos, neg, w = pos.to(dev, non_blocking=True), neg.to(dev, non_blocking=True), w.to(dev, non_blocking=True)
        ge, gr, gm, losses = m._grad_buffers()
        t1 = time.perf_counter()
        adam = opt.prepare_fused(m.entity_embedding, m.relation_embedding, None, write_grad=True)
        t2 = time.perf_counter()
        d = m.desc()
        t3 = time.perf_counter()
        ops.train_step_grads(d, mode, pos, neg, w, dev, adversarial=True, temperature=1.0, uni_weight=False,
                             regularization=0.0, grad_entity=ge, grad_relation=gr, grad_modulus=None, losses=losses,
                             adam=adam)
        t4 = time.perf_counter()
        m.entity_embedding.grad, m.relation_embedding.grad = ge, gr
        opt.step()
        t5 = time.perf_counter()
        vals = losses.cpu().tolist()
        t6 = time.perf_counter()
        for k, v in zip(acc, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            acc[k] += v
    total = time.perf_counter() - t_all
    print({k: round(v / N * 1e6, 1) for k, v in acc.items()}, "us/step; total", round(total / N * 1e6, 1), "us/step")


if __name__ == "__main__":
    main()
