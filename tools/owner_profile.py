#!/usr/bin/env python3
"""Kernel-level cost of one owner rank's step at N ranks (RotatE FB15k shape,
b = 1024 per rank): the rank's row pass in two pieces, the owner-range CSR of
the global batch beside it, then the owner step (kge_train_step_from_rows
over the rank's 1/N of the entity rows) — run under
`rocprofv3 --kernel-trace --stats` to see which kernels the N-fold global
work lands in.  No collectives (the gathered buffers are used as they are).

    rocprofv3 --kernel-trace --stats -d gpurun_out/owner_prof -- python3 tools/owner_profile.py --world 8
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEAdam, KGEModel, ops, synth  # noqa: E402

E, R, D, B, N = 14951, 1345, 1000, 1024, 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = KGEModel("RotatE", E, R, D, 24.0, True, False).to(dev)
    desc = m.desc()
    Le, Bg = m.entity_dim, B * a.world
    pg, ng, wg = (torch.from_numpy(x).to(dev) for x in synth.kge_batch(10 + a.world, Bg, N, E, R))
    wsum = torch.empty(1, device=dev)
    g_g, dq_g, st_g = torch.empty(Bg, N, device=dev), torch.empty(Bg, Le, device=dev), torch.empty(Bg, 4, device=dev)
    ge, gr, gm, losses = m._grad_buffers()
    rows_own = -(-E // a.world)
    shard = torch.nn.Parameter(m.entity_embedding.data[:rows_own])
    opt = KGEAdam([shard, m.relation_embedding], lr=1e-4)
    side = torch.cuda.Stream(dev)
    gws = ops.exchange_workspace(desc, Bg, N, dev)
    ops.weight_sum(wg, wsum)
    for k in range(a.world):  # every row's factors filled once, as after the exchange
        sl = slice(k * B, (k + 1) * B)
        ops.train_rows_slice(desc, "tail-batch", pg[sl], ng[sl], wg[sl], wsum, dev, adversarial=True, temperature=1.0,
                             uni_weight=False, uni_batch=Bg, g_out=g_g[sl], dq_out=dq_g[sl], stats_out=st_g[sl])
    for _ in range(a.reps):
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            ops.train_csr(desc, "tail-batch", pg, ng, dev, workspace=gws, entity_range=(0, rows_own))
        for a0, a1 in ((0, B // 2), (B // 2, B)):
            ops.train_rows_slice(desc, "tail-batch", pg[a0:a1], ng[a0:a1], wg[a0:a1], wsum, dev, adversarial=True,
                                 temperature=1.0, uni_weight=False, uni_batch=Bg, g_out=g_g[a0:a1],
                                 dq_out=dq_g[a0:a1], stats_out=st_g[a0:a1])
        torch.cuda.current_stream(dev).wait_stream(side)
        adam = opt.prepare_fused_rows(shard, m.entity_embedding, 0, m.relation_embedding, None, write_grad=True)
        ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, uni_weight=False, uni_batch=Bg,
                                 regularization=0.0, g_in=g_g, dq_in=dq_g, stats=st_g, grad_entity=ge,
                                 grad_relation=gr, grad_modulus=gm, losses=losses, adam=adam, csr_ready=True,
                                 entity_range=(0, rows_own), reg_relations=True, workspace=gws)
        opt.step()
    torch.cuda.synchronize()
    print("done", a.world)


if __name__ == "__main__":
    main()
