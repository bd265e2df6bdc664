#!/usr/bin/env python3
"""Compute side of the data-parallel factor exchange on one GPU (RotatE FB15k
shape): the per-rank row pass on 1024 rows (kge_train_rows_slice), the
global step (kge_train_step_from_rows, fused Adam) on N·1024 gathered rows,
and the owner-computes step (the same, entity pass + Adam on the 1/N of the
rows one rank owns, kge_train_step_from_rows_range), for N = 1, 2, 4, 8 —
against the single-device fused step.  Prints one JSON
line; the exchange itself moves (B·Le + B·n + 4B)·4 + B·(n+3)·8 bytes per rank.

    python tools/dp_factor_cost.py [--reps 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from argparse import Namespace  # noqa: E402

from knowledgegraphembedding_amd import KGEAdam, KGEModel, _lib, ops, synth  # noqa: E402

E, R, D, B, N = 14951, 1345, 1000, 1024, 256


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = KGEModel("RotatE", E, R, D, 24.0, True, False).to(dev)
    opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-4)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    desc = m.desc()
    Le = m.entity_dim
    res = {"workload": "RotatE FB15k shape d=1000 b=1024/rank n=256", "reps": a.reps}
    pos, neg, w = (torch.from_numpy(x).to(dev) for x in synth.kge_batch(9, B, N, E, R))

    def single():
        m.compute_train_grads(pos, neg, w, "tail-batch", args, optimizer=opt)
        opt.step()
    res["single_step_ms"] = timed(single, a.reps)

    for world in (1, 2, 4, 8):
        Bg = B * world
        pg, ng, wg = (torch.from_numpy(x).to(dev) for x in synth.kge_batch(10 + world, Bg, N, E, R))
        wsum = torch.empty(1, device=dev)
        g_g, dq_g, st_g = torch.empty(Bg, N, device=dev), torch.empty(Bg, Le, device=dev), torch.empty(Bg, 4, device=dev)
        ge, gr, gm, losses = m._grad_buffers()

        def rows():
            ops.weight_sum(wg, wsum)
            ops.train_rows_slice(desc, "tail-batch", pg[:B], ng[:B], wg[:B], wsum, dev, adversarial=True,
                                 temperature=1.0, uni_weight=False, uni_batch=Bg, g_out=g_g[:B], dq_out=dq_g[:B],
                                 stats_out=st_g[:B])

        def glob():
            adam = opt.prepare_fused(m.entity_embedding, m.relation_embedding, None, write_grad=True)
            ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, uni_weight=False, uni_batch=Bg,
                                     regularization=0.0, g_in=g_g, dq_in=dq_g, stats=st_g, grad_entity=ge,
                                     grad_relation=gr, grad_modulus=gm, losses=losses, adam=adam)
            opt.step()
        if world == 1:
            res["rows_slice_ms"] = timed(rows, a.reps)
        for k in range(world):  # every row's factors filled once, as after the exchange
            sl = slice(k * B, (k + 1) * B)
            ops.train_rows_slice(desc, "tail-batch", pg[sl], ng[sl], wg[sl], wsum, dev, adversarial=True,
                                 temperature=1.0, uni_weight=False, uni_batch=Bg, g_out=g_g[sl], dq_out=dq_g[sl],
                                 stats_out=st_g[sl])
        res[f"global_step_ms_N{world}"] = timed(glob, a.reps)

        def glob_csr():  # the CSR already built (kge_train_csr ran while the factors were on the wire)
            adam = opt.prepare_fused(m.entity_embedding, m.relation_embedding, None, write_grad=True)
            ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, uni_weight=False, uni_batch=Bg,
                                     regularization=0.0, g_in=g_g, dq_in=dq_g, stats=st_g, grad_entity=ge,
                                     grad_relation=gr, grad_modulus=gm, losses=losses, adam=adam, csr_ready=True)
            opt.step()
        ops.train_csr(desc, "tail-batch", pg, ng, dev)
        res[f"global_step_ms_N{world}_csr_ahead"] = timed(glob_csr, a.reps)

        # the "owner" exchange: the same global step, but the entity pass and
        # its fused Adam only over the 1/N of the rows rank 0 owns
        rows_own = -(-E // world)
        shard = torch.nn.Parameter(m.entity_embedding.data[:rows_own])
        oopt = KGEAdam([shard, m.relation_embedding], lr=1e-4)

        def owner():
            adam = oopt.prepare_fused_rows(shard, m.entity_embedding, 0, m.relation_embedding, None, write_grad=True)
            ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, uni_weight=False, uni_batch=Bg,
                                     regularization=0.0, g_in=g_g, dq_in=dq_g, stats=st_g, grad_entity=ge,
                                     grad_relation=gr, grad_modulus=gm, losses=losses, adam=adam, csr_ready=True,
                                     entity_range=(0, rows_own), reg_relations=True)
            oopt.step()
        ops.train_csr(desc, "tail-batch", pg, ng, dev, entity_range=(0, rows_own))
        res[f"owner_step_ms_N{world}_csr_ahead"] = timed(owner, a.reps)
        res[f"csr_owner_range_ms_N{world}"] = timed(
            lambda: ops.train_csr(desc, "tail-batch", pg, ng, dev, entity_range=(0, rows_own)), a.reps)

        # one owner rank's whole device timeline without the collectives, as
        # _exchange_row_factors + _owner_step issue it: the global CSR on a
        # side stream beside the rank's row pass (FX_CHUNKS pieces), then the
        # owner step — shows whether the CSR hides behind the row pass
        side = torch.cuda.Stream(dev)
        gws = ops.exchange_workspace(desc, Bg, N, dev)
        pieces = [(0, B // 2), (B // 2, B)]

        def rank_timeline(chunks=4):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                ops.train_csr(desc, "tail-batch", pg, ng, dev, workspace=gws, entity_range=(0, rows_own))
            ops.weight_sum(wg, wsum)
            for a0, a1 in pieces:
                ops.train_rows_slice(desc, "tail-batch", pg[a0:a1], ng[a0:a1], wg[a0:a1], wsum, dev, adversarial=True,
                                     temperature=1.0, uni_weight=False, uni_batch=Bg, g_out=g_g[a0:a1],
                                     dq_out=dq_g[a0:a1], stats_out=st_g[a0:a1])
            adam = oopt.prepare_fused_rows(shard, m.entity_embedding, 0, m.relation_embedding, None, write_grad=True)
            kw = dict(uni_weight=False, uni_batch=Bg, regularization=0.0, g_in=g_g, dq_in=dq_g, stats=st_g,
                      grad_entity=ge, grad_relation=gr, grad_modulus=gm, losses=losses, adam=adam, csr_ready=True,
                      reg_relations=True, workspace=gws)
            if chunks <= 1:  # one call (the owner step's unchunked form)
                torch.cuda.current_stream(dev).wait_stream(side)
                ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, entity_range=(0, rows_own), **kw)
            else:  # as partition._owner_step: the CSR joined, ROWS, entity chunks, FINALIZE
                torch.cuda.current_stream(dev).wait_stream(side)
                ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, entity_range=(0, rows_own),
                                         phases=_lib.PHASE_ROWS, **kw)
                step = -(-rows_own // chunks)
                for c0 in range(0, rows_own, step):
                    ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev,
                                             entity_range=(c0, min(rows_own, c0 + step)), phases=_lib.PHASE_ENTITY,
                                             **kw)
                ops.train_step_from_rows(desc, "tail-batch", pg, ng, wg, wsum, dev, entity_range=(0, rows_own),
                                         phases=_lib.PHASE_FINALIZE, **kw)
            oopt.step()
        res[f"owner_rank_compute_ms_N{world}_4chunks"] = timed(rank_timeline, a.reps)
        res[f"owner_rank_compute_ms_N{world}_1chunk"] = timed(lambda: rank_timeline(1), a.reps)
        res[f"owner_rank_compute_ms_N{world}_2chunks"] = timed(lambda: rank_timeline(2), a.reps)
        res[f"owner_rows_allgather_bytes_in_N{world}"] = (world - 1) * rows_own * Le * 4
        res[f"csr_ms_N{world}"] = timed(lambda: ops.train_csr(desc, "tail-batch", pg, ng, dev), a.reps)
        res[f"exchange_bytes_per_rank_N{world}"] = (B * Le + B * N + 4 * B) * 4 + B * (N + 3) * 8 + 4 * B
    res["allreduce_bytes_per_rank_grads"] = {f"N{k}": 2 * (k - 1) / k * E * Le * 4 for k in (2, 4, 8)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
