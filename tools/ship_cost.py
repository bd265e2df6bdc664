#!/usr/bin/env python3
"""Per-rank device cost of one query-shipping step (partition.py exchange
"queries", kge_ship_step) at a chosen world size, on ONE GPU: rank 0 of
`--world` ranks runs its five stages on the global batch (world × b rows)
with its shard of the table; the collectives between the stages are left
out (their buffers are used as they are), so the figures are the compute
side of the step only.  Prints one JSON line with the mean ms per stage and
the step's compute total, plus the collective bytes per rank the step moves.

  python tools/ship_cost.py --world 8            # config 5: YAGO3-10, b=1024, n=1024, d=1000
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--entities", type=int, default=123182)
    ap.add_argument("--relations", type=int, default=37)
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=1024, help="rows per rank")
    ap.add_argument("--negatives", type=int, default=1024)
    ap.add_argument("--mode", default="tail-batch")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W, E, R, D, n = a.world, a.entities, a.relations, a.dim, a.negatives
    Le, Lr, Bg = 2 * D, D, a.batch * a.world
    rows = -(-E // W)
    g = torch.Generator(device="cpu").manual_seed(0)
    rng = (24.0 + 2.0) / D
    shard = ((torch.rand(rows, Le, generator=g) * 2 - 1) * rng).to(dev)
    rel = ((torch.rand(R, Lr, generator=g) * 2 - 1) * rng).to(dev)
    m_e, v_e = torch.zeros_like(shard), torch.zeros_like(shard)
    desc = ops.make_desc("RotatE", shard, rel, 24.0, rng, None)
    desc.nentity = E  # rank 0: own_begin = 0, so the base is the shard itself
    pos = torch.stack([torch.randint(0, E, (Bg,), generator=g), torch.randint(0, R, (Bg,), generator=g),
                       torch.randint(0, E, (Bg,), generator=g)], 1).to(dev)
    neg = torch.randint(0, E, (Bg, n), generator=g).to(dev)
    w = (torch.rand(Bg, generator=g) * 0.3 + 0.1).to(dev)
    wsum = w.sum().reshape(1)
    f32 = dict(device=dev, dtype=torch.float32)
    qq = torch.zeros(2 * Bg * Le, **f32)
    part = torch.zeros(Bg, 4, **f32)
    parts = torch.zeros(W * Bg, 4, **f32)
    scores, gbuf = torch.zeros(Bg, n, **f32), torch.zeros(Bg, n, **f32)
    flat = torch.zeros(2 * Bg * Le + 4 * Bg, **f32)
    ent_c, rel_c, row_stats = torch.zeros(2 * Bg, Le, **f32), torch.zeros(Bg, Lr, **f32), torch.zeros(Bg, 4, **f32)
    gr, grad_e, losses = torch.zeros(R, Lr, **f32), torch.zeros(rows, Le, **f32), torch.zeros(5, **f32)
    sd = _lib.ShipDesc()
    sd.world, sd.rank, sd.own_begin, sd.own_end = W, 0, 0, min(rows, E)
    sd.pos, sd.neg, sd.batch, sd.nneg = pos.data_ptr(), neg.data_ptr(), Bg, n
    sd.subsampling_weight, sd.weight_sum = w.data_ptr(), wsum.data_ptr()
    sd.uni_weight, sd.adversarial, sd.uni_batch = 0, 1, Bg
    sd.adversarial_temperature, sd.regularization = 1.0, 0.0
    q_n = Bg * Le
    sd.q, sd.qp = qq.data_ptr(), qq[q_n:].data_ptr()
    sd.part, sd.parts = part.data_ptr(), parts.data_ptr()
    sd.scores, sd.g = scores.data_ptr(), gbuf.data_ptr()
    sd.dq, sd.pstats, sd.pq = flat.data_ptr(), flat[q_n:].data_ptr(), flat[q_n + 4 * Bg:].data_ptr()
    sd.ent_contrib, sd.rel_contrib, sd.row_stats = ent_c.data_ptr(), rel_c.data_ptr(), row_stats.data_ptr()
    adam = _lib.AdamDesc()
    adam.beta1, adam.beta2, adam.eps, adam.write_grad = 0.9, 0.999, 1e-8, 1
    adam.entity.param, adam.entity.exp_avg, adam.entity.exp_avg_sq = shard.data_ptr(), m_e.data_ptr(), v_e.data_ptr()
    adam.entity.step_size, adam.entity.bias_correction2_sqrt = 1e-4, 1.0
    ws = ops._train_ws(desc, Bg, n, dev)
    stages = [("q", _lib.SHIP_Q), ("rows", _lib.SHIP_ROWS), ("merge", _lib.SHIP_MERGE), ("chain", _lib.SHIP_CHAIN),
              ("entity", _lib.SHIP_ENTITY)]

    def run(stage):
        kw = {}
        if stage >= _lib.SHIP_CHAIN:
            kw["grad_relation"] = gr
        if stage == _lib.SHIP_ENTITY:
            kw.update(adam=adam, grad_entity_ptr=grad_e.data_ptr(), losses=losses)
        ops.ship_step(desc, a.mode, stage, sd, dev, workspace=ws, **kw)

    # fill the shipped buffers once the way the collectives would (this
    # rank's share standing in for every shard's), then time
    run(_lib.SHIP_Q)
    run(_lib.SHIP_ROWS)
    parts.view(W, Bg, 4).copy_(part.unsqueeze(0).expand(W, Bg, 4))
    torch.cuda.synchronize()
    ev = {k: [torch.cuda.Event(enable_timing=True) for _ in range(2)] for k, _ in stages}
    tot = {k: 0.0 for k, _ in stages}
    for it in range(a.iters + 1):
        for k, s in stages:
            ev[k][0].record()
            run(s)
            ev[k][1].record()
        torch.cuda.synchronize()
        if it:  # the first pass warms up
            for k, _ in stages:
                tot[k] += ev[k][0].elapsed_time(ev[k][1])
    ms = {k: v / a.iters for k, v in tot.items()}
    head = a.mode == "head-batch"
    ring = 2.0 * (W - 1) / W  # ring all-reduce bytes per rank / buffer bytes
    comm = {"ids_allgather": (W - 1) / W * Bg * (3 + n) * 8, "q_allreduce": ring * q_n * 4 * (2 if head else 1),
            "state_allgather": (W - 1) / W * Bg * 16,
            "dq_allreduce": ring * (q_n * (2 if head else 1) + 4 * Bg) * 4, "relation_allreduce": ring * R * Lr * 4}
    print(json.dumps({"world": W, "mode": a.mode, "global_batch": Bg, "negatives": n, "entities": E, "dim": D,
                      "shard_rows": rows, "stage_ms": ms, "compute_ms": sum(ms.values()),
                      "comm_bytes_per_rank": comm, "comm_total_MB": sum(comm.values()) / 1e6,
                      "row_allgather_MB_factors_exchange": (W - 1) / W * E * Le * 4 / 1e6}))


if __name__ == "__main__":
    main()
