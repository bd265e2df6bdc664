#!/usr/bin/env python3
"""Entity pass split across CUs: would a gather part on some
CUs and the dense Adam stream on the others beat the fused pass?

Streams restricted to a subset of the CUs (hipExtStreamCreateWithCUMask) time
(1) the dense Adam stream alone — kge_adam_step over the FB15k RotatE entity
table (read p, g, m, v; write p, m, v: 837 MB) — and (2) the entity-major
gradient pass alone (kge_train_step_grads_phased, ENTITY phase: the q-slice
gathers, gradient written, no Adam), each on 64 / 128 / 192 / 256 CUs, and
(3) both at once on complementary CU sets with no dependency between them:
the wall time of that pair is the floor of any pipelined cross-CU split (a
real one also waits for each gradient chunk before its Adam chunk).  The
fused pass (gradient + Adam, one launch) is timed on all CUs beside them.

    python tools/cu_split_probe.py [--reps 20]

Its gather_* columns (0.044 ms on 64 or 256 CUs, profiles/r05/train/
cu_split_probe.json) are NOT the kernel's time: the same ENTITY-phase launch
runs 0.140-0.165 ms in every rocprofv3 trace (in the step, repeated, after a
cache flush: tools/entity_gather_probe.py, profiles/r05/train/), so the
concurrent / pipeline rows built on it are not evidence either.  The adam_*
columns agree with the traced k_adam (0.145-0.149 ms).
"""
import argparse
import ctypes
import json
import os
import sys
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from knowledgegraphembedding_amd import KGEAdam, KGEModel, _lib, ops, synth  # noqa: E402

E, R, D, B, N = 14951, 1345, 1000, 1024, 256


def masked_stream(cus, total):
    hip = ctypes.CDLL("libamdhip64.so")
    words = (total + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value)


def timed(stream, fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        fn()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    torch.manual_seed(0)
    model = KGEModel("RotatE", E, R, D, 24.0, True, False).to(dev)
    desc = model.desc()
    pos, neg, w = synth.kge_batch(5, B, N, E, R)
    pos, neg, w = torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev)
    ge = torch.zeros_like(model.entity_embedding)
    gr = torch.zeros_like(model.relation_embedding)
    losses = torch.zeros(5, device=dev)
    kw = dict(adversarial=True, temperature=1.0, uni_weight=False, regularization=0.0, grad_entity=ge,
              grad_relation=gr, grad_modulus=None, losses=losses)
    ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ROWS, **kw)
    torch.cuda.synchronize()

    def gather():
        ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ENTITY, **kw)

    # the ENTITY phase alone must reproduce the unphased call's gradient
    gather()
    torch.cuda.synchronize()
    g_phased = ge.clone()
    ge2, gr2 = torch.zeros_like(ge), torch.zeros_like(gr)
    ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, **dict(kw, grad_entity=ge2, grad_relation=gr2))
    torch.cuda.synchronize()
    check = {"gather_equals_unphased": bool(torch.equal(g_phased, ge2)),
             "grad_rows_nonzero": int((g_phased.abs().sum(1) > 0).sum()), "grad_absmax": float(ge2.abs().max())}
    # the unphased call rewrote the workspace for the same batch: the ROWS phase again for the timing loops
    ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ROWS, **kw)
    torch.cuda.synchronize()

    p = torch.randn(E, 2 * D, device=dev) * 0.01
    g = torch.randn_like(p) * 1e-3
    m1, m2 = torch.zeros_like(p), torch.zeros_like(p)

    def adam():
        ops.adam_step(p, g, m1, m2, step=1, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8)

    # the fused pass, as train_step runs it (row pass + fused Adam entity pass): its entity launch
    opt = KGEAdam([q for q in model.parameters() if q.requires_grad], lr=1e-4)
    args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    lib = _lib.load()
    _lib.check(lib.kge_stage_timer(1, None, 1), "kge_stage_timer")
    for _ in range(a.reps):
        model.compute_train_grads(pos, neg, w, "tail-batch", args, optimizer=opt)
    torch.cuda.synchronize()
    import numpy as np
    st = np.zeros(7, dtype=np.float32)
    _lib.check(lib.kge_stage_timer(2, st.ctypes.data_as(ctypes.c_void_p), 7), "kge_stage_timer")
    lib.kge_stage_timer(0, None, 0)
    out = {"cus": ncu, "fused_entity_pass_ms": float(st[4] / max(st[6], 1)), **check}
    ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ROWS, **kw)
    torch.cuda.synchronize()
    for order in ("first", "strided"):
        for n in (64, 128, 192, ncu):
            cus = list(range(n)) if order == "first" else [int(i * ncu / n) for i in range(n)]
            s = masked_stream(cus, ncu)
            out[f"adam_{order}_{n}_ms"] = timed(s, adam, a.reps)
            out[f"gather_{order}_{n}_ms"] = timed(s, gather, a.reps)
    # both at once on complementary CU sets (no dependency): the split's floor
    for ng in (128, 160, 192, 224):
        cg = [int(i * ncu / ng) for i in range(ng)]
        ca = sorted(set(range(ncu)) - set(cg))
        sg, sa = masked_stream(cg, ncu), masked_stream(ca, ncu)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        ev0 = torch.cuda.Event()
        ev0.record()
        for s in (sg, sa):
            s.wait_event(ev0)
        with torch.cuda.stream(sg):
            for _ in range(a.reps):
                gather()
        with torch.cuda.stream(sa):
            for _ in range(a.reps):
                adam()
        torch.cuda.current_stream().wait_stream(sg)
        torch.cuda.current_stream().wait_stream(sa)
        t1.record()
        t1.synchronize()
        out[f"concurrent_gather{ng}_adam{ncu - ng}_ms"] = t0.elapsed_time(t1) / a.reps
    # the production shape of a split: the gradient pass in entity-row chunks
    # on the gather CUs, each chunk's Adam on the stream CUs behind an event
    pm, gm = model.entity_embedding.detach(), ge
    mm, vm = torch.zeros_like(pm), torch.zeros_like(pm)

    def pipeline(ng, chunks, reps):
        cg = [int(i * ncu / ng) for i in range(ng)]
        ca = sorted(set(range(ncu)) - set(cg))
        sg, sa = masked_stream(cg, ncu), masked_stream(ca, ncu)
        step = -(-E // chunks)
        bounds = [(e0, min(E, e0 + step)) for e0 in range(0, E, step)]
        evs = [torch.cuda.Event() for _ in bounds]
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            ev0 = torch.cuda.Event()
            ev0.record()
            sg.wait_event(ev0)
            sa.wait_event(ev0)
            for (e0, e1), ev in zip(bounds, evs):
                with torch.cuda.stream(sg):
                    ops.train_step_grads(desc, "tail-batch", pos, neg, w, dev, phases=_lib.PHASE_ENTITY,
                                         entity_range=(e0, e1), **kw)
                    ev.record()
                sa.wait_event(ev)
                with torch.cuda.stream(sa):
                    ops.adam_step(pm[e0:e1], gm[e0:e1], mm[e0:e1], vm[e0:e1], step=1, lr=1e-4, beta1=0.9,
                                  beta2=0.999, eps=1e-8)
            torch.cuda.current_stream().wait_stream(sg)
            torch.cuda.current_stream().wait_stream(sa)
        t1.record()
        t1.synchronize()
        return t0.elapsed_time(t1) / reps

    for ng in (160, 192, 224):
        for chunks in (4, 8):
            out[f"pipeline_gather{ng}_adam{ncu - ng}_chunks{chunks}_ms"] = pipeline(ng, chunks, a.reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
