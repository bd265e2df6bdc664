#!/usr/bin/env python3
"""bench.py — the BASELINE.json metric on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric: scored (positive + negative) triples per second of the training step,
RotatE FB15k shape (E=14951, R=1345) d=1000 -de, b=1024 per GPU, n=256,
self-adversarial (T=1.0), γ=24 — BASELINE config 2 (best_config.sh:3).
One step = KGEModel.train_step exactly as run.py calls it: fused scoring + loss +
backward (libkge_hip.so) + KGEAdam dense update + the loss read-back, with
batches pre-staged in HBM (the CPU sampler cannot feed this rate; SURVEY §7 v)
and alternating tail-/head-batch like BidirectionalOneShotIterator.
Data: synthetic (uniform ids, reference init U(-range, range) tables).

`--workload fb15k-237` runs BASELINE config 4's shape: RotatE FB15k-237
(E=14541, R=237) d=1000 -de, b=1024 per GPU (global 8192 on 8 GPUs), n=256,
data-parallel.  `--workload yago3-10-rowpart` runs BASELINE config 5: RotatE
YAGO3-10 shape (E=123182, R=37) d=1000 -de, b=1024 per GPU, n=1024, with the
entity table row-partitioned across the ranks (partition.py: reduce-scatter of
the dense entity gradient to the row owners, shard Adam, all-gather of the rows).

Prints one JSON line (rank 0).  `roofline` is the dominant kernel (the fused
row pass) timed live with HIP events on its launch stream, `roofline_entity`
the entity pass the same way; `step_roofline` sums both kernels' bytes over the
whole step time.  `traffic` fields are rocprofv3 PMC bytes per launch from the
committed profiles/ summaries.  `cpu_baseline` is the oracle's ATen op chain
(the reference's algorithm) on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from argparse import Namespace

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from knowledgegraphembedding_amd import KGEAdam, KGEModel, _lib  # noqa: E402
from knowledgegraphembedding_amd.distributed import dp_exchange_mode  # noqa: E402

E, R, D, B, NNEG, GAMMA, TEMP = 14951, 1345, 1000, 1024, 256, 24.0, 1.0
METRIC = "scored (pos+neg) triples/sec, RotatE FB15k d=1000 b=1024 n=256, 1/2/4/8 GPU"
WORKLOADS = {
    # BASELINE config 2 (the headline metric; the driver's default)
    "fb15k": dict(E=14951, R=1345, D=1000, B=1024, NNEG=256, partition=False,
                  name="RotatE FB15k-shape train_step (fused score+self-adv loss+bwd, dense Adam)"),
    # BASELINE config 4 (FB15k-237 shape, 1024 per rank; the 8-GPU driver run makes global 8192)
    "fb15k-237": dict(E=14541, R=237, D=1000, B=1024, NNEG=256, partition=False,
                      name="RotatE FB15k-237-shape train_step, data-parallel (fused score+self-adv loss+bwd, dense Adam)"),
    # BASELINE config 5
    "yago3-10-rowpart": dict(E=123182, R=37, D=1000, B=1024, NNEG=1024, partition=True,
                             name="RotatE YAGO3-10-shape train_step, entity rows partitioned over the ranks "
                                  "(reduce-scatter grads to owners, shard Adam, all-gather rows)"),
}
TIMER_PERIOD = 8
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def algorithmic_row_bytes(b: int, n: int, le: int, lr: int) -> int:
    """Bytes one fused row-pass launch (k_row) must move.  Reads:
    every negative row once, the positive h/r/t rows, indices and weights.
    Writes: dL/ds [b, n], q [b, le] for the entity pass, the row statistics, and
    (the epilogue is fused into the launch) the head/tail [2b, le] and relation
    [b, lr] gradient contributions."""
    reads = b * n * le * 4 + b * (le + lr + le) * 4 + b * n * 8 + b * 3 * 8 + b * 4
    writes = b * n * 4 + b * le * 4 + b * 16 + (2 * b * le + b * lr) * 4
    return reads + writes


def algorithmic_entity_bytes(e: int, r: int, b: int, n: int, le: int, lr: int) -> int:
    """Bytes the entity pass (k_entity_sl with the relation rows in its
    trailing blocks, Adam fused) must move: per table element the fused Adam
    stream reads param, exp_avg, exp_avg_sq and writes them back plus the dense
    gradient (28 B); plus one read of every input it gathers — q [b, le], the
    row contributions [2b, le] and [b, lr], dL/ds [b, n], the occurrence CSR
    (ids + offsets).  The q rows are gathered once per occurrence from L2; only
    their first touch is counted here."""
    adam = 28 * (e * le + r * lr)
    inputs = b * le * 4 + (2 * b * le + b * lr) * 4 + b * n * 4 + (b * n + 3 * b) * 4 + (e + r + 1) * 4
    return adam + inputs


def step_roofline(step_s: float, row_bytes: int, ent_bytes: int, row_traffic, ent_traffic) -> dict:
    """Whole-step view: the two kernels' algorithmic bytes (and their PMC bytes
    when a committed summary exists) over the measured step time.  Every
    figure counts each byte once, so no fraction can exceed 1 unless the
    kernels beat the HBM peak."""
    def gbs(nbytes):
        return nbytes / step_s / 1e9

    alg = row_bytes + ent_bytes
    out = {"algorithmic_bytes": alg, "achieved": gbs(alg), "frac": gbs(alg) / HBM_PEAK_GBS,
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "what": "k_row + entity pass algorithmic bytes / measured step time (includes launch gaps, CSR join, "
                   "finalize and the loss read-back)"}
    if row_traffic and ent_traffic:
        tr = row_traffic + ent_traffic
        out.update({"traffic": tr, "achieved_traffic": gbs(tr), "frac_traffic": gbs(tr) / HBM_PEAK_GBS})
    return out


def _pmc_bytes(path: str):
    """hbm_bytes_per_launch from a committed tools/pmc_traffic.py summary."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


class DeviceBatches:
    """Pre-staged device batches, tail-batch on odd steps and head-batch on even
    steps (dataloader.py:171-177)."""

    def __init__(self, dev, seed: int, nsets: int = 4):
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        self.sets = []
        for _ in range(nsets):
            h = torch.randint(0, E, (B,), device=dev, generator=g)
            r = torch.randint(0, R, (B,), device=dev, generator=g)
            t = torch.randint(0, E, (B,), device=dev, generator=g)
            pos = torch.stack([h, r, t], 1).contiguous()
            neg = torch.randint(0, E, (B, NNEG), device=dev, generator=g)
            w = torch.rand(B, device=dev, generator=g) * 0.3 + 0.1
            self.sets.append((pos, neg, w))
        self.step = 0

    def __iter__(self):
        return self

    def __next__(self):
        self.step += 1
        pos, neg, w = self.sets[self.step % len(self.sets)]
        return pos, neg, w, ('head-batch' if self.step % 2 == 0 else 'tail-batch')


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """CPUs this process may actually use: the affinity mask, capped by the
    cgroup CPU quota and OMP_NUM_THREADS when set (a GPU box shows all of the
    machine's cores in the mask but grants a share of them)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_baseline(model_cpu_state, budget_s: float = 90.0, b: int = B, max_steps: int = 2):
    """The oracle (the reference's ATen op chain on CPU fp32 + torch.optim.Adam)
    on the workload itself — BASELINE config 2's full b = 1024 × n = 256 step
     — on every host core this process may run on: one small
    warm-up step (b = 16: thread pool and allocator), then full-batch steps,
    tail- then head-batch, until `max_steps` are timed or `budget_s` has
    passed after the first (a full step takes ≈ 20-45 s on 8-16 cores, so the
    default budget times two)."""
    from oracle import kge_oracle as O
    ent, rel, erange = model_cpu_state
    cores = host_cores()
    torch.set_num_threads(cores)
    g = torch.Generator().manual_seed(7)

    def batch(nb):
        pos = torch.stack([torch.randint(0, E, (nb,), generator=g), torch.randint(0, R, (nb,), generator=g),
                           torch.randint(0, E, (nb,), generator=g)], 1)
        return pos, torch.randint(0, E, (nb, NNEG), generator=g), torch.rand(nb, generator=g) * 0.3 + 0.1

    params = [ent.clone().requires_grad_(True), rel.clone().requires_grad_(True)]
    opt = torch.optim.Adam(params, lr=1e-4)

    def step(mode, pos, neg, w):
        _, ge, gr, _ = O.train_grads("RotatE", params[0].detach(), params[1].detach(), None, pos, neg, w, mode,
                                     adversarial=True, temperature=TEMP, uni_weight=False, regularization=0.0,
                                     gamma=GAMMA, erange=erange)
        opt.zero_grad()
        params[0].grad, params[1].grad = ge, gr
        opt.step()

    step('tail-batch', *batch(16))  # warm-up
    full = batch(b)
    times = []
    while len(times) < max_steps and (not times or sum(times) < budget_s):
        t0 = time.perf_counter()
        step('head-batch' if len(times) % 2 else 'tail-batch', *full)
        times.append(time.perf_counter() - t0)
    dt = sum(times)
    return {"value": len(times) * b * (NNEG + 1) / dt, "unit": "triples/s", "cores": cores,
            "cpu_model": _cpu_model(), "kind": "port", "step_s": [round(x, 2) for x in times],
            "sample": f"oracle train step (ATen op chain fwd + autograd bwd + torch Adam), the workload's own "
                      f"RotatE E={E} R={R} d={D} b={b} n={NNEG} adv; {len(times)} timed full-batch steps "
                      f"(tail, head) after a b=16 warm-up, {dt:.1f} s, torch threads = {cores}"}


def rank_section(dev, reps: int = 10, distance_reps: int = 3) -> dict:
    """BASELINE config 3, measured live beside the training metric: filtered
    ranking (KGEModel.rank_queries_both → kge_rank_filtered: split-bf16 MFMA
    tile + near-tie refinement in the reference's order) of all 3134
    wn18rr-shape test triples in both directions (6268 queries, E=40943, d=500)
    against a synthetic filter graph of wn18rr's 93,003 true triples
    (tools/bench_rank.py, same data).  The tile computes each fp32 product as
    three bf16 MFMA products (x = x_hi + x_lo; the lo·lo product dropped,
    inside the window's bound): `frac` = the bf16 flops the
    matrix cores issue (tile padding included) / wall time of the whole pass
    (host CSR, bitmap, operand split, window, MFMA tile, refinement,
    read-back) / the 2.5 PF bf16 dense spec; `fp32_equivalent_tflops` =
    2·queries·E·K / the same time (tile alone: profiles/r0x/rank/)."""
    import numpy as np
    from knowledgegraphembedding_amd import synth
    from knowledgegraphembedding_amd.filters import FilterIndex
    Ew, Rw, ntrue, ntest, d = 40943, 11, 93003, 3134, 500
    h, r, t = synth.randint(901, (ntrue,), Ew), synth.randint(902, (ntrue,), Rw), synth.randint(903, (ntrue,), Ew)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(904, (ntest,), len(true))]
    index = FilterIndex(true, Ew, Rw)
    out = {"workload": "wn18rr-shape filtered ranking (config 3), synthetic graph, both directions",
           "queries": 2 * ntest, "entities": Ew, "hidden_dim": d}
    for name, cplx in (("DistMult", False), ("ComplEx", True)):
        torch.manual_seed(0)
        m = KGEModel(name, Ew, Rw, d, 12.0, cplx, cplx).to(dev)
        K = m.entity_dim
        times = []
        for rep in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            (rh, _), (rt, _) = m.rank_queries_both(test, index)
            torch.cuda.synchronize()
            if rep:  # (the first pass is the warm-up)
                times.append(time.perf_counter() - t0)
        best = min(times)
        flops = 2.0 * 2 * ntest * Ew * K  # fp32 products the ranking needs (both directions)
        # what the matrix cores issue: three bf16 products per fp32 product (hi·hi,
        # hi·lo, lo·hi) over the tile-padded shape (128-query and 128-candidate
        # tiles, 16-k slabs)
        pad = lambda x, m: -(-x // m) * m  # noqa: E731
        prods = 3
        issued = 2.0 * prods * pad(2 * ntest, 128) * pad(Ew, 128) * pad(K, 16)  # one tile over both directions
        out[name] = {"ms": best * 1e3, "ms_median": float(np.median(times)) * 1e3, "passes": len(times),
                     "queries_per_s": 2 * ntest / best,
                     "bf16_issued_tflops": issued / best / 1e12, "peak_tflops": 2500.0,
                     "frac": issued / best / 1e12 / 2500.0,
                     "fp32_equivalent_tflops": flops / best / 1e12,
                     "what": "whole pass wall time, the fastest of `passes` after a warm-up (`ms_median`: their "
                             "median; device filter table lookup, bitmap, operand split, window, MFMA tile, "
                             "refinement, read-back); frac = issued bf16 MFMA flops / 2.5 PF bf16 dense spec",
                     "path": f"split-bf16 MFMA tile ({prods} bf16 products per fp32 product) + reference-order "
                             "refinement",
                     "mrr": float(np.mean(1.0 / np.concatenate([rh, rt])))}
        del m
    torch.cuda.empty_cache()
    out.update(distance_rank_section(dev, distance_reps))
    return out


# VALU issue bound of the register tile (k_rank_tile) per pair-element —
# one reduction element of one (query, candidate) pair — from its inner loop's
# instruction mix: issue cycles per wave for 64 pair-elements, at
# 4 SIMDs × 256 CUs × 2.4 GHz (a wave64 VALU instruction, packed or not, 4
# cycles; v_sqrt 8).  RotatE (round 5): v_pk_add (q − e: re and im of two
# candidates, ½ each) + ½ v_pk_mul + ½ v_pk_fma + v_sqrt + ½ v_pk_add = 18
# (round 4's (re, im)-pair form: 22); TransE (round 5): ½ v_pk_add (q − e) +
# v_add with |·| = 6; pRotatE (round 5): ½ v_pk_mul + ½ v_pk_fma + v_add with
# |·| = 8.
TILE_ISSUE_CYC = {"RotatE": 18.0, "TransE": 6.0, "pRotatE": 8.0}


def _rank_timer_read(lib):
    import ctypes
    import numpy as np
    buf = np.zeros(4, dtype=np.float32)
    _lib.check(lib.kge_stage_timer(5, buf.ctypes.data_as(ctypes.c_void_p), 4), "kge_stage_timer")
    return buf


def distance_rank_section(dev, reps: int = 3) -> dict:
    """The distance models' filtered ranking — the register-tile streaming scan
    (k_rank_tile) + near-tie refinement — measured live: RotatE and TransE at
    the FB15k shape best_config.sh:3 / :27 evaluate (E=14951, R=1345, d=1000,
    γ=24; 4096 test triples × both directions against a synthetic filter graph
    of FB15k's 592,213 true triples), pRotatE at the wn18rr shape (E=40943,
    R=11, d=500, γ=6; 3134 × 2 queries, the config-3 graph) with the
    reference's own host sin for its near-ties (ranks bit-exact, three-call
    form).  Per model: the whole pass's wall time and queries/s, and from the
    ranking timer (HIP events on the launch stream, kge_stage_timer 4/5) the
    fast pass's average launch time per direction → pair-element terms/s
    against the tile's VALU issue bound, and the bytes the tile streams from
    L2 / Infinity Cache (every query tile of 64 reads the whole table, every
    candidate tile the query block) over that time."""
    import numpy as np
    from knowledgegraphembedding_amd import synth
    from knowledgegraphembedding_amd.filters import FilterIndex
    lib = _lib.load()
    cases = []
    # FB15k shape: train + valid + test = 592,213 triples (483,142 + 50,000 + 59,071)
    Ef, Rf, nq_f = 14951, 1345, 4096
    tf = np.unique(np.stack([synth.randint(911, (592213,), Ef), synth.randint(912, (592213,), Rf),
                             synth.randint(913, (592213,), Ef)], 1), axis=0)
    test_f = tf[synth.randint(914, (nq_f,), len(tf))]
    idx_f = FilterIndex(tf, Ef, Rf)
    cases.append(("RotatE", True, False, 1000, 24.0, Ef, Rf, test_f, idx_f, "FB15k"))
    cases.append(("TransE", False, False, 1000, 24.0, Ef, Rf, test_f, idx_f, "FB15k"))
    Ew, Rw, ntest = 40943, 11, 3134
    tw = np.unique(np.stack([synth.randint(901, (93003,), Ew), synth.randint(902, (93003,), Rw),
                             synth.randint(903, (93003,), Ew)], 1), axis=0)
    test_w = tw[synth.randint(904, (ntest,), len(tw))]
    cases.append(("pRotatE", False, False, 500, 6.0, Ew, Rw, test_w, FilterIndex(tw, Ew, Rw), "wn18rr"))
    out = {}
    for name, de, dr, d, gamma, En, Rn, test, index, shape in cases:
        torch.manual_seed(0)
        m = KGEModel(name, En, Rn, d, gamma, de, dr).to(dev)
        m.rank_trig = "reference"
        nq = 2 * len(test)
        best, stages = None, None
        for rep in range(reps + 1):
            if rep == 1:
                _lib.check(lib.kge_stage_timer(4, None, 0), "kge_stage_timer")  # warm-up pass untimed
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            (rh, _), (rt, _) = m.rank_queries_both(test, index)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if rep and (best is None or dt < best):
                best = dt
        stages = _rank_timer_read(lib)
        lib.kge_stage_timer(0, None, 0)
        calls = max(1.0, float(stages[3]))
        fast_ms = float(stages[1]) / calls
        Kred = d  # reduction length per pair: complex dims (RotatE) or floats (TransE, pRotatE)
        Le = m.entity_dim
        terms = (nq / 2) * En * Kred  # one direction per call
        bound = 4 * 256 * 2.4e9 * 64 / TILE_ISSUE_CYC[name]
        tiles_q, tiles_e = -(-(nq // 2) // 64), -(-En // 64)
        streamed = 4.0 * Le * (tiles_q * En + tiles_e * (nq // 2))
        out[name] = {
            "shape": f"{shape} E={En} R={Rn} d={d} (entity_dim {Le}), {nq} queries (both directions), "
                     f"synthetic filter graph, rank_trig=reference",
            "ms": best * 1e3, "queries_per_s": nq / best,
            "fast_pass_ms_per_direction": fast_ms,
            "prep_ms_per_direction": float(stages[0]) / calls,
            "refine_ms_per_direction": float(stages[2]) / calls,
            "timed_calls": int(stages[3]),
            "valu": {"bound": "valu", "achieved_terms_per_s": terms / (fast_ms * 1e-3),
                     "peak_terms_per_s": bound, "frac": terms / (fast_ms * 1e-3) / bound,
                     "issue_cycles_per_wave_per_64_terms": TILE_ISSUE_CYC[name],
                     "what": "pair-element terms (query × candidate × reduction element) per second of the "
                             "register tile against its VALU issue bound (DESIGN §5)"},
            "streamed": {"bytes_per_direction": streamed, "achieved_GBps": streamed / (fast_ms * 1e-3) / 1e9,
                         "what": "table + query bytes the tile reads from L2 / Infinity Cache per launch "
                                 "(64-query × 64-candidate tiles) over its launch time; HBM: the table once"},
            "mrr": float(np.mean(1.0 / np.concatenate([rh, rt]))),
        }
        del m
    torch.cuda.empty_cache()
    return out


def test_step_section(dev) -> dict:
    """What run.sh's --do_test waits on (run.py → KGEModel.test_step,
    model.py:346-429): filtered MRR / MR / HITS over a whole FB15k-size test
    split, end to end — the reference's list-of-tuples inputs, FilterIndex
    construction over train + valid + test, query blocks, both directions,
    reference-order refinement and the metric aggregation.  RotatE FB15k
    (E = 14951, R = 1345, d = 1000 -de, γ = 24, best_config.sh:3), synthetic
    483,142 train + 50,000 valid + 59,071 test triples (all_true = their
    union), 118,142 queries.  `host_s` = the wall time not covered by the
    ranking calls' device spans (kge_stage_timer 4/5: call start → ranks
    written), i.e. index build, per-block filter CSRs, launches, read-back and
    the metric sums."""
    import numpy as np
    from knowledgegraphembedding_amd import synth
    from knowledgegraphembedding_amd.filters import FilterIndex
    Ef, Rf = 14951, 1345

    def trip(seed, n):
        return np.stack([synth.randint(seed, (n,), Ef), synth.randint(seed + 1, (n,), Rf),
                         synth.randint(seed + 2, (n,), Ef)], 1).astype(np.int64)

    train, valid, test = trip(11, 483142), trip(21, 50000), trip(31, 59071)
    all_true = [tuple(x) for x in np.concatenate([train, valid, test]).tolist()]  # run.py's read_triple lists
    test_l = [tuple(x) for x in test.tolist()]
    torch.manual_seed(0)
    m = KGEModel("RotatE", Ef, Rf, 1000, 24.0, True, False).to(dev)
    args = Namespace(countries=False, nentity=Ef, nrelation=Rf, test_batch_size=16, cpu_num=10,
                     test_log_steps=10 ** 9, cuda=True)
    KGEModel.test_step(m, test_l[:64], all_true[:4096], args)  # warm-up: first-use state, not timed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    FilterIndex(all_true, Ef, Rf, device=dev)  # as test_step builds it (on the GPU)
    torch.cuda.synchronize()
    t_index = time.perf_counter() - t0
    lib = _lib.load()
    _lib.check(lib.kge_stage_timer(4, None, 0), "kge_stage_timer")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    met = KGEModel.test_step(m, test_l, all_true, args)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = _rank_timer_read(lib)
    lib.kge_stage_timer(0, None, 0)
    dev_s = float(st[0] + st[1] + st[2]) * 1e-3
    del m
    torch.cuda.empty_cache()
    return {"workload": "KGEModel.test_step, RotatE FB15k E=14951 R=1345 d=1000 -de, 59,071 test triples "
                        "(118,142 filtered queries), synthetic 592,213-triple filter graph, list-of-tuples inputs",
            "seconds": dt, "queries_per_s": 2 * len(test_l) / dt, "filter_index_build_s": t_index,
            "ranking_device_s": dev_s, "host_s": max(0.0, dt - dev_s), "host_share": max(0.0, dt - dev_s) / dt,
            "directions_timed": int(st[3]), "MRR": met["MRR"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=90.0,
                    help="seconds after which no further full CPU step starts (two are timed when the first ends sooner)")
    ap.add_argument("--no-stage-timer", action="store_true",
                    help="skip the per-stage HIP events (roofline then comes from the committed rocprof summary)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="fb15k")
    ap.add_argument("--no-rank", action="store_true", help="skip the config-3 ranking section (rank 0, 1 GPU)")
    ap.add_argument("--hidden-dim", type=int, default=None,
                    help="override the workload's hidden_dim (diagnostics; the headline is the workload's own)")
    ap.add_argument("--batch", type=int, default=None,
                    help="override the workload's batch size (diagnostics; the headline is the workload's own)")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 PMC summary (tools/pmc_traffic.py output) for roofline.traffic "
                         "(default: the committed profiles/pmc_traffic.json of this workload)")
    a = ap.parse_args()
    global E, R, D, B, NNEG
    wl = WORKLOADS[a.workload]
    E, R, D, B, NNEG = wl["E"], wl["R"], wl["D"], wl["B"], wl["NNEG"]
    if a.hidden_dim:
        D = a.hidden_dim
    if a.batch:
        B = a.batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("KGE_DIST_BACKEND", "nccl") != "nccl":
        local %= torch.cuda.device_count()  # rehearsal: several ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        # RCCL ("nccl") over xGMI; KGE_DIST_BACKEND=gloo rehearses N ranks on one GPU
        backend = os.environ.get("KGE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        group = dist.group.WORLD

    torch.manual_seed(0)
    model = KGEModel("RotatE", E, R, D, GAMMA, double_entity_embedding=True, double_relation_embedding=False)
    erange = model.embedding_range.item()
    cpu_state = (model.entity_embedding.detach().clone(), model.relation_embedding.detach().clone(), erange)
    model = model.to(dev)
    model.fuse_optimizer = os.environ.get("KGE_FUSED_ADAM", "1") == "1"
    model.keep_grads = os.environ.get("KGE_KEEP_GRADS", "1") == "1"
    args = Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=TEMP, uni_weight=False,
                     regularization=0.0, dp_group=group)
    part = None
    dp_mode = None if group is None else dp_exchange_mode(world)
    if group is not None and (wl["partition"] or dp_mode == "owner"):
        # config 5's row-partitioned table (KGE_PART_EXCHANGE, default the
        # owner-computes "factors"), or the data-parallel "owner" exchange
        from knowledgegraphembedding_amd.partition import EntityRowPartition
        exchange = os.environ.get("KGE_PART_EXCHANGE", "factors") if wl["partition"] else "factors"
        part = EntityRowPartition(model, group, exchange=exchange)
        params = part.parameters()
    else:
        params = [p for p in model.parameters() if p.requires_grad]
    opt = KGEAdam(params, lr=1e-4)
    sampler = os.environ.get("KGE_BENCH_SAMPLER", "staged")
    if sampler == "device":
        # end-to-end variant: every batch drawn inside the timed loop by the
        # device sampler (sampler.py) from a synthetic FB15k-sized train set
        from knowledgegraphembedding_amd.sampler import DeviceTrainIterator
        g = torch.Generator().manual_seed(4242)
        ntrain = 483142  # FB15k train.txt size
        train = torch.stack([torch.randint(0, E, (ntrain,), generator=g), torch.randint(0, R, (ntrain,), generator=g),
                             torch.randint(0, E, (ntrain,), generator=g)], 1).numpy()
        it = DeviceTrainIterator(train, E, R, NNEG, B, dev, seed=1000 + rank)
    else:
        it = DeviceBatches(dev, seed=1000 + rank)

    for _ in range(a.warmup):
        KGEModel.train_step(model, opt, it, args)
    torch.cuda.synchronize()

    lib = _lib.load()
    # per-stage HIP events on one step in TIMER_PERIOD (every step's events cost ~4 %)
    _lib.check(lib.kge_stage_timer(0 if a.no_stage_timer else 1, None, TIMER_PERIOD), "kge_stage_timer")
    if group is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        KGEModel.train_step(model, opt, it, args)
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    stage = (torch.zeros(7, dtype=torch.float32)).numpy()
    import ctypes
    _lib.check(lib.kge_stage_timer(2, stage.ctypes.data_as(ctypes.c_void_p), 7), "kge_stage_timer")
    lib.kge_stage_timer(0, None, 0)
    replica_check = None
    if group is not None:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        # after the timed steps (outside the clock): every exchange that keeps a
        # replicated table must leave it bit-identical on every rank
        from knowledgegraphembedding_amd.distributed import replicas_disagree, table_fingerprint
        fp = part.replica_checksums() if part is not None else \
            table_fingerprint(model.entity_embedding, model.relation_embedding)
        bad = replicas_disagree(fp, group)
        replica_check = {"tables": "relation only (query shipping keeps no replica)" if fp.numel() == 1 else
                         "entity replica + relation", "ranks_differing_from_rank0": bad, "agree": not bad}

    calls = max(1.0, float(stage[6]))
    here = os.path.dirname(os.path.abspath(__file__))
    row_ms = float(stage[1]) / calls
    ent_ms = float(stage[4]) / calls
    # the factor / owner exchanges run the row pass in pieces (each timed call
    # is one piece) and the entity pass outside the timed call: the entity and
    # whole-step rooflines are single-process figures only
    exchanged = group is not None and (part is not None or dp_mode in ("factors", "owner"))
    row_rows = B
    if exchanged:
        from knowledgegraphembedding_amd.distributed import fx_pieces
        row_rows = fx_pieces(B)[0][1]
        ent_ms = 0.0
    row_bytes = algorithmic_row_bytes(row_rows, NNEG, 2 * D, D)
    ent_bytes = algorithmic_entity_bytes(E, R, B, NNEG, 2 * D, D)
    achieved = row_bytes / (row_ms * 1e-3) / 1e9 if row_ms > 0 else None
    ent_achieved = ent_bytes / (ent_ms * 1e-3) / 1e9 if ent_ms > 0 else None
    row_traffic = ent_traffic = None
    # the committed PMC summaries and pattern ceilings were measured on the
    # workload's own shape (d = 1000): not applicable to a --hidden-dim run
    own_shape = (not a.hidden_dim or a.hidden_dim == wl["D"]) and (not a.batch or a.batch == wl["B"])
    if a.workload == "fb15k" and not exchanged and own_shape:  # PMC summaries of this workload (tools/profile.sh + tools/pmc_traffic.py)
        row_traffic = _pmc_bytes(a.traffic_json or os.path.join(here, "profiles", "pmc_traffic.json"))
        ent_traffic = _pmc_bytes(os.path.join(here, "profiles", "pmc_traffic_entity.json"))

    ceiling = None  # k_row's access pattern alone (tools/dbg/gather_ceiling.hip), measured on MI355X
    cj = os.path.join(here, "profiles", "r01", "gather_ceiling.jsonl")
    if a.workload == "fb15k" and own_shape and os.path.exists(cj) and achieved:
        with open(cj) as f:
            c0 = json.loads(f.readline())
        ceiling = {"GBps": c0["GBps"], "frac": achieved / c0["GBps"], "source": "profiles/r01/gather_ceiling.jsonl",
                   "what": "same grid and buffer loads over the same table, no arithmetic"}

    ent_ceiling = None  # the entity pass's HBM stream alone (tools/dbg/stream_ceiling.hip), measured on MI355X
    sj = os.path.join(here, "profiles", "entity_stream_ceiling.jsonl")
    if a.workload == "fb15k" and own_shape and os.path.exists(sj) and ent_achieved:
        with open(sj) as f:
            best = max((json.loads(line) for line in f if line.strip()), key=lambda r: r["GBps"])
        ent_ceiling = {"GBps": best["GBps"], "frac": ent_achieved / best["GBps"],
                       "source": "profiles/entity_stream_ceiling.jsonl",
                       "what": "the dense Adam stream alone (read p/m/v, write p/m/v/grad, 837 MB, coalesced, "
                               "non-temporal), without the entity pass's 2.1 GB of q-slice gathers from L2"}

    value = a.steps * B * (NNEG + 1) * world / dt
    # what the process group itself saw (the driver's multi-GPU record can
    # check that RCCL ran over N ranks): backend, its world size, RCCL version
    dist_info = {"backend": None, "world_size": 1, "rccl_version": None}
    if group is not None:
        dist_info["backend"] = str(dist.get_backend(group))
        dist_info["world_size"] = dist.get_world_size(group)
        dist_info["replica_check"] = replica_check
    try:
        dist_info["rccl_version"] = ".".join(str(x) for x in torch.cuda.nccl.version())
    except Exception:  # noqa: BLE001 — reported as unknown, never fatal
        pass
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "triples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (uniform ids, U(-range,range) tables), batches pre-staged in HBM",
        "variant": {"fused_adam": model.fuse_optimizer, "keep_grads": model.keep_grads, "batches": sampler,
                    "dp_exchange": dp_mode,
                    "partition_exchange": None if part is None else part.exchange},
        "config": {"workload": wl["name"],
                   "entities": E, "relations": R, "hidden_dim": D, "batch_per_gpu": B, "global_batch": B * world,
                   "negatives": NNEG, "adversarial_temperature": TEMP, "gamma": GAMMA,
                   "parallelism": (f"rowpart{world}" if wl["partition"] and part is not None else f"dp{world}")},
        "dist": dist_info,
        "stage_timed_steps": int(stage[6]),
        # HIP-event stage times of one step in TIMER_PERIOD, on the launching
        # stream; the CSR runs on a side stream beside the row pass, so these
        # are not a decomposition of ms_per_step
        "stage_ms": {"row_pass": row_ms, "csr_join": float(stage[3]) / calls, "entity_pass": ent_ms,
                     "relation_join_finalize": float(stage[5]) / calls},
        "roofline": {"bound": "hbm", "kernel": "k_row (q build + negative scoring + self-adversarial loss + q-side backward + positive epilogue)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS if achieved else None,
                     "traffic": row_traffic, "algorithmic_bytes_per_launch": row_bytes,
                     "avg_launch_ms": row_ms, "pattern_ceiling": ceiling},
        "roofline_entity": {"bound": "hbm", "kernel": "k_entity_sl (entity-major gradient + fused Adam; loss finalisation and relation rows in leading blocks)",
                            "achieved": ent_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": ent_achieved / HBM_PEAK_GBS if ent_achieved else None, "traffic": ent_traffic,
                            "algorithmic_bytes_per_launch": ent_bytes, "avg_launch_ms": ent_ms,
                            "pattern_ceiling": ent_ceiling},
        "step_roofline": None if exchanged else step_roofline(dt / a.steps, row_bytes, ent_bytes, row_traffic,
                                                                 ent_traffic),
    }
    if exchanged:
        out["roofline"]["rows_per_launch"] = row_rows
        out["roofline_entity"] = None
    if a.workload != "fb15k":
        out["metric"] = f"scored (pos+neg) triples/sec, RotatE {a.workload} d={D} b={B} n={NNEG}"
    fr = [out["roofline"]["frac"]]
    if not exchanged:
        fr += [out["roofline_entity"]["frac"], out["step_roofline"]["frac"], out["step_roofline"].get("frac_traffic")]
    fr = [x for x in fr if x is not None]
    if any(f > 1.0 for f in fr):
        print(f"bench.py: a roofline fraction exceeds 1 ({fr}); the byte model is wrong", file=sys.stderr)
    if rank == 0 and world == 1 and not a.no_rank and a.workload == "fb15k":
        out["ranking"] = rank_section(dev)
        out["test_step"] = test_step_section(dev)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        # the full batch at config 2's n = 256; config 5's n = 1024 at a quarter of the rows (one full
        # step there would hold ~40 GB of temporaries and take minutes)
        out["cpu_baseline"] = cpu_baseline(cpu_state, budget_s=a.cpu_budget, b=B if NNEG <= 256 else B // 4)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if group is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
