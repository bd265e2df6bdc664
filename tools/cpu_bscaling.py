"""Per-triple rate of the CPU baseline (oracle train step) against the batch
size b, so bench.py's bounded b=32 sample can stand for the b=1024 workload.

    python tools/cpu_bscaling.py > profiles/r02/cpu_baseline_bscaling.json
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import kge_oracle as O  # noqa: E402

E, R, D, NNEG = 14951, 1345, 1000, 256


def rate(b, steps):
    g = torch.Generator().manual_seed(7)
    erange = (24.0 + 2.0) / D
    ent = (torch.rand(E, 2 * D, generator=g) * 2 - 1) * erange
    rel = (torch.rand(R, D, generator=g) * 2 - 1) * erange
    pos = torch.stack([torch.randint(0, E, (b,), generator=g), torch.randint(0, R, (b,), generator=g),
                       torch.randint(0, E, (b,), generator=g)], 1)
    neg = torch.randint(0, E, (b, NNEG), generator=g)
    w = torch.rand(b, generator=g) * 0.3 + 0.1
    params = [ent.requires_grad_(True), rel.requires_grad_(True)]
    opt = torch.optim.Adam(params, lr=1e-4)

    def step(mode):
        _, ge, gr, _ = O.train_grads("RotatE", params[0].detach(), params[1].detach(), None, pos, neg, w, mode,
                                     adversarial=True, temperature=1.0, uni_weight=False, regularization=0.0,
                                     gamma=24.0, erange=erange)
        opt.zero_grad()
        params[0].grad, params[1].grad = ge, gr
        opt.step()

    step("tail-batch")
    t0 = time.perf_counter()
    for k in range(steps):
        step("head-batch" if k % 2 else "tail-batch")
    dt = time.perf_counter() - t0
    return {"b": b, "steps": steps, "seconds": dt, "triples_per_s": steps * b * (NNEG + 1) / dt}


if __name__ == "__main__":
    cores = len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    out = {"cores": cores, "torch": torch.__version__, "cpu_capability": torch.backends.cpu.get_cpu_capability(),
           "runs": [rate(32, 8), rate(1024, 2)]}
    print(json.dumps(out))
