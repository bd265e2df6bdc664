"""HBM rate of the standalone dense Adam (kge_adam_step) and of a plain float4
copy on tables of the FB15k / YAGO3-10 RotatE shapes — the stream the fused
entity pass carries, without its q gathers.  Prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from knowledgegraphembedding_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


for name, rows in (("fb15k", 14951), ("yago3-10", 123182)):
    n = rows * 2000
    p, g, m, v = (torch.rand(n, device=dev) for _ in range(4))
    for var in ("0", "1", "2", "3", "0"):  # KGE_ADAM_VARIANT (kge_common.hip k_adam)
        os.environ["KGE_ADAM_VARIANT"] = var
        t = timed(lambda: ops.adam_step(p, g, m, v, step=3, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8))
        print(json.dumps({"case": name, "kernel": "kge_adam_step", "variant": var, "elems": n, "bytes": 28 * n,
                          "ms": t * 1e3, "GBps": 28 * n / t / 1e9}), flush=True)
    dst = torch.empty_like(p)
    t = timed(lambda: dst.copy_(p))
    print(json.dumps({"case": name, "kernel": "torch copy_", "bytes": 8 * n, "ms": t * 1e3,
                      "GBps": 8 * n / t / 1e9}), flush=True)
    del p, g, m, v, dst
