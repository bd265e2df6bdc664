#!/usr/bin/env python3
"""Row pass (k_row alone, kge_train_rows_slice) at B = 512 … 4096 rows of the
RotatE FB15k shape (n = 256): does a second round of blocks (B > 1024: more
blocks than fit the chip at once) amortise the blocks' serial prologue /
epilogue phases?  Prints ms per launch and per 1024 rows."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knowledgegraphembedding_amd import KGEModel, ops, synth  # noqa: E402

E, R, D, N = 14951, 1345, 1000, 256


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = KGEModel("RotatE", E, R, D, 24.0, True, False).to(dev)
    desc = m.desc()
    out = {}
    for B in (512, 1024, 1536, 2048, 3072, 4096):
        pos, neg, w = (torch.from_numpy(x).to(dev) for x in synth.kge_batch(3, B, N, E, R))
        wsum = torch.empty(1, device=dev)
        ops.weight_sum(w, wsum)
        g, dq, st = torch.empty(B, N, device=dev), torch.empty(B, 2 * D, device=dev), torch.empty(B, 4, device=dev)

        def run():
            ops.train_rows_slice(desc, "tail-batch", pos, neg, w, wsum, dev, adversarial=True, temperature=1.0,
                                 uni_weight=False, uni_batch=B, g_out=g, dq_out=dq, stats_out=st)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 50
        out[B] = {"ms": round(ms, 4), "ms_per_1024_rows": round(ms * 1024 / B, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
