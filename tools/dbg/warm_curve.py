"""Per-block step time over the first seconds of a bench.py-shaped run
(RotatE FB15k, b=1024, n=256): how long until the step time settles."""
import os
import sys
import time
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from knowledgegraphembedding_amd import KGEAdam, KGEModel  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    m = KGEModel("RotatE", bench.E, bench.R, bench.D, bench.GAMMA, True, False).to(dev)
    opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-4)
    args = Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0, dp_group=None)
    it = bench.DeviceBatches(dev, seed=1000)
    t_start = time.perf_counter()
    nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    reset_at = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # zero the Adam moments in place at this block
    for blk in range(nblk):
        if blk == reset_at:
            for st in opt.state.values():
                for v in st.values():
                    if torch.is_tensor(v) and v.is_floating_point() and v.numel() > 1:
                        v.zero_()
            print("-- Adam moments zeroed in place", flush=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            KGEModel.train_step(m, opt, it, args)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if blk < 10 or blk % 10 == 0 or (reset_at >= 0 and reset_at <= blk < reset_at + 6):
            print(f"block {blk:4d} t={t0 - t_start:7.3f}s  {dt / 20 * 1e3:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
