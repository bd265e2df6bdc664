"""Host-side cost of one KGEModel.train_step (tiny model: the GPU work is
negligible, so the loop rate is the Python/ctypes enqueue rate)."""
import os
import sys
import time
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from knowledgegraphembedding_amd import KGEAdam, KGEModel, synth  # noqa: E402

dev = torch.device("cuda", 0)
m = KGEModel("RotatE", 100, 5, 8, 12.0, True, False).to(dev)
opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)
args = Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                 regularization=0.0, dp_group=None)
pos, neg, w = (torch.from_numpy(x).to(dev) for x in synth.kge_batch(1, 8, 4, 100, 5))
batches = [(pos, neg, w, "tail-batch"), (pos, neg, w, "head-batch")]


class It:
    k = 0

    def __next__(self):
        self.k += 1
        return batches[self.k % 2]


it = It()
for _ in range(20):
    KGEModel.train_step(m, opt, it, args)
torch.cuda.synchronize()
t0 = time.perf_counter()
N = 500
for _ in range(N):
    KGEModel.train_step(m, opt, it, args)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print({"host_us_per_step": (t1 - t0) / N * 1e6, "with_drain_us_per_step": (t2 - t0) / N * 1e6})
