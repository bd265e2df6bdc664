"""Is k_row reading the 120 MB entity table from the Infinity Cache or from HBM?
Time the row phase alone, back to back (table hot, nothing else streaming),
against the row phase of full fused train steps (the entity pass streams
~840 MB of table/Adam/gradient between two row passes)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from argparse import Namespace
from knowledgegraphembedding_amd import KGEModel, KGEAdam, synth, ops, _lib
dev = torch.device("cuda", 0)
E, R, d, B, n = 14951, 1345, 1000, 1024, 256
torch.manual_seed(0)
m = KGEModel("RotatE", E, R, d, 24.0, True, False).to(dev)
opt = KGEAdam([p for p in m.parameters() if p.requires_grad], lr=1e-4)
pos, neg, w = synth.kge_batch(5, B, n, E, R)
P, N, W = (torch.from_numpy(x).to(dev) for x in (pos, neg, w))
args = Namespace(negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False, regularization=0.0)
ge, gr, gm, losses = m._grad_buffers()
desc = m.desc()
def rows():
    ops.train_step_grads(desc, "tail-batch", P, N, W, dev, adversarial=True, temperature=1.0, uni_weight=False,
                         regularization=0.0, grad_entity=ge, grad_relation=gr, grad_modulus=None, losses=losses,
                         phases=_lib.PHASE_ROWS)
def full():
    m.compute_train_grads(P, N, W, "tail-batch", args, optimizer=opt)
    opt.step()
def timed(fn, k=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(k): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / k
r_only = timed(rows)
def alt():
    full(); rows()
f_only = timed(full)
both = timed(alt)
# flush the Infinity Cache with a 1 GB stream between row passes
junk = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device=dev)
def cold():
    junk.add_(1.0); rows()
junk_t = timed(lambda: junk.add_(1.0))
cold_t = timed(cold) - junk_t
print(json.dumps({"rows_phase_hot_ms": r_only, "full_step_ms": f_only, "rows_after_full_ms": both - f_only,
                  "rows_after_1GB_flush_ms": cold_t, "flush_ms": junk_t}))
