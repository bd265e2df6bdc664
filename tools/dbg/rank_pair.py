"""GPU diagnostic for single RotatE rank disagreements at the FB15k fixture:
for the given head-batch queries, the oracle's reference-order scores of the
true entity and its nearest competitors (CPU, the committed trig bits) against
(a) the device's ranks (auto / scan, listed counts) and (b) a mini table made
of just those rows, so the refinement alone decides every pair.

    python tools/dbg/rank_pair.py 50 81
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from knowledgegraphembedding_amd import KGEModel, synth  # noqa: E402
from knowledgegraphembedding_amd.filters import FilterIndex  # noqa: E402
from oracle import kge_oracle as O  # noqa: E402
from test_rank_parity_gpu import reference_trig  # noqa: E402

DEV = torch.device("cuda", 0)
E, R, d, gamma, seed = 14951, 1345, 1000, 24.0, 62
g = np.load(ROOT / "tests/golden/ranks_full.npz")
m = KGEModel("RotatE", E, R, d, gamma, True, False)
rng = m.embedding_range.item()
ent, rel = synth.kge_tables(seed, E, R, 2 * d, d, rng)
with torch.no_grad():
    m.entity_embedding.copy_(torch.from_numpy(ent))
    m.relation_embedding.copy_(torch.from_numpy(rel))
m = m.to(DEV)
trig, phase, ids = reference_trig("fb15k", rel, rng)
cos_t, sin_t = trig[:, 0].numpy(), trig[:, 1].numpy()
queries, filters = g["fb15k/queries"], g["fb15k/filters"]
index = FilterIndex([tuple(x) for x in filters.tolist()], E, R)
mode = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2].endswith("batch") else "head-batch"
qids = [int(a) for a in sys.argv[1:] if a.isdigit()]
for qi in qids:
    q = queries[qi:qi + 1]
    for path in ("auto", "scan"):
        r_, t_, l_ = m.rank_queries(q, index, mode, path=path, listed=True, relation_trig=trig)
        print(f"q{qi} {path}: rank {r_[0]} ties {t_[0]} listed {l_[0]} | fixture rank "
              f"{g[f'fb15k/RotatE/{mode}/rank'][qi]} ties {g[f'fb15k/RotatE/{mode}/ties'][qi]}")
    h, r, t = (int(x) for x in q[0])
    tid = h if mode == "head-batch" else t
    # reference-order scores of all candidates (oracle, committed trig bits for relation r)
    P = torch.from_numpy(q)
    N = torch.arange(E).view(1, -1)
    cs_row, sn_row = cos_t[r], sin_t[r]

    def cosf(a, _c=cs_row):
        return np.broadcast_to(_c, np.shape(a)).astype(np.float32)

    def sinf(a, _s=sn_row):
        return np.broadcast_to(_s, np.shape(a)).astype(np.float32)
    s = O.ref_order_scores("RotatE", ent, rel, None, (P, N), mode, torch.Tensor([gamma]).item(), rng,
                           trig=(cosf, sinf))[0]
    off, fid = index.filter_csr(q, mode)
    excl = set(fid[off[0]:off[1]].tolist()) | {tid}
    comp = np.array([e not in excl for e in range(E)])
    gt = int((comp & (s > s[tid])).sum())
    print(f"  oracle (committed trig): s_true {s[tid]!r} greater {gt} -> rank {gt + 1}")
    gap = np.where(comp, s.astype(np.float64) - s[tid], np.inf)
    near = np.argsort(np.abs(gap))[:12]
    print("  nearest competitors", near.tolist(), gap[near].tolist())
    # the device's fast scores of those rows (kge_score: the training-path reduction order)
    with torch.no_grad():
        fs = m((P.to(DEV), torch.from_numpy(np.concatenate([[tid], near])).view(1, -1).to(DEV)), mode).cpu().numpy()[0]
    print("  device fast scores - oracle:", (fs - s[np.concatenate([[tid], near])]).tolist())
    # mini table: true row, anchor row, the 12 competitors; the anchor filtered
    rows = [tid, t if mode == "head-batch" else h] + near.tolist()
    mini = KGEModel("RotatE", len(rows), R, d, gamma, True, False)
    with torch.no_grad():
        mini.entity_embedding.copy_(torch.from_numpy(ent[rows]))
        mini.relation_embedding.copy_(torch.from_numpy(rel))
    mini = mini.to(DEV)
    mq = np.array([[0, r, 1]] if mode == "head-batch" else [[1, r, 0]], dtype=np.int64)
    mfilt = [(1, r, 1)] if mode == "head-batch" else [(1, r, 1)]
    mr, mt, ml = mini.rank_queries(mq, mfilt, mode, listed=True, relation_trig=trig)
    print(f"  mini table: rank {mr[0]} ties {mt[0]} listed {ml[0]}; oracle: {1 + int((gap[near] > 0).sum())}")
