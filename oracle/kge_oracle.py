"""CPU oracle for the KGE hot path — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker (or the timed CPU baseline) —
never as a compute path of knowledgegraphembedding_amd.

It restates the reference's algorithm (kahrabian/KnowledgeGraphEmbedding,
codes/model.py + codes/dataloader.py) as the same ATen op chain on CPU fp32
tensors, so on one machine it reproduces the reference's floats; integer
work (filters, ranks) is numpy.  Pinning: tests/test_oracle_golden.py checks
every function below against tests/golden/*.npz, generated in the build
container by importing the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

PI = 3.14159265358979323846        # model.py:202
PI_PROTATE = 3.14159262358979323846  # model.py:232 (typo kept: it is the reference's behaviour)


# --------------------------------------------------------------- gather
def gather(ent: torch.Tensor, rel: torch.Tensor, sample, mode: str):
    """Row gathers of KGEModel.forward (model.py:83-149) → (head, relation, tail)."""
    sel = lambda table, idx: torch.index_select(table, 0, idx)  # noqa: E731
    if mode == 'single':
        s = sample
        return sel(ent, s[:, 0]).unsqueeze(1), sel(rel, s[:, 1]).unsqueeze(1), sel(ent, s[:, 2]).unsqueeze(1)
    if mode == 'head-batch':
        pos, neg = sample
        b, n = neg.shape
        return (sel(ent, neg.reshape(-1)).view(b, n, -1), sel(rel, pos[:, 1]).unsqueeze(1),
                sel(ent, pos[:, 2]).unsqueeze(1))
    if mode == 'tail-batch':
        pos, neg = sample
        b, n = neg.shape
        return (sel(ent, pos[:, 0]).unsqueeze(1), sel(rel, pos[:, 1]).unsqueeze(1),
                sel(ent, neg.reshape(-1)).view(b, n, -1))
    raise ValueError('mode %s not supported' % mode)


# --------------------------------------------------------------- scores
def _transe(h, r, t, mode, gamma, erange, modulus):  # model.py:166-173
    x = h + (r - t) if mode == 'head-batch' else (h + r) - t
    return gamma - torch.norm(x, p=1, dim=2)


def _distmult(h, r, t, mode, gamma, erange, modulus):  # model.py:175-182
    x = h * (r * t) if mode == 'head-batch' else (h * r) * t
    return x.sum(dim=2)


def _complex(h, r, t, mode, gamma, erange, modulus):  # model.py:184-199
    hr, hi = torch.chunk(h, 2, dim=2)
    rr, ri = torch.chunk(r, 2, dim=2)
    tr, ti = torch.chunk(t, 2, dim=2)
    if mode == 'head-batch':
        a = rr * tr + ri * ti
        b = rr * ti - ri * tr
        x = hr * a + hi * b
    else:
        a = hr * rr - hi * ri
        b = hr * ri + hi * rr
        x = a * tr + b * ti
    return x.sum(dim=2)


def _rotate(h, r, t, mode, gamma, erange, modulus):  # model.py:201-229
    hr, hi = torch.chunk(h, 2, dim=2)
    tr, ti = torch.chunk(t, 2, dim=2)
    phase = r / (erange / PI)
    c, s = torch.cos(phase), torch.sin(phase)
    if mode == 'head-batch':
        a = (c * tr + s * ti) - hr
        b = (c * ti - s * tr) - hi
    else:
        a = (hr * c - hi * s) - tr
        b = (hr * s + hi * c) - ti
    mod = torch.stack([a, b], dim=0).norm(dim=0)
    return gamma - mod.sum(dim=2)


def _protate(h, r, t, mode, gamma, erange, modulus):  # model.py:231-249
    k = erange / PI_PROTATE
    ph, pr, pt = h / k, r / k, t / k
    x = ph + (pr - pt) if mode == 'head-batch' else (ph + pr) - pt
    return gamma - torch.abs(torch.sin(x)).sum(dim=2) * modulus


SCORE_FNS = {'TransE': _transe, 'DistMult': _distmult, 'ComplEx': _complex, 'RotatE': _rotate,
             'pRotatE': _protate}


def forward(name, ent, rel, modulus, sample, mode, gamma: float, erange: float):
    """KGEModel.forward (model.py:72-164): [B, n] scores."""
    h, r, t = gather(ent, rel, sample, mode)
    return SCORE_FNS[name](h, r, t, mode, gamma, erange, modulus)


# --------------------------------------------------------------- training
def train_grads(name, ent, rel, modulus, pos, neg, w, mode, *, adversarial: bool, temperature: float,
                uni_weight: bool, regularization: float, gamma: float, erange: float):
    """train_step up to loss.backward() (model.py:268-301).

    Returns ({'positive_sample_loss', 'negative_sample_loss', 'loss'[, 'regularization']},
             grad_entity, grad_relation, grad_modulus-or-None) — dense gradients.
    """
    E = ent.detach().clone().requires_grad_(True)
    R = rel.detach().clone().requires_grad_(True)
    Mo = modulus.detach().clone().requires_grad_(True) if modulus is not None else None
    neg_s = forward(name, E, R, Mo, (pos, neg), mode, gamma, erange)
    if adversarial:
        wts = F.softmax(neg_s * temperature, dim=1).detach()
        neg_term = (wts * F.logsigmoid(-neg_s)).sum(dim=1)
    else:
        neg_term = F.logsigmoid(-neg_s).mean(dim=1)
    pos_term = F.logsigmoid(forward(name, E, R, Mo, pos, 'single', gamma, erange)).squeeze(dim=1)
    if uni_weight:
        p_loss, n_loss = -pos_term.mean(), -neg_term.mean()
    else:
        p_loss = -(w * pos_term).sum() / w.sum()
        n_loss = -(w * neg_term).sum() / w.sum()
    loss = (p_loss + n_loss) / 2
    out = {}
    if regularization != 0.0:
        reg = regularization * (E.norm(p=3) ** 3 + R.norm(p=3).norm(p=3) ** 3)
        loss = loss + reg
        out['regularization'] = reg.item()
    loss.backward()
    out.update({'positive_sample_loss': p_loss.item(), 'negative_sample_loss': n_loss.item(), 'loss': loss.item()})
    return out, E.grad, R.grad, (Mo.grad if Mo is not None else None)


def adam_steps(params, grads_per_step, lr: float):
    """torch.optim.Adam(params, lr) stepped once per entry of grads_per_step
    (run.py:266-269, model.py:303); returns (params, state tensors)."""
    ps = [p.detach().clone().requires_grad_(True) for p in params]
    opt = torch.optim.Adam(ps, lr=lr)
    for grads in grads_per_step:
        opt.zero_grad()
        for p, g in zip(ps, grads):
            p.grad = g.clone()
        opt.step()
    states = [(opt.state[p]['exp_avg'].clone(), opt.state[p]['exp_avg_sq'].clone()) for p in ps]
    return [p.detach() for p in ps], states


# --------------------------------------------------------------- ranking
def filtered_candidates(triple, all_true_set, nentity: int, mode: str):
    """TestDataset.__getitem__ (dataloader.py:134-154): (negative_sample [E], filter_bias [E])."""
    h, r, t = triple
    cand = np.arange(nentity, dtype=np.int64)
    bias = np.zeros(nentity, dtype=np.float32)
    for e in range(nentity):
        key = (e, r, t) if mode == 'head-batch' else (h, r, e)
        if key in all_true_set:
            cand[e] = h if mode == 'head-batch' else t
            bias[e] = -1.0
    true_id = h if mode == 'head-batch' else t
    cand[true_id] = true_id
    bias[true_id] = 0.0
    return cand, bias


def filtered_ranks(name, ent, rel, modulus, triples, all_true_triples, mode, gamma: float, erange: float):
    """test_step's rank per query (model.py:383-418), plus diagnostics.

    Returns dict of numpy arrays:
      rank_argsort  1 + position of the true entity in argsort(desc) — the reference's number
      rank_count    1 + #{unfiltered e != true : s_e > s_true} (strict count, tie-free definition)
      ties          #{unfiltered e != true : s_e == s_true}
      margin64      min over unfiltered e != true of |s_e - s_true| recomputed in float64
      score64       s_true in float64
    """
    all_true_set = set(map(tuple, np.asarray(all_true_triples).tolist()))
    E = ent.shape[0]
    out = {k: [] for k in ('rank_argsort', 'rank_count', 'ties', 'margin64', 'score64')}
    for tr in np.asarray(triples, dtype=np.int64).tolist():
        cand, bias = filtered_candidates(tr, all_true_set, E, mode)
        pos = torch.tensor([tr], dtype=torch.int64)
        negt = torch.from_numpy(cand).view(1, -1)
        s = forward(name, ent, rel, modulus, (pos, negt), mode, gamma, erange)
        s = s + torch.from_numpy(bias).view(1, -1)
        arg = torch.argsort(s, dim=1, descending=True)
        true_id = tr[0] if mode == 'head-batch' else tr[2]
        out['rank_argsort'].append(1 + int((arg[0] == true_id).nonzero().item()))
        s0 = s[0].numpy()
        keep = (bias == 0) & (np.arange(E) != true_id)
        st = s0[true_id]
        out['rank_count'].append(1 + int((s0[keep] > st).sum()))
        out['ties'].append(int((s0[keep] == st).sum()))
        s64 = forward(name, ent.double(), rel.double(), None if modulus is None else modulus.double(), (pos, negt),
                      mode, gamma, erange)[0].numpy()
        out['margin64'].append(float(np.min(np.abs(s64[keep] - s64[true_id]))) if keep.any() else np.inf)
        out['score64'].append(float(s64[true_id]))
    return {k: np.asarray(v) for k, v in out.items()}


def metrics_from_ranks(ranks):
    """MRR / MR / HITS@k averaged the way model.py:412-427 averages its log dicts."""
    logs = [{'MRR': 1.0 / r, 'MR': float(r), 'HITS@1': 1.0 if r <= 1 else 0.0, 'HITS@3': 1.0 if r <= 3 else 0.0,
             'HITS@10': 1.0 if r <= 10 else 0.0} for r in np.asarray(ranks).tolist()]
    return {k: sum(l[k] for l in logs) / len(logs) for k in logs[0]}


# --------------------------------------------------------------- sampler
# The device sampler (kge_sample_negatives) restated.  Semantics follow
# TrainDataset.__getitem__ (dataloader.py:34-61): uniform draws over
# [0, nentity), true heads of (r, t) / true tails of (h, r) rejected, the
# first n survivors kept in draw order; weights dataloader.py:40-42.  The
# random stream is the build's (splitmix64 per batch row), not numpy's.
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64_np(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over='ignore'):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _mulhi_small(x, E: int):
    """floor(x * E / 2^64) for uint64 x and E < 2^31, exactly."""
    e = np.uint64(E)
    lo = x & np.uint64(0xFFFFFFFF)
    hi = x >> np.uint64(32)
    with np.errstate(over='ignore'):
        return ((hi * e + ((lo * e) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


def true_lists(triples, mode: str):
    """{key: sorted true members} — get_true_head_and_tail (dataloader.py:77-85) keyed per mode."""
    out = {}
    for h, r, t in np.asarray(triples).tolist():
        if mode == 'head-batch':
            out.setdefault((r, t), set()).add(h)
        else:
            out.setdefault((h, r), set()).add(t)
    return {k: np.array(sorted(v), dtype=np.int64) for k, v in out.items()}


def subsampling_weights(triples):
    """sqrt(1 / (count(h,r) + count(t,-r-1))) per triple, counts from 4 (dataloader.py:40-42, :68-75)."""
    cnt = {}
    for h, r, t in np.asarray(triples).tolist():
        cnt[(h, r)] = cnt.get((h, r), 3) + 1
        cnt[(t, -r - 1)] = cnt.get((t, -r - 1), 3) + 1
    return np.array([torch.sqrt(1 / torch.Tensor([cnt[(h, r)] + cnt[(t, -r - 1)]])).item()
                     for h, r, t in np.asarray(triples).tolist()], dtype=np.float32)


def sample_negatives(triples, batch, nentity: int, n: int, mode: str, key: int, max_draws: int):
    """(pos [B,3], neg [B,n], ok [B]) for the device sampler's stream; ok=False where max_draws ran out."""
    triples = np.asarray(triples, dtype=np.int64)
    lists = true_lists(triples, mode)
    B = len(batch)
    pos = triples[np.asarray(batch)]
    neg = np.zeros((B, n), dtype=np.int64)
    ok = np.ones(B, dtype=bool)
    lanes = np.arange(64, dtype=np.uint64)
    for i in range(B):
        h, r, t = pos[i].tolist()
        tl = lists[(r, t)] if mode == 'head-batch' else lists[(h, r)]
        with np.errstate(over='ignore'):
            krow = _mix64_np(np.uint64(key) ^ (np.uint64(i) * np.uint64(0xD1B54A32D192ED03)))
        got = []
        d = 0
        while len(got) < n:
            if d >= max_draws:
                ok[i] = False
                break
            with np.errstate(over='ignore'):
                x = _mix64_np(krow + (np.uint64(d) + lanes) * np.uint64(0x9E3779B97F4A7C15))
            e = _mulhi_small(x, nentity)
            got.extend(e[~np.isin(e, tl)].tolist())
            d += 64
        take = got[:n]
        neg[i, :len(take)] = take
    return pos, neg, ok


# ------------------------------------- reference operation order (numpy)
# The sequence of fp32 operations the reference's CPU forward performs,
# written out element by element — what the HIP ranking refinement
# (csrc/kge_rank_ref.h) reproduces.  Pinned by tests/test_oracle_golden.py
# against the golden scores the reference itself produced (bit for bit).
U32 = np.float32


def aten_sum_lastdim(x: np.ndarray) -> np.ndarray:
    """ATen CPU `sum(dim=-1)` of a contiguous fp32 array, in its own order
    (SumKernel.cpp vectorized_inner_sum → row_sum → multi_row_sum: 8-float
    vectors, 4 interleaved accumulators, a 4-level cascade of 2^lp rows, tail
    vectors into accumulator 0, then the scalar tail from 0 and the 8 vector
    lanes in order).  Requires the last dim >= 8."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    d = x.shape[-1]
    nvec = d // 8
    vecs = np.moveaxis(x[..., :nvec * 8].reshape(x.shape[:-1] + (nvec, 8)), -2, 0)  # [nvec, ..., 8]
    size = nvec // 4
    rows = vecs[:size * 4].reshape((size, 4) + vecs.shape[1:])
    lp = max(4, (int(np.ceil(np.log2(size))) if size > 1 else 0) // 4)
    step, mask = 1 << lp, (1 << lp) - 1
    acc = np.zeros((4, 4) + vecs.shape[1:], np.float32)  # [level, column, ..., 8]
    i = 0
    while i + step <= size:
        for _ in range(step):
            acc[0] = acc[0] + rows[i]
            i += 1
        for lv in range(1, 4):
            acc[lv] = acc[lv] + acc[lv - 1]
            acc[lv - 1] = 0
            if i & (mask << (lv * lp)):
                break
    while i < size:
        acc[0] = acc[0] + rows[i]
        i += 1
    cols = acc[0]
    for lv in range(1, 4):
        cols = cols + acc[lv]
    ps0 = cols[0]
    for v in range(size * 4, nvec):
        ps0 = ps0 + vecs[v]
    vacc = ps0
    for k in range(1, 4):
        vacc = vacc + cols[k]
    fin = np.zeros(x.shape[:-1], np.float32)
    for k in range(nvec * 8, d):
        fin = fin + x[..., k]
    for p in range(8):
        fin = fin + vacc[..., p]
    return fin


def ref_order_scores(name: str, ent: np.ndarray, rel: np.ndarray, modulus, sample, mode: str, gamma: float,
                     erange: float, trig=None) -> np.ndarray:
    """Scores of KGEModel.forward (model.py:72-249) as explicit fp32 element
    operations + aten_sum_lastdim / a sequential L1 sum.  `trig` (cos, sin)
    evaluates the transcendentals; default: torch's CPU ones (the reference's)."""
    cos, sin = trig or ((lambda a: torch.cos(torch.from_numpy(np.array(a, np.float32))).numpy()),
                        (lambda a: torch.sin(torch.from_numpy(np.array(a, np.float32))).numpy()))
    h, r, t = (a.numpy() for a in gather(torch.from_numpy(ent), torch.from_numpy(rel), sample, mode))
    head = mode == 'head-batch'
    g = U32(gamma)
    if name == 'TransE':
        x = np.abs(h + (r - t) if head else (h + r) - t)
        acc = np.zeros(x.shape[:-1], np.float32)
        for k in range(x.shape[-1]):
            acc = acc + x[..., k]
        return g - acc
    if name == 'DistMult':
        return aten_sum_lastdim(h * (r * t) if head else (h * r) * t)
    if name == 'ComplEx':
        hr, hi = np.split(h, 2, axis=2)
        rr, ri = np.split(r, 2, axis=2)
        tr, ti = np.split(t, 2, axis=2)
        if head:
            a, b = rr * tr + ri * ti, rr * ti - ri * tr
            x = hr * a + hi * b
        else:
            a, b = hr * rr - hi * ri, hr * ri + hi * rr
            x = a * tr + b * ti
        return aten_sum_lastdim(x)
    if name == 'RotatE':
        hr, hi = np.split(h, 2, axis=2)
        tr, ti = np.split(t, 2, axis=2)
        ph = r / U32(erange / PI)
        cr, sr = cos(ph), sin(ph)
        if head:
            re, im = (cr * tr + sr * ti) - hr, (cr * ti - sr * tr) - hi
        else:
            re, im = (hr * cr - hi * sr) - tr, (hr * sr + hi * cr) - ti
        re, im = np.broadcast_arrays(re, im)
        el = np.sqrt((im.astype(np.float64) * im + (re * re).astype(np.float64)).astype(np.float32))
        return g - aten_sum_lastdim(el)
    if name == 'pRotatE':
        div = U32(erange / PI_PROTATE)
        ph, pr, pt = h / div, r / div, t / div
        x = ph + (pr - pt) if head else (ph + pr) - pt
        return g - aten_sum_lastdim(np.abs(sin(np.ascontiguousarray(np.broadcast_to(x, np.broadcast_shapes(
            ph.shape, pr.shape, pt.shape)))))) * U32(modulus.reshape(-1)[0])
    raise ValueError('model %s not supported' % name)
