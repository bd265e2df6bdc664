"""Edge shapes through the HIP path, against the CPU oracle (GPU box):
one positive with one negative, a "hot" entity that takes every negative of
the batch (one occurrence bucket of 1600 ids: the entity pass's 64-id chunks
and the CSR's long bucket), many negatives per row (n = 2000: the row pass's
LDS score buffer), a two-entity graph, an empty scoring batch, and filtered
ranking where the filter removes every candidate (rank 1).  Tolerances as in
test_gpu_parity.py."""
from argparse import Namespace

import numpy as np
import pytest
import torch

from conftest import score_tol
from knowledgegraphembedding_amd import KGEModel, synth
from knowledgegraphembedding_amd import ops
from oracle import kge_oracle as O
from test_gpu_parity import DEV, NAMES, assert_close_grad, build_model

pytestmark = pytest.mark.gpu


def _check_train(name, E, R, d, pos, neg, w, mode, adv=True, gamma=12.0, seed=3):
    m, ent, rel, mod, rng = build_model(name, E, R, d, gamma, seed)
    args = Namespace(negative_adversarial_sampling=adv, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)
    losses = m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                                   torch.from_numpy(w).to(DEV), mode, args).cpu().numpy()
    ops.raise_on_device_error(DEV)
    log, ge, gr, gm = O.train_grads(name, torch.from_numpy(ent), torch.from_numpy(rel),
                                    None if mod is None else torch.from_numpy(mod), torch.from_numpy(pos),
                                    torch.from_numpy(neg), torch.from_numpy(w), mode, adversarial=adv,
                                    temperature=1.0, uni_weight=False, regularization=0.0,
                                    gamma=torch.Tensor([gamma]).item(), erange=rng)
    ref = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"]])
    assert np.all(np.abs(losses[:3] - ref) <= score_tol(ref)), (losses[:3], ref)
    assert_close_grad(m.entity_embedding.grad.cpu().numpy(), ge.numpy(), f"{name} ent")
    assert_close_grad(m.relation_embedding.grad.cpu().numpy(), gr.numpy(), f"{name} rel")
    if gm is not None:
        assert_close_grad(m.modulus.grad.cpu().numpy(), gm.numpy(), f"{name} modulus")


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_one_positive_one_negative(name, mode):
    E, R, d = 50, 3, 40
    pos, neg, w = synth.kge_batch(21, 1, 1, E, R)
    _check_train(name, E, R, d, pos, neg, w, mode)


@pytest.mark.parametrize("name", ["RotatE", "DistMult", "pRotatE"])
def test_hot_entity_bucket(name):
    """Every negative of the batch is entity 7 (1600 occurrences in one bucket)."""
    E, R, d, B, n = 120, 5, 48, 8, 200
    pos, _, w = synth.kge_batch(22, B, n, E, R)
    neg = np.full((B, n), 7, dtype=np.int64)
    _check_train(name, E, R, d, pos, neg, w, "tail-batch")


@pytest.mark.parametrize("name", ["RotatE", "TransE"])
def test_many_negatives_per_row(name):
    E, R, d, B, n = 3000, 4, 24, 4, 2000
    pos, neg, w = synth.kge_batch(23, B, n, E, R)
    _check_train(name, E, R, d, pos, neg, w, "head-batch", adv=True)


@pytest.mark.parametrize("name", NAMES)
def test_two_entity_graph(name):
    E, R, d, B, n = 2, 1, 16, 6, 5
    pos, neg, w = synth.kge_batch(24, B, n, E, R)
    _check_train(name, E, R, d, pos, neg, w, "tail-batch")


def test_empty_scoring_batch():
    m, *_ = build_model("RotatE", 30, 3, 16, 12.0, 1)
    with torch.no_grad():
        out = m((torch.zeros(0, 3, dtype=torch.int64, device=DEV), torch.zeros(0, 4, dtype=torch.int64, device=DEV)),
                "tail-batch")
    assert tuple(out.shape) == (0, 4)


@pytest.mark.parametrize("name", NAMES)
def test_everything_filtered_ranks_first(name):
    """With every entity a true tail of (h, r), each query's rank is 1 (the
    reference's filter_bias leaves only the true entity unfiltered)."""
    E, R, d = 40, 2, 32
    m, *_ = build_model(name, E, R, d, 12.0, 2)
    true = np.array([[0, 1, t] for t in range(E)], dtype=np.int64)
    ranks, ties = m.rank_queries(true[:10], true, "tail-batch")
    assert np.array_equal(ranks, np.ones(10, dtype=np.int64)) and not ties.any()


@pytest.mark.parametrize("name", ["DistMult", "RotatE"])
def test_rank_queries_both_directions_pipelined(name):
    """rank_queries_both (both directions queued, one read-back — what bench.py's
    ranking section and test_step do) returns exactly rank_queries' per-direction
    ranks and ties."""
    E, R, d = 300, 5, 32
    m, *_ = build_model(name, E, R, d, 12.0, 7)
    rng = np.random.default_rng(3)
    true = np.unique(np.stack([rng.integers(0, E, 2000), rng.integers(0, R, 2000), rng.integers(0, E, 2000)], 1),
                     axis=0)
    q = true[:257]
    (rh, th), (rt, tt) = m.rank_queries_both(q, true)
    rh1, th1 = m.rank_queries(q, true, "head-batch")
    rt1, tt1 = m.rank_queries(q, true, "tail-batch")
    assert np.array_equal(rh, rh1) and np.array_equal(th, th1)
    assert np.array_equal(rt, rt1) and np.array_equal(tt, tt1)


@pytest.mark.parametrize("ftab", ["1", "0"])
@pytest.mark.parametrize("name", ["DistMult", "ComplEx", "pRotatE"])
def test_test_step_query_blocks_reuse_the_table(name, ftab, monkeypatch):
    """test_step ranks in query blocks (both directions of a block in one
    pass, kge_rank_filtered_both, except pRotatE with the library sin; the
    filter as the device table or, ftab = "0", per-query lists) and, from the second
    block (and direction) on, reuses the table statistics and split operands
    the first call left in the workspace (KGE_RANK_REUSE_TABLE); its ranks
    must equal one unblocked rank_queries call per direction without reuse.
    A training step between two evaluations must drop the reuse (the step
    writes the shared workspace and the table)."""
    monkeypatch.setenv("KGE_RANK_FILTER_TABLE", ftab)
    E, R, d = 300, 7, 24
    m, *_ = build_model(name, E, R, d, 12.0, 9)
    g = np.random.default_rng(4)
    test = np.stack([g.integers(0, E, 20000), g.integers(0, R, 20000), g.integers(0, E, 20000)], 1).astype(np.int64)
    true = np.unique(test, axis=0)
    args = Namespace(countries=False, nentity=E, nrelation=R, test_batch_size=16, cpu_num=2, test_log_steps=10 ** 9,
                     cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0)

    def expected():
        ranks = np.concatenate([m.rank_queries(test, true, mode)[0] for mode in ("head-batch", "tail-batch")])
        return float(np.mean(1.0 / ranks)), float(np.mean(ranks))

    for rnd in range(2):
        met = KGEModel.test_step(m, [tuple(x) for x in test.tolist()], [tuple(x) for x in true.tolist()], args)
        mrr, mr = expected()
        assert abs(met["MRR"] - mrr) < 1e-9 and abs(met["MR"] - mr) < 1e-6, (rnd, met, mrr, mr)
        # one training step changes the table before the next evaluation
        pos, neg, w = synth.kge_batch(50 + rnd, 32, 16, E, R)
        m.compute_train_grads(torch.from_numpy(pos).to(DEV), torch.from_numpy(neg).to(DEV),
                              torch.from_numpy(w).to(DEV), "tail-batch", args)
        with torch.no_grad():
            m.entity_embedding.add_(m.entity_embedding.grad, alpha=-100.0)


@pytest.mark.parametrize("kind", ["identical_rows", "zero_modulus"])
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_protate_degenerate_table_library_sin(kind, mode, monkeypatch):
    """pRotatE with the reference's host sin on a degenerate
    table — every candidate scores exactly the true score (identical entity
    rows, or modulus 0), so every query's near-tie window overflows the
    1024-entry list.  The list stage scans such queries with score intervals
    (k_rank_exact_iv): more undecided candidates than a list, so they are
    ranked on the device (correctly rounded sin; identical arguments give
    identical values under any sin) and NO item goes to the host — the host
    buffer stays bounded instead of 1 + E items per query.  Ranks: 1, ties:
    every unfiltered candidate; the same as the device-sin path."""
    E, R, d = 1500, 3, 16
    m, *_ = build_model("pRotatE", E, R, d, 6.0, 4)
    with torch.no_grad():
        if kind == "identical_rows":
            m.entity_embedding.copy_(m.entity_embedding[0].expand(E, -1))
        else:
            m.modulus.zero_()
    g = np.random.default_rng(8)
    q = np.stack([g.integers(0, E, 40), g.integers(0, R, 40), g.integers(0, E, 40)], 1).astype(np.int64)
    true = np.unique(np.concatenate([q, np.stack([g.integers(0, E, 300), g.integers(0, R, 300),
                                                  g.integers(0, E, 300)], 1)]), axis=0)
    calls = []
    real_sin = torch.sin

    def counting_sin(x, *a, **k):
        calls.append(int(x.numel()))
        return real_sin(x, *a, **k)

    monkeypatch.setattr(torch, "sin", counting_sin)
    m.rank_trig = "reference"
    ops.device_sin_queries(DEV)  # reset
    ranks, ties, listed = m.rank_queries(q, true, mode, listed=True)
    monkeypatch.setattr(torch, "sin", real_sin)
    assert sum(calls) == 0, calls  # nothing left for the host sin
    assert (listed > 1024).all()
    # those queries are reported as ranked without the library sin
    assert ops.device_sin_queries(DEV) == len(q)
    m.rank_trig = "device"
    r_dev, t_dev = m.rank_queries(q, true, mode, path="scan")
    assert np.array_equal(ranks, r_dev) and np.array_equal(ties, t_dev)
    assert (ranks == 1).all() and (ties > 0).all()


def test_protate_three_call_protocol_checks():
    """kge_rank_sin_args / kge_rank_finish_sin check that they
    follow their list stage — the same mode, nq and table, nothing else
    ranked on the workspace in between — and that a query's items arrive
    once, with 1 + listed entries; a violation sets KGE_DEVERR_ARG (raised
    as RuntimeError) instead of returning wrong ranks."""
    from knowledgegraphembedding_amd import _lib
    E, R, d = 400, 3, 32
    m, *_ = build_model("pRotatE", E, R, d, 6.0, 6)
    with torch.no_grad():  # ten exact copies of entity 5: near-ties only the host sin can order
        m.entity_embedding[100:110].copy_(m.entity_embedding[5].expand(10, -1))
    g = np.random.default_rng(2)
    qs = np.stack([g.integers(0, E, 64), g.integers(0, R, 64), np.full(64, 5)], 1).astype(np.int64)
    true = np.unique(np.concatenate([qs, np.stack([g.integers(0, E, 900), g.integers(0, R, 900),
                                                   g.integers(0, E, 900)], 1)]), axis=0)
    q = torch.from_numpy(qs).to(DEV)
    from knowledgegraphembedding_amd.filters import FilterIndex
    off, ids = FilterIndex(true, E, R).filter_csr(qs, "tail-batch")
    off, ids = torch.from_numpy(off).to(DEV), torch.from_numpy(ids).to(DEV)
    lib = _lib.load()
    desc = m.desc()
    mode = _lib.MODE_IDS["tail-batch"]
    st = ops.state(DEV)
    nq = 64
    ws = st.workspace(lib.kge_rank_workspace_bytes(desc, nq))
    st.rank_ws_ptr = None
    ranks = torch.empty(nq, dtype=torch.int64, device=DEV)
    ties = torch.empty(nq, dtype=torch.int32, device=DEV)
    cnt = torch.empty(nq, dtype=torch.int32, device=DEV)
    s = ops._stream(DEV)
    args_ = (ws.data_ptr(), ws.numel(), st.err.data_ptr(), s)

    def list_stage():
        _lib.check(lib.kge_rank_filtered_ex(desc, mode, q.data_ptr(), nq, off.data_ptr(), ids.data_ptr(),
                                            ranks.data_ptr(), ties.data_ptr(), cnt.data_ptr(),
                                            _lib.RANK_STAGE_LIST, *args_), "list")
        c = cnt.cpu().numpy().astype(np.int64)
        items = np.where((c >= 1) & (c <= 1024), 1 + c, 0)
        io = np.zeros(nq + 1, dtype=np.int64)
        np.cumsum(items, out=io[1:])
        return torch.from_numpy(io).to(DEV), int(io[-1])

    # a well-formed round: no error
    io, total = list_stage()
    buf = torch.zeros((max(total, 1), d), device=DEV)
    _lib.check(lib.kge_rank_sin_args(desc, mode, nq, io.data_ptr(), buf.data_ptr(), *args_), "args")
    buf = torch.sin(buf.cpu()).to(DEV)
    _lib.check(lib.kge_rank_finish_sin(desc, mode, nq, io.data_ptr(), buf.data_ptr(), ranks.data_ptr(),
                                       ties.data_ptr(), None, *args_), "finish")
    ops.raise_on_device_error(DEV)
    if total:
        # the same items delivered a second time
        _lib.check(lib.kge_rank_finish_sin(desc, mode, nq, io.data_ptr(), buf.data_ptr(), ranks.data_ptr(),
                                           ties.data_ptr(), None, *args_), "finish")
        with pytest.raises(RuntimeError, match="list stage"):
            ops.raise_on_device_error(DEV)
    # another mode than the list stage's
    io, total = list_stage()
    buf = torch.zeros((max(total, 1), d), device=DEV)
    other = _lib.MODE_IDS["head-batch"]
    _lib.check(lib.kge_rank_sin_args(desc, other, nq, io.data_ptr(), buf.data_ptr(), *args_), "args")
    if total:
        with pytest.raises(RuntimeError, match="list stage"):
            ops.raise_on_device_error(DEV)
    # another ranking call on the workspace between the list stage and finish
    io, total = list_stage()
    _lib.check(lib.kge_rank_filtered_ex(desc, mode, q.data_ptr(), nq, off.data_ptr(), ids.data_ptr(),
                                        ranks.data_ptr(), ties.data_ptr(), None, 0, *args_), "all")
    buf = torch.zeros((max(total, 1), d), device=DEV)
    _lib.check(lib.kge_rank_sin_args(desc, mode, nq, io.data_ptr(), buf.data_ptr(), *args_), "args")
    if total:
        with pytest.raises(RuntimeError, match="list stage"):
            ops.raise_on_device_error(DEV)
    assert total > 0, "the fixture should leave some near-ties for the host"


def test_rank_reuse_checks_the_derived_table_kind():
    """The workspace's derived table is the split-bf16 operands (DistMult /
    ComplEx) or pRotatE's phase table (k_prot_phase), at the same workspace
    offset.  A pRotatE call with KGE_RANK_REUSE_TABLE right after a DistMult
    call on the SAME entity tensor (same pointer and shape) must not take the
    split for phases (k_rank_tag's kind word), nor a phase table made with
    another phase divisor (its parameter word): its ranks equal a call on a
    fresh workspace."""
    from knowledgegraphembedding_amd import _lib
    from knowledgegraphembedding_amd.filters import FilterIndex
    E, R, d = 700, 4, 64
    md, *_ = build_model("DistMult", E, R, d, 6.0, 11)
    mp, *_ = build_model("pRotatE", E, R, d, 6.0, 11)
    mp2, *_ = build_model("pRotatE", E, R, d, 9.0, 11)  # another embedding range: another phase divisor
    with torch.no_grad():
        mp.entity_embedding.data = md.entity_embedding.data
        mp2.entity_embedding.data = md.entity_embedding.data
    g = np.random.default_rng(12)
    qs = np.stack([g.integers(0, E, 96), g.integers(0, R, 96), g.integers(0, E, 96)], 1).astype(np.int64)
    true = np.unique(np.concatenate([qs, np.stack([g.integers(0, E, 800), g.integers(0, R, 800),
                                                   g.integers(0, E, 800)], 1)]), axis=0)
    q = torch.from_numpy(qs).to(DEV)
    off, ids = FilterIndex(true, E, R).filter_csr(qs, "tail-batch")
    off, ids = torch.from_numpy(off).to(DEV), torch.from_numpy(ids).to(DEV)
    lib = _lib.load()
    mode = _lib.MODE_IDS["tail-batch"]
    nq = qs.shape[0]
    descs = {"d": md.desc(), "p": mp.desc(), "p2": mp2.desc()}
    need = max(lib.kge_rank_workspace_bytes(x, nq) for x in descs.values())
    ws = torch.zeros(need, dtype=torch.uint8, device=DEV)
    fresh = torch.zeros(need, dtype=torch.uint8, device=DEV)
    err = ops.state(DEV).err
    s = ops._stream(DEV)

    def rank(key, buf, flags):
        r = torch.empty(nq, dtype=torch.int64, device=DEV)
        t = torch.empty(nq, dtype=torch.int32, device=DEV)
        _lib.check(lib.kge_rank_filtered_ex(descs[key], mode, q.data_ptr(), nq, off.data_ptr(), ids.data_ptr(),
                                            r.data_ptr(), t.data_ptr(), None, flags, buf.data_ptr(), buf.numel(),
                                            err.data_ptr(), s), key)
        ops.raise_on_device_error(DEV)
        return r.cpu().numpy(), t.cpu().numpy()

    reuse = ops.RANK_REUSE_TABLE
    want_p = rank("p", fresh, 0)
    fresh.zero_()
    want_p2 = rank("p2", fresh, 0)
    rank("d", ws, 0)  # the split-bf16 operands land where pRotatE keeps its phases
    for got, want in ((rank("p", ws, reuse), want_p), (rank("p", ws, reuse), want_p),
                      (rank("p2", ws, reuse), want_p2), (rank("d", ws, reuse), rank("d", fresh, 0))):
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_protate_library_sin_in_chunks(mode, monkeypatch):
    """the three-call form's chunked delivery — the host sin's
    arguments in pieces of at most SIN_CHUNK_BYTES (the C++ op's budget:
    KGE_SIN_CHUNK_BYTES), each piece's queries finished before the next —
    gives the single-delivery ranks and ties.  Every listed near-tie goes to
    the host (KGE_RANK_SIN_SCREEN=0) and the budget is a few rows, so both
    paths run many chunks (counted)."""
    E, R, d = 1200, 5, 24
    m, *_ = build_model("pRotatE", E, R, d, 6.0, 12)
    m.rank_trig = "reference"
    g = np.random.default_rng(21)
    with torch.no_grad():  # rows 100..399: one row with relative noise ~1e-7 (near-ties, not exact ones)
        blk = m.entity_embedding[100].detach().cpu().numpy()[None, :] * \
            (1.0 + 1e-7 * g.standard_normal((300, d))).astype(np.float32)
        m.entity_embedding[100:400].copy_(torch.from_numpy(blk.astype(np.float32)))
    q = np.stack([g.integers(0, E, 120), g.integers(0, R, 120), g.integers(0, E, 120)], 1).astype(np.int64)
    q[:60, 0 if mode == "head-batch" else 2] = g.integers(100, 400, 60)  # true entities inside the block
    true = np.unique(np.concatenate([q, np.stack([g.integers(0, E, 900), g.integers(0, R, 900),
                                                  g.integers(0, E, 900)], 1)]), axis=0)
    monkeypatch.setenv("KGE_RANK_SIN_SCREEN", "0")
    r1, t1, listed = m.rank_queries(q, true, mode, listed=True)
    assert listed.sum() > 1000, int(listed.sum())
    calls = []
    real_sin = torch.sin

    def counting_sin(x, *a, **k):  # the host sin runs once per chunk
        calls.append(int(x.numel()))
        return real_sin(x, *a, **k)

    budget = 8 * 4 * d  # eight item rows
    monkeypatch.setattr(ops, "SIN_CHUNK_BYTES", budget)
    monkeypatch.setattr(torch, "sin", counting_sin)
    r2, t2 = m.rank_queries(q, true, mode)
    monkeypatch.setattr(torch, "sin", real_sin)
    assert len(calls) >= 3, calls
    assert np.array_equal(r1, r2) and np.array_equal(t1, t2)
    # the C++ op's own chunk loop (the binding a libtorch caller uses)
    from knowledgegraphembedding_amd.filters import FilterIndex
    from knowledgegraphembedding_amd._lib import MODE_IDS, MODEL_IDS
    off, ids = FilterIndex(true, E, R).filter_csr(q, mode)
    gm, rng = m._host_scalars()
    args = (m.entity_embedding.detach(), m.relation_embedding.detach(), m.modulus.detach(),
            torch.from_numpy(q).to(DEV), torch.from_numpy(off).to(DEV), torch.from_numpy(ids).to(DEV),
            MODE_IDS[mode], MODEL_IDS["pRotatE"], gm, rng, 0, None)
    monkeypatch.setenv("KGE_SIN_CHUNK_BYTES", str(budget))
    r3, t3 = torch.ops.kge.rank_filtered(*args)
    assert np.array_equal(r3.cpu().numpy(), r1) and np.array_equal(t3.cpu().numpy(), t1)
