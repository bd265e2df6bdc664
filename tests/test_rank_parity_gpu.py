"""Filtered-rank parity with the reference: the HIP
ranking against ranks the reference's own test_step produced (tests/golden/
make_golden.py: `ranks` on synthetic KGs, `ranks_full` at config-3 scale — the
real wn18rr split with DistMult / ComplEx / pRotatE at d = 500 and E = 40943,
512 queries per direction, the FB15k entity set with TransE / RotatE at
d = 1000).

What is asserted, per query (rank = 1 + #{unfiltered e ≠ true: s_e > s_true}):
  * all five models: the kernel's near-ties are re-scored in the reference's
    fp32 operation order (kge_rank_ref.h), so ranks AND tie counts equal the
    reference's on every query (0 untied disagreements); where the reference
    has exact ties (its argsort is not stable) its position lies in
    [rank, rank + ties].
    RotatE's rotation comes from the reference's own cos / sin bits of the
    relation phases (tests/golden/rotate_trig.npz, made by the reference's
    ATen CPU ops in make_golden.py `gen_rotate_trig`), fed to the kernels as
    kge_model_desc.relation_trig — the table KGEModel builds itself with
    ops.reference_rotation on the host it runs on.
    pRotatE's sin acts on per-candidate phase sums (model.py:241-245): the
    device lists the near-ties, writes their phase sums, the host takes the
    sin with the reference's own torch.sin (ops.reference_sin), and the device
    re-scores them (kge_rank_sin_args / kge_rank_finish_sin); by default the
    listed candidates are first re-scored with correctly rounded sin and only
    those within the library sin's bound of the true score go to the host
    ("auto/noscreen": all of them — the same ranks).
  * pRotatE with correctly rounded DEVICE sin (rank_trig = "device"): equal on
    every query decidable under the rigorous last-bit-of-sin bound δ below,
    within the competitors inside δ otherwise.
  * Every fast path (split-bf16 MFMA tile = "auto" for DistMult / ComplEx,
    fp32 MFMA tile, register tile, wave scan) returns the same ranks and ties
    bit for bit: their windows differ, the refinement does not.
  * test_host_trig_matches_reference / test_host_sin_matches_reference: this
    host's torch.cos / torch.sin (what KGEModel.test_step uses) against the
    reference's committed bits, and that torch.sin's bits do not depend on how
    its input is batched (the reference takes the sin of a [B, E, d] tensor,
    the ranking of a [items, d] one).

δ for pRotatE with device sin (u = 2^-24, K dims, S = (γ − s_true)/mod): |sin|
moves by ≤ u per element; every partial sum of the reference's reduction
(≤ K/32 + 24 per lane column and fold) may round the other way by ≤ 2u of its
value; both the candidate and the true score move:
δ = 2·mod·(K·u + (4 + 2·(K/32 + 24))·u·S).
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_npz, synth_tables
from knowledgegraphembedding_amd import KGEModel

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
U = 2.0 ** -24
EXACT = ("TransE", "DistMult", "ComplEx", "RotatE", "pRotatE")
PATHS = {"DistMult": ("auto", "mfma32", "tile", "scan"), "ComplEx": ("auto", "mfma32", "tile", "scan"),
         "TransE": ("auto", "scan"), "RotatE": ("auto", "scan"), "pRotatE": ("auto", "auto/noscreen", "scan")}


def build(name, E, R, d, gamma, seed):
    de, dr = {"TransE": (0, 0), "DistMult": (0, 0), "ComplEx": (1, 1), "RotatE": (1, 0), "pRotatE": (0, 0)}[name]
    m = KGEModel(name, E, R, d, gamma, bool(de), bool(dr))
    ent, rel, mod, rng = synth_tables(name, E, R, d, gamma, seed)
    with torch.no_grad():
        m.entity_embedding.copy_(torch.from_numpy(ent))
        m.relation_embedding.copy_(torch.from_numpy(rel))
    return m.to(DEV), ent, rel, mod, rng


def reference_trig(tag, rel, rng):
    """[R, 2, d] reference (cos | sin) of the relation phases: the committed
    XOR (rotate_trig.npz) applied to correctly rounded values for the queried
    relations (the others are never read by the fixture's queries); plus the
    phases, computed as model.py:209 does (an IEEE division, host-independent)."""
    g = load_npz("rotate_trig.npz")
    phase = (torch.from_numpy(rel) / (rng / 3.14159265358979323846)).numpy()
    ph64 = phase.astype(np.float64)
    cs, sn = np.cos(ph64).astype(np.float32), np.sin(ph64).astype(np.float32)
    ids = g[f"{tag}/rel_ids"]
    cs.view(np.uint32)[ids] ^= g[f"{tag}/cos_xor"]
    sn.view(np.uint32)[ids] ^= g[f"{tag}/sin_xor"]
    return torch.from_numpy(np.stack([cs, sn], 1)), phase, ids


def trig_bound(name, mod, queries, d, gamma, s_true, exact=True):
    """δ above (0 for the models whose operations are all reproduced)."""
    if exact:
        return np.zeros(len(queries))
    K = d
    fold = 4 + 2 * (K / 32 + 24)
    m = float(mod[0, 0])
    S = np.abs(gamma - s_true.astype(np.float64)) / m
    return 2 * m * (K * U + fold * U * S)


def check(tag, name, mode, ranks, ties, ref, bound, exact=True):
    """The assertions of the module docstring; returns (decidable, differing, ambiguous)."""
    r_rank, r_ties, gaps = ref["rank"].astype(np.int64), ref["ties"], ref["gap"]
    near = (np.abs(gaps) <= bound[:, None]).sum(1)
    decidable = (r_ties == 0) & (near == 0)
    bad = decidable & (ranks != r_rank)
    assert not bad.any(), f"{tag} {name} {mode}: queries {np.nonzero(bad)[0][:8]} {ranks[bad][:8]} vs {r_rank[bad][:8]}"
    if exact:
        assert np.array_equal(ties, r_ties), f"{tag} {name} {mode}: tie counts differ"
        assert np.all((r_rank >= ranks) & (r_rank <= ranks + ties)), f"{tag} {name} {mode}: tie interval"
    else:
        amb = ~decidable & (near < 16)
        assert np.all(np.abs(ranks[amb] - r_rank[amb]) <= near[amb] + r_ties[amb]), f"{tag} {name} {mode}"
    differ = ranks != r_rank
    # a query the reference ties at the true score is placed by its non-stable
    # argsort somewhere in [rank, rank + ties] (checked above); the others may
    # differ only through device sin's bound (pRotatE, rank_trig "device"), on
    # at most 5 % of the queries
    untied_differ = int((differ & (r_ties == 0)).sum())
    cap = 0 if exact else 0.05 * len(ranks)
    assert untied_differ <= cap, f"{tag} {name} {mode}: {untied_differ} of {len(ranks)} ranks differ"
    return int(decidable.sum()), int((r_ties > 0).sum()), int((~decidable).sum()), int(differ.sum()), untied_differ


def run_case(tag, name, E, R, d, gamma, seed, queries, filters, refs, report):
    m, ent, rel, mod, rng = build(name, E, R, d, gamma, seed)
    trig = reference_trig(tag, rel, rng)[0] if name == "RotatE" else None
    bases = {}
    for mode in ("head-batch", "tail-batch"):
        ref = refs(mode)
        nq = len(ref["rank"])
        qs = queries[:nq]
        bound = trig_bound(name, mod, qs, d, gamma, ref["s_true"])
        base = None
        for path in PATHS[name]:
            import os
            # "/noscreen": pRotatE's listed candidates all go to the host sin
            # (the diagnostic switch KGE_RANK_SIN_SCREEN=0: no device screen)
            os.environ["KGE_RANK_SIN_SCREEN"] = "0" if path.endswith("/noscreen") else "1"
            ranks, ties, listed = m.rank_queries(qs, filters, mode, path=path.split("/")[0], listed=True,
                                                 relation_trig=trig)
            os.environ.pop("KGE_RANK_SIN_SCREEN", None)
            if base is None:
                base = (ranks, ties)
            else:
                assert np.array_equal(ranks, base[0]) and np.array_equal(ties, base[1]), f"{name} {mode} {path}"
            dec, tied, amb, diff, udiff = check(tag, name, mode, ranks, ties, ref, bound)
            report.append((tag, name, mode, path, nq, dec, tied, amb, diff, udiff, round(float(listed.mean()), 1),
                           int(listed.max())))
        bases[mode] = base
        if name == "pRotatE":  # correctly rounded device sin: within the last-bit bound
            m.rank_trig = "device"
            ranks, ties, listed = m.rank_queries(qs, filters, mode, listed=True)
            m.rank_trig = "reference"
            bound = trig_bound(name, mod, qs, d, gamma, ref["s_true"], exact=False)
            dec, tied, amb, diff, udiff = check(tag, name, mode, ranks, ties, ref, bound, exact=False)
            report.append((tag, name, mode, "auto/device-sin", nq, dec, tied, amb, diff, udiff,
                           round(float(listed.mean()), 1), int(listed.max())))
    # both directions in one pass (rank_queries_both → kge_rank_filtered_both;
    # pRotatE with the library sin stays per direction): every path's ranks
    # and ties equal the per-direction calls' above, i.e. the reference's
    nq = len(bases["head-batch"][0])
    if nq == len(bases["tail-batch"][0]):
        for path in dict.fromkeys(p.split("/")[0] for p in PATHS[name]):
            (rh, th), (rt, tt) = m.rank_queries_both(queries[:nq], filters, path=path, relation_trig=trig)
            for mode, r, t in (("head-batch", rh, th), ("tail-batch", rt, tt)):
                assert np.array_equal(r, bases[mode][0]) and np.array_equal(t, bases[mode][1]), \
                    f"{tag} {name} {mode} {path}: both-directions pass"
            report.append((tag, name, "both", path, 2 * nq, "ranks and ties = per-direction"))
    del m
    torch.cuda.empty_cache()


def _print(report):
    print("\n(tag, model, mode, path, queries, decidable, reference-tied, ambiguous, differing, differing untied, "
          "mean listed, max listed)")
    for r in report:
        print("  ", r)


def test_ranks_vs_reference_small(g_ranks, golden_info):
    report = []
    for kg in golden_info["ranks"]:
        tag, E, R, d, seed = kg["tag"], kg["E"], kg["R"], kg["d"], kg["seed"]
        gamma = torch.Tensor([kg["gamma"]]).item()
        for name in kg["models"]:
            def refs(mode, name=name, tag=tag):
                k = f"{tag}/{name}/{mode}"
                return {f: g_ranks[f"{k}/{f}"] for f in ("rank", "ties", "gap", "s_true")}
            run_case(tag, name, E, R, d, gamma, seed, g_ranks[f"{tag}/test"], g_ranks[f"{tag}/all_true"], refs,
                     report)
    _print(report)


@pytest.fixture(scope="module")
def g_full():
    if not (GOLDEN / "ranks_full.npz").exists():
        pytest.skip("ranks_full.npz not generated")
    return load_npz("ranks_full.npz")


def _full_cases(info):
    for kg in info.get("ranks_full", []):
        for mdl in kg["models"]:
            yield kg, mdl


@pytest.mark.parametrize("case", ["wn18rr/DistMult", "wn18rr/ComplEx", "wn18rr/pRotatE", "fb15k/TransE",
                                  "fb15k/RotatE"])
def test_ranks_vs_reference_full_size(g_full, golden_info, case):
    tag, name = case.split("/")
    kg = next(k for k in golden_info["ranks_full"] if k["tag"] == tag)
    mdl = next(x for x in kg["models"] if x["name"] == name)
    gamma = torch.Tensor([kg["gamma"]]).item()

    def refs(mode):
        k = f"{tag}/{name}/{mode}"
        return {f: g_full[f"{k}/{f}"] for f in ("rank", "ties", "gap", "s_true")}

    report = []
    run_case(tag, name, kg["E"], kg["R"], mdl["d"], gamma, kg["seed"], g_full[f"{tag}/queries"],
             g_full[f"{tag}/filters"], refs, report)
    _print(report)


def test_host_trig_matches_reference(g_full, golden_info, capsys):
    """This host's torch.cos / torch.sin of the FB15k fixture's relation phases
    (what KGEModel.test_step rotates RotatE's queries by, ops.reference_rotation)
    against the reference's bits.  Equal: test_step's RotatE ranks on this host
    are the reference's.  Different: the reference's own ranks depend on the
    CPU's vector library; the test then reports how many fixture ranks this
    host's table moves (asserting only that the committed-bit ranks above are
    exact, which test_ranks_vs_reference_full_size does)."""
    from knowledgegraphembedding_amd import ops
    kg = next(k for k in golden_info["ranks_full"] if k["tag"] == "fb15k")
    d, gamma = 1000, torch.Tensor([kg["gamma"]]).item()
    m, ent, rel, mod, rng = build("RotatE", kg["E"], kg["R"], d, gamma, kg["seed"])
    ref_tab, phase, ids = reference_trig("fb15k", rel, rng)
    host_tab = ops.reference_rotation(torch.from_numpy(rel), m._host_scalars()[1])
    same = (host_tab.numpy().view(np.uint32)[ids] == ref_tab.numpy().view(np.uint32)[ids])
    frac = 1.0 - float(same.mean())
    with capsys.disabled():
        print(f"\nhost torch.cos/sin vs the reference's bits on {same.size} fixture values: {frac:.4%} differ "
              f"(MKL {torch.backends.mkl.is_available()}, cpu capability "
              f"{torch.backends.cpu.get_cpu_capability()})")
    if frac == 0.0:
        return
    # the bits differ: measure what this host's table does to the reference's ranks (reported, not asserted)
    nq = len(g_full["fb15k/RotatE/head-batch/rank"])
    qs, filters = g_full["fb15k/queries"][:nq], g_full["fb15k/filters"]
    for mode in ("head-batch", "tail-batch"):
        ranks, _ = m.rank_queries(qs, filters, mode, relation_trig=host_tab)
        r_rank = g_full[f"fb15k/RotatE/{mode}/rank"]
        with capsys.disabled():
            print(f"  {mode}: ranks from this host's cos/sin differ from the reference's on "
                  f"{int((ranks != r_rank).sum())} of {nq} queries")


def test_host_sin_matches_reference(golden_info, g_full, capsys):
    """pRotatE: this host's torch.sin (ops.reference_sin, what the ranking's
    near-ties are re-scored from) on the true entities' phase sums of the
    first 128 wn18rr fixture queries, both associations (model.py:240-243),
    against the reference's bits (tests/golden/protate_sin.npz); and the same
    values from the arguments batched differently (a permuted [items, d] block
    and odd-length slices, as the ranking batches them) — the reference took
    the sin of a [B, E, d] tensor."""
    from knowledgegraphembedding_amd import ops
    info = golden_info["protate_sin"]
    E, R, d, gamma, seed, nq = (info[k] for k in ("E", "R", "d", "gamma", "seed", "queries"))
    ent, rel, _, rng = synth_tables("pRotatE", E, R, d, torch.Tensor([gamma]).item(), seed)
    q = torch.from_numpy(g_full["wn18rr/queries"][:nq])
    div = rng / 3.14159262358979323846  # model.py:232-238 (a Python float, as the reference's)
    ph = torch.from_numpy(ent)[q[:, 0]] / div
    pr = torch.from_numpy(rel)[q[:, 1]] / div
    pt = torch.from_numpy(ent)[q[:, 2]] / div
    args = torch.stack([ph + (pr - pt), (ph + pr) - pt])
    mine = ops.reference_sin(args).numpy()
    cr = np.sin(args.numpy().astype(np.float64)).astype(np.float32)
    ref = (cr.view(np.uint32) ^ load_npz("protate_sin.npz")["sin_xor"]).view(np.float32)
    differ = float((mine.view(np.uint32) != ref.view(np.uint32)).mean())
    flat = args.reshape(-1)
    perm = torch.from_numpy(np.random.default_rng(3).permutation(flat.numel()))
    batched = torch.empty_like(flat)
    batched[perm] = ops.reference_sin(flat[perm].contiguous())
    for a0, n in ((1, 7), (13, 501), (1000, 4099)):
        assert torch.equal(ops.reference_sin(flat[a0:a0 + n].clone()), batched[a0:a0 + n])
    with capsys.disabled():
        print(f"\nhost torch.sin vs the reference's bits on {mine.size} pRotatE phase sums: {differ:.4%} differ "
              f"(MKL {torch.backends.mkl.is_available()}, cpu capability {torch.backends.cpu.get_cpu_capability()})")
    assert torch.equal(batched.view(mine.shape), torch.from_numpy(mine)), "torch.sin depends on the batching"
    assert differ == 0.0, "this host's sin differs from the reference's: pRotatE ranks would follow this host's"


@pytest.mark.parametrize("name,E,d", [("DistMult", 300, 50), ("DistMult", 257, 37), ("DistMult", 1000, 130),
                                      ("ComplEx", 300, 25), ("ComplEx", 513, 33), ("DistMult", 129, 16),
                                      ("DistMult", 300, 1100), ("ComplEx", 257, 530)])
def test_split_bf16_tile_matches_other_paths(name, E, d):
    """The split-bf16 MFMA tile ("auto" for DistMult / ComplEx) against the
    fp32 paths on shapes its layout pads: E not a multiple of the 128-row
    block, reduction lengths not a multiple of the 16-k slab (and odd ones,
    whose rows are not float4-aligned), plus exact ties — a block of entity
    rows copied from a true entity.  Ranks and tie counts must be identical
    to the wave scan's (reference order after refinement on every path).
    Rows of more than 1024 floats (d = 1100, ComplEx 2·530) take the tile's
    own gather mode for s_true instead of the reference-order true score
    (whose LDS staging holds ≤ 1024 floats), with the window covering both
    fast scores."""
    R = 7
    m, ent, rel, _, _ = build(name, E, R, d, 12.0, 17)
    with torch.no_grad():
        m.entity_embedding[E - 9:E - 1].copy_(m.entity_embedding[3].expand(8, -1))  # 8 exact copies of entity 3
    g = np.random.default_rng(5)
    q = np.stack([g.integers(0, E, 200), g.integers(0, R, 200), g.integers(0, E, 200)], 1).astype(np.int64)
    q[:20, 0] = 3
    q[20:40, 2] = 3
    true = np.unique(np.concatenate([q, np.stack([g.integers(0, E, 600), g.integers(0, R, 600),
                                                  g.integers(0, E, 600)], 1)]), axis=0)
    le = 2 * d if name == "ComplEx" else d
    paths = ["scan", "auto"] + (["mfma32"] if le % 4 == 0 else [])
    for mode in ("head-batch", "tail-batch"):
        out = {p: m.rank_queries(q, true, mode, path=p, listed=True) for p in paths}
        r0, t0, _ = out["scan"]
        tied = slice(0, 20) if mode == "head-batch" else slice(20, 40)  # true entity 3, copied 8 times
        assert (t0[tied] > 0).any(), (name, mode)
        for p in paths[1:]:
            r, t, _ = out[p]
            assert np.array_equal(r, r0) and np.array_equal(t, t0), (name, E, d, mode, p)


@pytest.mark.parametrize("name,d", [("DistMult", 48), ("ComplEx", 48), ("DistMult", 1040)])
def test_split_bf16_tile_wide_dynamic_range(name, d):
    """The split tile's error bound is rigorous, not statistical: entity and
    relation values spread over 10^-30 … 10^3 (bf16 lo pieces and products
    that underflow, rows that differ by 30 orders of magnitude, exact zeros)
    must still give the wave scan's ranks and ties (d = 1040: s_true from the
    tile's gather mode)."""
    E, R = 500, 5
    m, ent, rel, _, _ = build(name, E, R, d, 12.0, 23)
    g = np.random.default_rng(11)
    with torch.no_grad():
        ee = m.entity_embedding.detach().cpu().numpy()
        ee *= 10.0 ** g.uniform(-30, 3, size=ee.shape)
        ee[g.random(ee.shape) < 0.05] = 0.0
        ee[:20] *= 1e-25  # whole rows near the underflow range
        m.entity_embedding.copy_(torch.from_numpy(ee.astype(np.float32)))
        rr = m.relation_embedding.detach().cpu().numpy()
        rr *= 10.0 ** g.uniform(-5, 2, size=rr.shape)
        m.relation_embedding.copy_(torch.from_numpy(rr.astype(np.float32)))
    q = np.stack([g.integers(0, E, 150), g.integers(0, R, 150), g.integers(0, E, 150)], 1).astype(np.int64)
    q[:30, 2] = g.integers(0, 20, 30)  # true tails among the tiny rows
    q[30:60, 0] = g.integers(0, 20, 30)
    true = np.unique(q, axis=0)
    for mode in ("head-batch", "tail-batch"):
        r0, t0 = m.rank_queries(q, true, mode, path="scan")
        r1, t1 = m.rank_queries(q, true, mode, path="auto")
        assert np.array_equal(r0, r1) and np.array_equal(t0, t1), (name, mode)


@pytest.mark.parametrize("name", ["DistMult", "ComplEx", "RotatE", "TransE", "pRotatE"])
def test_filter_table_matches_query_lists(name, monkeypatch):
    """KGE_RANK_FILTER_TABLE (rank_queries_both's default for a dense filter
    index: the device looks each query's filtered ids up in the whole index)
    gives the ranks and ties of per-query filter lists built on the host
    (rank_queries), on a wn18rr-shaped synthetic graph with repeated keys —
    through rank_queries_both's two-direction pass (kge_rank_filtered_both),
    with the table and with per-query lists, against one call per direction."""
    from knowledgegraphembedding_amd import synth
    from knowledgegraphembedding_amd.filters import FilterIndex
    E, R, d = 3000, 11, 64
    h, r, t = synth.randint(911, (20000,), E), synth.randint(912, (20000,), R), synth.randint(913, (20000,), E)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(914, (700,), len(true))]
    index = FilterIndex(true, E, R)
    cplx = name in ("ComplEx", "RotatE")
    torch.manual_seed(3)
    m = KGEModel(name, E, R, d, 12.0, cplx, name == "ComplEx").to(DEV)
    if name == "pRotatE":  # the device sin: rank_queries_both takes the two-direction pass (its register tile)
        m.rank_trig = "device"
    (rh, th), (rt, tt) = m.rank_queries_both(test, index)
    assert index.device_table("head-batch", DEV) is not None
    ref_h = m.rank_queries(test, index, "head-batch")
    ref_t = m.rank_queries(test, index, "tail-batch")
    assert np.array_equal(rh, ref_h[0]) and np.array_equal(th, ref_h[1])
    assert np.array_equal(rt, ref_t[0]) and np.array_equal(tt, ref_t[1])
    monkeypatch.setenv("KGE_RANK_FILTER_TABLE", "0")
    (rh2, th2), (rt2, tt2) = m.rank_queries_both(test, index)
    assert np.array_equal(rh2, rh) and np.array_equal(rt2, rt) and np.array_equal(th2, th) and np.array_equal(tt2, tt)
    # key spaces above DENSE_KEYS: the start table searched on the device (FB15k's path)
    monkeypatch.delenv("KGE_RANK_FILTER_TABLE")
    host = [index.device_table(md, DEV) for md in ("head-batch", "tail-batch")]
    monkeypatch.setattr(FilterIndex, "DENSE_KEYS", 16)
    index.__dict__.pop("_dev_tables", None)
    searched = [index.device_table(md, DEV) for md in ("head-batch", "tail-batch")]
    assert all(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) for a, b in zip(host, searched))
    (rh3, th3), (rt3, tt3) = m.rank_queries_both(test, index)
    assert np.array_equal(rh3, rh) and np.array_equal(rt3, rt) and np.array_equal(th3, th) and np.array_equal(tt3, tt)


def test_device_sinf_within_declared_floats():
    """The pRotatE list stage's interval screen bounds the library's sin around
    the device's own sinf (kge_rank_ref.h SIN_FAST_*): at most 1 float from the
    correctly rounded sin for |x| <= 16 and 2 for |x| <= 65536.  Checked here
    on every float of both ranges, with the library's own compiled sinf
    (kge_selftest_sin), so a toolchain whose sinf drifts fails this test
    instead of producing wrong ranks."""
    from knowledgegraphembedding_amd import _lib, ops
    lib = _lib.load()
    for rng, bound in ((16.0, 1), (65536.0, 2)):
        out = torch.zeros(1, dtype=torch.int32, device=DEV)
        _lib.check(lib.kge_selftest_sin(rng, out.data_ptr(), ops._stream(DEV)), "kge_selftest_sin")
        assert int(out.item()) <= bound, (rng, int(out.item()))


@pytest.mark.parametrize("name", ["TransE"])
def test_tile_staging_switch_same_ranks(name, monkeypatch):
    """The register tile's round-6 staging for TransE (queries
    pre-splatted, padded k-rows, pipelined LDS reads) and round 5's
    (KGE_TILE_SPL=0, diagnostic) give the same ranks, ties and listed counts —
    the same arithmetic in the same order."""
    from knowledgegraphembedding_amd import synth
    E, R, d = 3000, 11, 64
    h, r, t = synth.randint(921, (12000,), E), synth.randint(922, (12000,), R), synth.randint(923, (12000,), E)
    true = np.unique(np.stack([h, r, t], 1), axis=0)
    test = true[synth.randint(924, (500,), len(true))]
    torch.manual_seed(4)
    m = KGEModel(name, E, R, d, 12.0, False, False).to(DEV)
    m.rank_trig = "device"
    for mode in ("head-batch", "tail-batch"):
        a = m.rank_queries(test, true, mode, listed=True)
        monkeypatch.setenv("KGE_TILE_SPL", "0")
        b = m.rank_queries(test, true, mode, listed=True)
        monkeypatch.delenv("KGE_TILE_SPL")
        for x, y in zip(a, b):
            assert np.array_equal(x, y), (name, mode)
