"""Pin the CPU oracle (oracle/kge_oracle.py) to the reference's own outputs
(tests/golden/*.npz, made by tests/golden/make_golden.py from the imported
reference).  CPU only."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN, dims, erange_of, load_npz, synth_tables  # noqa: F401
from knowledgegraphembedding_amd import synth
from oracle import kge_oracle as O

MODES = ("single", "head-batch", "tail-batch")


def _tables(name, E, R, d, gamma, seed):
    ent, rel, mod, rng = synth_tables(name, E, R, d, gamma, seed)
    return torch.from_numpy(ent), torch.from_numpy(rel), (None if mod is None else torch.from_numpy(mod)), rng


@pytest.mark.parametrize("tag,E,R,d,B,n,gamma,seed", [("small", 64, 8, 16, 4, 8, 12.0, 11),
                                                       ("d1000", 128, 16, 1000, 8, 16, 24.0, 12)])
@pytest.mark.parametrize("name", ["TransE", "DistMult", "ComplEx", "RotatE", "pRotatE"])
def test_oracle_scores(g_scores, tag, E, R, d, B, n, gamma, seed, name):
    ent, rel, mod, rng = _tables(name, E, R, d, gamma, seed)
    pos, neg, _ = synth.kge_batch(seed, B, n, E, R)
    P, N = torch.from_numpy(pos), torch.from_numpy(neg)
    g = torch.Tensor([gamma]).item()
    for mode in MODES:
        s = O.forward(name, ent, rel, mod, P if mode == "single" else (P, N), mode, g, rng).numpy()
        ref = g_scores[f"{tag}/{name}/{mode}"]
        # same ATen op chain: bitwise on the generating machine, ~1 ulp across SIMD levels
        np.testing.assert_allclose(s, ref, rtol=2e-6, atol=2e-6 * max(1.0, np.abs(ref).max()))


@pytest.mark.parametrize("tag,E,R,d,B,n,gamma,seed", [("small", 64, 8, 16, 4, 8, 12.0, 11),
                                                       ("d1000", 128, 16, 1000, 8, 16, 24.0, 12)])
@pytest.mark.parametrize("name", ["TransE", "DistMult", "ComplEx", "RotatE", "pRotatE"])
def test_reference_operation_order(g_scores, tag, E, R, d, B, n, gamma, seed, name):
    """The element-by-element restatement of the reference's fp32 operations
    (O.ref_order_scores: ATen's sum(dim=2) order, torch.norm(p=1)'s sequential
    sum, RotatE's sqrt(fma(im, im, re*re))) reproduces the reference's golden
    scores BIT FOR BIT — the order the HIP ranking refinement implements
    (csrc/kge_rank_ref.h).  The transcendentals here are torch's, as in the
    reference; the kernels round cos/sin correctly instead."""
    if torch.backends.cpu.get_cpu_capability() not in ("AVX2", "AVX512"):
        pytest.skip("the golden scores were made with AVX2/AVX512 ATen kernels")
    ent, rel, mod, rng = synth_tables(name, E, R, d, gamma, seed)
    pos, neg, _ = synth.kge_batch(seed, B, n, E, R)
    P, N = torch.from_numpy(pos), torch.from_numpy(neg)
    g = torch.Tensor([gamma]).item()
    for mode in MODES:
        s = O.ref_order_scores(name, ent, rel, mod, P if mode == "single" else (P, N), mode, g, rng)
        ref = g_scores[f"{tag}/{name}/{mode}"]
        assert s.dtype == np.float32 and s.shape == ref.shape
        np.testing.assert_array_equal(s.view(np.int32), ref.view(np.int32), err_msg=f"{name} {mode}")


@pytest.mark.parametrize("d", [8, 9, 15, 16, 17, 31, 100, 127, 128, 500, 511, 512, 1000, 2000, 4100])
def test_aten_sum_order(d):
    """O.aten_sum_lastdim is torch's CPU sum(dim=-1), bit for bit, for every
    tail shape (scalar tail, vector tail, partial and full cascade blocks)."""
    if torch.backends.cpu.get_cpu_capability() not in ("AVX2", "AVX512"):
        pytest.skip("order restated for the AVX2/AVX512 ATen kernels")
    x = (np.random.default_rng(d).standard_normal((37, d)) * 0.01).astype(np.float32)
    np.testing.assert_array_equal(O.aten_sum_lastdim(x).view(np.int32), torch.from_numpy(x).sum(-1).numpy().view(np.int32))


def test_oracle_train(g_train, golden_info):
    ti = golden_info["train"]
    E, R, d, B, n, gamma, seed = ti["E"], ti["R"], ti["d"], ti["B"], ti["n"], ti["gamma"], ti["seed"]
    g = torch.Tensor([gamma]).item()
    for ci, case in enumerate(ti["cases"]):
        name = case["model"]
        ent, rel, mod, rng = _tables(name, E, R, d, gamma, seed)
        pos, neg, w = synth.kge_batch(seed + ci, B, n, E, R)
        log, ge, gr, gm = O.train_grads(name, ent, rel, mod, torch.from_numpy(pos), torch.from_numpy(neg),
                                        torch.from_numpy(w), case["mode"], adversarial=case["adversarial"],
                                        temperature=ti["adversarial_temperature"], uni_weight=case["uni_weight"],
                                        regularization=case["regularization"], gamma=g, erange=rng)
        ref_log = g_train[f"{ci}/log"]
        got = np.array([log["positive_sample_loss"], log["negative_sample_loss"], log["loss"],
                        log.get("regularization", 0.0)])
        np.testing.assert_allclose(got, ref_log, rtol=1e-6, atol=1e-7, err_msg=str(case))
        for key, val in (("grad_entity", ge), ("grad_relation", gr)):
            ref = g_train[f"{ci}/{key}"]
            np.testing.assert_allclose(val.numpy(), ref, rtol=1e-5, atol=1e-6 * max(1e-3, np.abs(ref).max()),
                                       err_msg=f"{case} {key}")
        if name == "pRotatE":
            np.testing.assert_allclose(gm.numpy(), g_train[f"{ci}/grad_modulus"], rtol=1e-5)
        # two Adam steps (the second recomputed on the updated tables) against the reference's params
        if ci % 5 == 0:
            params = [ent, rel] + ([mod] if mod is not None else [])
            grads1 = [ge, gr] + ([gm] if gm is not None else [])
            p1, _ = O.adam_steps(params, [grads1], lr=ti["lr"])
            _, ge2, gr2, gm2 = O.train_grads(name, p1[0], p1[1], p1[2] if mod is not None else None,
                                            torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w),
                                            case["mode"], adversarial=case["adversarial"],
                                            temperature=ti["adversarial_temperature"], uni_weight=case["uni_weight"],
                                            regularization=case["regularization"], gamma=g, erange=rng)
            grads2 = [ge2, gr2] + ([gm2] if gm2 is not None else [])
            p2, _ = O.adam_steps(params, [grads1, grads2], lr=ti["lr"])
            np.testing.assert_allclose(p2[0].numpy(), g_train[f"{ci}/param2_entity"], rtol=1e-5, atol=1e-7)
            np.testing.assert_allclose(p2[1].numpy(), g_train[f"{ci}/param2_relation"], rtol=1e-5, atol=1e-7)


def test_oracle_ranks(g_ranks, golden_info):
    for kg in golden_info["ranks"]:
        tag, E, R, d, seed = kg["tag"], kg["E"], kg["R"], kg["d"], kg["seed"]
        all_true = g_ranks[f"{tag}/all_true"]
        test = g_ranks[f"{tag}/test"]
        for name in kg["models"]:
            ent, rel, mod, rng = _tables(name, E, R, d, kg["gamma"], seed)
            g = torch.Tensor([kg["gamma"]]).item()
            ranks_all = []
            for mode in ("head-batch", "tail-batch"):
                r = O.filtered_ranks(name, ent, rel, mod, test, all_true, mode, g, rng)
                ref = g_ranks[f"{tag}/{name}/{mode}/rank"]
                # the reference's argsort position: identical where no exact tie with the positive
                clean = r["ties"] == 0
                np.testing.assert_array_equal(r["rank_argsort"][clean], ref[clean], err_msg=f"{tag} {name} {mode}")
                np.testing.assert_array_equal(r["rank_count"][clean], ref[clean])
                # with ties, the reference rank lies in [count, count + ties]
                assert np.all(ref >= r["rank_count"]) and np.all(ref <= r["rank_count"] + r["ties"])
                ranks_all.append(ref)
            met = O.metrics_from_ranks(np.concatenate(ranks_all))
            ref_met = g_ranks[f"{tag}/{name}/metrics"]
            got = np.array([met[k] for k in golden_info["metric_order"]])
            np.testing.assert_allclose(got, ref_met, rtol=0, atol=1e-12)


def test_oracle_testdataset_semantics(g_ranks):
    all_true = set(map(tuple, g_ranks["kg_small/all_true"].tolist()))
    test = g_ranks["kg_small/test"].tolist()
    for mode in ("head-batch", "tail-batch"):
        for k in range(3):
            cand, bias = O.filtered_candidates(test[k], all_true, 40, mode)
            np.testing.assert_array_equal(cand, g_ranks[f"testds/{mode}/{k}/neg"])
            np.testing.assert_array_equal(bias, g_ranks[f"testds/{mode}/{k}/bias"])


def test_oracle_countries(g_countries, golden_info):
    from sklearn.metrics import average_precision_score
    ci = golden_info["countries"]
    ent, rel, mod, rng = _tables("TransE", ci["nentity"], ci["nrelation"], ci["d"], ci["gamma"], ci["seed"])
    test, regions = g_countries["test"], g_countries["regions"]
    sample = torch.LongTensor([(h, r, c) for h, r, _ in test.tolist() for c in regions.tolist()])
    y = O.forward("TransE", ent, rel, None, sample, "single", torch.Tensor([ci["gamma"]]).item(), rng)
    y = y.squeeze(1).numpy()
    np.testing.assert_allclose(y, g_countries["y_score"], rtol=1e-6, atol=1e-7)
    y_true = np.array([1 if c == t else 0 for _, _, t in test.tolist() for c in regions.tolist()])
    assert abs(average_precision_score(y_true, y) - g_countries["auc_pr"][0]) < 1e-9


def test_reference_trig_fixture_against_host():
    """tests/golden/rotate_trig.npz holds the reference's own cos / sin bits of
    RotatE's relation phases (model.py:209-212) as an XOR against correctly
    rounded values.  The XOR is sparse (the vector library is within an ulp),
    and this host's torch.cos / torch.sin (ops.reference_rotation — what
    KGEModel's ranking uses) give exactly the committed bits when the host's
    CPU vector library matches the one the fixtures were made with."""
    import torch
    from conftest import erange_of
    from knowledgegraphembedding_amd import ops, synth
    g = load_npz("rotate_trig.npz")
    info = {c["tag"]: c for c in json.load(open(GOLDEN / "golden.json"))["rotate_trig"]}
    seeds = {"kg_small": (40, 31, 12.0), "kg_mid": (1500, 32, 12.0), "fb15k": (14951, 62, 24.0)}
    differ = []
    for tag, (E, seed, gamma) in seeds.items():
        R, d = info[tag]["R"], info[tag]["d"]
        rng = erange_of(gamma, d)
        _, rel = synth.kge_tables(seed, E, R, 2 * d, d, rng)
        ids = g[f"{tag}/rel_ids"]
        xc, xs = g[f"{tag}/cos_xor"], g[f"{tag}/sin_xor"]
        assert xc.shape == (len(ids), d) and 0 < (xc != 0).mean() < 0.1 and 0 < (xs != 0).mean() < 0.1
        ph64 = (torch.from_numpy(rel) / (rng / ops.PI)).numpy().astype(np.float64)[ids]
        ref_c = np.cos(ph64).astype(np.float32).view(np.uint32) ^ xc
        ref_s = np.sin(ph64).astype(np.float32).view(np.uint32) ^ xs
        host = ops.reference_rotation(torch.from_numpy(rel), rng).numpy()[ids]
        differ.append(float((host[:, 0].view(np.uint32) != ref_c).mean() + (host[:, 1].view(np.uint32) != ref_s).mean()))
    if any(differ):
        pytest.skip(f"this host's CPU cos/sin differ from the reference's on {differ} of the fixture values "
                    "(the GPU parity test ranks with the committed bits)")
