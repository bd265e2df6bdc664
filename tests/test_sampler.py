"""Device negative sampler (sampler.py, kge_sample_negatives) — SURVEY §8f row 1.

Pinning: the true-head/true-tail lists and the subsampling weights are
checked against the oracle restatement of dataloader.py:68-85 and against the
reference's own weights (tests/golden/sampler.npz, made by importing the
reference).  The negatives come from the build's counter-based stream, not
numpy's MT19937, so a reference run's negatives are not reproducible; the GPU
tests check the kernel bit-exact against the oracle's restatement of that
stream, and the reference's invariants: no true head/tail is ever drawn, the
draws are uniform over the allowed entities, shapes/dtypes/modes follow
TrainDataset + BidirectionalOneShotIterator.
"""
import numpy as np
import pytest
import torch
from scipy import stats

from knowledgegraphembedding_amd import synth
from knowledgegraphembedding_amd.sampler import TrueLists, batch_key
from oracle import kge_oracle as O


def _graph(seed, E, R, T):
    h = synth.randint(seed * 3 + 1, (T,), E)
    r = synth.randint(seed * 3 + 2, (T,), R)
    t = synth.randint(seed * 3 + 3, (T,), E)
    return np.stack([h, r, t], 1).astype(np.int64)


# ------------------------------------------------------------------ CPU
def test_true_lists_match_reference_semantics(g_sampler):
    for triples, E, R in ((g_sampler["triples"], 50, 4), (_graph(7, 200, 9, 3000), 200, 9)):
        tl = TrueLists(triples, E, R)
        for mode in ("head-batch", "tail-batch"):
            ref = O.true_lists(triples, mode)
            off, ln, ids = tl.lists(mode)
            for k, (h, r, t) in enumerate(triples.tolist()):
                want = ref[(r, t)] if mode == "head-batch" else ref[(h, r)]
                np.testing.assert_array_equal(ids[off[k]:off[k] + ln[k]], want)


def test_weights_match_reference(g_sampler):
    triples = g_sampler["triples"]
    tl = TrueLists(triples, 50, 4)
    # the reference's own weights for triples 0..11 (TrainDataset[k], dataloader.py:40-42)
    for mode in ("head-batch", "tail-batch"):
        np.testing.assert_array_equal(tl.weights[:12], g_sampler[f"{mode}/w"])
    np.testing.assert_array_equal(tl.weights, O.subsampling_weights(triples))
    big = _graph(8, 300, 5, 4000)
    np.testing.assert_array_equal(TrueLists(big, 300, 5).weights, O.subsampling_weights(big))


def test_oracle_sampler_invariants():
    triples = _graph(9, 40, 3, 500)
    for mode in ("head-batch", "tail-batch"):
        pos, neg, ok = O.sample_negatives(triples, np.arange(64), 40, 32, mode, batch_key(1, 0), 1 << 16)
        assert ok.all()
        lists = O.true_lists(triples, mode)
        for i, (h, r, t) in enumerate(pos.tolist()):
            tl = lists[(r, t)] if mode == "head-batch" else lists[(h, r)]
            assert not np.isin(neg[i], tl).any()
            assert ((neg[i] >= 0) & (neg[i] < 40)).all()


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_device_sampler_bit_exact_vs_oracle(g_sampler, mode):
    from knowledgegraphembedding_amd.sampler import DeviceTrainIterator
    triples = g_sampler["triples"]
    it = DeviceTrainIterator(triples, 50, 4, 16, 300, "cuda:0", seed=11)
    batch = torch.arange(len(triples), device="cuda:0").flip(0).contiguous()
    key = batch_key(11, it.batch_no)
    pos, neg, w, m = it.sample(batch, mode)
    opos, oneg, ok = O.sample_negatives(triples, batch.cpu().numpy(), 50, 16, mode, key, it.max_draws)
    assert ok.all() and m == mode
    np.testing.assert_array_equal(pos.cpu().numpy(), opos)
    np.testing.assert_array_equal(neg.cpu().numpy(), oneg)
    np.testing.assert_array_equal(w.cpu().numpy(), TrueLists(triples, 50, 4).weights[batch.cpu().numpy()])


@pytest.mark.gpu
def test_device_sampler_uniform_over_allowed():
    """One positive repeated: its negatives must be uniform over the non-true entities."""
    from knowledgegraphembedding_amd.sampler import DeviceTrainIterator
    E = 60
    triples = np.array([[3, 0, t] for t in range(0, 60, 3)] + [[5, 1, 7]], dtype=np.int64)  # (3, 0) has 20 tails
    it = DeviceTrainIterator(triples, E, 2, 128, 1, "cuda:0", seed=3)
    batch = torch.zeros(2048, dtype=torch.int64, device="cuda:0")  # triple 0 = (3, 0, 0)
    _, neg, _, _ = it.sample(batch, "tail-batch")
    v = neg.cpu().numpy().ravel()
    allowed = np.array([e for e in range(E) if e % 3 != 0])
    assert np.isin(v, allowed).all()
    counts = np.bincount(v, minlength=E)[allowed]
    chi2, p = stats.chisquare(counts)
    assert p > 1e-4, (chi2, p)


@pytest.mark.gpu
def test_device_iterator_epochs_and_modes():
    from knowledgegraphembedding_amd.sampler import DeviceTrainIterator
    triples = _graph(10, 100, 6, 1000)
    it = DeviceTrainIterator(triples, 100, 6, 8, 96, "cuda:0", seed=5)
    seen = {"head-batch": [], "tail-batch": []}
    sizes = []
    for k in range(22):  # 11 batches per mode = one epoch of 1000 triples (10 × 96 + 40)
        pos, neg, w, mode = next(it)
        assert mode == ("tail-batch" if k % 2 == 0 else "head-batch")
        assert pos.dtype == torch.int64 and neg.dtype == torch.int64 and w.dtype == torch.float32
        assert neg.shape == (pos.shape[0], 8) and w.shape == (pos.shape[0],)
        seen[mode].append(pos.cpu().numpy())
        sizes.append(pos.shape[0])
    assert sizes[-2:] == [40, 40]
    for mode in seen:
        got = np.concatenate(seen[mode])
        key = lambda a: np.sort(a[:, 0] * 10 ** 6 + a[:, 1] * 10 ** 3 + a[:, 2])  # noqa: E731
        np.testing.assert_array_equal(key(got), key(triples))  # every triple exactly once per epoch


@pytest.mark.gpu
def test_device_sampler_exhaustion_raises():
    from knowledgegraphembedding_amd import ops
    from knowledgegraphembedding_amd.sampler import DeviceTrainIterator
    triples = np.array([[0, 0, t] for t in range(10)], dtype=np.int64)  # every entity is a true tail of (0, 0)
    it = DeviceTrainIterator(triples, 10, 1, 4, 2, "cuda:0", max_draws=4096)
    it.sample(torch.zeros(1, dtype=torch.int64, device="cuda:0"), "tail-batch")
    with pytest.raises(RuntimeError, match="negative sampler"):
        ops.raise_on_device_error(torch.device("cuda:0"))
