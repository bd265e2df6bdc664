"""TrainDataset / TestDataset / BidirectionalOneShotIterator — the reference's
data API (codes/dataloader.py), unchanged in behaviour.

TrainDataset draws its negatives with the same numpy calls in the same order
(dataloader.py:39-61), so a seeded numpy RNG yields the reference's exact
batches; it remains host-side CPU work feeding the device.
TestDataset keeps its item format for API users; KGEModel.test_step itself
ranks through filters.FilterIndex + the ranking kernel instead.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import Dataset

from .filters import FilterIndex


class TrainDataset(Dataset):
    def __init__(self, triples, nentity, nrelation, negative_sample_size, mode):
        self.len = len(triples)
        self.triples = triples
        self.triple_set = set(triples)
        self.nentity = nentity
        self.nrelation = nrelation
        self.negative_sample_size = negative_sample_size
        self.mode = mode
        self.count = self.count_frequency(triples)
        self.true_head, self.true_tail = self.get_true_head_and_tail(self.triples)

    def __len__(self):
        return self.len

    def __getitem__(self, idx):
        positive_sample = self.triples[idx]
        head, relation, tail = positive_sample

        # word2vec-style subsampling weight, fp32 like dataloader.py:33-34
        subsampling_weight = self.count[(head, relation)] + self.count[(tail, -relation - 1)]
        subsampling_weight = torch.sqrt(1 / torch.Tensor([subsampling_weight]))

        if self.mode == 'head-batch':
            true_ids = self.true_head[(relation, tail)]
        elif self.mode == 'tail-batch':
            true_ids = self.true_tail[(head, relation)]
        else:
            raise ValueError('Training batch mode %s not supported' % self.mode)

        # rejection sampling: draw 2n uniform ids per round, drop the true ones
        chunks = []
        have = 0
        while have < self.negative_sample_size:
            draw = np.random.randint(self.nentity, size=self.negative_sample_size * 2)
            draw = draw[np.isin(draw, true_ids, assume_unique=True, invert=True)]
            chunks.append(draw)
            have += draw.size
        negative_sample = torch.from_numpy(np.concatenate(chunks)[:self.negative_sample_size])
        return torch.LongTensor(positive_sample), negative_sample, subsampling_weight, self.mode

    @staticmethod
    def collate_fn(data):
        positive_sample = torch.stack([d[0] for d in data], dim=0)
        negative_sample = torch.stack([d[1] for d in data], dim=0)
        subsample_weight = torch.cat([d[2] for d in data], dim=0)
        return positive_sample, negative_sample, subsample_weight, data[0][3]

    @staticmethod
    def count_frequency(triples, start=4):
        '''Frequency of (head, relation) and (tail, -relation-1), starting at `start`.'''
        count = {}
        for head, relation, tail in triples:
            count[(head, relation)] = count.get((head, relation), start - 1) + 1
            count[(tail, -relation - 1)] = count.get((tail, -relation - 1), start - 1) + 1
        return count

    @staticmethod
    def get_true_head_and_tail(triples):
        '''True heads per (relation, tail) and true tails per (head, relation).'''
        true_head, true_tail = {}, {}
        for head, relation, tail in triples:
            true_tail.setdefault((head, relation), []).append(tail)
            true_head.setdefault((relation, tail), []).append(head)
        true_head = {k: np.array(list(set(v))) for k, v in true_head.items()}
        true_tail = {k: np.array(list(set(v))) for k, v in true_tail.items()}
        return true_head, true_tail

    # The copy a DataLoader worker receives.  run.py starts its workers from a
    # forkserver (run.worker_context), so every worker unpickles the dataset;
    # the reference's dicts keyed by tuples take ≈ 8 s to pickle at FB15k's
    # size (483 k triples), once per worker and epoch.  Workers only call
    # __getitem__, so they get the triples and this mode's tables as flat
    # sorted arrays (≈ 15 MB, milliseconds) and look them up by binary search:
    # the same values (counts, the same true id sets — np.isin's result does
    # not depend on their order) and the same numpy calls in the same order,
    # so the same batches (tests/test_run_shard.py).
    def __getstate__(self):
        cached = self.__dict__.get('_compact')
        if cached is not None:  # built once: every later worker start pickles only the arrays
            return cached
        t = np.asarray(self.triples, dtype=np.int64).reshape(-1, 3)
        E, R = int(self.nentity), int(self.nrelation)
        h, r, tl = t[:, 0], t[:, 1], t[:, 2]
        # count[(x, y)] = start - 1 + occurrences, y = relation or -relation - 1
        ck, cn = np.unique(np.concatenate([h * (2 * R) + (r + R), tl * (2 * R) + (R - 1 - r)]), return_counts=True)
        if self.mode == 'head-batch':
            key, val = r * E + tl, h        # true_head[(relation, tail)]
        else:
            key, val = h * R + r, tl        # true_tail[(head, relation)]
        kv = np.unique(np.stack([key, val], 1), axis=0)
        tk, start = np.unique(kv[:, 0], return_index=True)
        state = {'compact': True, 'len': self.len, 'nentity': E, 'nrelation': R,
                 'negative_sample_size': self.negative_sample_size, 'mode': self.mode, 'triples': t,
                 'count_keys': ck, 'count_vals': cn + 3, 'true_keys': tk,
                 'true_off': np.append(start, len(kv)), 'true_ids': kv[:, 1].copy()}
        self.__dict__['_compact'] = state
        return state

    def __setstate__(self, st):
        E, R = st['nentity'], st['nrelation']
        self.len, self.nentity, self.nrelation = st['len'], E, R
        self.negative_sample_size, self.mode = st['negative_sample_size'], st['mode']
        self.triples = _TripleRows(st['triples'])
        self.count = _CountTable(st['count_keys'], st['count_vals'], R)
        table = _TrueTable(st['true_keys'], st['true_off'], st['true_ids'], E if self.mode == 'head-batch' else R)
        self.true_head, self.true_tail = (table, None) if self.mode == 'head-batch' else (None, table)


class _TripleRows:
    """triples[idx] → (h, r, t) of Python ints, from an [n, 3] array."""

    def __init__(self, arr):
        self.arr = arr

    def __len__(self):
        return len(self.arr)

    def __getitem__(self, idx):
        h, r, t = self.arr[idx].tolist()
        return h, r, t


class _CountTable:
    """count[(x, y)] of TrainDataset.count_frequency from sorted keys x·2R + (y + R)."""

    def __init__(self, keys, vals, R):
        self.keys, self.vals, self.R = keys, vals, R

    def __getitem__(self, k):
        key = k[0] * (2 * self.R) + (k[1] + self.R)
        i = int(np.searchsorted(self.keys, key))
        if i == len(self.keys) or self.keys[i] != key:
            raise KeyError(k)
        return int(self.vals[i])


class _TrueTable:
    """true_head[(r, t)] / true_tail[(h, r)] from sorted keys a·M + b and a CSR of ids."""

    def __init__(self, keys, off, ids, M):
        self.keys, self.off, self.ids, self.M = keys, off, ids, M

    def __getitem__(self, k):
        key = k[0] * self.M + k[1]
        i = int(np.searchsorted(self.keys, key))
        if i == len(self.keys) or self.keys[i] != key:
            raise KeyError(k)
        return self.ids[self.off[i]:self.off[i + 1]]


class TestDataset(Dataset):
    def __init__(self, triples, all_true_triples, nentity, nrelation, mode):
        self.len = len(triples)
        self.triple_set = set(all_true_triples)
        self.triples = triples
        self.nentity = nentity
        self.nrelation = nrelation
        self.mode = mode
        self._index = FilterIndex(list(self.triple_set), nentity, nrelation) if self.triple_set else None

    def __len__(self):
        return self.len

    def __getitem__(self, idx):
        head, relation, tail = self.triples[idx]
        if self.mode == 'head-batch':
            true_id = head
        elif self.mode == 'tail-batch':
            true_id = tail
        else:
            raise ValueError('negative batch mode %s not supported' % self.mode)
        negative_sample = torch.arange(self.nentity, dtype=torch.int64)
        filter_bias = torch.zeros(self.nentity, dtype=torch.float32)
        if self._index is not None:
            f = torch.from_numpy(self._index.filtered((head, relation, tail), self.mode))
            negative_sample[f] = true_id  # filtered candidate -> (-1, true id), dataloader.py:138-144
            filter_bias[f] = -1.0
        positive_sample = torch.LongTensor((head, relation, tail))
        return positive_sample, negative_sample, filter_bias, self.mode

    @staticmethod
    def collate_fn(data):
        positive_sample = torch.stack([d[0] for d in data], dim=0)
        negative_sample = torch.stack([d[1] for d in data], dim=0)
        filter_bias = torch.stack([d[2] for d in data], dim=0)
        return positive_sample, negative_sample, filter_bias, data[0][3]


class BidirectionalOneShotIterator(object):
    '''Alternates tail-batch (odd steps) and head-batch (even steps) batches.'''

    def __init__(self, dataloader_head, dataloader_tail):
        self.iterator_head = self.one_shot_iterator(dataloader_head)
        self.iterator_tail = self.one_shot_iterator(dataloader_tail)
        self.step = 0

    def __iter__(self):
        return self

    def __next__(self):
        self.step += 1
        if self.step % 2 == 0:
            return next(self.iterator_head)
        return next(self.iterator_tail)

    @staticmethod
    def one_shot_iterator(dataloader):
        '''Endless iterator over a DataLoader.'''
        while True:
            for data in dataloader:
                yield data


class RankShardSampler(torch.utils.data.Sampler):
    """Data-parallel training order: each epoch one permutation of the whole
    train set, drawn from a generator seeded by (seed, epoch) and therefore the
    same on every rank, of which rank r takes positions r, r + world, ... of
    the first world·⌊n/world⌋.  Every rank's shard has the same length, so the
    ranks' batches have the same size at every step (the factor / owner /
    query-shipping exchanges all-gather per-row buffers of equal shape); the
    n mod world positives at the end of an epoch's permutation — different
    ones every epoch, as each epoch's permutation is drawn independently —
    are not visited in that epoch.  `seed` must be the same on every rank
    (run.py broadcasts rank 0's).  The ranks' positives are disjoint
    within an epoch; the epoch advances on every new iteration
    (BidirectionalOneShotIterator restarts the DataLoader endlessly), so no
    set_epoch call is needed.  With world = 1 this is a plain reshuffle per
    epoch."""

    def __init__(self, n: int, rank: int, world: int, seed: int):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        if n < world:  # every rank's shard would be empty: the DataLoader would yield nothing, forever
            raise ValueError(f"{n} training triples cannot be sharded over {world} ranks")
        self.n, self.rank, self.world, self.seed = int(n), int(rank), int(world), int(seed)
        self.epoch = 0

    def __len__(self):
        return self.n // self.world

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed * 1000003 + self.epoch)
        self.epoch += 1
        perm = torch.randperm(self.n, generator=g)
        return iter(perm[self.rank:self.world * len(self):self.world].tolist())
