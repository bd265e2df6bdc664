"""Training batches produced on the GPU.

The reference builds every training batch on CPU worker processes:
``TrainDataset.__getitem__`` draws negatives with numpy and rejects true
heads/tails (dataloader.py:34-61), ``collate_fn`` stacks them (:63-66), a
shuffling ``DataLoader`` orders the triples (run.py:240-255) and
``BidirectionalOneShotIterator`` alternates tail-/head-batch forever
(dataloader.py:165-186).  That host pipeline delivers ~14 k positives/s per
process, far below what the fused training kernels consume.

``DeviceTrainIterator`` is the same iterator protocol with the whole batch
built on the device by one kernel launch (kge_sample_negatives):

  * per-epoch shuffle: ``torch.randperm`` of the triple ids on the device
    (DataLoader(shuffle=True)), consecutive slices of ``batch_size`` with the
    last one short (drop_last=False);
  * negatives: for each positive, the first n draws of a per-row uniform
    stream over [0, nentity) that are not true heads of (r, t) (head-batch) /
    true tails of (h, r) (tail-batch) — the distribution of the reference's
    draw-2n-reject-repeat-truncate loop;
  * subsampling weights ``sqrt(1 / (count(h,r) + count(t,-r-1)))`` computed
    once with the reference's fp32 arithmetic (dataloader.py:40-42, :68-85).

The per-triple true lists are a CSR built once on the host (``TrueLists``).
The reference's stream is numpy's MT19937, so batches are not
sample-identical to a reference run; the sampler is tested bit-exact against
its own restatement (oracle) and against the reference's invariants.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops

_MASK64 = (1 << 64) - 1
_WEYL = 0x9E3779B97F4A7C15


def _mix64(z: int) -> int:
    z &= _MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def batch_key(seed: int, batch_no: int) -> int:
    """The kernel key of the batch_no-th batch of a stream seeded with `seed`."""
    return _mix64(_mix64(seed) + batch_no * _WEYL)


def _group_lists(key: np.ndarray, member: np.ndarray, span: int):
    """Sorted unique members per key; per-row (offset, length) into the id array."""
    pair = np.unique(key * span + member)
    gkey = pair // span
    ids = (pair - gkey * span).astype(np.int64)
    ukey, start = np.unique(gkey, return_index=True)
    length = np.diff(np.append(start, len(pair)))
    slot = np.searchsorted(ukey, key)
    return start[slot].astype(np.int64), length[slot].astype(np.int32), ids


class TrueLists:
    """Per-triple true-tail / true-head lists and subsampling weights
    (TrainDataset.get_true_head_and_tail / count_frequency, dataloader.py:68-85)."""

    def __init__(self, triples, nentity: int, nrelation: int):
        tr = np.asarray(triples, dtype=np.int64).reshape(-1, 3)
        h, r, t = tr[:, 0], tr[:, 1], tr[:, 2]
        E, R = int(nentity), int(nrelation)
        if R * E * E >= 2 ** 62:
            raise ValueError("entity/relation counts too large for the packed (key, member) sort")
        self.triples = tr
        # true tails of (h, r) for tail-batch, true heads of (r, t) for head-batch
        self.tail_off, self.tail_len, self.tail_ids = _group_lists(h * R + r, t, E)
        self.head_off, self.head_len, self.head_ids = _group_lists(r * E + t, h, E)
        # count(h, r) + count(t, -r-1), each starting at 4 (count_frequency(start=4)), over the triple list
        _, inv_hr, cnt_hr = np.unique(h * R + r, return_inverse=True, return_counts=True)
        _, inv_tr, cnt_tr = np.unique(t * R + r, return_inverse=True, return_counts=True)
        total = (cnt_hr[inv_hr] + 3) + (cnt_tr[inv_tr] + 3)
        # torch.sqrt(1 / torch.Tensor([w])) per positive, dataloader.py:41-42 (fp32 throughout)
        self.weights = torch.sqrt(1 / torch.tensor(total.astype(np.float64), dtype=torch.float32)).numpy()

    def lists(self, mode: str):
        if mode == 'head-batch':
            return self.head_off, self.head_len, self.head_ids
        if mode == 'tail-batch':
            return self.tail_off, self.tail_len, self.tail_ids
        raise ValueError('negative batch mode %s not supported' % mode)


class DeviceTrainIterator:
    """``next()`` → (positive_sample [B,3] int64, negative_sample [B,n] int64,
    subsampling_weight [B] fp32, mode), all on `device`, tail-batch first and
    then alternating — BidirectionalOneShotIterator's protocol
    (dataloader.py:165-186) over two shuffled TrainDataset loaders.

    Data parallel (world > 1): every rank draws the same per-epoch permutation
    (from `perm_seed`, which must be equal on all ranks) and takes positions
    rank, rank + world, ... of its first world·⌊T/world⌋ — disjoint shards of
    equal length, as RankShardSampler gives the host loaders; the negatives'
    streams are keyed by the rank's own `seed`."""

    def __init__(self, train_triples, nentity: int, nrelation: int, negative_sample_size: int, batch_size: int,
                 device, seed: int = 0, max_draws: int | None = None, rank: int = 0, world: int = 1,
                 perm_seed: int | None = None):
        dev = torch.device(device)
        ops._require_device(torch.empty(0, device=dev))
        self.lists = TrueLists(train_triples, nentity, nrelation)
        self.dev = dev
        self.nentity, self.n, self.batch_size = int(nentity), int(negative_sample_size), int(batch_size)
        if self.batch_size <= 0 or self.n < 0 or len(self.lists.triples) == 0:
            raise ValueError('empty training set or non-positive batch size')
        self.max_draws = int(max_draws) if max_draws else max(1 << 20, 1024 * (self.n + 64))
        self.triples = torch.from_numpy(self.lists.triples).to(dev)
        self.weights = torch.from_numpy(self.lists.weights).to(dev)
        self._dev_lists = {}
        for mode in ('head-batch', 'tail-batch'):
            off, ln, ids = self.lists.lists(mode)
            self._dev_lists[mode] = (torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev),
                                     torch.from_numpy(ids).to(dev) if len(ids) else torch.zeros(1, dtype=torch.int64,
                                                                                                device=dev))
        self.seed = int(seed)
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        if self.triples.shape[0] < world:  # each rank's epoch shard would be empty: endless empty batches
            raise ValueError(f"{self.triples.shape[0]} training triples cannot be sharded over {world} ranks")
        self.rank, self.world = int(rank), int(world)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(self.seed if perm_seed is None else int(perm_seed))
        self._perm = {'head-batch': None, 'tail-batch': None}
        self._cursor = {'head-batch': 0, 'tail-batch': 0}
        self.step = 0
        self.batch_no = 0

    def __iter__(self):
        return self

    def _indices(self, mode: str) -> torch.Tensor:
        T = self.triples.shape[0] // self.world  # this rank's shard of an epoch
        if self._perm[mode] is None or self._cursor[mode] >= T:  # a new epoch of this loader
            perm = torch.randperm(self.triples.shape[0], device=self.dev, generator=self.gen)
            self._perm[mode] = perm[self.rank:self.world * T:self.world]
            self._cursor[mode] = 0
        c = self._cursor[mode]
        self._cursor[mode] = c + self.batch_size
        return self._perm[mode][c:c + self.batch_size]

    def sample(self, batch: torch.Tensor, mode: str):
        """The TrainDataset batch for the given triple ids (one kernel launch)."""
        B = batch.shape[0]
        pos = torch.empty(B, 3, dtype=torch.int64, device=self.dev)
        neg = torch.empty(B, self.n, dtype=torch.int64, device=self.dev)
        w = torch.empty(B, dtype=torch.float32, device=self.dev)
        off, ln, ids = self._dev_lists[mode]
        key = batch_key(self.seed, self.batch_no)
        self.batch_no += 1
        ops.sample_negatives(self.triples, batch.contiguous(), self.nentity, self.n, off, ln, ids, self.weights, key,
                             self.max_draws, pos, neg, w)
        return pos, neg, w, mode

    def __next__(self):
        self.step += 1
        mode = 'head-batch' if self.step % 2 == 0 else 'tail-batch'
        return self.sample(self._indices(mode), mode)
