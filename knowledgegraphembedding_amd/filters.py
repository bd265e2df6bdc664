"""Host-side index of true triples for filtered ranking.

The reference builds, per test query, an nentity-long Python list in which
every candidate that forms a true triple (all_true_triples = train + valid +
test, run.py:225) is replaced by (-1, true_id) (dataloader.py:134-154).  Here
the same set is kept as two sorted arrays (tails by (h, r), heads by (r, t))
and handed to the ranking kernel as a CSR of the filtered candidate ids of
each query — the true entity itself excluded, exactly as tmp[head] /
tmp[tail] = (0, id) re-admits it (dataloader.py:140, 144).
"""
from __future__ import annotations

import itertools

import numpy as np


def triples_array(triples) -> np.ndarray:
    """[n, 3] int64 from an array or from the reference's list of (h, r, t)
    tuples (run.py:225 passes lists): np.fromiter over the flattened tuples
    takes ≈0.4× np.asarray's time on a 592 k-triple list."""
    if isinstance(triples, list) and triples and isinstance(triples[0], tuple) and set(map(len, triples)) == {3}:
        return np.fromiter(itertools.chain.from_iterable(triples), dtype=np.int64,
                           count=3 * len(triples)).reshape(-1, 3)
    return np.asarray(triples, dtype=np.int64).reshape(-1, 3)


class FilterIndex:
    """`device`: the two sorted key orders are built there with torch (unique
    / sort of the packed keys — on a GPU, test_step's index for an FB15k-size
    graph in a few ms instead of ≈20 ms of numpy) and the host arrays are
    made from them only when a host method needs them (filter_csr)."""

    _HOST = ('_k_hr', '_tails', '_k_rt', '_heads')

    def __init__(self, all_true_triples, nentity: int, nrelation: int, device=None):
        t = triples_array(all_true_triples)
        self.nentity = int(nentity)
        self.nrelation = int(nrelation)
        R, E = self.nrelation, self.nentity
        self._on = None  # (device, {mode: (sorted keys, ids)}) when built on a GPU
        if device is not None and R * E * E < 2 ** 62 and len(t):
            import torch
            td = torch.from_numpy(t).to(device)
            hr_t = torch.unique((td[:, 0] * R + td[:, 1]) * E + td[:, 2])  # sorted: set(all_true_triples)
            k_hr, tails = hr_t // E, hr_t % E
            h, r = k_hr // R, k_hr % R
            rt_h = torch.sort((r * E + tails) * E + h).values
            self._on = (str(device), {'tail-batch': (k_hr, tails), 'head-batch': (rt_h // E, rt_h % E)})
            return
        self._build_host(t)

    def __getattr__(self, name):
        # the host arrays of an index built on the device, made on first use
        if name in FilterIndex._HOST and self.__dict__.get('_on') is not None:
            d = self._on[1]
            (kh, tl), (kr, hd) = d['tail-batch'], d['head-batch']
            for n, v in zip(FilterIndex._HOST, (kh, tl, kr, hd)):
                self.__dict__[n] = v.cpu().numpy()
            return self.__dict__[name]
        raise AttributeError(name)

    def _build_host(self, t):
        R, E = self.nrelation, self.nentity
        if R * E * E < 2 ** 62:
            # set(all_true_triples) (dataloader.py:125) and both orders as sorts
            # of packed int64 keys: ((h·R + r)·E + t) and ((r·E + t)·E + h)
            hr_t = np.unique((t[:, 0] * R + t[:, 1]) * E + t[:, 2])
            self._k_hr, self._tails = hr_t // E, hr_t % E
            h, r = self._k_hr // R, self._k_hr % R
            rt_h = np.sort((r * E + self._tails) * E + h)
            self._k_rt, self._heads = rt_h // E, rt_h % E
        else:
            t = np.unique(t, axis=0)
            k_hr = t[:, 0] * R + t[:, 1]
            o = np.lexsort((t[:, 2], k_hr))
            self._k_hr, self._tails = k_hr[o], t[o, 2]
            k_rt = t[:, 1] * E + t[:, 2]
            o = np.lexsort((t[:, 0], k_rt))
            self._k_rt, self._heads = k_rt[o], t[o, 0]

    # query keys (h·R + r or r·E + t) span E·R values: up to this many, the
    # [lo, hi) range of every key is tabulated once (two int32 arrays per mode)
    # and a lookup is one gather; above, binary searches of the sorted keys
    DENSE_KEYS = 1 << 22

    def _range(self, cand, keys, tag):
        if self.nentity * self.nrelation <= self.DENSE_KEYS:
            tab = getattr(self, tag, None)
            if tab is None:
                n = self.nentity * self.nrelation
                start = np.searchsorted(cand, np.arange(n + 1, dtype=np.int64), side='left').astype(np.int32)
                tab = start
                setattr(self, tag, tab)
            return tab[keys].astype(np.int64), tab[keys + 1].astype(np.int64)
        o = np.argsort(keys, kind='stable')  # sorted probes: the searches walk the array forward
        ks = keys[o]
        lo, hi = np.empty_like(keys), np.empty_like(keys)
        lo[o] = np.searchsorted(cand, ks, side='left')
        hi[o] = np.searchsorted(cand, ks, side='right')
        return lo, hi

    # key spaces up to this many get a dense start table on the device, built
    # there (8 B per key: FB15k's 20.1 M keys are 161 MB per direction)
    DEVICE_DENSE_KEYS = 1 << 26

    def device_table(self, mode: str, dev):
        """(start table [E·R + 1], ids) int64 on `dev` for KGE_RANK_FILTER_TABLE:
        key h·R + r → the true tails (tail-batch), r·E + t → the true heads
        (head-batch), sorted by key; None when the key space is too large for
        a dense table (filter_csr then).  Up to DENSE_KEYS keys the host's
        table is uploaded; above, the table is the device's binary search of
        every key in the sorted keys (the same start offsets).  Cached per
        device."""
        n = self.nentity * self.nrelation
        if n > self.DEVICE_DENSE_KEYS:
            return None
        cache = self.__dict__.setdefault('_dev_tables', {})
        k = (mode, str(dev))
        if k not in cache:
            import torch
            if self._on is not None and self._on[0] == str(dev):
                # built on this device: the table is the search of every key in its sorted keys
                self._sorted(mode)  # (mode check)
                cd, vals = self._on[1][mode]
                cache[k] = (torch.searchsorted(cd, torch.arange(n + 1, dtype=torch.int64, device=dev)), vals)
            elif n <= self.DENSE_KEYS:
                cache[k] = self._host_table_on(mode, dev)
            else:
                cand, vals = self._sorted(mode)
                cd = torch.from_numpy(np.ascontiguousarray(cand, dtype=np.int64)).to(dev)
                tab = torch.searchsorted(cd, torch.arange(n + 1, dtype=torch.int64, device=dev))
                cache[k] = (tab, torch.from_numpy(np.ascontiguousarray(vals, dtype=np.int64)).to(dev))
        return cache[k]

    def _sorted(self, mode: str):
        if mode not in ('tail-batch', 'head-batch'):
            raise ValueError('negative batch mode %s not supported' % mode)
        if self._on is not None:
            return self._on[1][mode]
        return (self._k_hr, self._tails) if mode == 'tail-batch' else (self._k_rt, self._heads)

    def _host_table_on(self, mode: str, dev):
        import torch
        self._sorted(mode)  # (mode check)
        cand, vals = (self._k_hr, self._tails) if mode == 'tail-batch' else (self._k_rt, self._heads)
        tag = '_tab_hr' if mode == 'tail-batch' else '_tab_rt'
        self._range(cand, np.zeros(1, dtype=np.int64), tag)  # builds the dense start table
        return (torch.from_numpy(getattr(self, tag).astype(np.int64)).to(dev),
                torch.from_numpy(np.ascontiguousarray(vals, dtype=np.int64)).to(dev))

    def filter_csr(self, queries, mode: str):
        """(offsets [nq+1] int64, ids int64) of the filtered candidates per query."""
        q = np.asarray(queries, dtype=np.int64).reshape(-1, 3)
        if mode == 'tail-batch':
            keys, vals, cand = q[:, 0] * self.nrelation + q[:, 1], self._tails, self._k_hr
            true = q[:, 2]
        elif mode == 'head-batch':
            keys, vals, cand = q[:, 1] * self.nentity + q[:, 2], self._heads, self._k_rt
            true = q[:, 0]
        else:
            raise ValueError('negative batch mode %s not supported' % mode)
        lo, hi = self._range(cand, keys, '_tab_hr' if mode == 'tail-batch' else '_tab_rt')
        cnt = hi - lo
        total = int(cnt.sum())
        if total == 0:
            return np.zeros(len(q) + 1, dtype=np.int64), np.zeros(0, dtype=np.int64)
        starts = np.repeat(lo - np.concatenate(([0], np.cumsum(cnt)[:-1])), cnt)
        ids = vals[starts + np.arange(total)]
        owner = np.repeat(np.arange(len(q)), cnt)
        keep = ids != true[owner]
        ids, owner = ids[keep], owner[keep]
        per = np.bincount(owner, minlength=len(q))
        off = np.zeros(len(q) + 1, dtype=np.int64)
        np.cumsum(per, out=off[1:])
        return off, ids.astype(np.int64)

    def filtered(self, triple, mode: str) -> np.ndarray:
        off, ids = self.filter_csr([triple], mode)
        return ids[off[0]:off[1]]
