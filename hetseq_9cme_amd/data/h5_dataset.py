"""BERT pre-training shards in the NVIDIA HDF5 schema (reference
hetseq/data/h5pyDataset.py:13-134; schema SURVEY App. D).

Each sample is ``[input_ids, segment_ids, input_mask, masked_lm_labels,
next_sentence_labels]`` (int64; the positional order of
``BertForPreTraining.forward``), with ``masked_lm_labels`` = -1 except
``labels[pos[:n]] = ids[:n]`` where n is the first 0 in ``masked_lm_positions``.

Reads go through the native ``BertShardReader`` (keeps the file open, one
hyperslab read per key per run of consecutive rows, GIL released).  Besides
the per-sample ``__getitem__`` of the reference, ``read_batch(indices)`` returns
an already-collated batch written straight into (optionally pinned) host
tensors -- the path the training loader uses.
"""
import bisect
import threading

import numpy as np
import torch
import torch.utils.data
from torch.utils.data.dataloader import default_collate


def _native():
    from .. import _data_native
    return _data_native


class BertH5pyData(torch.utils.data.Dataset):
    def __init__(self, path, max_pred_length=512):
        super().__init__()
        self.keys = ('input_ids', 'input_mask', 'segment_ids', 'masked_lm_positions', 'masked_lm_ids',
                     'next_sentence_labels')
        self.max_pred_length = max_pred_length
        self.path = path
        self._local = threading.local()
        r = _native().BertShardReader(path)
        self._len = len(r)
        self.seq_len = r.seq_len
        self.max_pred = r.max_pred
        r.close()

    # one open reader per thread (HDF5 is thread-safe but handles are cheap)
    def _reader(self):
        r = getattr(self._local, 'reader', None)
        if r is None:
            r = _native().BertShardReader(self.path)
            self._local.reader = r
        return r

    def __getstate__(self):
        d = dict(self.__dict__)
        d.pop('_local', None)
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)
        self._local = threading.local()

    def check_index(self, i):
        if i < 0 or i >= self._len:
            raise IndexError('index out of range')

    def __getitem__(self, index):
        self.check_index(index)
        b = self.read_batch(np.asarray([index], dtype=np.int64))
        return [t[0] for t in b]

    def read_batch(self, indices, pin_memory=False, out=None):
        B, S = len(indices), self.seq_len
        if out is None:
            out = [torch.empty((B, S), dtype=torch.int64, pin_memory=pin_memory) for _ in range(4)]
            out.append(torch.empty((B,), dtype=torch.int64, pin_memory=pin_memory))
        ids, seg, mask, lab, nsp = out
        self._reader().read_into(np.asarray(indices, dtype=np.int64), ids.numpy(), seg.numpy(), mask.numpy(),
                                 lab.numpy(), nsp.numpy())
        return [ids, seg, mask, lab, nsp]

    def __len__(self):
        return self._len

    def size(self, idx):
        return self.max_pred_length   # reference quirk (App. A6): always max_pred_length

    def set_epoch(self, epoch):
        pass


class ConBertH5pyData(torch.utils.data.Dataset):
    """Concatenation of shards with bisect over cumulative sizes."""

    @staticmethod
    def cumsum(sequence, sample_ratios):
        r, s = [], 0
        for e, ratio in zip(sequence, sample_ratios):
            curr_len = int(ratio * len(e))
            r.append(curr_len + s)
            s += curr_len
        return r

    def __init__(self, datasets, sample_ratios=1):
        super().__init__()
        assert len(datasets) > 0, 'datasets should not be an empty iterable'
        self.datasets = list(datasets)
        if isinstance(sample_ratios, int):
            sample_ratios = [sample_ratios] * len(self.datasets)
        self.sample_ratios = sample_ratios
        self.cumulative_sizes = self.cumsum(self.datasets, sample_ratios)
        self.real_sizes = [len(d) for d in self.datasets]
        self.seq_len = self.datasets[0].seq_len
        self.max_pred = max(d.max_pred for d in self.datasets)
        # every BERT sample has the same token count -> vectorised batching fast path
        self.fixed_num_tokens = int(self.datasets[0].size(0))

    def __len__(self):
        return self.cumulative_sizes[-1]

    def __getitem__(self, idx):
        d, s = self._get_dataset_and_sample_index(idx)
        return self.datasets[d][s]

    def _get_dataset_and_sample_index(self, idx):
        dataset_idx = bisect.bisect_right(self.cumulative_sizes, idx)
        sample_idx = idx if dataset_idx == 0 else idx - self.cumulative_sizes[dataset_idx - 1]
        sample_idx = sample_idx % self.real_sizes[dataset_idx]
        return dataset_idx, sample_idx

    def read_batch(self, indices, pin_memory=False):
        indices = np.asarray(indices, dtype=np.int64)
        B, S = len(indices), self.seq_len
        out = [torch.empty((B, S), dtype=torch.int64, pin_memory=pin_memory) for _ in range(4)]
        out.append(torch.empty((B,), dtype=torch.int64, pin_memory=pin_memory))
        cs = np.asarray(self.cumulative_sizes, dtype=np.int64)
        ds_idx = np.searchsorted(cs, indices, side='right')
        start = 0
        while start < B:
            d = ds_idx[start]
            end = start + 1
            while end < B and ds_idx[end] == d:
                end += 1
            base = 0 if d == 0 else cs[d - 1]
            local = (indices[start:end] - base) % self.real_sizes[d]
            self.datasets[d].read_batch(local, out=[t[start:end] for t in out])
            start = end
        return out

    def collater(self, samples):
        if len(samples) == 0:
            return None
        if hasattr(self.datasets[0], 'collater'):
            return self.datasets[0].collater(samples)
        return default_collate(samples)

    def ordered_indices(self):
        return np.arange(len(self))

    def num_tokens(self, index):
        return np.max(self.size(index))

    def size(self, idx):
        d, s = self._get_dataset_and_sample_index(idx)
        return self.datasets[d].size(s)

    def set_epoch(self, epoch):
        pass


class CombineBertData(torch.utils.data.Dataset):
    """Eager in-memory loader over many shards (reference hetseq/data/BERT_DATA.py:11-43,
    ``CombineBertData``).

    The reference reads every key of every shard into RAM with h5py, one file after
    another (its own comment: ~20 GB and ~25 min for Wikipedia).  Here each shard is
    read key by key through the native reader (GIL released) on a thread pool, and
    the arrays are concatenated once.  ``__getitem__`` returns the raw key tuple in
    the reference's order ``keys``; ``read_batch`` builds the same collated
    training batch as :class:`BertH5pyData` (masked-LM labels from positions/ids),
    so the in-memory variant is a drop-in for the streaming one when a corpus fits
    in host memory.
    """

    DEFAULT_KEYS = ('input_ids', 'input_mask', 'segment_ids', 'masked_lm_positions', 'masked_lm_ids',
                    'next_sentence_labels')

    def __init__(self, files, max_pred_length=512, keys=DEFAULT_KEYS, num_threads=8):
        super().__init__()
        from concurrent.futures import ThreadPoolExecutor
        self.max_pred_length = max_pred_length
        self.keys = tuple(keys)
        files = list(files)
        assert len(files) > 0, 'no shard files given'

        def load(path):
            r = _native().BertShardReader(path)
            try:
                n = len(r)
                return {k: r.read_key(k, 0, n) for k in self.keys}
            finally:
                r.close()

        with ThreadPoolExecutor(max_workers=max(1, min(num_threads, len(files)))) as ex:
            parts = list(ex.map(load, files))
        self.inputs = {k: np.concatenate([p[k] for p in parts]) for k in self.keys}
        self.seq_len = int(self.inputs[self.keys[0]].shape[1])
        self.max_pred = int(self.inputs['masked_lm_positions'].shape[1]) \
            if 'masked_lm_positions' in self.inputs else 0
        self.fixed_num_tokens = max_pred_length

    def __len__(self):
        return len(self.inputs[self.keys[0]])

    def __getitem__(self, index):
        return [self.inputs[key][index] for key in self.keys]

    def read_batch(self, indices, pin_memory=False, out=None):
        idx = np.asarray(indices, dtype=np.int64)
        ids = self.inputs['input_ids'][idx]
        pos = self.inputs['masked_lm_positions'][idx]
        mid = self.inputs['masked_lm_ids'][idx]
        labels = np.full_like(ids, -1)
        # first zero position ends the prediction list (h5pyDataset.py:47-53)
        valid = np.cumprod(pos != 0, axis=1).astype(bool)
        rows = np.broadcast_to(np.arange(len(idx))[:, None], pos.shape)
        labels[rows[valid], pos[valid]] = mid[valid]
        arrays = [ids, self.inputs['segment_ids'][idx], self.inputs['input_mask'][idx], labels,
                  self.inputs['next_sentence_labels'][idx].reshape(-1)]
        if out is None:
            out = [torch.empty(a.shape, dtype=torch.int64, pin_memory=pin_memory) for a in arrays]
        for t, a in zip(out, arrays):
            t.copy_(torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)))
        return out

    def size(self, idx):
        return self.max_pred_length

    def num_tokens(self, index):
        return self.max_pred_length

    def ordered_indices(self):
        return np.arange(len(self))

    def set_epoch(self, epoch):
        pass
