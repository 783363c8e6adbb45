"""Epoch / batch iterators with deterministic sharding (reference
hetseq/data/iterators.py:10-274).

Semantics kept bit-for-bit:
  * ``frozen_batches`` are built once; each epoch the BATCH ORDER is shuffled with
    ``np.random.seed(seed + epoch)`` -- identical on every rank, so no
    communication is needed;
  * rank r takes batches r, r+W, r+2W, ... and the shard is padded with ``[]`` to
    ``ceil(N / W)``; an empty batch collates to ``None`` and triggers the
    controller's dummy-batch path;
  * ``state_dict`` = {epoch, iterations_in_epoch}; resume fast-forwards by offset.

MI355X-native loader: datasets that implement ``read_batch(indices)`` (the native
HDF5 BERT shards) are served by ``BatchReaderLoader`` -- worker THREADS call the
GIL-free C++ reader, each producing one collated batch in (pinned) host memory,
``prefetch`` batches ahead -- instead of torch's DataLoader with per-sample
``__getitem__`` in worker processes.  Other datasets keep the DataLoader path.
"""
import abc
import concurrent.futures as cf
import itertools
import os

import numpy as np
import torch

from .data_utils import numpy_seed


class CountingIterator(object):
    """Iterator over ``iterable`` that knows how many items have been consumed
    (``count``, starting at ``start`` when resuming mid-epoch).  Same contract as the
    reference's (hetseq/data/iterators.py:10-40: ``len`` = start + len(iterable),
    ``has_next``, ``skip``); written as a plain stateful iterator."""

    def __init__(self, iterable, start=0):
        self.iterable = iterable
        self.count = start
        self.len = start + len(iterable)
        self._it = iter(iterable)

    def __len__(self):
        return self.len

    def __iter__(self):
        return self

    def __next__(self):
        item = next(self._it)
        self.count += 1
        return item

    def has_next(self):
        return self.count < self.len

    def skip(self, num_to_skip):
        """Consume ``num_to_skip`` items (fewer if the iterable runs out)."""
        for _ in range(num_to_skip):
            try:
                next(self)
            except StopIteration:
                break
        return self


class EpochBatchIterating(abc.ABC):
    """Interface of an epoch-aware batch iterator (the reference's base class,
    hetseq/data/iterators.py:43-64)."""

    @abc.abstractmethod
    def __len__(self):
        pass

    @abc.abstractmethod
    def next_epoch_itr(self, shuffle=True, fix_batches_to_gpus=False):
        pass

    @abc.abstractmethod
    def end_of_epoch(self):
        pass

    @property
    @abc.abstractmethod
    def iterations_in_epoch(self):
        pass

    @abc.abstractmethod
    def state_dict(self):
        pass

    @abc.abstractmethod
    def load_state_dict(self, state_dict):
        pass


class BatchReaderLoader(object):
    """Ordered, threaded batch loader for datasets with a native ``read_batch``."""

    def __init__(self, dataset, batches, num_workers=2, prefetch=4, pin_memory=False, device=None):
        self.dataset = dataset
        self.batches = list(batches)
        self.num_workers = max(1, num_workers)
        self.prefetch = max(1, prefetch)
        self.device = torch.device(device) if device is not None else None
        self.stage = self.device is not None and self.device.type == 'cuda'
        self.pin_memory = pin_memory or self.stage

    def __len__(self):
        return len(self.batches)

    def _load(self, b):
        if len(b) == 0:
            return None
        host = self.dataset.read_batch(np.asarray(b, dtype=np.int64), pin_memory=self.pin_memory)
        if self.stage:
            from .prefetch import stage_to_device
            return stage_to_device(host, self.device)
        return host

    def __iter__(self):
        if self.num_workers <= 0 or len(self.batches) == 0:
            for b in self.batches:
                yield self._load(b)
            return
        with cf.ThreadPoolExecutor(max_workers=self.num_workers) as ex:
            futs = []
            it = iter(self.batches)
            for b in itertools.islice(it, self.prefetch):
                futs.append(ex.submit(self._load, b))
            while futs:
                f = futs.pop(0)
                nxt = next(it, None)
                if nxt is not None:
                    futs.append(ex.submit(self._load, nxt))
                yield f.result()


def _auto_workers(num_workers):
    if num_workers is None or num_workers < 0:
        return min(4, max(1, (os.cpu_count() or 2) // 2))
    return num_workers


class EpochBatchIterator(EpochBatchIterating):
    def __init__(self, dataset, collate_fn, batch_sampler, seed=1, num_shards=1, shard_id=0, num_workers=0,
                 epoch=0, pin_memory=False, device=None):
        assert isinstance(dataset, torch.utils.data.Dataset)
        self.dataset = dataset
        self.collate_fn = collate_fn
        self.frozen_batches = tuple(batch_sampler)
        self.seed = seed
        self.num_shards = num_shards
        self.shard_id = shard_id
        self.num_workers = _auto_workers(num_workers)
        self.pin_memory = pin_memory
        self.device = device
        self.epoch = epoch
        self._cur_epoch_itr = None
        self._next_epoch_itr = None
        self._supports_prefetch = getattr(dataset, 'supports_prefetch', False)

    def __len__(self):
        return len(self.frozen_batches)

    def next_epoch_itr(self, shuffle=True, fix_batches_to_gpus=False):
        if self._next_epoch_itr is not None:
            self._cur_epoch_itr = self._next_epoch_itr
            self._next_epoch_itr = None
        else:
            self.epoch += 1
            self._cur_epoch_itr = self._get_iterator_for_epoch(self.epoch, shuffle,
                                                               fix_batches_to_gpus=fix_batches_to_gpus)
        if hasattr(self.dataset, 'set_epoch'):
            self.dataset.set_epoch(self.epoch)
        return self._cur_epoch_itr

    def end_of_epoch(self):
        return not self._cur_epoch_itr.has_next()

    @property
    def iterations_in_epoch(self):
        if self._cur_epoch_itr is not None:
            return self._cur_epoch_itr.count
        if self._next_epoch_itr is not None:
            return self._next_epoch_itr.count
        return 0

    def state_dict(self):
        return {'epoch': self.epoch, 'iterations_in_epoch': self.iterations_in_epoch}

    def load_state_dict(self, state_dict):
        self.epoch = state_dict['epoch']
        itr_pos = state_dict.get('iterations_in_epoch', 0)
        if itr_pos > 0:
            self._next_epoch_itr = self._get_iterator_for_epoch(self.epoch, shuffle=state_dict.get('shuffle', True),
                                                                offset=itr_pos)

    def shard_batches(self, epoch, shuffle, fix_batches_to_gpus=False):
        """The list of index batches this shard consumes in ``epoch`` (exposed for tests).

        Order contract (reference hetseq/data/iterators.py:166-195, kept bit for bit so a
        run resumes and shards exactly as the reference does): the frozen batch list is
        permuted by ``np.random.shuffle`` under seed ``seed + epoch`` -- the same on every
        rank -- then dealt round-robin; a prefetching dataset with
        ``fix_batches_to_gpus`` instead keeps the global order and permutes each shard
        under ``seed + epoch + shard_id``."""
        per_shard = not self._supports_prefetch or not fix_batches_to_gpus
        order = list(self.frozen_batches)
        if shuffle and per_shard:
            _seeded_shuffle(order, self.seed + epoch)
        mine = _deal(order, self.num_shards, self.shard_id, fill=[])
        if self._supports_prefetch:
            self.dataset.prefetch([i for b in mine for i in b])
            if shuffle and not per_shard:
                _seeded_shuffle(mine, self.seed + epoch + self.shard_id)
        return mine

    def _get_iterator_for_epoch(self, epoch, shuffle, fix_batches_to_gpus=False, offset=0):
        batches = self.shard_batches(epoch, shuffle, fix_batches_to_gpus)
        if offset > 0 and offset >= len(batches):
            return None
        if hasattr(self.dataset, 'read_batch'):
            loader = BatchReaderLoader(self.dataset, batches[offset:], num_workers=self.num_workers,
                                       pin_memory=self.pin_memory, device=self.device)
        else:
            # no DataLoader pin thread: it competes with the training loop for the GIL;
            # the step pins its (small) batch itself before the asynchronous H2D copy
            # (utils.misc.move_to_device)
            loader = torch.utils.data.DataLoader(self.dataset, collate_fn=self.collate_fn,
                                                 batch_sampler=[list(b) for b in batches[offset:]],
                                                 num_workers=self.num_workers, pin_memory=self.pin_memory)
        return CountingIterator(loader, start=offset)


def _seeded_shuffle(items, seed):
    """In-place ``np.random.shuffle`` under a temporary global numpy seed."""
    with numpy_seed(seed):
        np.random.shuffle(items)
    return items


def _deal(items, num_shards, shard_id, fill=None):
    """Round-robin shard ``shard_id`` of ``items``: items shard_id, shard_id + W, ...,
    padded with ``fill`` to ceil(len / W) entries (every shard the same length)."""
    if not 0 <= shard_id < num_shards:
        raise ValueError('shard_id must be between 0 and num_shards')
    n = -(-len(items) // num_shards)
    mine = list(items[shard_id::num_shards])
    return mine + [fill] * (n - len(mine))


class GroupedIterator(object):
    """Lists of ``chunk_size`` consecutive items: the micro-batches of one optimizer step
    under --update-freq (the last group may be short).  ``offset`` = groups already
    consumed when resuming from a partly consumed CountingIterator."""

    def __init__(self, iterable, chunk_size):
        self.itr = iterable
        self.chunk_size = chunk_size
        self._len = -(-len(iterable) // chunk_size)
        self.offset = -(-getattr(iterable, 'count', 0) // chunk_size)

    def __len__(self):
        return self._len

    def __iter__(self):
        return self

    def __next__(self):
        chunk = list(itertools.islice(self.itr, self.chunk_size))
        if not chunk:
            raise StopIteration
        return chunk


class ShardedIterator(object):
    """Iterator over shard ``shard_id`` of ``num_shards`` (see :func:`_deal`)."""

    def __init__(self, iterable, num_shards, shard_id, fill_value=None):
        self._items = _deal(list(iterable), num_shards, shard_id, fill_value)
        self._it = iter(self._items)

    def __len__(self):
        return len(self._items)

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._it)
