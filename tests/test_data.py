"""Native batch packer, HDF5 shard IO, iterators / sharding / resume offsets."""
import os

import numpy as np
import pytest
import torch

from hetseq_9cme_amd import _data_native
from hetseq_9cme_amd.data import data_utils, iterators
from hetseq_9cme_amd.data.h5_dataset import BertH5pyData, ConBertH5pyData
from hetseq_9cme_amd.data.synthetic import make_bert_samples, write_synthetic_bert_shards


@pytest.mark.parametrize('max_tokens,max_sentences,mult', [(None, 7, 1), (200, None, 1), (300, 16, 4),
                                                            (150, 5, 3), (None, None, 1)])
def test_batch_by_size_matches_reference_algorithm(max_tokens, max_sentences, mult):
    rng = np.random.RandomState(0)
    lens = rng.randint(1, 40, size=500)
    idx = rng.permutation(500).astype(np.int64)
    fn = lambda i: int(lens[i])  # noqa: E731
    ref = data_utils.batch_by_size_py(idx, fn, max_tokens, max_sentences, mult)
    got = data_utils.batch_by_size(idx, fn, max_tokens, max_sentences, mult)
    assert [list(b) for b in got] == ref


def test_batch_by_size_fixed_tokens_fast_path():
    class D(object):
        fixed_num_tokens = 512

        def num_tokens(self, i):
            return 512
    got = data_utils.batch_by_size(np.arange(100), D().num_tokens, None, 32, 1)
    assert [len(b) for b in got] == [32, 32, 32, 4]
    with pytest.raises(RuntimeError):
        data_utils.batch_by_size(np.arange(10), D().num_tokens, 100, 32, 1)


def _shards(tmp_path, n_files=3, per=37, S=32, P=5):
    return write_synthetic_bert_shards(str(tmp_path), n_files=n_files, samples_per_file=per, seq_len=S,
                                       max_pred=P, vocab_size=500, seed=3)


def test_h5_roundtrip_and_labels(tmp_path):
    rng = np.random.RandomState(1)
    ids, mask, seg, pos, mids, nsp = make_bert_samples(20, 32, 6, 500, rng)
    pos[3, 2:] = 0  # padded positions -> only first 2 used
    p = str(tmp_path / 'train_a.hdf5')
    _data_native.write_bert_shard(p, ids, mask, seg, pos, mids, nsp)
    d = BertH5pyData(p)
    assert len(d) == 20 and d.seq_len == 32 and d.max_pred == 6
    s = d[3]
    assert torch.equal(s[0], torch.from_numpy(ids[3]).long())
    assert torch.equal(s[1], torch.from_numpy(seg[3]).long())
    assert torch.equal(s[2], torch.from_numpy(mask[3]).long())
    lab = torch.full((32,), -1, dtype=torch.long)
    lab[torch.from_numpy(pos[3, :2]).long()] = torch.from_numpy(mids[3, :2]).long()
    assert torch.equal(s[3], lab)
    assert s[4].item() == nsp[3]
    # batched read of scattered rows == per-item reads
    rows = np.array([5, 6, 7, 1, 19, 0])
    b = d.read_batch(rows)
    for k, r in enumerate(rows):
        it = d[int(r)]
        for f in range(5):
            assert torch.equal(b[f][k], it[f])


def test_concat_dataset_read_batch(tmp_path):
    paths = _shards(tmp_path)
    ds = ConBertH5pyData([BertH5pyData(p) for p in paths])
    assert len(ds) == 111
    rows = np.array([35, 36, 37, 38, 80, 110, 0])
    b = ds.read_batch(rows)
    for k, r in enumerate(rows):
        it = ds[int(r)]
        for f in range(5):
            assert torch.equal(b[f][k], it[f])


def test_combine_bert_data_in_memory(tmp_path):
    """Eager in-memory loader (reference BERT_DATA.py:11-43): raw key tuples equal the
    shard contents, and its collated batches equal the streaming reader's."""
    from hetseq_9cme_amd.data.h5_dataset import CombineBertData
    paths = _shards(tmp_path)
    mem = CombineBertData(paths)
    stream = ConBertH5pyData([BertH5pyData(p) for p in paths])
    assert len(mem) == len(stream) == 111
    r = _data_native.BertShardReader(paths[1])
    first = len(BertH5pyData(paths[0]))
    raw = mem[first + 2]
    for k, key in enumerate(CombineBertData.DEFAULT_KEYS):
        assert np.array_equal(raw[k], r.read_key(key, 2, 1)[0])
    rows = np.array([35, 36, 37, 38, 80, 110, 0, 3])
    a, b = mem.read_batch(rows), stream.read_batch(rows)
    for f in range(5):
        assert torch.equal(a[f], b[f])


def _ref_shard_order(n_batches, W, r, seed, epoch):
    """Reference algorithm: shuffle batch list with seed+epoch, take r::W, pad []."""
    batches = [[i] for i in range(n_batches)]
    state = np.random.get_state()
    np.random.seed(seed + epoch)
    np.random.shuffle(batches)
    np.random.set_state(state)
    mine = batches[r::W]
    L = (n_batches + W - 1) // W
    return mine + [[]] * (L - len(mine))


@pytest.mark.parametrize('W', [1, 3, 4])
def test_sharding_shuffle_padding_matches_reference(tmp_path, W):
    paths = _shards(tmp_path, n_files=1, per=10)
    ds = ConBertH5pyData([BertH5pyData(p) for p in paths])
    for r in range(W):
        it = iterators.EpochBatchIterator(ds, ds.collater, [[i] for i in range(10)], seed=11, num_shards=W,
                                          shard_id=r, num_workers=0)
        got = [list(b) for b in it.shard_batches(epoch=2, shuffle=True)]
        assert got == _ref_shard_order(10, W, r, 11, 2)


def test_epoch_iterator_resume_offset(tmp_path):
    paths = _shards(tmp_path, n_files=1, per=40)
    ds = ConBertH5pyData([BertH5pyData(p) for p in paths])
    bs = data_utils.batch_by_size(ds.ordered_indices(), ds.num_tokens, None, 4, 1)
    it = iterators.EpochBatchIterator(ds, ds.collater, bs, seed=1, num_workers=2)
    e = it.next_epoch_itr()
    first = [next(e)[0].clone() for _ in range(3)]
    st = it.state_dict()
    assert st == {'epoch': 1, 'iterations_in_epoch': 3}
    rest = []
    while e.has_next():
        rest.append(next(e)[0].clone())
    it2 = iterators.EpochBatchIterator(ds, ds.collater, bs, seed=1, num_workers=2)
    it2.load_state_dict(st)
    e2 = it2.next_epoch_itr()
    rest2 = []
    while e2.has_next():
        rest2.append(next(e2)[0].clone())
    assert len(rest2) == len(rest) == 7
    assert all(torch.equal(a, b) for a, b in zip(rest, rest2))
    assert len(first) == 3


def test_grouped_iterator():
    it = iterators.CountingIterator(list(range(7)))
    g = iterators.GroupedIterator(it, 3)
    assert len(g) == 3
    assert list(g) == [[0, 1, 2], [3, 4, 5], [6]]
