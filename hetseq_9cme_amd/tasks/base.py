"""Task base class (reference hetseq/tasks/tasks.py:22-192).

A task owns dictionaries and datasets, builds the model, creates the cached,
sharded ``EpochBatchIterator`` and runs one forward/backward micro-batch.

``train_step`` keeps the reference contract exactly:
  loss = model(*sample); loss *= 0 if ignore_grad;
  sample_size = len(sample[0][0])   (= seq_len for BERT, 1 for MNIST: App. A3);
  logging_output = {nsentences, loss, nll_loss, ntokens: 0, sample_size};
  optimizer.backward(loss).
``loss`` stays a DEVICE tensor in the logging output (no per-step host sync).
"""
import collections

import torch

from ..data import data_utils, iterators
from ..utils.misc import ensure_train


class Task(object):
    def __init__(self, args):
        self.args = args
        self.datasets = {}
        self.dataset_to_epoch_iter = {}

    @staticmethod
    def load_dictionary(vocab_file):
        vocab = collections.OrderedDict()
        if vocab_file is None:
            return vocab
        with open(vocab_file, 'r', encoding='utf-8') as reader:
            for index, token in enumerate(reader):
                vocab[token.strip()] = index
        print('| loaded dictionary with {} subwords  from: {}'.format(len(vocab), vocab_file))
        return vocab

    def load_dataset(self, split, **kwargs):
        raise NotImplementedError

    def dataset(self, split):
        if split not in self.datasets:
            raise KeyError('Dataset not loaded: ' + split)
        if not isinstance(self.datasets[split], torch.utils.data.Dataset):
            raise TypeError('Datasets are expected to be of type torch.utils.data.Dataset')
        return self.datasets[split]

    def get_batch_iterator(self, dataset, max_tokens=None, max_sentences=None, max_positions=None,
                           ignore_invalid_inputs=False, required_batch_size_multiple=1, seed=1, num_shards=1,
                           shard_id=0, num_workers=0, epoch=0, device=None):
        if dataset in self.dataset_to_epoch_iter:
            return self.dataset_to_epoch_iter[dataset]
        with data_utils.numpy_seed(seed):
            indices = dataset.ordered_indices()
        print('| build batch sampler')
        batch_sampler = data_utils.batch_by_size(indices, dataset.num_tokens, max_tokens=max_tokens,
                                                 max_sentences=max_sentences,
                                                 required_batch_size_multiple=required_batch_size_multiple)
        print('| finish building batch sampler')
        epoch_iter = iterators.EpochBatchIterator(dataset=dataset, collate_fn=dataset.collater,
                                                  batch_sampler=batch_sampler, seed=seed, num_shards=num_shards,
                                                  shard_id=shard_id, num_workers=num_workers, epoch=epoch,
                                                  device=device)
        self.dataset_to_epoch_iter[dataset] = epoch_iter
        return epoch_iter

    def build_model(self, args):
        raise NotImplementedError

    def configure_model(self, model):
        """Hook called once datasets are known (e.g. MLM gather capacity)."""
        pass

    @staticmethod
    def _sample_size(sample):
        if sample is None or len(sample) == 0 or len(sample[0][0]) == 0:
            return 0
        return len(sample[0][0])

    def train_step(self, sample, model, optimizer, ignore_grad=False):
        ensure_train(model)
        loss = model(*sample)
        if ignore_grad:
            loss = loss * 0
        sample_size = self._sample_size(sample)
        logging_output = {
            'nsentences': sample_size,
            'loss': loss.detach(),
            'nll_loss': loss.detach(),
            'ntokens': 0,
            'sample_size': sample_size,
        }
        optimizer.backward(loss)
        return loss, sample_size, logging_output

    def update_step(self, num_updates):
        pass
