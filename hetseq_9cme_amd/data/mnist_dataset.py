"""MNIST dataset (reference hetseq/data/mnist_dataset.py:9-82).

Accepts, in order of preference, the layouts a reference user already has:
  * torchvision "processed" files (``training.pt`` / ``test.pt``: a (uint8
    [N,28,28], int64 [N]) tuple) -- loaded with ``weights_only=True``;
  * torchvision "raw" IDX files (``train-images-idx3-ubyte`` / ``t10k-...``),
    parsed here with numpy (torchvision is not required);
  * ``*.npz`` with ``images``/``labels`` arrays.
Per-item transform = ToTensor + Normalize(0.1307, 0.3081), done vectorised on
the whole uint8 tensor once (no PIL round trip per item).
There is no download path (offline); ``data.synthetic.write_synthetic_mnist``
creates IDX files of the right shape for plumbing runs.
"""
import gzip
import os
import struct

import numpy as np
import torch
import torch.utils.data
from torch.utils.data.dataloader import default_collate

MEAN, STD = 0.1307, 0.3081


def read_idx(path):
    opener = gzip.open if path.endswith('.gz') else open
    with opener(path, 'rb') as f:
        data = f.read()
    zero, dtype, ndim = struct.unpack('>HBB', data[:4])
    assert zero == 0 and dtype == 0x08, 'only uint8 IDX files are supported'
    dims = struct.unpack('>' + 'I' * ndim, data[4:4 + 4 * ndim])
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim)
    return arr.reshape(dims)


def load_mnist_file(path):
    if path.endswith('.pt'):
        images, labels = torch.load(path, map_location='cpu', weights_only=True)
        return images.numpy().astype(np.uint8), labels.numpy().astype(np.int64)
    if path.endswith('.npz'):
        z = np.load(path)
        return z['images'].astype(np.uint8), z['labels'].astype(np.int64)
    raise ValueError('unsupported MNIST file: {}'.format(path))


def find_mnist_split(path, split):
    """Return (images, labels) numpy arrays for ``split`` ('train'/'test'/...)."""
    cands = []
    if os.path.isdir(path):
        for sub in ['', 'MNIST/processed', 'processed', 'MNIST/raw', 'raw']:
            d = os.path.join(path, sub)
            if os.path.isdir(d):
                cands.append(d)
    else:
        return load_mnist_file(path)
    for d in cands:
        files = sorted(f for f in os.listdir(d) if split in f and (f.endswith('.pt') or f.endswith('.npz')))
        if len(files) == 1:
            return load_mnist_file(os.path.join(d, files[0]))
    idx_prefix = {'train': 'train', 'training': 'train', 'test': 't10k', 'valid': 't10k'}.get(split, split)
    for d in cands:
        img = [f for f in os.listdir(d) if f.startswith(idx_prefix + '-images-idx3-ubyte')]
        lab = [f for f in os.listdir(d) if f.startswith(idx_prefix + '-labels-idx1-ubyte')]
        if img and lab:
            return read_idx(os.path.join(d, sorted(img)[0])), read_idx(os.path.join(d, sorted(lab)[0])).astype(np.int64)
    raise FileNotFoundError('no MNIST data for split "{}" under {} (offline: no download)'.format(split, path))


class MNISTDataset(torch.utils.data.Dataset):
    def __init__(self, images, labels):
        images = torch.from_numpy(np.array(images, dtype=np.uint8, copy=True))
        self.image = ((images.to(torch.float32) / 255.0 - MEAN) / STD).unsqueeze(1).contiguous()
        self.label = torch.from_numpy(np.ascontiguousarray(labels)).to(torch.int64)
        self._len = len(self.label)
        self.fixed_num_tokens = 1

    @classmethod
    def from_path(cls, path, split='train'):
        return cls(*find_mnist_split(path, split))

    def __getitem__(self, index):
        return self.image[index], self.label[index]

    def read_batch(self, indices, pin_memory=False):
        idx = torch.as_tensor(np.asarray(indices), dtype=torch.int64)
        x = self.image.index_select(0, idx)
        y = self.label.index_select(0, idx)
        if pin_memory:
            x, y = x.pin_memory(), y.pin_memory()
        return [x, y]

    def __len__(self):
        return self._len

    def ordered_indices(self):
        return np.arange(len(self))

    def num_tokens(self, index):
        return 1

    def size(self, index):
        return 1

    def collater(self, samples):
        if len(samples) == 0:
            return None
        return default_collate(samples)

    def set_epoch(self, epoch):
        pass
