"""Synthetic data generators (there is no network: no corpora, no downloads).

* BERT shards in the NVIDIA HDF5 schema via the native writer;
  shapes match phase 1 (S=128, P=20) / phase 2 (S=512, P=80).
* MNIST-shaped IDX files (torchvision raw layout).
* CoNLL-2003-style NER files and a WordPiece vocab covering their tokens.
* BERT configs (base / large / tiny).
"""
import json
import os
import struct

import numpy as np

BERT_BASE = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_act='gelu', hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02)
BERT_LARGE = dict(BERT_BASE, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                  intermediate_size=4096)
BERT_TINY = dict(BERT_BASE, vocab_size=1024, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=512, max_position_embeddings=128)


def write_bert_config(path, **overrides):
    cfg = dict(BERT_BASE)
    cfg.update(overrides)
    with open(path, 'w') as f:
        json.dump(cfg, f, indent=2)
    return path


def _zipf_tokens(rng, size, vocab_size):
    r = np.minimum(rng.zipf(1.3, size=size), vocab_size - 5)
    return (r + 4).astype(np.int64)


def make_bert_samples(n, seq_len, max_pred, vocab_size, rng, pad_frac=0.0, pattern=None):
    """``pattern=None``: uniform random tokens (shape-only data, nothing to learn).
    ``pattern='bigram'``: a learnable corpus -- Zipf unigrams, each token followed by a
    fixed successor with probability 0.7, and the NSP label says whether segment B
    continues segment A's chain -- so loss curves actually move (parity runs)."""
    if pattern == 'bigram':
        split = rng.randint(seq_len // 4, 3 * seq_len // 4, size=n)
        nsp = rng.randint(0, 2, size=n).astype(np.int32)
        t = np.zeros((n, seq_len), dtype=np.int64)
        t[:, 1] = _zipf_tokens(rng, n, vocab_size)
        for j in range(2, seq_len):
            succ = (t[:, j - 1] * 7919 + 13) % (vocab_size - 5) + 5
            fresh = _zipf_tokens(rng, n, vocab_size)
            keep = rng.rand(n) < 0.7
            brk = (j == split) & (nsp == 0)        # "random next sentence": the chain restarts
            t[:, j] = np.where(keep & ~brk, succ, fresh)
        ids = t.astype(np.int32)
    else:
        ids = rng.randint(5, vocab_size, size=(n, seq_len)).astype(np.int32)
        split = rng.randint(seq_len // 4, 3 * seq_len // 4, size=n)   # (draw order kept: same data as before)
        nsp = None
    ids[:, 0] = 2  # [CLS]
    mask = np.ones((n, seq_len), dtype=np.int32)
    seg = np.zeros((n, seq_len), dtype=np.int32)
    for i in range(n):
        seg[i, split[i]:] = 1
        if pad_frac > 0:
            L = seq_len - int(rng.rand() * pad_frac * seq_len)
            mask[i, L:] = 0
            ids[i, L:] = 0
            seg[i, L:] = 0
    pos = np.zeros((n, max_pred), dtype=np.int32)
    mids = np.zeros((n, max_pred), dtype=np.int32)
    for i in range(n):
        valid = int(mask[i].sum())
        k = min(max_pred, max(1, int(round(0.15 * valid))))
        p = np.sort(rng.choice(np.arange(1, valid), size=k, replace=False))
        pos[i, :k] = p
        mids[i, :k] = ids[i, p]
        ids[i, p] = 4  # [MASK]
    if nsp is None:
        nsp = rng.randint(0, 2, size=n).astype(np.int32)
    return ids, mask, seg, pos, mids, nsp


def write_synthetic_bert_shards(out_dir, n_files=2, samples_per_file=256, seq_len=128, max_pred=20,
                                vocab_size=30522, seed=1234, split='train', pad_frac=0.0, pattern=None):
    """Write ``n_files`` shards named ``{split}_shard_{k}.hdf5`` into ``out_dir``
    (``pattern``: see :func:`make_bert_samples`)."""
    from .. import _data_native
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.RandomState(seed)
    paths = []
    for k in range(n_files):
        ids, mask, seg, pos, mids, nsp = make_bert_samples(samples_per_file, seq_len, max_pred, vocab_size, rng,
                                                           pad_frac, pattern)
        p = os.path.join(out_dir, '{}_shard_{:03d}.hdf5'.format(split, k))
        _data_native.write_bert_shard(p, ids, mask, seg, pos, mids, nsp)
        paths.append(p)
    return paths


def write_vocab(path, vocab_size=30522, extra_words=()):
    special = ['[PAD]', '[UNK]', '[CLS]', '[SEP]', '[MASK]']
    words = list(dict.fromkeys(w.lower() for w in extra_words))
    toks = special + words
    i = 0
    while len(toks) < vocab_size:
        toks.append('tok{}'.format(i))
        i += 1
    with open(path, 'w', encoding='utf-8') as f:
        f.write('\n'.join(toks[:max(vocab_size, len(special) + len(words))]) + '\n')
    return path


def _write_idx(path, arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    with open(path, 'wb') as f:
        f.write(struct.pack('>HBB', 0, 0x08, arr.ndim))
        f.write(struct.pack('>' + 'I' * arr.ndim, *arr.shape))
        f.write(arr.tobytes())


def write_synthetic_mnist(root, n_train=1024, n_test=256, seed=0):
    """torchvision raw layout under ``root/MNIST/raw``; digits are class-dependent
    blobs so a CNN can actually learn them."""
    rng = np.random.RandomState(seed)
    raw = os.path.join(root, 'MNIST', 'raw')
    os.makedirs(raw, exist_ok=True)

    def gen(n):
        labels = rng.randint(0, 10, size=n).astype(np.uint8)
        imgs = rng.randint(0, 40, size=(n, 28, 28)).astype(np.float32)
        for i, c in enumerate(labels):
            r, cc = 4 + (c // 5) * 10, 2 + (c % 5) * 5
            imgs[i, r:r + 9, cc:cc + 5] += 200
        return np.clip(imgs, 0, 255).astype(np.uint8), labels

    xi, yi = gen(n_train)
    xt, yt = gen(n_test)
    _write_idx(os.path.join(raw, 'train-images-idx3-ubyte'), xi)
    _write_idx(os.path.join(raw, 'train-labels-idx1-ubyte'), yi)
    _write_idx(os.path.join(raw, 't10k-images-idx3-ubyte'), xt)
    _write_idx(os.path.join(raw, 't10k-labels-idx1-ubyte'), yt)
    return root


WORDS = ['john', 'smith', 'paris', 'london', 'acme', 'corp', 'went', 'to', 'the', 'city', 'of', 'and', 'visited',
         'germany', 'france', 'bank', 'united', 'nations', 'said', 'on', 'monday', 'in', 'a', 'report', 'mary',
         'berlin', 'google', 'river', 'league', 'cup']
TAGS = {'john': 'B-PER', 'smith': 'I-PER', 'mary': 'B-PER', 'paris': 'B-LOC', 'london': 'B-LOC',
        'berlin': 'B-LOC', 'germany': 'B-LOC', 'france': 'B-LOC', 'acme': 'B-ORG', 'corp': 'I-ORG',
        'google': 'B-ORG', 'united': 'B-ORG', 'nations': 'I-ORG', 'league': 'B-MISC', 'cup': 'I-MISC'}


def write_synthetic_conll(path, n_sents=64, seed=0, with_entities=False, min_len=4, max_len=14):
    rng = np.random.RandomState(seed)
    lines = ['-DOCSTART- -X- -X- O', '']
    for _ in range(n_sents):
        L = rng.randint(min_len, max_len)
        for _ in range(L):
            w = WORDS[rng.randint(len(WORDS))]
            tag = TAGS.get(w, 'O')
            cols = [w.capitalize(), 'NN', 'O', tag]
            if with_entities:
                cols.append(w.capitalize() if tag.startswith('B') else '')
            lines.append('\t'.join(cols))
        lines.append('')
    with open(path, 'w', encoding='utf-8') as f:
        f.write('\n'.join(lines) + '\n')
    return path
