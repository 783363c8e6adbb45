"""Batching utilities (reference hetseq/data/data_utils.py:14-61).

``batch_by_size`` runs the native C++ packer (``_data_native.batch_by_size``) over
a vector of token counts -- bit-identical batches to the reference's Cython
``batch_by_size_fast`` but without a Python callback per index.
"""
import contextlib
import sys

import numpy as np


@contextlib.contextmanager
def numpy_seed(seed, *addl_seeds):
    """Seed the NumPy PRNG for the duration of the context, then restore it."""
    if seed is None:
        yield
        return
    if len(addl_seeds) > 0:
        seed = int(hash((seed, *addl_seeds)) % 1e6)
    state = np.random.get_state()
    np.random.seed(seed)
    try:
        yield
    finally:
        np.random.set_state(state)


def _token_counts(indices, num_tokens_fn):
    """Vectorised token counts: datasets may expose ``num_tokens_vec(indices)`` or a
    constant ``fixed_num_tokens``; otherwise fall back to the per-index callback."""
    owner = getattr(num_tokens_fn, '__self__', None)
    if owner is not None:
        fixed = getattr(owner, 'fixed_num_tokens', None)
        if fixed is not None:
            return np.asarray([int(fixed)], dtype=np.int64)
        vec = getattr(owner, 'num_tokens_vec', None)
        if vec is not None:
            return np.asarray(vec(indices), dtype=np.int64)
    return np.fromiter((num_tokens_fn(int(i)) for i in indices), dtype=np.int64, count=len(indices))


def batch_by_size(indices, num_tokens_fn, max_tokens=None, max_sentences=None,
                  required_batch_size_multiple=1):
    """Yield mini-batches of indices bucketed by size (greedy, order preserving)."""
    from .. import _data_native
    max_tokens = max_tokens if max_tokens is not None else sys.maxsize
    max_sentences = max_sentences if max_sentences is not None else sys.maxsize
    indices = np.asarray(indices, dtype=np.int64)
    counts = _token_counts(indices, num_tokens_fn)
    return _data_native.batch_by_size(indices, counts, int(max_tokens), int(max_sentences),
                                      int(required_batch_size_multiple))


def batch_by_size_py(indices, num_tokens_fn, max_tokens=None, max_sentences=None,
                     required_batch_size_multiple=1):
    """Pure-Python transcription of the reference algorithm (test oracle)."""
    max_tokens = max_tokens if max_tokens is not None else sys.maxsize
    max_sentences = max_sentences if max_sentences is not None else sys.maxsize
    bsz_mult = required_batch_size_multiple
    sample_len = 0
    sample_lens, batch, batches = [], [], []
    for idx in indices:
        idx = int(idx)
        n = num_tokens_fn(idx)
        sample_lens.append(n)
        sample_len = max(sample_len, n)
        assert sample_len <= max_tokens
        num_tokens = (len(batch) + 1) * sample_len
        full = len(batch) > 0 and (len(batch) == max_sentences or num_tokens > max_tokens)
        if full:
            mod_len = max(bsz_mult * (len(batch) // bsz_mult), len(batch) % bsz_mult)
            batches.append(batch[:mod_len])
            batch = batch[mod_len:]
            sample_lens = sample_lens[mod_len:]
            sample_len = max(sample_lens) if len(sample_lens) > 0 else 0
        batch.append(idx)
    if len(batch) > 0:
        batches.append(batch)
    return batches
