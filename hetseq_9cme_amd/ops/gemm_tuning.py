"""Per-shape GEMM solution selection for the library GEMMs (hipBLASLt / rocBLAS).

The plain GEMMs of a BERT step (QKV / attention-out / FFN projections, their
dgrad and wgrad, the MLM decoder) go to the vendor libraries.  Their default
heuristics pick a reasonable but not the fastest solution for the tall-skinny
fp32 shapes of BERT (M = tokens per GPU = 16384): measured on MI355X, the FFN
GEMMs run at ~128-135 TF/s with the default choice and ~149 TF/s (95% of the
157 TF/s fp32 MFMA peak) with the best rocBLAS solution, i.e. ~5% of the whole
step.  PyTorch-ROCm's TunableOp layer lets us pin a solution per
(op, transpose, shape, leading-dims) key, so this module

* ``table`` (default): loads the solution table shipped in
  ``hetseq_9cme_amd/tuning/gemm_gfx950.csv`` (tuned on an MI355X with
  ``tools/tune_gemm.sh``; fp32 keys for BERT-base phase 1/2 and BERT-large
  phase 1 at their per-GPU batches, and -- round 5 (its one-off GPU script is in git history) -- the bf16 keys of
  the ``--precision bf16`` BERT-base phase-1 products: 15.49-15.59 vs 15.74-15.90 ms/step,
  ``profiles/r5bw_bf16_tuned_table_ab.txt``), with tuning disabled -- shapes not in the table keep the
  library default, nothing is benchmarked at run time;
* ``online``: additionally benchmarks every new shape the first time it runs
  (a few hundred ms per shape) and writes the merged table to
  ``--gemm-tuning-file`` (rank-suffixed) at exit;
* ``retune``: like ``online`` but without loading the shipped table, so every
  shape is benchmarked again (after a ROCm / PyTorch / library upgrade);
* ``off``: library defaults.

The table carries validators (PyTorch / HIP / hipBLASLt / rocBLAS versions and
the gfx arch); PyTorch refuses a table whose validators do not match the
running stack, in which case we warn and fall back to the defaults.
"""
import os
import tempfile
import warnings

import torch

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tuning', 'gemm_gfx950.csv')

_state = {'mode': None}


def configure(mode='table', out_file=None, table=TABLE, max_tuning_ms=None):
    """Enable the per-shape GEMM selection on the current GPU process.

    Must run before the first GEMM of interest; idempotent.  Returns True when
    a solution table was loaded.
    """
    if not torch.cuda.is_available() or mode in (None, 'off'):
        _state['mode'] = 'off'
        return False
    if _state['mode'] == mode:
        return True
    tun = torch.cuda.tunable
    tun.enable(True)
    tuning = mode in ('online', 'retune')
    tun.tuning_enable(tuning)
    if mode == 'retune':
        table = None
    if tuning:
        if max_tuning_ms is not None:
            tun.set_max_tuning_duration(int(max_tuning_ms))
        tun.set_filename(out_file or os.path.join(tempfile.gettempdir(), 'hx_gemm_tuning.csv'),
                         insert_device_ordinal=True)
    else:
        # results are only read; keep any exit-time dump out of the working tree
        tun.set_filename(os.path.join(tempfile.gettempdir(), 'hx_gemm_table_{}.csv'.format(os.getpid())),
                         insert_device_ordinal=True)
    ok = False
    if table and os.path.exists(table):
        ok = bool(tun.read_file(table))
        if not ok:
            warnings.warn('GEMM solution table {} does not match this ROCm/PyTorch stack; '
                          'using library defaults'.format(table))
    _state['mode'] = mode
    return ok


def mode():
    return _state['mode']


def merge_tables(paths, out):
    """Union several TunableOp CSV dumps (first file's validators win)."""
    validators, rows, seen = [], [], set()
    for i, p in enumerate(paths):
        with open(p) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                if line.startswith('Validator,'):
                    if i == 0:
                        validators.append(line)
                    continue
                key = tuple(line.split(',')[:2])
                if key not in seen:
                    seen.add(key)
                    rows.append(line)
    with open(out, 'w') as f:
        f.write('\n'.join(validators + rows) + '\n')
    return len(rows)
