"""Training-level fp32 parity of the default fp32 GEMM mode.

BERT-tiny, 60 Adam updates, dropout on, learnable synthetic corpus: ``fp16x3`` (the default fp32
path: scaled fp16 pieces, ops/gemm16.py) must track ``--fp32-gemm native`` (fp32 MFMA) per update
and in the final weights.  The long BERT-base horizon (300 updates) is ``tools/parity_run.py`` ->
``profiles/r4_parity_bert_base_300.md``.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_fp16x3_tracks_native_60_updates(tmp_path):
    out = tmp_path / 'parity'
    r = subprocess.run([sys.executable, '-u', os.path.join(ROOT, 'tools', 'parity_run.py'), '--model', 'tiny',
                        '--updates', '60', '--batch', '32', '--lr', '5e-4', '--warmup-updates', '10',
                        '--out', str(out), '--work', str(tmp_path / 'work')],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.load(open(out / 'parity.json'))
    curve = res['loss_curve']['native']
    assert curve[-1] < curve[0] - 0.5 * abs(curve[0] - curve[-1]) or curve[-1] < 0.9 * curve[0], \
        'corpus should be learnable: {} -> {}'.format(curve[0], curve[-1])
    for mode, tol in (('fp16x3', 1e-4),):
        s = res['modes'][mode]
        assert s['finite']
        assert s['loss_reldiff_max'] < tol, (mode, s)
        assert s['gnorm_reldiff_max'] < 10 * tol, (mode, s)
        assert s['param_diff_over_update'] < 10 * tol, (mode, s)
