import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (ROCm GPU) and the built _C extension')
    config.addinivalue_line('markers', 'slow: longer CPU tests')
    # The native extensions (C++ data runtime, gradient reducer, gfx950 kernels) are part of
    # every code path the CPU tests exercise.  Build them in-tree when missing (incremental,
    # hipcc cross-compiles for gfx950 without a GPU); the GPU box gets the prebuilt .so files.
    import glob
    pkg = os.path.join(ROOT, 'hetseq_9cme_amd')
    if not (glob.glob(os.path.join(pkg, '_C*.so')) and glob.glob(os.path.join(pkg, '_data_native*.so'))):
        from hetseq_9cme_amd import build_ext
        build_ext.build_all(force=False, jobs=min(8, os.cpu_count() or 4))


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def dev():
    import torch
    if not gpu_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)
