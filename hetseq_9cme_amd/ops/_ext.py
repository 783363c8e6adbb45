"""Loader for the in-tree gfx950 kernel extension (``hetseq_9cme_amd/_C*.so``).

GPU tensors ALWAYS go through the HIP kernels; if the extension is missing on a
GPU run this raises instead of silently falling back to torch ops (the CPU path
exists for CPU tensors only: tests, plumbing runs, and as the numerics oracle).
``HETSEQ_NO_FUSED=1`` (or ``set_fused(False)``) disables the kernels explicitly
for A/B comparisons.
"""
import os

_C = None
_ERR = None
_FUSED = os.environ.get('HETSEQ_NO_FUSED', '0') != '1'


def set_fused(flag):
    global _FUSED
    _FUSED = bool(flag)


def fused_enabled():
    return _FUSED


def C():
    global _C, _ERR
    if _C is None:
        try:
            from .. import _C as ext  # noqa: N814
            _C = ext
        except ImportError as e:  # pragma: no cover - depends on build state
            _ERR = e
            raise RuntimeError(
                'hetseq_9cme_amd GPU kernels are not built (hetseq_9cme_amd/_C*.so missing): {}. '
                'Run `python -m hetseq_9cme_amd.build_ext`.'.format(e))
    return _C


def use_kernels(t):
    """True when ``t`` lives on the GPU and the fused kernels are enabled."""
    return _FUSED and t.is_cuda
