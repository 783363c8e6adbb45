"""Packaging: ``pip install -e .`` / ``python setup.py build_ext --inplace``.

The native extensions are built by ``hetseq_9cme_amd/build_ext.py`` (hipcc for
gfx950 kernels, g++ for the torch bindings and the libhdf5 data runtime) --
no hipify, no torch JIT cache.
"""
from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext as _build_ext
from setuptools import Extension


class NativeBuild(_build_ext):
    def run(self):
        import sys
        sys.path.insert(0, '.')
        from hetseq_9cme_amd import build_ext
        build_ext.build_all(force=self.force)

    def build_extension(self, ext):  # handled in run()
        pass


setup(
    name='hetseq_9cme_amd',
    version='0.1.0',
    description='MI355X-native heterogeneous data-parallel training engine (HetSeq capabilities)',
    packages=find_packages(include=['hetseq_9cme_amd', 'hetseq_9cme_amd.*']),
    package_data={'hetseq_9cme_amd': ['csrc/**/*', '*.so']},
    ext_modules=[Extension('hetseq_9cme_amd._C', sources=[])],
    cmdclass={'build_ext': NativeBuild},
    python_requires='>=3.8',
    install_requires=['torch', 'numpy'],
    extras_require={'finetune': ['transformers', 'datasets']},
    entry_points={'console_scripts': ['hetseq-train=hetseq_9cme_amd.train:cli_main']},
)
