"""In-tree build of the native extensions (no hipify, no torch JIT cache).

* ``hetseq_9cme_amd/_C*.so``           -- CDNA4 (gfx950) HIP kernels + torch bindings.
  Kernel TUs (``csrc/kernels/*.hip``) are compiled by ``hipcc --offload-arch=gfx950``
  WITHOUT torch headers (fast, seconds per file); the one binding TU
  (``csrc/bindings.cpp``) is host-only C++ against the torch/ROCm headers.
* ``hetseq_9cme_amd/_data_native*.so`` -- host C++ data runtime (batch packing,
  libhdf5 shard reader/writer), pybind11 only, no HIP dependency, so data
  worker threads/processes never touch the GPU runtime.

Incremental: an object is rebuilt only when its source or a header changed.
Usage: ``python -m hetseq_9cme_amd.build_ext [--force] [-j N]``.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(HERE, '..', 'build', 'obj')
EXT = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')
HIPCC = os.path.join(ROCM, 'bin', 'hipcc')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')
HDF5_ROOT = os.environ.get('HDF5_ROOT', '/opt/conda')
# what the last build_* call did per output: {basename: {'mode': 'compiled' | 'reused', 'objects': n}}
LAST = {}


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, 'include'), os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include')]
    lib = os.path.join(tdir, 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _pybind_inc():
    import pybind11
    return pybind11.get_include()


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError('build command failed:\n{}\n{}'.format(' '.join(cmd), r.stdout))
    return r.stdout


def _headers():
    return glob.glob(os.path.join(CSRC, '**', '*.h'), recursive=True)


def build_kernels(force=False, jobs=8, verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    tinc, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()['include']
    srcs = sorted(glob.glob(os.path.join(CSRC, 'kernels', '*.hip')))
    hdrs = _headers()
    out_so = os.path.join(HERE, '_C' + EXT)
    objs, jobs_list = [], []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + '.o')
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs_list.append([HIPCC, '--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-c', s, '-o', o,
                              '-I' + os.path.join(CSRC, 'include'), '-munsafe-fp-atomics',
                              '-Wno-unused-result'])
    # host-only TUs against the torch / ROCm headers: the bindings and the native
    # gradient reducer (c10d process groups, autograd hooks, HIP events)
    for b_src in (os.path.join(CSRC, 'bindings.cpp'), os.path.join(CSRC, 'native', 'reducer.cpp')):
        b_obj = os.path.join(BUILD, os.path.basename(b_src) + '.o')
        objs.append(b_obj)
        if force or _newer(b_obj, [b_src] + hdrs):
            jobs_list.append(['g++', '-O2', '-std=c++17', '-fPIC', '-c', b_src, '-o', b_obj,
                              '-I' + os.path.join(CSRC, 'include'), '-I' + py_inc,
                              '-I' + os.path.join(ROCM, 'include')]
                             + ['-I' + i for i in tinc]
                             + ['-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1', '-DUSE_C10D_NCCL=1',
                                '-DUSE_DISTRIBUTED=1', '-DTORCH_EXTENSION_NAME=_C',
                                '-DTORCH_API_INCLUDE_EXTENSION_H', '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi,
                                '-Wno-deprecated-declarations'])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    linked = bool(force or jobs_list or _newer(out_so, objs))
    if linked:
        _run([HIPCC, '-shared', '-fPIC', '--offload-arch=' + ARCH] + objs + ['-o', out_so, '-L' + tlib,
             '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip', '-ltorch_python',
             '-Wl,-rpath,' + tlib])
    LAST[os.path.basename(out_so)] = {'mode': 'compiled' if linked else 'reused', 'objects': len(jobs_list),
                                      'arch': ARCH}
    return out_so


def build_data_native(force=False):
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(CSRC, 'native', 'data_native.cpp')
    out_so = os.path.join(HERE, '_data_native' + EXT)
    built = bool(force or _newer(out_so, [src]))
    LAST[os.path.basename(out_so)] = {'mode': 'compiled' if built else 'reused', 'objects': int(built)}
    if built:
        py_inc = sysconfig.get_paths()['include']
        # the compiler's own libstdc++ directory goes first in the rpath: the HDF5 prefix
        # (/opt/conda/lib) ships an older libstdc++ that lacks symbols g++ 11 emits, and
        # the module must import on its own (data workers), not only after torch
        stdcxx = os.path.dirname(os.path.realpath(
            subprocess.run(['g++', '-print-file-name=libstdc++.so.6'], stdout=subprocess.PIPE,
                           text=True).stdout.strip()))
        _run(['g++', '-O3', '-std=c++17', '-fPIC', '-shared', src, '-o', out_so, '-I' + _pybind_inc(),
              '-I' + py_inc, '-I' + os.path.join(HDF5_ROOT, 'include'), '-L' + os.path.join(HDF5_ROOT, 'lib'),
              '-lhdf5', '-Wl,-rpath,' + stdcxx, '-Wl,-rpath,' + os.path.join(HDF5_ROOT, 'lib'), '-pthread'])
    return out_so


def build_all(force=False, jobs=8, verbose=False):
    with cf.ThreadPoolExecutor(max_workers=2) as ex:
        f1 = ex.submit(build_data_native, force)
        f2 = ex.submit(build_kernels, force, jobs, verbose)
        return f1.result(), f2.result()


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument('-v', action='store_true')
    a = ap.parse_args()
    for so in build_all(a.force, a.j, a.v):
        print(LAST[os.path.basename(so)]['mode'], so)
    sys.exit(0)
