#!/usr/bin/env python
"""Build the in-tree native extensions.

* ``_native``      : C++ runtime (src/native/*.cc) — engine, storage, recordio.
* ``_hip_kernels`` : gfx950 HIP kernels (src/kernels/*.hip) + pybind11 bindings,
                     compiled with ``hipcc --offload-arch=gfx950``.

Outputs go to ``mxnet_maintenance_amd/_lib/`` (git-ignored, shipped to the GPU
box with the snapshot).  Incremental: an object is rebuilt only when a source or
header is newer.  Usage: ``python tools/build_native.py [--only native|hip] [-j N]``.
"""
import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'mxnet_maintenance_amd', '_lib')
BUILD = os.path.join(ROOT, 'build')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('MXAMD_OFFLOAD_ARCH', 'gfx950')


def _ext_suffix():
    return sysconfig.get_config_var('EXT_SUFFIX') or '.so'


def _includes():
    import pybind11
    return ['-I' + pybind11.get_include(), '-I' + sysconfig.get_paths()['include']]


def _newer(src_files, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(' '.join(cmd) + '\n' + r.stdout + '\n')
        raise RuntimeError('build step failed: %s' % cmd[-1])
    return r.stdout


def build_native(jobs):
    srcdir = os.path.join(ROOT, 'src', 'native')
    srcs = sorted(glob.glob(os.path.join(srcdir, '*.cc')))
    hdrs = glob.glob(os.path.join(srcdir, '*.h'))
    objdir = os.path.join(BUILD, 'native')
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    flags = ['-O2', '-fPIC', '-std=c++17', '-fvisibility=hidden', '-Wall', '-Wno-unused-variable'] + _includes()
    objs = []
    tasks = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + '.o')
        objs.append(o)
        if _newer([s] + hdrs, o):
            tasks.append(['g++'] + flags + ['-c', s, '-o', o])
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, tasks))
    out = os.path.join(LIB, '_native' + _ext_suffix())
    if tasks or _newer(objs, out):
        _run(['g++', '-shared', '-o', out] + objs + ['-ldl', '-lpthread'])
    return out


def build_hip(jobs):
    srcdir = os.path.join(ROOT, 'src', 'kernels')
    srcs = sorted(glob.glob(os.path.join(srcdir, '*.hip')))
    hdrs = glob.glob(os.path.join(srcdir, '*.h')) + glob.glob(os.path.join(srcdir, '*.cuh'))
    bind = sorted(glob.glob(os.path.join(srcdir, '*.cc')))
    if not srcs:
        return None
    objdir = os.path.join(BUILD, 'hip')
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    hflags = ['-O3', '-fPIC', '-std=c++17', '--offload-arch=' + ARCH, '-munsafe-fp-atomics',
              '-Wno-unused-result'] + _includes()
    objs, tasks = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + '.o')
        objs.append(o)
        if _newer([s] + hdrs, o):
            tasks.append([HIPCC] + hflags + ['-c', s, '-o', o])
    for s in bind:
        o = os.path.join(objdir, os.path.basename(s) + '.o')
        objs.append(o)
        if _newer([s] + hdrs, o):
            tasks.append([HIPCC, '-O2', '-fPIC', '-std=c++17', '-fvisibility=hidden'] + _includes() +
                         ['-I/opt/rocm/include', '-c', s, '-o', o])
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, tasks))
    out = os.path.join(LIB, '_hip_kernels' + _ext_suffix())
    if tasks or _newer(objs, out):
        _run([HIPCC, '-shared', '--offload-arch=' + ARCH, '-o', out] + objs +
             ['-L/opt/rocm/lib', '-lamdhip64'])
    return out


def build_capi(jobs):
    """``libmxamd_predict.so`` / ``libmxamd.so``: the C predict API and the general C API (src/capi), a C
    ABI over the framework in an embedded (or the host's) CPython."""
    import sysconfig
    srcs = sorted(glob.glob(os.path.join(ROOT, 'src', 'capi', '*.cc')))
    if not srcs:
        return None
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, 'libmxamd_predict.so')
    if not _newer(srcs, out) and os.path.exists(os.path.join(LIB, 'libmxamd.so')):
        return out
    inc = sysconfig.get_paths()['include']
    libdir = sysconfig.get_config_var('LIBDIR')
    ver = sysconfig.get_config_var('LDVERSION') or sysconfig.get_python_version()
    _run(['g++', '-O2', '-fPIC', '-shared', '-std=c++17', '-fvisibility=hidden', '-I' + inc] + srcs +
         ['-o', out, '-L' + libdir, '-lpython' + ver, '-ldl', '-Wl,-rpath,' + libdir])
    # the same library under the general C API's name (include/mxamd/c_api.h)
    import shutil
    shutil.copyfile(out, os.path.join(LIB, 'libmxamd.so'))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', choices=['native', 'hip', 'capi'], default=None)
    ap.add_argument('-j', type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    if a.only in (None, 'native'):
        print('built', build_native(a.j))
    if a.only in (None, 'hip'):
        print('built', build_hip(a.j))
    if a.only in (None, 'capi'):
        print('built', build_capi(a.j))


if __name__ == '__main__':
    main()
