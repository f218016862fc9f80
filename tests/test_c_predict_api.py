"""The C predict API (libmxamd_predict.so): a plain C program embeds the framework through
MXPredCreate / SetInput / Forward / GetOutputShape / GetOutput / Reshape / Free and MXNDList*,
and its outputs equal the Python executor's; the same library also works loaded into a running
Python process (ctypes)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import mxnet_maintenance_amd as mx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'mxnet_maintenance_amd', '_lib', 'libmxamd_predict.so')

C_PROGRAM = r'''
#include <stdio.h>
#include <stdlib.h>
#include "mxamd/c_predict_api.h"

static char* slurp(const char* path, long* n) {
  FILE* f = fopen(path, "rb"); fseek(f, 0, SEEK_END); *n = ftell(f); fseek(f, 0, SEEK_SET);
  char* buf = (char*)malloc(*n + 1); fread(buf, 1, *n, f); buf[*n] = 0; fclose(f); return buf;
}

int main(int argc, char** argv) {
  long js, ps, ins;
  char* json = slurp(argv[1], &js);
  char* params = slurp(argv[2], &ps);
  char* input = slurp(argv[3], &ins);
  const char* keys[1] = {"data"};
  uint32_t indptr[2] = {0, 2}, shape[2] = {4, 8};
  PredictorHandle h;
  if (MXPredCreate(json, params, (int)ps, 1, 0, 1, keys, indptr, shape, &h)) { printf("ERR %s\n", MXGetLastError()); return 1; }
  if (MXPredSetInput(h, "data", (const float*)input, 32) || MXPredForward(h)) { printf("ERR %s\n", MXGetLastError()); return 1; }
  uint32_t *osh, ond;
  MXPredGetOutputShape(h, 0, &osh, &ond);
  printf("SHAPE %u %u %u\n", ond, osh[0], osh[1]);
  float out[40];
  if (MXPredGetOutput(h, 0, out, osh[0] * osh[1])) { printf("ERR %s\n", MXGetLastError()); return 1; }
  printf("OUT");
  for (uint32_t i = 0; i < osh[0] * osh[1]; ++i) printf(" %.7g", out[i]);
  printf("\n");
  /* reshape to batch 2: a second predictor sharing the weights */
  uint32_t shape2[2] = {2, 8};
  PredictorHandle h2;
  if (MXPredReshape(1, keys, indptr, shape2, h, &h2)) { printf("ERR %s\n", MXGetLastError()); return 1; }
  MXPredSetInput(h2, "data", (const float*)input, 16);
  MXPredForward(h2);
  MXPredGetOutputShape(h2, 0, &osh, &ond);
  printf("SHAPE2 %u %u\n", osh[0], osh[1]);
  /* a bad key reports an error instead of crashing */
  int rc = MXPredSetInput(h2, "nope", (const float*)input, 16);
  printf("BADKEY %d %s\n", rc, MXGetLastError());
  NDListHandle nl; uint32_t n;
  if (MXNDListCreate(params, (int)ps, &nl, &n)) { printf("ERR %s\n", MXGetLastError()); return 1; }
  const char* k; const float* d; const uint32_t* s; uint32_t nd;
  MXNDListGet(nl, 0, &k, &d, &s, &nd);
  printf("NDLIST %u %s %u\n", n, k, nd);
  MXNDListFree(nl);
  MXPredFree(h2);
  MXPredFree(h);
  return 0;
}
'''


def _model(tmp):
    data = mx.sym.Variable('data')
    net = mx.sym.FullyConnected(data, num_hidden=16, name='fc1')
    net = mx.sym.Activation(net, act_type='relu')
    net = mx.sym.FullyConnected(net, num_hidden=5, name='fc2')
    net = mx.sym.softmax(net, name='prob')
    rng = np.random.RandomState(0)
    params = {'arg:fc1_weight': mx.nd.array(rng.randn(16, 8) * 0.3), 'arg:fc1_bias': mx.nd.array(rng.randn(16)),
              'arg:fc2_weight': mx.nd.array(rng.randn(5, 16) * 0.3), 'arg:fc2_bias': mx.nd.array(rng.randn(5))}
    js, ps, xs = (os.path.join(tmp, n) for n in ('net.json', 'net.params', 'input.bin'))
    with open(js, 'w') as f:
        f.write(net.tojson())
    mx.nd.save(ps, params)
    x = rng.randn(4, 8).astype(np.float32)
    x.tofile(xs)
    ex = net.bind(mx.cpu(), {'data': mx.nd.array(x), **{k[4:]: v for k, v in params.items()}})
    ref = ex.forward()[0].asnumpy()
    return js, ps, xs, x, ref


@pytest.fixture(scope='module')
def lib_path():
    if not os.path.exists(LIB):
        pytest.skip('libmxamd_predict.so not built (tools/build_native.py)')
    return LIB


def test_c_program_embeds_the_framework(tmp_path, lib_path):
    js, ps, xs, x, ref = _model(str(tmp_path))
    src = tmp_path / 'predict.c'
    src.write_text(C_PROGRAM)
    exe = tmp_path / 'predict'
    subprocess.check_call(['gcc', '-O1', str(src), '-I', os.path.join(ROOT, 'include'), '-o', str(exe),
                           lib_path, '-Wl,-rpath,' + os.path.dirname(lib_path)])
    env = {k: v for k, v in os.environ.items() if k != 'PYTHONPATH'}
    out = subprocess.run([str(exe), js, ps, xs], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = {l.split()[0]: l.split()[1:] for l in out.stdout.splitlines() if l}
    assert lines['SHAPE'] == ['2', '4', '5']
    np.testing.assert_allclose(np.array(lines['OUT'], dtype=np.float32).reshape(4, 5), ref, rtol=1e-5, atol=1e-6)
    assert lines['SHAPE2'] == ['2', '5']
    assert lines['BADKEY'][0] == '-1' and 'nope' in ' '.join(lines['BADKEY'])
    assert lines['NDLIST'][0] == '4'


def test_ctypes_inside_python(tmp_path, lib_path):
    js, ps, xs, x, ref = _model(str(tmp_path))
    lib = ctypes.CDLL(lib_path)
    h = ctypes.c_void_p()
    keys = (ctypes.c_char_p * 1)(b'data')
    indptr = (ctypes.c_uint32 * 2)(0, 2)
    shape = (ctypes.c_uint32 * 2)(4, 8)
    pbytes = open(ps, 'rb').read()
    assert lib.MXPredCreate(open(js).read().encode(), pbytes, len(pbytes), 1, 0, 1, keys, indptr, shape,
                            ctypes.byref(h)) == 0, lib.MXGetLastError
    buf = np.ascontiguousarray(x)
    assert lib.MXPredSetInput(h, b'data', buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 32) == 0
    assert lib.MXPredForward(h) == 0
    out = np.zeros((4, 5), dtype=np.float32)
    assert lib.MXPredGetOutput(h, 0, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 20) == 0
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)
    assert lib.MXPredFree(h) == 0
