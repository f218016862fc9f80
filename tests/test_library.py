"""mx.library.load: a native extension library (C ABI, built here with gcc) registers operators
usable imperatively, under autograd and in symbolic graphs (reference library.py / lib_api.h)."""
import os
import subprocess

import numpy as np
import pytest

import mxnet_maintenance_amd as mx

_SRC = r'''
#include <stdint.h>
const char* mxamd_ext_ops(void) {
  return "[{\"name\": \"ext_scale2\", \"num_inputs\": 1, \"backward\": true},"
         " {\"name\": \"ext_addmul\", \"num_inputs\": 2, \"backward\": false}]";
}
static int64_t numel(const int64_t* s, int nd) { int64_t n = 1; for (int i = 0; i < nd; ++i) n *= s[i]; return n; }
int ext_scale2_forward(int n_in, const void** in, void* out, const int64_t* shape, int nd, int dtype, void* stream) {
  if (dtype != 0) return 1;
  const float* x = (const float*)in[0]; float* y = (float*)out;
  for (int64_t i = 0; i < numel(shape, nd); ++i) y[i] = 2.f * x[i];
  return 0;
}
int ext_scale2_backward(int n_in, const void** in, const void* gout, void** gin, const int64_t* shape, int nd,
                        int dtype, void* stream) {
  const float* g = (const float*)gout; float* gx = (float*)gin[0];
  for (int64_t i = 0; i < numel(shape, nd); ++i) gx[i] = 2.f * g[i];
  return 0;
}
int ext_addmul_forward(int n_in, const void** in, void* out, const int64_t* shape, int nd, int dtype, void* stream) {
  const float* a = (const float*)in[0]; const float* b = (const float*)in[1]; float* y = (float*)out;
  for (int64_t i = 0; i < numel(shape, nd); ++i) y[i] = (a[i] + b[i]) * b[i];
  return 0;
}
'''


@pytest.fixture(scope='module')
def extlib(tmp_path_factory):
    d = tmp_path_factory.mktemp('ext')
    src = d / 'ext.c'
    src.write_text(_SRC)
    so = str(d / 'libext.so')
    subprocess.check_call(['gcc', '-shared', '-fPIC', '-O2', str(src), '-o', so])
    mx.library.load(so, verbose=False)
    return so


def test_extension_ops_imperative_autograd_symbolic(extlib):
    x = mx.nd.array(np.arange(6, dtype='float32').reshape(2, 3))
    np.testing.assert_allclose(mx.nd.ext_scale2(x).asnumpy(), 2 * x.asnumpy())
    b = mx.nd.ones((2, 3)) * 3
    np.testing.assert_allclose(mx.nd.ext_addmul(x, b).asnumpy(), (x.asnumpy() + 3) * 3)
    x.attach_grad()
    with mx.autograd.record():
        y = (mx.nd.ext_scale2(x) * x).sum()
    y.backward()
    np.testing.assert_allclose(x.grad.asnumpy(), 4 * x.asnumpy())
    data = mx.sym.var('data')
    net = mx.sym.ext_scale2(data) + 1
    ex = net.bind(mx.cpu(), {'data': x})
    np.testing.assert_allclose(ex.forward()[0].asnumpy(), 2 * x.asnumpy() + 1)
    assert extlib in mx.library.loaded_libraries()


def test_load_rejects_bad_paths(tmp_path):
    with pytest.raises(mx.MXNetError):
        mx.library.load('/nonexistent/lib.so')
    with pytest.raises(mx.MXNetError):
        mx.library.load('relative.so')
    p = tmp_path / 'x.txt'
    p.write_text('')
    with pytest.raises(mx.MXNetError):
        mx.library.load(str(p))
