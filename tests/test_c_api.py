"""The general C API (libmxamd.so, include/mxamd/c_api.h): a plain C program creates NDArrays, invokes
operators imperatively with autograd, builds a symbol from JSON and composes one from atomic symbols,
binds an executor (forward + backward) and round-trips a kvstore -- checked against the framework."""
import os
import subprocess

import numpy as np
import pytest

import mxnet_maintenance_amd as mx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'mxnet_maintenance_amd', '_lib', 'libmxamd.so')

C_PROGRAM = r'''
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "mxamd/c_api.h"

#define CHECK(x) do { if ((x) != 0) { printf("ERR %s: %s\n", #x, MXGetLastError()); return 1; } } while (0)

static char* slurp(const char* path) {
  FILE* f = fopen(path, "rb"); fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
  char* buf = (char*)malloc(n + 1); size_t got = fread(buf, 1, n, f); buf[got] = 0; fclose(f); return buf;
}

int main(int argc, char** argv) {
  int ver; CHECK(MXGetVersion(&ver)); printf("VERSION %d\n", ver);
  /* NDArrays */
  uint32_t shp[2] = {2, 3};
  NDArrayHandle a, b;
  CHECK(MXNDArrayCreateEx(shp, 2, 1, 0, 0, 0, &a));
  CHECK(MXNDArrayCreateEx(shp, 2, 1, 0, 0, 0, &b));
  float va[6] = {1, 2, 3, 4, 5, 6}, vb[6] = {0.5f, -1, 2, 0, 1, 3};
  CHECK(MXNDArraySyncCopyFromCPU(a, va, 6));
  CHECK(MXNDArraySyncCopyFromCPU(b, vb, 6));
  uint32_t nd; const uint32_t* pd; int dt, dev, did;
  CHECK(MXNDArrayGetShape(a, &nd, &pd)); CHECK(MXNDArrayGetDType(a, &dt)); CHECK(MXNDArrayGetContext(a, &dev, &did));
  printf("SHAPE %u %u %u DTYPE %d CTX %d %d\n", nd, pd[0], pd[1], dt, dev, did);
  /* imperative invoke with autograd: y = sum(a * b) -> da = b */
  OpHandle mul, sum;
  CHECK(NNGetOpHandle("elemwise_mul", &mul)); CHECK(NNGetOpHandle("sum", &sum));
  NDArrayHandle ga; CHECK(MXNDArrayCreateEx(shp, 2, 1, 0, 0, 0, &ga));
  uint32_t req = 1;
  CHECK(MXAutogradMarkVariables(1, &a, &req, &ga));
  int prev; CHECK(MXAutogradSetIsRecording(1, &prev));
  NDArrayHandle in2[2] = {a, b}; int nout = 0; NDArrayHandle* outs = NULL;
  CHECK(MXImperativeInvoke(mul, 2, in2, &nout, &outs, 0, NULL, NULL));
  NDArrayHandle prod = outs[0];
  nout = 0; outs = NULL;
  CHECK(MXImperativeInvoke(sum, 1, &prod, &nout, &outs, 0, NULL, NULL));
  NDArrayHandle s = outs[0];
  CHECK(MXAutogradSetIsRecording(0, &prev));
  CHECK(MXAutogradBackward(1, &s, NULL, 0));
  float sv[1]; CHECK(MXNDArraySyncCopyToCPU(s, sv, 1)); printf("SUM %.4f\n", sv[0]);
  NDArrayHandle g; CHECK(MXNDArrayGetGrad(a, &g));
  float gv[6]; CHECK(MXNDArraySyncCopyToCPU(g, gv, 6));
  printf("GRAD"); for (int i = 0; i < 6; ++i) printf(" %.3f", gv[i]); printf("\n");
  /* operator with parameters */
  const char* keys[1] = {"axis"}; const char* vals[1] = {"1"};
  nout = 0; outs = NULL;
  CHECK(MXImperativeInvoke(sum, 1, &a, &nout, &outs, 1, keys, vals));
  float rs[2]; CHECK(MXNDArraySyncCopyToCPU(outs[0], rs, 2)); printf("ROWSUM %.1f %.1f\n", rs[0], rs[1]);
  /* bad operator name reports an error */
  OpHandle bad; printf("BADOP %d\n", NNGetOpHandle("no_such_op_xyz", &bad));
  /* save / load */
  const char* names[2] = {"a", "b"}; NDArrayHandle ab[2] = {a, b};
  CHECK(MXNDArraySave(argv[2], 2, ab, names));
  uint32_t nl, nn; NDArrayHandle* la; const char** ln;
  CHECK(MXNDArrayLoad(argv[2], &nl, &la, &nn, &ln));
  printf("LOADED %u %u %s %s\n", nl, nn, ln[0], ln[1]);
  /* symbols: JSON file, list arguments, compose FC from atomic symbols */
  char* json = slurp(argv[1]);
  SymbolHandle net; CHECK(MXSymbolCreateFromJSON(json, &net));
  uint32_t na; const char** an; CHECK(MXSymbolListArguments(net, &na, &an));
  printf("ARGS %u", na); for (uint32_t i = 0; i < na; ++i) printf(" %s", an[i]); printf("\n");
  SymbolHandle data, fc; CHECK(MXSymbolCreateVariable("data", &data));
  OpHandle fcop; CHECK(NNGetOpHandle("FullyConnected", &fcop));
  const char* fk[1] = {"num_hidden"}; const char* fv[1] = {"4"};
  CHECK(MXSymbolCreateAtomicSymbol(fcop, 1, fk, fv, &fc));
  const char* ck[1] = {"data"};
  CHECK(MXSymbolCompose(fc, "fcx", 1, ck, &data));
  CHECK(MXSymbolListArguments(fc, &na, &an));
  printf("FCARGS %u", na); for (uint32_t i = 0; i < na; ++i) printf(" %s", an[i]); printf("\n");
  const char* ik[1] = {"data"}; uint32_t ip[2] = {0, 2}, isd[2] = {5, 7};
  uint32_t ins, outsz, auxs; const uint32_t *ind, *ond, *aund; const uint32_t **idat, **odat, **adat; int complete;
  CHECK(MXSymbolInferShape(fc, 1, ik, ip, isd, &ins, &ind, &idat, &outsz, &ond, &odat, &auxs, &aund, &adat, &complete));
  printf("INFER %u %u %u %u complete %d\n", ins, idat[1][0], idat[1][1], odat[0][1], complete);
  /* executor on the JSON net: forward + backward */
  uint32_t xs[2] = {4, 8}, ws[2] = {3, 8}, bs[1] = {3};
  NDArrayHandle x, w, bb, gx, gw, gb;
  CHECK(MXNDArrayCreateEx(xs, 2, 1, 0, 0, 0, &x)); CHECK(MXNDArrayCreateEx(ws, 2, 1, 0, 0, 0, &w));
  CHECK(MXNDArrayCreateEx(bs, 1, 1, 0, 0, 0, &bb));
  CHECK(MXNDArrayCreateEx(xs, 2, 1, 0, 0, 0, &gx)); CHECK(MXNDArrayCreateEx(ws, 2, 1, 0, 0, 0, &gw));
  CHECK(MXNDArrayCreateEx(bs, 1, 1, 0, 0, 0, &gb));
  float xv[32], wv[24], bv[3] = {0.1f, 0.2f, 0.3f};
  for (int i = 0; i < 32; ++i) xv[i] = (float)((i % 7) - 3) * 0.25f;
  for (int i = 0; i < 24; ++i) wv[i] = (float)((i % 5) - 2) * 0.5f;
  CHECK(MXNDArraySyncCopyFromCPU(x, xv, 32)); CHECK(MXNDArraySyncCopyFromCPU(w, wv, 24));
  CHECK(MXNDArraySyncCopyFromCPU(bb, bv, 3));
  NDArrayHandle args[3] = {x, w, bb}, grads[3] = {gx, gw, gb}; uint32_t reqs[3] = {1, 1, 1};
  ExecutorHandle ex;
  CHECK(MXExecutorBind(net, 1, 0, 3, args, grads, reqs, 0, NULL, &ex));
  CHECK(MXExecutorForward(ex, 1));
  uint32_t no; NDArrayHandle* eo; CHECK(MXExecutorOutputs(ex, &no, &eo));
  float ov[12]; CHECK(MXNDArraySyncCopyToCPU(eo[0], ov, 12));
  printf("FWD"); for (int i = 0; i < 12; ++i) printf(" %.5f", ov[i]); printf("\n");
  uint32_t os2[2] = {4, 3}; NDArrayHandle head; CHECK(MXNDArrayCreateEx(os2, 2, 1, 0, 0, 0, &head));
  float ones[12]; for (int i = 0; i < 12; ++i) ones[i] = 1.0f;
  CHECK(MXNDArraySyncCopyFromCPU(head, ones, 12));
  CHECK(MXExecutorBackward(ex, 1, &head));
  float gbv[3]; CHECK(MXNDArraySyncCopyToCPU(gb, gbv, 3)); printf("GB %.1f %.1f %.1f\n", gbv[0], gbv[1], gbv[2]);
  /* kvstore */
  KVStoreHandle kv; CHECK(MXKVStoreCreate("local", &kv));
  int key = 3; CHECK(MXKVStoreInit(kv, 1, &key, &a));
  CHECK(MXKVStorePush(kv, 1, &key, &b, 0));
  NDArrayHandle pulled; CHECK(MXNDArrayCreateEx(shp, 2, 1, 0, 0, 0, &pulled));
  CHECK(MXKVStorePull(kv, 1, &key, &pulled, 0));
  float pv[6]; CHECK(MXNDArraySyncCopyToCPU(pulled, pv, 6));
  printf("KV"); for (int i = 0; i < 6; ++i) printf(" %.2f", pv[i]); printf("\n");
  CHECK(MXKVStoreFree(kv)); CHECK(MXExecutorFree(ex)); CHECK(MXSymbolFree(net)); CHECK(MXSymbolFree(fc));
  CHECK(MXNDArrayFree(a)); CHECK(MXNDArrayFree(b));
  CHECK(MXNDArrayWaitAll());
  printf("DONE\n");
  return 0;
}
'''


@pytest.fixture(scope='module')
def lib_path():
    if not os.path.exists(LIB):
        pytest.skip('libmxamd.so not built (tools/build_native.py)')
    return LIB


def test_c_program_drives_ndarray_autograd_symbol_executor_kvstore(tmp_path, lib_path):
    data = mx.sym.Variable('data')
    net = mx.sym.FullyConnected(data, num_hidden=3, name='fc')
    js = tmp_path / 'net.json'
    js.write_text(net.tojson())
    src = tmp_path / 'capi.c'
    src.write_text(C_PROGRAM)
    exe = tmp_path / 'capi'
    subprocess.check_call(['gcc', '-O1', str(src), '-I', os.path.join(ROOT, 'include'), '-o', str(exe),
                           lib_path, '-Wl,-rpath,' + os.path.dirname(lib_path)])
    env = {k: v for k, v in os.environ.items() if k != 'PYTHONPATH'}
    out = subprocess.run([str(exe), str(js), str(tmp_path / 'arrs.params')], capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    L = {l.split()[0]: l.split()[1:] for l in out.stdout.splitlines() if l}
    assert 'DONE' in L
    assert L['SHAPE'] == ['2', '2', '3', 'DTYPE', '0', 'CTX', '1', '0']
    va = np.array([1, 2, 3, 4, 5, 6], np.float32)
    vb = np.array([0.5, -1, 2, 0, 1, 3], np.float32)
    assert abs(float(L['SUM'][0]) - float((va * vb).sum())) < 1e-4
    np.testing.assert_allclose(np.array(L['GRAD'], np.float32), vb, atol=1e-3)
    assert L['ROWSUM'] == ['6.0', '15.0']
    assert L['BADOP'] == ['-1']
    assert L['LOADED'] == ['2', '2', 'a', 'b']
    assert L['ARGS'] == ['3', 'data', 'fc_weight', 'fc_bias']
    assert L['FCARGS'] == ['3', 'data', 'fcx_weight', 'fcx_bias']
    assert L['INFER'][:4] == ['3', '4', '7', '4'] and L['INFER'][-1] == '1'
    xv = np.array([((i % 7) - 3) * 0.25 for i in range(32)], np.float32).reshape(4, 8)
    wv = np.array([((i % 5) - 2) * 0.5 for i in range(24)], np.float32).reshape(3, 8)
    ref = xv @ wv.T + np.array([0.1, 0.2, 0.3], np.float32)
    np.testing.assert_allclose(np.array(L['FWD'], np.float32).reshape(4, 3), ref, rtol=1e-5, atol=1e-5)
    assert L['GB'] == ['4.0', '4.0', '4.0']
    np.testing.assert_allclose(np.array(L['KV'], np.float32), vb, atol=1e-6)   # local store: push replaces
