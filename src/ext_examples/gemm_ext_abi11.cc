// A self-contained operator library speaking the extension ABI version 11 (the C entry points a
// library built on the reference's include/mxnet/lib_api.h exports; see
// mxnet_maintenance_amd/library.py).  Written from the ABI's function signatures only, so the
// loader can be tested without compiling third-party code.  Two CPU operators:
//   ext_gemm        C = A . B        (stateless; backward dA = dC . B^T, dB = A^T . dC)
//   ext_state_gemm  the same through a stateful op object (counts its forward calls)
// Build: g++ -shared -fPIC -O2 gemm_ext_abi11.cc -o libgemm_ext_abi11.so
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

typedef void* (*xpu_malloc_t)(void*, int);

std::vector<std::string> g_msgs;

const char* kCpu = "cpu";
// per-op tables handed out by _opRegGet (stable addresses)
const char* g_ctx[1] = {kCpu};
void* g_fwd_fp[1];
void* g_bwd_fp[1];
void* g_state_fp[1];

int fail(const std::string& m) {
  g_msgs.push_back(m);
  return 0;
}

void gemm(const float* a, const float* b, float* c, int n, int k, int m, bool ta, bool tb) {
  // c[n,m] = op(a)[n,k] . op(b)[k,m]; ta: a stored [k,n]; tb: b stored [m,k]
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      float s = 0.f;
      for (int p = 0; p < k; ++p) s += (ta ? a[p * n + i] : a[i * k + p]) * (tb ? b[j * k + p] : b[p * m + j]);
      c[i * m + j] = s;
    }
}

// marker functions: the loader only passes these pointers back to _opCallFCompute
int fwd_marker() { return 1; }
int bwd_marker() { return 2; }
int state_marker() { return 3; }

struct GemmState {
  int calls = 0;
};

int run(bool forward, const int64_t** inshapes, void** indata, int* intypes, int num_in, void** outdata,
        int num_out) {
  for (int i = 0; i < num_in; ++i)
    if (intypes[i] != 0) return fail("ext_gemm: float32 inputs only");
  if (forward) {
    if (num_in != 2 || num_out != 1) return fail("ext_gemm: forward takes 2 inputs, 1 output");
    const int n = (int)inshapes[0][0], k = (int)inshapes[0][1], m = (int)inshapes[1][1];
    gemm((const float*)indata[0], (const float*)indata[1], (float*)outdata[0], n, k, m, false, false);
    return 1;
  }
  // backward inputs: [dC, A, B, C], outputs: [dA, dB]
  if (num_in != 4 || num_out != 2) return fail("ext_gemm: backward takes 4 inputs, 2 outputs");
  const int n = (int)inshapes[1][0], k = (int)inshapes[1][1], m = (int)inshapes[2][1];
  const float* dc = (const float*)indata[0];
  gemm(dc, (const float*)indata[2], (float*)outdata[0], n, m, k, false, true);   // dA = dC . B^T
  gemm((const float*)indata[1], dc, (float*)outdata[1], k, n, m, true, false);   // dB = A^T . dC
  return 1;
}

}  // namespace

extern "C" {

int initialize(int version) { return version >= 10700 ? 1 : 0; }
int _opVersion() { return 11; }
int _opRegSize() { return 2; }

void _opRegGet(int idx, const char** name, int* isSGop, const char*** forward_ctx, void*** forward_fp,
               int* forward_count, const char*** backward_ctx, void*** backward_fp, int* backward_count,
               const char*** create_op_ctx, void*** create_op_fp, int* create_op_count, void** parse,
               void** type, void** stype, void** shape, void** mutate) {
  g_fwd_fp[0] = (void*)&fwd_marker;
  g_bwd_fp[0] = (void*)&bwd_marker;
  g_state_fp[0] = (void*)&state_marker;
  *name = idx == 0 ? "ext_gemm" : "ext_state_gemm";
  *isSGop = 0;
  *forward_ctx = g_ctx;
  *backward_ctx = g_ctx;
  *create_op_ctx = g_ctx;
  *forward_fp = g_fwd_fp;
  *backward_fp = g_bwd_fp;
  *create_op_fp = g_state_fp;
  *forward_count = idx == 0 ? 1 : 0;
  *backward_count = idx == 0 ? 1 : 0;
  *create_op_count = idx == 0 ? 0 : 1;
  *parse = (void*)&fwd_marker;
  *type = (void*)&fwd_marker;
  *stype = nullptr;
  *shape = (void*)&fwd_marker;
  *mutate = nullptr;
}

void _opCallFree(void* ptr) { free(ptr); }

int _opCallParseAttrs(void*, const char* const*, const char* const*, int, int* num_in, int* num_out) {
  *num_in = 2;
  *num_out = 1;
  return 1;
}

int _opCallInferShape(void*, const char* const*, const char* const*, int, unsigned int** inshapes, int* indims,
                      int num_in, unsigned int*** mod_inshapes, int** mod_indims, unsigned int*** outshapes,
                      int** outdims, int num_out) {
  if (num_in != 2 || indims[0] != 2 || indims[1] != 2) return fail("ext_gemm: two 2-D inputs expected");
  if (inshapes[0][1] != inshapes[1][0]) return fail("ext_gemm: inner dimensions differ");
  *mod_indims = (int*)malloc(num_in * sizeof(int));
  *mod_inshapes = (unsigned**)malloc(num_in * sizeof(unsigned*));
  for (int i = 0; i < num_in; ++i) {
    (*mod_indims)[i] = 2;
    (*mod_inshapes)[i] = (unsigned*)malloc(2 * sizeof(unsigned));
    memcpy((*mod_inshapes)[i], inshapes[i], 2 * sizeof(unsigned));
  }
  *outdims = (int*)malloc(num_out * sizeof(int));
  *outshapes = (unsigned**)malloc(num_out * sizeof(unsigned*));
  (*outdims)[0] = 2;
  (*outshapes)[0] = (unsigned*)malloc(2 * sizeof(unsigned));
  (*outshapes)[0][0] = inshapes[0][0];
  (*outshapes)[0][1] = inshapes[1][1];
  return 1;
}

int _opCallInferType(void*, const char* const*, const char* const*, int, int* intypes, int num_in, int* outtypes,
                     int) {
  for (int i = 0; i < num_in; ++i)
    if (intypes[i] != 0) return fail("ext_gemm: float32 inputs only");
  outtypes[0] = intypes[0];
  return 1;
}

int _opCallFCompute(void* fcomp, const char* const*, const char* const*, int, const int64_t** inshapes, int*,
                    void** indata, int* intypes, size_t*, const char**, int*, int num_in, const int64_t**, int*,
                    void** outdata, int*, size_t*, const char**, int*, int num_out, xpu_malloc_t cpu_malloc,
                    void* cpu_alloc, xpu_malloc_t, void*, void*, void*, void*, int*, int*, void**, void**, void**,
                    void**, int64_t*, int64_t*, int64_t*, int64_t*, void*, void*) {
  // exercise the workspace callback like a real library would (res.alloc_cpu)
  void* ws = cpu_malloc(cpu_alloc, 64);
  if (ws == nullptr) return fail("ext_gemm: workspace allocation failed");
  return run(fcomp == (void*)&fwd_marker, inshapes, indata, intypes, num_in, outdata, num_out);
}

int _opCallCreateOpState(void*, const char* const*, const char* const*, int, const char* dev_type, int,
                         unsigned int**, int*, int, const int*, void** state_op) {
  if (strcmp(dev_type, "cpu") != 0) return fail("ext_state_gemm: cpu only");
  *state_op = new GemmState();
  return 1;
}

void _opCallDestroyOpState(void* state_op) { delete static_cast<GemmState*>(state_op); }

int _opCallFStatefulCompute(int is_forward, void* state_op, const int64_t** inshapes, int*, void** indata,
                            int* intypes, size_t*, const char**, int*, int num_in, const int64_t**, int*,
                            void** outdata, int*, size_t*, const char**, int*, int num_out, xpu_malloc_t, void*,
                            xpu_malloc_t, void*, void*, void*, void*, int*, int*, void**, void**, void**, void**,
                            int64_t*, int64_t*, int64_t*, int64_t*, void*, void*) {
  if (is_forward) static_cast<GemmState*>(state_op)->calls++;
  return run(is_forward != 0, inshapes, indata, intypes, num_in, outdata, num_out);
}

int _opCallMutateInputs(void*, const char* const*, const char* const*, int, int**, int* indices_size) {
  *indices_size = 0;
  return 1;
}

int _partRegSize() { return 0; }
int _passRegSize() { return 0; }
int _msgSize() { return (int)g_msgs.size(); }
void _msgGet(int idx, const char** msg) { *msg = g_msgs[idx].c_str(); }

}  // extern "C"
