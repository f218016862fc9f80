// C predict API: libmxamd_predict.so.
//
// Parity: include/mxnet/c_predict_api.h (MXPredCreate / CreateEx / CreatePartialOut / Reshape /
// SetInput / Forward / GetOutputShape / GetOutputType / GetOutput / Free, MXNDListCreate / Get /
// Free, MXGetLastError) -- the reference implements them over its C++ executor
// (src/c_api/c_predict_api.cc).  Here the executor is the Python framework (HIP kernels on the
// GPU), so this library embeds CPython when the host application has no interpreter (a plain C/C++
// program) or joins the running one when loaded into Python (ctypes).  Every entry point takes the
// GIL, forwards to mxnet_maintenance_amd.c_predict and converts errors into the -1 return code +
// MXGetLastError() contract.  Pointers returned to the caller (shapes, keys, data) stay valid
// until the next call on the same handle, as the reference documents.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_last_error;

struct Predictor {
  PyObject* obj = nullptr;             // mxnet_maintenance_amd.c_predict.Predictor
  std::vector<uint32_t> shape;         // last MXPredGetOutputShape result
};

struct NDList {
  std::vector<std::string> keys;
  std::vector<std::vector<float>> data;
  std::vector<std::vector<uint32_t>> shapes;
};

// Directory that holds the package: the library lives in <root>/mxnet_maintenance_amd/_lib/.
std::string package_root() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&package_root), &info) == 0 || info.dli_fname == nullptr) return "";
  std::string path(info.dli_fname);
  for (int up = 0; up < 3; ++up) {
    const size_t cut = path.find_last_of('/');
    if (cut == std::string::npos) return "";
    path.resize(cut);
  }
  return path;
}

bool ensure_python() {
  if (Py_IsInitialized()) return true;
  Py_InitializeEx(0);
  PyGILState_STATE st = PyGILState_Ensure();
  const std::string root = package_root();
  if (!root.empty()) {
    PyObject* sys_path = PySys_GetObject("path");  // borrowed
    PyObject* entry = PyUnicode_FromString(root.c_str());
    if (sys_path && entry) PyList_Insert(sys_path, 0, entry);
    Py_XDECREF(entry);
  }
  PyGILState_Release(st);
  // the embedding thread keeps no GIL: every API call takes it through PyGILState_Ensure
  PyEval_SaveThread();
  return true;
}

// RAII GIL holder
struct Gil {
  PyGILState_STATE st;
  Gil() { st = PyGILState_Ensure(); }
  ~Gil() { PyGILState_Release(st); }
};

int fail_from_python() {
  PyObject *type = nullptr, *value = nullptr, *tb = nullptr;
  PyErr_Fetch(&type, &value, &tb);
  PyErr_NormalizeException(&type, &value, &tb);
  g_last_error = "unknown error";
  if (value) {
    PyObject* s = PyObject_Str(value);
    if (s) {
      const char* c = PyUnicode_AsUTF8(s);
      if (c) g_last_error = c;
      Py_DECREF(s);
    }
  }
  if (type) {
    PyObject* name = PyObject_GetAttrString(type, "__name__");
    if (name) {
      const char* c = PyUnicode_AsUTF8(name);
      if (c) g_last_error = std::string(c) + ": " + g_last_error;
      Py_DECREF(name);
    }
  }
  PyErr_Clear();
  Py_XDECREF(type);
  Py_XDECREF(value);
  Py_XDECREF(tb);
  return -1;
}

int fail(const char* msg) {
  g_last_error = msg;
  return -1;
}

PyObject* module() {
  static PyObject* mod = nullptr;  // kept for the process lifetime
  if (mod == nullptr) mod = PyImport_ImportModule("mxnet_maintenance_amd.c_predict");
  return mod;
}

PyObject* str_list(uint32_t n, const char** items) {
  PyObject* lst = PyList_New(n);
  for (uint32_t i = 0; lst && i < n; ++i) PyList_SET_ITEM(lst, i, PyUnicode_FromString(items[i]));
  return lst;
}

PyObject* shape_list(uint32_t n, const uint32_t* indptr, const uint32_t* data) {
  PyObject* lst = PyList_New(n);
  for (uint32_t i = 0; lst && i < n; ++i) {
    PyObject* shp = PyTuple_New(indptr[i + 1] - indptr[i]);
    for (uint32_t j = indptr[i]; j < indptr[i + 1]; ++j)
      PyTuple_SET_ITEM(shp, j - indptr[i], PyLong_FromUnsignedLong(data[j]));
    PyList_SET_ITEM(lst, i, shp);
  }
  return lst;
}

int create_impl(const char* json, const void* params, int param_size, int dev_type, int dev_id, uint32_t num_in,
                const char** keys, const uint32_t* indptr, const uint32_t* shapes, uint32_t num_dt,
                const char** dt_names, const int* dt_codes, uint32_t num_out, const char** out_keys, void** out) {
  if (!json || !out) return fail("MXPredCreate: null symbol or output handle");
  ensure_python();
  Gil gil;
  PyObject* mod = module();
  if (!mod) return fail_from_python();
  PyObject* codes_list = PyList_New(num_dt);
  for (uint32_t i = 0; i < num_dt; ++i) PyList_SET_ITEM(codes_list, i, PyLong_FromLong(dt_codes[i]));
  PyObject* res = PyObject_CallMethod(
      mod, "create", "sy#iiNNNNN", json, static_cast<const char*>(params), static_cast<Py_ssize_t>(param_size),
      dev_type, dev_id, str_list(num_in, keys), shape_list(num_in, indptr, shapes), str_list(num_dt, dt_names),
      codes_list, str_list(num_out, out_keys));
  if (!res) return fail_from_python();
  Predictor* p = new Predictor();
  p->obj = res;
  *out = p;
  return 0;
}

}  // namespace

// shared with c_api.cc (same library): the embedded interpreter and the last-error slot
namespace mxamd_capi {
bool ensure_python() { return ::ensure_python(); }
int fail_from_python() { return ::fail_from_python(); }
int fail(const char* msg) { return ::fail(msg); }
}  // namespace mxamd_capi

extern "C" {

typedef void* PredictorHandle;
typedef void* NDListHandle;

__attribute__((visibility("default"))) const char* MXGetLastError() { return g_last_error.c_str(); }

__attribute__((visibility("default"))) int MXPredCreate(const char* symbol_json_str, const void* param_bytes,
                                                        int param_size, int dev_type, int dev_id,
                                                        uint32_t num_input_nodes, const char** input_keys,
                                                        const uint32_t* input_shape_indptr,
                                                        const uint32_t* input_shape_data, PredictorHandle* out) {
  return create_impl(symbol_json_str, param_bytes, param_size, dev_type, dev_id, num_input_nodes, input_keys,
                     input_shape_indptr, input_shape_data, 0, nullptr, nullptr, 0, nullptr, out);
}

__attribute__((visibility("default"))) int MXPredCreateEx(
    const char* symbol_json_str, const void* param_bytes, int param_size, int dev_type, int dev_id,
    const uint32_t num_input_nodes, const char** input_keys, const uint32_t* input_shape_indptr,
    const uint32_t* input_shape_data, const uint32_t num_provided_arg_dtypes, const char** provided_arg_dtype_names,
    const int* provided_arg_dtypes, PredictorHandle* out) {
  return create_impl(symbol_json_str, param_bytes, param_size, dev_type, dev_id, num_input_nodes, input_keys,
                     input_shape_indptr, input_shape_data, num_provided_arg_dtypes, provided_arg_dtype_names,
                     provided_arg_dtypes, 0, nullptr, out);
}

__attribute__((visibility("default"))) int MXPredCreatePartialOut(
    const char* symbol_json_str, const void* param_bytes, int param_size, int dev_type, int dev_id,
    uint32_t num_input_nodes, const char** input_keys, const uint32_t* input_shape_indptr,
    const uint32_t* input_shape_data, uint32_t num_output_nodes, const char** output_keys, PredictorHandle* out) {
  return create_impl(symbol_json_str, param_bytes, param_size, dev_type, dev_id, num_input_nodes, input_keys,
                     input_shape_indptr, input_shape_data, 0, nullptr, nullptr, num_output_nodes, output_keys, out);
}

__attribute__((visibility("default"))) int MXPredReshape(uint32_t num_input_nodes, const char** input_keys,
                                                         const uint32_t* input_shape_indptr,
                                                         const uint32_t* input_shape_data, PredictorHandle handle,
                                                         PredictorHandle* out) {
  if (!handle || !out) return fail("MXPredReshape: null handle");
  Gil gil;
  Predictor* p = static_cast<Predictor*>(handle);
  PyObject* shapes = PyDict_New();
  PyObject* keys = str_list(num_input_nodes, input_keys);
  PyObject* vals = shape_list(num_input_nodes, input_shape_indptr, input_shape_data);
  for (uint32_t i = 0; i < num_input_nodes; ++i)
    PyDict_SetItem(shapes, PyList_GET_ITEM(keys, i), PyList_GET_ITEM(vals, i));
  Py_DECREF(keys);
  Py_DECREF(vals);
  PyObject* res = PyObject_CallMethod(p->obj, "reshape", "N", shapes);
  if (!res) return fail_from_python();
  Predictor* q = new Predictor();
  q->obj = res;
  *out = q;
  return 0;
}

__attribute__((visibility("default"))) int MXPredSetInput(PredictorHandle handle, const char* key, const float* data,
                                                          uint32_t size) {
  if (!handle || !key || (!data && size)) return fail("MXPredSetInput: null argument");
  Gil gil;
  Predictor* p = static_cast<Predictor*>(handle);
  PyObject* res = PyObject_CallMethod(p->obj, "set_input", "sy#", key, reinterpret_cast<const char*>(data),
                                      static_cast<Py_ssize_t>(size) * static_cast<Py_ssize_t>(sizeof(float)));
  if (!res) return fail_from_python();
  Py_DECREF(res);
  return 0;
}

__attribute__((visibility("default"))) int MXPredForward(PredictorHandle handle) {
  if (!handle) return fail("MXPredForward: null handle");
  Gil gil;
  PyObject* res = PyObject_CallMethod(static_cast<Predictor*>(handle)->obj, "forward", nullptr);
  if (!res) return fail_from_python();
  Py_DECREF(res);
  return 0;
}

__attribute__((visibility("default"))) int MXPredPartialForward(PredictorHandle handle, int step, int* step_left) {
  // the whole graph runs as one program: the first step does all the work
  if (step_left) *step_left = 0;
  return step == 0 ? MXPredForward(handle) : 0;
}

__attribute__((visibility("default"))) int MXPredGetOutputShape(PredictorHandle handle, uint32_t index,
                                                                uint32_t** shape_data, uint32_t* shape_ndim) {
  if (!handle || !shape_data || !shape_ndim) return fail("MXPredGetOutputShape: null argument");
  Gil gil;
  Predictor* p = static_cast<Predictor*>(handle);
  PyObject* res = PyObject_CallMethod(p->obj, "output_shape", "I", index);
  if (!res) return fail_from_python();
  p->shape.clear();
  for (Py_ssize_t i = 0; i < PyList_Size(res); ++i)
    p->shape.push_back(static_cast<uint32_t>(PyLong_AsUnsignedLong(PyList_GET_ITEM(res, i))));
  Py_DECREF(res);
  *shape_data = p->shape.data();
  *shape_ndim = static_cast<uint32_t>(p->shape.size());
  return 0;
}

__attribute__((visibility("default"))) int MXPredGetOutputType(PredictorHandle handle, uint32_t index,
                                                               int* out_dtype) {
  if (!handle || !out_dtype) return fail("MXPredGetOutputType: null argument");
  Gil gil;
  PyObject* res = PyObject_CallMethod(static_cast<Predictor*>(handle)->obj, "output_dtype", "I", index);
  if (!res) return fail_from_python();
  *out_dtype = static_cast<int>(PyLong_AsLong(res));
  Py_DECREF(res);
  return 0;
}

__attribute__((visibility("default"))) int MXPredGetOutput(PredictorHandle handle, uint32_t index, float* data,
                                                           uint32_t size) {
  if (!handle || (!data && size)) return fail("MXPredGetOutput: null argument");
  Gil gil;
  PyObject* res = PyObject_CallMethod(static_cast<Predictor*>(handle)->obj, "output_bytes", "I", index);
  if (!res) return fail_from_python();
  char* buf = nullptr;
  Py_ssize_t len = 0;
  if (PyBytes_AsStringAndSize(res, &buf, &len) != 0) {
    Py_DECREF(res);
    return fail_from_python();
  }
  if (static_cast<size_t>(len) != static_cast<size_t>(size) * sizeof(float)) {
    Py_DECREF(res);
    return fail("MXPredGetOutput: size does not match the output's element count");
  }
  std::memcpy(data, buf, static_cast<size_t>(len));
  Py_DECREF(res);
  return 0;
}

__attribute__((visibility("default"))) int MXPredFree(PredictorHandle handle) {
  if (!handle) return 0;
  {
    Gil gil;
    Py_XDECREF(static_cast<Predictor*>(handle)->obj);
  }
  delete static_cast<Predictor*>(handle);
  return 0;
}

__attribute__((visibility("default"))) int MXNDListCreate(const char* nd_file_bytes, int nd_file_size,
                                                          NDListHandle* out, uint32_t* out_length) {
  if (!nd_file_bytes || !out || !out_length) return fail("MXNDListCreate: null argument");
  ensure_python();
  Gil gil;
  PyObject* mod = module();
  if (!mod) return fail_from_python();
  PyObject* res = PyObject_CallMethod(mod, "nd_list", "y#", nd_file_bytes, static_cast<Py_ssize_t>(nd_file_size));
  if (!res) return fail_from_python();
  NDList* lst = new NDList();
  for (Py_ssize_t i = 0; i < PyList_Size(res); ++i) {
    PyObject* item = PyList_GET_ITEM(res, i);
    const char* key = PyUnicode_AsUTF8(PyTuple_GET_ITEM(item, 0));
    char* buf = nullptr;
    Py_ssize_t len = 0;
    PyBytes_AsStringAndSize(PyTuple_GET_ITEM(item, 1), &buf, &len);
    PyObject* shp = PyTuple_GET_ITEM(item, 2);
    lst->keys.emplace_back(key ? key : "");
    lst->data.emplace_back(reinterpret_cast<float*>(buf), reinterpret_cast<float*>(buf) + len / sizeof(float));
    std::vector<uint32_t> s;
    for (Py_ssize_t j = 0; j < PyList_Size(shp); ++j)
      s.push_back(static_cast<uint32_t>(PyLong_AsUnsignedLong(PyList_GET_ITEM(shp, j))));
    lst->shapes.push_back(std::move(s));
  }
  Py_DECREF(res);
  *out = lst;
  *out_length = static_cast<uint32_t>(lst->keys.size());
  return 0;
}

__attribute__((visibility("default"))) int MXNDListGet(NDListHandle handle, uint32_t index, const char** out_key,
                                                       const float** out_data, const uint32_t** out_shape,
                                                       uint32_t* out_ndim) {
  NDList* lst = static_cast<NDList*>(handle);
  if (!lst || index >= lst->keys.size()) return fail("MXNDListGet: index out of range");
  *out_key = lst->keys[index].c_str();
  *out_data = lst->data[index].data();
  *out_shape = lst->shapes[index].data();
  *out_ndim = static_cast<uint32_t>(lst->shapes[index].size());
  return 0;
}

__attribute__((visibility("default"))) int MXNDListFree(NDListHandle handle) {
  delete static_cast<NDList*>(handle);
  return 0;
}

}  // extern "C"
