// C API (include/mxamd/c_api.h): NDArray / imperative invoke + autograd / Symbol / Executor / KVStore.
//
// Parity: include/mxnet/c_api.h (:591 MXNDArrayCreate, :1242 MXImperativeInvoke, :1551
// MXSymbolCreateFromJSON, :2307 MXExecutorBind) and nnvm's NNGetOpHandle.  The reference backs these
// with its C++ runtime (src/c_api/c_api*.cc); here the runtime is the framework itself (HIP kernels on
// the GPU, the C++ engine/storage underneath), so every handle is a reference to a framework object
// held by the embedded (or host) interpreter -- the same embedding the predict API uses
// (c_predict_api.cc, which also owns MXGetLastError).  Each entry point takes the GIL, forwards to
// mxnet_maintenance_amd.c_api_impl and turns a Python exception into -1 + MXGetLastError().
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mxamd/c_api.h"

#include "capi_internal.h"



MXAPI int MXGetVersion(int* out) {
  Gil g;
  PyObject* mod = impl();
  if (!mod) return fail_from_python();
  PyObject* v = PyObject_GetAttrString(mod, "VERSION");
  if (!v) return fail_from_python();
  *out = static_cast<int>(PyLong_AsLong(v));
  Py_DECREF(v);
  return 0;
}

// ------------------------------------------------------------------------------------------ NDArray
MXAPI int MXNDArrayCreateNone(NDArrayHandle* out) {
  Gil g;
  return new_handle(call("nd_none", PyTuple_New(0)), out);
}

MXAPI int MXNDArrayCreateEx(const uint32_t* shape, uint32_t ndim, int dev_type, int dev_id, int delay_alloc, int dtype,
                            NDArrayHandle* out) {
  (void)delay_alloc;
  Gil g;
  return new_handle(call("nd_create", Py_BuildValue("(Niii)", u32_list(ndim, shape), dev_type, dev_id, dtype)), out);
}

MXAPI int MXNDArrayCreate(const uint32_t* shape, uint32_t ndim, int dev_type, int dev_id, int delay_alloc,
                          NDArrayHandle* out) {
  return MXNDArrayCreateEx(shape, ndim, dev_type, dev_id, delay_alloc, 0, out);
}

MXAPI int MXNDArrayFree(NDArrayHandle handle) { return free_handle(handle); }

MXAPI int MXNDArrayGetShape(NDArrayHandle handle, uint32_t* out_dim, const uint32_t** out_pdata) {
  Gil g;
  Obj* o = static_cast<Obj*>(handle);
  PyObject* r = call("nd_shape", Py_BuildValue("(O)", o->o));
  if (!r) return fail_from_python();
  const bool ok = to_u32(r, &o->u32);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *out_dim = static_cast<uint32_t>(o->u32.size());
  *out_pdata = o->u32.data();
  return 0;
}

MXAPI int MXNDArrayGetDType(NDArrayHandle handle, int* out_dtype) {
  Gil g;
  PyObject* r = call("nd_dtype", Py_BuildValue("(O)", obj(handle)));
  if (!r) return fail_from_python();
  *out_dtype = static_cast<int>(PyLong_AsLong(r));
  Py_DECREF(r);
  return 0;
}

MXAPI int MXNDArrayGetContext(NDArrayHandle handle, int* out_dev_type, int* out_dev_id) {
  Gil g;
  PyObject* r = call("nd_context", Py_BuildValue("(O)", obj(handle)));
  if (!r) return fail_from_python();
  int a = 0, b = 0;
  const int ok = PyArg_ParseTuple(r, "ii", &a, &b);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *out_dev_type = a;
  *out_dev_id = b;
  return 0;
}

static int elem_bytes(void* h, int64_t* nb) {
  int dt = 0;
  if (MXNDArrayGetDType(h, &dt) != 0) return -1;
  static const int sizes[] = {4, 8, 2, 1, 4, 1, 8, 1, 0, 0, 0, 0, 2};
  *nb = (dt >= 0 && dt <= 12) ? sizes[dt] : 0;
  return *nb > 0 ? 0 : fail("unsupported dtype");
}

MXAPI int MXNDArraySyncCopyFromCPU(NDArrayHandle handle, const void* data, size_t size) {
  int64_t nb = 0;
  if (elem_bytes(handle, &nb) != 0) return -1;
  Gil g;
  PyObject* buf = PyBytes_FromStringAndSize(static_cast<const char*>(data), static_cast<Py_ssize_t>(size * nb));
  return done(call("nd_from_bytes", Py_BuildValue("(ONn)", obj(handle), buf, static_cast<Py_ssize_t>(size))));
}

MXAPI int MXNDArraySyncCopyToCPU(NDArrayHandle handle, void* data, size_t size) {
  int64_t nb = 0;
  if (elem_bytes(handle, &nb) != 0) return -1;
  Gil g;
  PyObject* r = call("nd_to_bytes", Py_BuildValue("(On)", obj(handle), static_cast<Py_ssize_t>(size)));
  if (!r) return fail_from_python();
  char* p = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(r, &p, &n) != 0) {
    Py_DECREF(r);
    return fail_from_python();
  }
  if (static_cast<size_t>(n) != size * nb) {
    Py_DECREF(r);
    return fail("MXNDArraySyncCopyToCPU: size mismatch");
  }
  std::memcpy(data, p, n);
  Py_DECREF(r);
  return 0;
}

MXAPI int MXNDArrayWaitToRead(NDArrayHandle handle) {
  Gil g;
  return done(call("nd_wait", Py_BuildValue("(O)", obj(handle))));
}

MXAPI int MXNDArrayWaitAll() {
  Gil g;
  return done(call("nd_waitall", PyTuple_New(0)));
}

MXAPI int MXNDArraySave(const char* fname, uint32_t num_args, NDArrayHandle* args, const char** keys) {
  Gil g;
  PyObject* k = keys ? str_list(num_args, keys) : PyList_New(0);
  return done(call("nd_save", Py_BuildValue("(sNN)", fname, obj_list(num_args, args), k)));
}

MXAPI int MXNDArrayLoad(const char* fname, uint32_t* out_size, NDArrayHandle** out_arr, uint32_t* out_name_size,
                        const char*** out_names) {
  Gil g;
  PyObject* r = call("nd_load", Py_BuildValue("(s)", fname));
  if (!r) return fail_from_python();
  PyObject *arrs = nullptr, *names = nullptr;
  if (!PyArg_ParseTuple(r, "OO", &arrs, &names) || !to_handles(arrs) || !to_strs(names, &tl_strs, &tl_cstrs)) {
    Py_DECREF(r);
    return fail_from_python();
  }
  Py_DECREF(r);
  *out_size = static_cast<uint32_t>(tl_handles.size());
  *out_arr = tl_handles.data();
  *out_name_size = static_cast<uint32_t>(tl_cstrs.size());
  *out_names = tl_cstrs.data();
  return 0;
}

MXAPI int MXNDArrayReshape(NDArrayHandle handle, int ndim, int* dims, NDArrayHandle* out) {
  Gil g;
  return new_handle(call("nd_reshape", Py_BuildValue("(ON)", obj(handle), int_list(ndim, dims))), out);
}

MXAPI int MXNDArraySlice(NDArrayHandle handle, uint32_t slice_begin, uint32_t slice_end, NDArrayHandle* out) {
  Gil g;
  return new_handle(call("nd_slice", Py_BuildValue("(OII)", obj(handle), slice_begin, slice_end)), out);
}

MXAPI int MXNDArrayAt(NDArrayHandle handle, uint32_t idx, NDArrayHandle* out) {
  Gil g;
  return new_handle(call("nd_at", Py_BuildValue("(OI)", obj(handle), idx)), out);
}

MXAPI int MXNDArrayGetGrad(NDArrayHandle handle, NDArrayHandle* out) {
  Gil g;
  PyObject* r = call("nd_grad", Py_BuildValue("(O)", obj(handle)));
  if (!r) return fail_from_python();
  if (r == Py_None) {
    Py_DECREF(r);
    *out = nullptr;
    return 0;
  }
  *out = wrap(r);
  return 0;
}

// --------------------------------------------------------------------------- operators + autograd
MXAPI int MXListAllOpNames(uint32_t* out_size, const char*** out_array) {
  Gil g;
  PyObject* r = call("op_names", PyTuple_New(0));
  if (!r) return fail_from_python();
  const bool ok = to_strs(r, &tl_strs, &tl_cstrs);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *out_size = static_cast<uint32_t>(tl_cstrs.size());
  *out_array = tl_cstrs.data();
  return 0;
}

MXAPI int NNGetOpHandle(const char* op_name, OpHandle* op_out) {
  Gil g;
  PyObject* r = call("op_exists", Py_BuildValue("(s)", op_name));
  if (!r) return fail_from_python();
  const bool ok = PyObject_IsTrue(r) == 1;
  Py_DECREF(r);
  if (!ok) return fail((std::string("operator not registered: ") + op_name).c_str());
  *op_out = new OpRec{op_name};  // one per lookup, kept for the process lifetime (like the registry's)
  return 0;
}

MXAPI int MXImperativeInvoke(AtomicSymbolCreator creator, int num_inputs, NDArrayHandle* inputs, int* num_outputs,
                             NDArrayHandle** outputs, int num_params, const char** param_keys,
                             const char** param_vals) {
  if (!creator) return fail("MXImperativeInvoke: null operator handle");
  Gil g;
  const bool given = outputs && *outputs && *num_outputs > 0;
  PyObject* outs = given ? obj_list(*num_outputs, *outputs) : PyList_New(0);
  PyObject* r = call("invoke", Py_BuildValue("(sNNNN)", static_cast<OpRec*>(creator)->name.c_str(),
                                             obj_list(num_inputs, inputs), str_list(num_params, param_keys),
                                             str_list(num_params, param_vals), outs));
  if (!r) return fail_from_python();
  if (given) {  // results were written into the caller's arrays
    Py_DECREF(r);
    return 0;
  }
  const bool ok = to_handles(r);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *num_outputs = static_cast<int>(tl_handles.size());
  *outputs = tl_handles.data();
  return 0;
}

MXAPI int MXAutogradSetIsRecording(int is_recording, int* prev) {
  Gil g;
  PyObject* r = call("set_recording", Py_BuildValue("(i)", is_recording));
  if (!r) return fail_from_python();
  if (prev) *prev = static_cast<int>(PyLong_AsLong(r));
  Py_DECREF(r);
  return 0;
}

MXAPI int MXAutogradSetIsTraining(int is_training, int* prev) {
  Gil g;
  PyObject* r = call("set_training", Py_BuildValue("(i)", is_training));
  if (!r) return fail_from_python();
  if (prev) *prev = static_cast<int>(PyLong_AsLong(r));
  Py_DECREF(r);
  return 0;
}

MXAPI int MXAutogradMarkVariables(uint32_t num_var, NDArrayHandle* var_handles, uint32_t* reqs_array,
                                  NDArrayHandle* grad_handles) {
  Gil g;
  return done(call("mark_variables", Py_BuildValue("(NNN)", obj_list(num_var, var_handles),
                                                   u32_list(num_var, reqs_array), obj_list(num_var, grad_handles))));
}

MXAPI int MXAutogradBackward(uint32_t num_output, NDArrayHandle* output_handles, NDArrayHandle* ograd_handles,
                             int retain_graph) {
  Gil g;
  PyObject* og = ograd_handles ? obj_list(num_output, ograd_handles) : PyList_New(0);
  return done(call("backward", Py_BuildValue("(NNi)", obj_list(num_output, output_handles), og, retain_graph)));
}

// ------------------------------------------------------------------------------------------ Symbol
MXAPI int MXSymbolCreateFromJSON(const char* json, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_from_json", Py_BuildValue("(s)", json)), out);
}

MXAPI int MXSymbolCreateFromFile(const char* fname, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_from_file", Py_BuildValue("(s)", fname)), out);
}

MXAPI int MXSymbolSaveToJSON(SymbolHandle symbol, const char** out_json) {
  Gil g;
  Obj* o = static_cast<Obj*>(symbol);
  PyObject* r = call("sym_to_json", Py_BuildValue("(O)", o->o));
  if (!r) return fail_from_python();
  const char* c = PyUnicode_AsUTF8(r);
  o->str = c ? c : "";
  Py_DECREF(r);
  *out_json = o->str.c_str();
  return 0;
}

MXAPI int MXSymbolFree(SymbolHandle symbol) { return free_handle(symbol); }

MXAPI int MXSymbolGetName(SymbolHandle symbol, const char** out, int* success) {
  Gil g;
  Obj* o = static_cast<Obj*>(symbol);
  PyObject* r = call("sym_name", Py_BuildValue("(O)", o->o));
  if (!r) return fail_from_python();
  const char* c = nullptr;
  int ok = 0;
  if (!PyArg_ParseTuple(r, "si", &c, &ok)) {
    Py_DECREF(r);
    return fail_from_python();
  }
  o->str = c ? c : "";
  Py_DECREF(r);
  *out = o->str.c_str();
  *success = ok;
  return 0;
}

MXAPI int MXSymbolListArguments(SymbolHandle symbol, uint32_t* out_size, const char*** out_str_array) {
  return list_strings(symbol, "sym_list", 0, out_size, out_str_array);
}

MXAPI int MXSymbolListOutputs(SymbolHandle symbol, uint32_t* out_size, const char*** out_str_array) {
  return list_strings(symbol, "sym_list", 1, out_size, out_str_array);
}

MXAPI int MXSymbolListAuxiliaryStates(SymbolHandle symbol, uint32_t* out_size, const char*** out_str_array) {
  return list_strings(symbol, "sym_list", 2, out_size, out_str_array);
}

MXAPI int MXSymbolCreateVariable(const char* name, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_var", Py_BuildValue("(s)", name)), out);
}

MXAPI int MXSymbolCreateAtomicSymbol(AtomicSymbolCreator creator, uint32_t num_param, const char** keys,
                                     const char** vals, SymbolHandle* out) {
  if (!creator) return fail("MXSymbolCreateAtomicSymbol: null operator handle");
  Gil g;
  return new_handle(call("sym_atomic", Py_BuildValue("(sNN)", static_cast<OpRec*>(creator)->name.c_str(),
                                                     str_list(num_param, keys), str_list(num_param, vals))),
                    out);
}

MXAPI int MXSymbolCompose(SymbolHandle sym, const char* name, uint32_t num_args, const char** keys,
                          SymbolHandle* args) {
  Gil g;
  Obj* o = static_cast<Obj*>(sym);
  PyObject* k = keys ? str_list(num_args, keys) : PyList_New(0);
  PyObject* r = call("sym_compose", Py_BuildValue("(OsNN)", o->o, name ? name : "", k, obj_list(num_args, args)));
  if (!r) return fail_from_python();
  // the handle now denotes the composed symbol (the reference composes in place)
  Py_DECREF(o->o);
  o->o = r;
  return 0;
}

static bool fill_shapes(PyObject* lst, int slot) {
  tl_shapes[slot].clear();
  tl_ndim[slot].clear();
  tl_ptr[slot].clear();
  PyObject* it = PyObject_GetIter(lst);
  if (!it) return false;
  while (PyObject* x = PyIter_Next(it)) {
    std::vector<uint32_t> v;
    to_u32(x, &v);
    Py_DECREF(x);
    tl_shapes[slot].push_back(v);
  }
  Py_DECREF(it);
  for (auto& v : tl_shapes[slot]) {
    tl_ndim[slot].push_back(static_cast<uint32_t>(v.size()));
    tl_ptr[slot].push_back(v.data());
  }
  return !PyErr_Occurred();
}

MXAPI int MXSymbolInferShape(SymbolHandle sym, uint32_t num_args, const char** keys, const uint32_t* arg_ind_ptr,
                             const uint32_t* arg_shape_data, uint32_t* in_shape_size, const uint32_t** in_shape_ndim,
                             const uint32_t*** in_shape_data, uint32_t* out_shape_size,
                             const uint32_t** out_shape_ndim, const uint32_t*** out_shape_data,
                             uint32_t* aux_shape_size, const uint32_t** aux_shape_ndim,
                             const uint32_t*** aux_shape_data, int* complete) {
  Gil g;
  PyObject* shapes = PyList_New(num_args);
  for (uint32_t i = 0; i < num_args; ++i)
    PyList_SET_ITEM(shapes, i, u32_list(arg_ind_ptr[i + 1] - arg_ind_ptr[i], arg_shape_data + arg_ind_ptr[i]));
  PyObject* k = keys ? str_list(num_args, keys) : PyList_New(0);
  PyObject* r = call("sym_infer_shape", Py_BuildValue("(ONN)", obj(sym), k, shapes));
  if (!r) return fail_from_python();
  PyObject *a = nullptr, *o = nullptr, *x = nullptr;
  int c = 0;
  if (!PyArg_ParseTuple(r, "OOOi", &a, &o, &x, &c) || !fill_shapes(a, 0) || !fill_shapes(o, 1) ||
      !fill_shapes(x, 2)) {
    Py_DECREF(r);
    return fail_from_python();
  }
  Py_DECREF(r);
  *in_shape_size = static_cast<uint32_t>(tl_ndim[0].size());
  *in_shape_ndim = tl_ndim[0].data();
  *in_shape_data = tl_ptr[0].data();
  *out_shape_size = static_cast<uint32_t>(tl_ndim[1].size());
  *out_shape_ndim = tl_ndim[1].data();
  *out_shape_data = tl_ptr[1].data();
  *aux_shape_size = static_cast<uint32_t>(tl_ndim[2].size());
  *aux_shape_ndim = tl_ndim[2].data();
  *aux_shape_data = tl_ptr[2].data();
  *complete = c;
  return 0;
}

// ---------------------------------------------------------------------------------------- Executor
MXAPI int MXExecutorBind(SymbolHandle symbol_handle, int dev_type, int dev_id, uint32_t len, NDArrayHandle* in_args,
                         NDArrayHandle* arg_grad_store, uint32_t* grad_req_type, uint32_t aux_states_len,
                         NDArrayHandle* aux_states, ExecutorHandle* out) {
  Gil g;
  return new_handle(call("bind", Py_BuildValue("(OiiNNNN)", obj(symbol_handle), dev_type, dev_id,
                                              obj_list(len, in_args), obj_list(len, arg_grad_store),
                                              u32_list(len, grad_req_type), obj_list(aux_states_len, aux_states))),
                    out);
}

MXAPI int MXExecutorForward(ExecutorHandle handle, int is_train) {
  Gil g;
  return done(call("exec_forward", Py_BuildValue("(Oi)", obj(handle), is_train)));
}

MXAPI int MXExecutorBackward(ExecutorHandle handle, uint32_t len, NDArrayHandle* head_grads) {
  Gil g;
  PyObject* hg = (len && head_grads) ? obj_list(len, head_grads) : PyList_New(0);
  return done(call("exec_backward", Py_BuildValue("(ON)", obj(handle), hg)));
}

MXAPI int MXExecutorOutputs(ExecutorHandle handle, uint32_t* out_size, NDArrayHandle** out) {
  Gil g;
  PyObject* r = call("exec_outputs", Py_BuildValue("(O)", obj(handle)));
  if (!r) return fail_from_python();
  const bool ok = to_handles(r);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *out_size = static_cast<uint32_t>(tl_handles.size());
  *out = tl_handles.data();
  return 0;
}

MXAPI int MXExecutorFree(ExecutorHandle handle) { return free_handle(handle); }

// ----------------------------------------------------------------------------------------- KVStore
MXAPI int MXKVStoreCreate(const char* type, KVStoreHandle* out) {
  Gil g;
  return new_handle(call("kv_create", Py_BuildValue("(s)", type)), out);
}

MXAPI int MXKVStoreInit(KVStoreHandle handle, uint32_t num, const int* keys, NDArrayHandle* vals) {
  Gil g;
  return done(call("kv_init", Py_BuildValue("(ONN)", obj(handle), int_list(num, keys), obj_list(num, vals))));
}

MXAPI int MXKVStorePush(KVStoreHandle handle, uint32_t num, const int* keys, NDArrayHandle* vals, int priority) {
  Gil g;
  return done(call("kv_push", Py_BuildValue("(ONNi)", obj(handle), int_list(num, keys), obj_list(num, vals),
                                            priority)));
}

MXAPI int MXKVStorePull(KVStoreHandle handle, uint32_t num, const int* keys, NDArrayHandle* vals, int priority) {
  Gil g;
  return done(call("kv_pull", Py_BuildValue("(ONNi)", obj(handle), int_list(num, keys), obj_list(num, vals),
                                            priority)));
}

MXAPI int MXKVStoreFree(KVStoreHandle handle) { return free_handle(handle); }
