// C API, second half (include/mxamd/c_api.h): NDArray extras, autograd extras, CachedOp, profiler,
// data iterators, RecordIO, KVStore extras, runtime controls and Symbol / Executor extras.
//
// Parity: include/mxnet/c_api.h (:983 MXNDArrayGetData, :1353 MXAutogradBackwardEx, :1372-1417
// CachedOp, :303-482 profiler, :2609-2698 MXDataIter*, :3151-3217 MXRecordIO*, :2947
// MXKVStorePushPull, :255 MXRandomSeed, ...).  Same embedding as c_api.cc: the GIL is taken per call,
// the work is done by mxnet_maintenance_amd.c_api_impl, failures become -1 + MXGetLastError().
#include "../../include/mxamd/c_api.h"
#include "capi_internal.h"

namespace {

thread_local std::string tl_str;
thread_local std::vector<uint64_t> tl_u64;
thread_local std::vector<int> tl_ints;
thread_local std::vector<void*> tl_creators;
thread_local std::vector<std::string> tl_names2[3];
thread_local std::vector<const char*> tl_cnames2[3];

struct IterCreator {
  std::string name;
};

// a python str -> std::string (false with the error set on failure)
bool to_string(PyObject* o, std::string* out) {
  const char* c = PyUnicode_AsUTF8(o);
  if (!c) return false;
  *out = c;
  return true;
}

int ret_string(PyObject* r, std::string* store, const char** out) {
  if (!r) return fail_from_python();
  const bool ok = to_string(r, store);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *out = store->c_str();
  return 0;
}

int ret_int(PyObject* r, int* out) {
  if (!r) return fail_from_python();
  const long v = PyLong_AsLong(r);
  Py_DECREF(r);
  if (PyErr_Occurred()) return fail_from_python();
  if (out) *out = static_cast<int>(v);
  return 0;
}

int ret_size(PyObject* r, size_t* out) {
  if (!r) return fail_from_python();
  const unsigned long long v = PyLong_AsUnsignedLongLong(r);
  Py_DECREF(r);
  if (PyErr_Occurred()) return fail_from_python();
  *out = static_cast<size_t>(v);
  return 0;
}

// (handles, stypes) tuple -> tl_handles / tl_ints
bool to_handles_stypes(PyObject* r) {
  PyObject *hs = nullptr, *st = nullptr;
  if (!PyArg_ParseTuple(r, "OO", &hs, &st) || !to_handles(hs)) return false;
  tl_ints.clear();
  PyObject* it = PyObject_GetIter(st);
  if (!it) return false;
  while (PyObject* x = PyIter_Next(it)) {
    tl_ints.push_back(static_cast<int>(PyLong_AsLong(x)));
    Py_DECREF(x);
  }
  Py_DECREF(it);
  return !PyErr_Occurred();
}

}  // namespace

// ------------------------------------------------------------------------------------- NDArray extras
MXAPI int MXNDArrayGetData(NDArrayHandle handle, void** out_pdata) {
  Gil g;
  PyObject* r = call("nd_data_ptr", Py_BuildValue("(O)", obj(handle)));
  if (!r) return fail_from_python();
  const unsigned long long p = PyLong_AsUnsignedLongLong(r);
  Py_DECREF(r);
  if (PyErr_Occurred()) return fail_from_python();
  *out_pdata = reinterpret_cast<void*>(static_cast<uintptr_t>(p));
  return 0;
}

MXAPI int MXNDArrayGetStorageType(NDArrayHandle handle, int* out_storage_type) {
  Gil g;
  return ret_int(call("nd_storage_type", Py_BuildValue("(O)", obj(handle))), out_storage_type);
}

MXAPI int MXNDArrayDetach(NDArrayHandle handle, NDArrayHandle* out) {
  Gil g;
  return new_handle(call("nd_detach", Py_BuildValue("(O)", obj(handle))), out);
}

MXAPI int MXNDArraySetGradState(NDArrayHandle handle, int state) {
  Gil g;
  return done(call("nd_set_grad_state", Py_BuildValue("(Oi)", obj(handle), state)));
}

MXAPI int MXNDArrayGetGradState(NDArrayHandle handle, int* out) {
  Gil g;
  return ret_int(call("nd_get_grad_state", Py_BuildValue("(O)", obj(handle))), out);
}

MXAPI int MXNDArraySaveRawBytes(NDArrayHandle handle, size_t* out_size, const char** out_buf) {
  Gil g;
  Obj* o = static_cast<Obj*>(handle);
  PyObject* r = call("nd_save_raw", Py_BuildValue("(O)", o->o));
  if (!r) return fail_from_python();
  char* p = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(r, &p, &n) != 0) {
    Py_DECREF(r);
    return fail_from_python();
  }
  o->str.assign(p, static_cast<size_t>(n));
  Py_DECREF(r);
  *out_size = o->str.size();
  *out_buf = o->str.data();
  return 0;
}

MXAPI int MXNDArrayLoadFromRawBytes(const void* buf, size_t size, NDArrayHandle* out) {
  Gil g;
  PyObject* b = PyBytes_FromStringAndSize(static_cast<const char*>(buf), static_cast<Py_ssize_t>(size));
  return new_handle(call("nd_load_raw", Py_BuildValue("(N)", b)), out);
}

MXAPI int MXNDArraySyncCopyFromNDArray(NDArrayHandle handle_dst, const NDArrayHandle handle_src, const int i) {
  Gil g;
  return done(call("nd_copy_from_nd", Py_BuildValue("(OOi)", obj(handle_dst), obj(handle_src), i)));
}

MXAPI int MXNDArrayWaitToWrite(NDArrayHandle handle) {
  Gil g;
  return done(call("nd_wait_write", Py_BuildValue("(O)", obj(handle))));
}

// ------------------------------------------------------------------------------------ autograd extras
MXAPI int MXAutogradIsRecording(bool* curr) {
  Gil g;
  int v = 0;
  if (ret_int(call("is_recording", PyTuple_New(0)), &v) != 0) return -1;
  *curr = v != 0;
  return 0;
}

MXAPI int MXAutogradIsTraining(bool* curr) {
  Gil g;
  int v = 0;
  if (ret_int(call("is_training", PyTuple_New(0)), &v) != 0) return -1;
  *curr = v != 0;
  return 0;
}

MXAPI int MXAutogradBackwardEx(uint32_t num_output, NDArrayHandle* output_handles, NDArrayHandle* ograd_handles,
                               uint32_t num_variables, NDArrayHandle* var_handles, int retain_graph,
                               int create_graph, int is_train, NDArrayHandle** grad_handles, int** grad_stypes) {
  Gil g;
  PyObject* og = ograd_handles ? obj_list(num_output, ograd_handles) : PyList_New(0);
  PyObject* vars = (num_variables && var_handles) ? obj_list(num_variables, var_handles) : PyList_New(0);
  PyObject* r = call("backward_ex", Py_BuildValue("(NNNiii)", obj_list(num_output, output_handles), og, vars,
                                                  retain_graph, create_graph, is_train));
  if (!r) return fail_from_python();
  const bool ok = to_handles_stypes(r);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  if (grad_handles) *grad_handles = tl_handles.empty() ? nullptr : tl_handles.data();
  if (grad_stypes) *grad_stypes = tl_ints.empty() ? nullptr : tl_ints.data();
  return 0;
}

// ------------------------------------------------------------------------------------------ CachedOp
MXAPI int MXCreateCachedOpEx(SymbolHandle handle, int num_flags, const char** keys, const char** vals,
                             CachedOpHandle* out) {
  Gil g;
  return new_handle(call("cached_op_create", Py_BuildValue("(ONN)", obj(handle), str_list(num_flags, keys),
                                                           str_list(num_flags, vals))),
                    out);
}

MXAPI int MXCreateCachedOp(SymbolHandle handle, CachedOpHandle* out) {
  return MXCreateCachedOpEx(handle, 0, nullptr, nullptr, out);
}

MXAPI int MXFreeCachedOp(CachedOpHandle handle) { return free_handle(handle); }

MXAPI int MXInvokeCachedOpEx(CachedOpHandle handle, int num_inputs, NDArrayHandle* inputs, int* num_outputs,
                             NDArrayHandle** outputs, const int** out_stypes) {
  Gil g;
  const bool given = outputs && *outputs && *num_outputs > 0;
  PyObject* outs = given ? obj_list(*num_outputs, *outputs) : PyList_New(0);
  PyObject* r = call("cached_op_invoke", Py_BuildValue("(ONN)", obj(handle), obj_list(num_inputs, inputs), outs));
  if (!r) return fail_from_python();
  const bool ok = to_handles_stypes(r);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  if (out_stypes) *out_stypes = tl_ints.data();
  if (given) {  // results were written into the caller's arrays; drop the fresh wrappers
    for (void* h : tl_handles) free_handle(h);
    tl_handles.clear();
    return 0;
  }
  *num_outputs = static_cast<int>(tl_handles.size());
  *outputs = tl_handles.data();
  return 0;
}

MXAPI int MXInvokeCachedOp(CachedOpHandle handle, int num_inputs, NDArrayHandle* inputs, int* num_outputs,
                           NDArrayHandle** outputs) {
  return MXInvokeCachedOpEx(handle, num_inputs, inputs, num_outputs, outputs, nullptr);
}

// ------------------------------------------------------------------------------------------ profiler
MXAPI int MXSetProfilerConfig(int num_params, const char* const* keys, const char* const* vals) {
  Gil g;
  return done(call("prof_config", Py_BuildValue("(NN)", str_list(num_params, const_cast<const char**>(keys)),
                                                str_list(num_params, const_cast<const char**>(vals)))));
}

MXAPI int MXSetProfilerState(int state) {
  Gil g;
  return done(call("prof_state", Py_BuildValue("(i)", state)));
}

MXAPI int MXDumpProfile(int finished) {
  Gil g;
  return done(call("prof_dump", Py_BuildValue("(i)", finished)));
}

MXAPI int MXAggregateProfileStatsPrint(const char** out_str, int reset) {
  Gil g;
  return ret_string(call("prof_dumps", Py_BuildValue("(i)", reset)), &tl_str, out_str);
}

MXAPI int MXProfilePause(int paused) {
  Gil g;
  return done(call("prof_pause", Py_BuildValue("(i)", paused)));
}

MXAPI int MXProfileCreateDomain(const char* domain, ProfileHandle* out) {
  Gil g;
  return new_handle(call("prof_domain", Py_BuildValue("(s)", domain)), out);
}

MXAPI int MXProfileCreateTask(ProfileHandle domain, const char* task_name, ProfileHandle* out) {
  Gil g;
  return new_handle(call("prof_task", Py_BuildValue("(Os)", obj(domain), task_name)), out);
}

MXAPI int MXProfileDurationStart(ProfileHandle duration_handle) {
  Gil g;
  return done(call("prof_start", Py_BuildValue("(O)", obj(duration_handle))));
}

MXAPI int MXProfileDurationStop(ProfileHandle duration_handle) {
  Gil g;
  return done(call("prof_stop", Py_BuildValue("(O)", obj(duration_handle))));
}

MXAPI int MXProfileSetMarker(ProfileHandle domain, const char* instant_marker_name, const char* scope) {
  Gil g;
  return done(call("prof_marker", Py_BuildValue("(Oss)", obj(domain), instant_marker_name, scope ? scope : "")));
}

MXAPI int MXProfileDestroyHandle(ProfileHandle frame_handle) { return free_handle(frame_handle); }

// ------------------------------------------------------------------------------------ data iterators
MXAPI int MXListDataIters(uint32_t* out_size, DataIterCreator** out_array) {
  Gil g;
  PyObject* r = call("iter_names", PyTuple_New(0));
  if (!r) return fail_from_python();
  std::vector<std::string> names;
  std::vector<const char*> cs;
  const bool ok = to_strs(r, &names, &cs);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  // creators live for the process (like the reference's registry entries): one per name, reused
  static std::vector<IterCreator*> registry;
  tl_creators.clear();
  for (const auto& n : names) {
    IterCreator* c = nullptr;
    for (IterCreator* e : registry)
      if (e->name == n) c = e;
    if (!c) {
      c = new IterCreator{n};
      registry.push_back(c);
    }
    tl_creators.push_back(c);
  }
  *out_size = static_cast<uint32_t>(tl_creators.size());
  *out_array = tl_creators.data();
  return 0;
}

MXAPI int MXDataIterGetIterInfo(DataIterCreator creator, const char** name, const char** description,
                                uint32_t* num_args, const char*** arg_names, const char*** arg_type_infos,
                                const char*** arg_descriptions) {
  if (!creator) return fail("MXDataIterGetIterInfo: null creator");
  Gil g;
  PyObject* r = call("iter_info", Py_BuildValue("(s)", static_cast<IterCreator*>(creator)->name.c_str()));
  if (!r) return fail_from_python();
  PyObject *nm = nullptr, *doc = nullptr, *an = nullptr, *at = nullptr, *ad = nullptr;
  static thread_local std::string s_name, s_doc;
  if (!PyArg_ParseTuple(r, "OOOOO", &nm, &doc, &an, &at, &ad) || !to_string(nm, &s_name) ||
      !to_string(doc, &s_doc) || !to_strs(an, &tl_names2[0], &tl_cnames2[0]) ||
      !to_strs(at, &tl_names2[1], &tl_cnames2[1]) || !to_strs(ad, &tl_names2[2], &tl_cnames2[2])) {
    Py_DECREF(r);
    return fail_from_python();
  }
  Py_DECREF(r);
  *name = s_name.c_str();
  *description = s_doc.c_str();
  *num_args = static_cast<uint32_t>(tl_cnames2[0].size());
  *arg_names = tl_cnames2[0].data();
  *arg_type_infos = tl_cnames2[1].data();
  *arg_descriptions = tl_cnames2[2].data();
  return 0;
}

MXAPI int MXDataIterCreateIter(DataIterCreator handle, uint32_t num_param, const char** keys, const char** vals,
                               DataIterHandle* out) {
  if (!handle) return fail("MXDataIterCreateIter: null creator");
  Gil g;
  return new_handle(call("iter_create", Py_BuildValue("(sNN)", static_cast<IterCreator*>(handle)->name.c_str(),
                                                      str_list(num_param, keys), str_list(num_param, vals))),
                    out);
}

MXAPI int MXDataIterFree(DataIterHandle handle) { return free_handle(handle); }

MXAPI int MXDataIterNext(DataIterHandle handle, int* out) {
  Gil g;
  return ret_int(call("iter_next", Py_BuildValue("(O)", obj(handle))), out);
}

MXAPI int MXDataIterBeforeFirst(DataIterHandle handle) {
  Gil g;
  return done(call("iter_reset", Py_BuildValue("(O)", obj(handle))));
}

MXAPI int MXDataIterGetData(DataIterHandle handle, NDArrayHandle* out) {
  Gil g;
  return new_handle(call("iter_data", Py_BuildValue("(O)", obj(handle))), out);
}

MXAPI int MXDataIterGetLabel(DataIterHandle handle, NDArrayHandle* out) {
  Gil g;
  return new_handle(call("iter_label", Py_BuildValue("(O)", obj(handle))), out);
}

MXAPI int MXDataIterGetPadNum(DataIterHandle handle, int* pad) {
  Gil g;
  return ret_int(call("iter_pad", Py_BuildValue("(O)", obj(handle))), pad);
}

MXAPI int MXDataIterGetIndex(DataIterHandle handle, uint64_t** out_index, uint64_t* out_size) {
  Gil g;
  PyObject* r = call("iter_index", Py_BuildValue("(O)", obj(handle)));
  if (!r) return fail_from_python();
  tl_u64.clear();
  PyObject* it = PyObject_GetIter(r);
  if (it) {
    while (PyObject* x = PyIter_Next(it)) {
      tl_u64.push_back(static_cast<uint64_t>(PyLong_AsUnsignedLongLong(x)));
      Py_DECREF(x);
    }
    Py_DECREF(it);
  }
  Py_DECREF(r);
  if (PyErr_Occurred()) return fail_from_python();
  *out_index = tl_u64.data();
  *out_size = tl_u64.size();
  return 0;
}

// ------------------------------------------------------------------------------------------ RecordIO
MXAPI int MXRecordIOWriterCreate(const char* uri, RecordIOHandle* out) {
  Gil g;
  return new_handle(call("rec_writer", Py_BuildValue("(s)", uri)), out);
}

MXAPI int MXRecordIOReaderCreate(const char* uri, RecordIOHandle* out) {
  Gil g;
  return new_handle(call("rec_reader", Py_BuildValue("(s)", uri)), out);
}

static int rec_free(RecordIOHandle handle) {
  if (!handle) return 0;
  {
    Gil g;
    PyObject* r = call("rec_close", Py_BuildValue("(O)", obj(handle)));
    if (!r) return fail_from_python();
    Py_DECREF(r);
  }
  return free_handle(handle);
}

MXAPI int MXRecordIOWriterFree(RecordIOHandle handle) { return rec_free(handle); }
MXAPI int MXRecordIOReaderFree(RecordIOHandle handle) { return rec_free(handle); }

MXAPI int MXRecordIOWriterWriteRecord(RecordIOHandle handle, const char* buf, size_t size) {
  Gil g;
  PyObject* b = PyBytes_FromStringAndSize(buf, static_cast<Py_ssize_t>(size));
  return done(call("rec_write", Py_BuildValue("(ON)", obj(handle), b)));
}

MXAPI int MXRecordIOWriterTell(RecordIOHandle handle, size_t* pos) {
  Gil g;
  return ret_size(call("rec_tell", Py_BuildValue("(O)", obj(handle))), pos);
}

MXAPI int MXRecordIOReaderTell(RecordIOHandle handle, size_t* pos) {
  Gil g;
  return ret_size(call("rec_tell", Py_BuildValue("(O)", obj(handle))), pos);
}

MXAPI int MXRecordIOReaderSeek(RecordIOHandle handle, size_t pos) {
  Gil g;
  return done(call("rec_seek", Py_BuildValue("(On)", obj(handle), static_cast<Py_ssize_t>(pos))));
}

MXAPI int MXRecordIOReaderReadRecord(RecordIOHandle handle, char const** buf, size_t* size) {
  Gil g;
  Obj* o = static_cast<Obj*>(handle);
  PyObject* r = call("rec_read", Py_BuildValue("(O)", o->o));
  if (!r) return fail_from_python();
  if (r == Py_None) {  // end of file
    Py_DECREF(r);
    *buf = nullptr;
    *size = 0;
    return 0;
  }
  char* p = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(r, &p, &n) != 0) {
    Py_DECREF(r);
    return fail_from_python();
  }
  o->str.assign(p, static_cast<size_t>(n));
  Py_DECREF(r);
  *buf = o->str.data();
  *size = o->str.size();
  return 0;
}

// ------------------------------------------------------------------------------------ KVStore extras
MXAPI int MXKVStoreInitEx(KVStoreHandle handle, uint32_t num, const char** keys, NDArrayHandle* vals) {
  Gil g;
  return done(call("kv_init", Py_BuildValue("(ONN)", obj(handle), str_list(num, keys), obj_list(num, vals))));
}

MXAPI int MXKVStorePushEx(KVStoreHandle handle, uint32_t num, const char** keys, NDArrayHandle* vals, int priority) {
  Gil g;
  return done(call("kv_push", Py_BuildValue("(ONNi)", obj(handle), str_list(num, keys), obj_list(num, vals),
                                            priority)));
}

MXAPI int MXKVStorePullEx(KVStoreHandle handle, uint32_t num, const char** keys, NDArrayHandle* vals, int priority) {
  Gil g;
  return done(call("kv_pull", Py_BuildValue("(ONNi)", obj(handle), str_list(num, keys), obj_list(num, vals),
                                            priority)));
}

MXAPI int MXKVStorePushPull(KVStoreHandle handle, uint32_t vnum, const int* vkeys, uint32_t onum, const int* okeys,
                            NDArrayHandle* vals, NDArrayHandle* outs, int priority) {
  Gil g;
  return done(call("kv_pushpull", Py_BuildValue("(ONNNNi)", obj(handle), int_list(vnum, vkeys), int_list(onum, okeys),
                                                obj_list(vnum, vals), obj_list(onum, outs), priority)));
}

MXAPI int MXKVStorePushPullEx(KVStoreHandle handle, uint32_t vnum, const char** vkeys, uint32_t onum,
                              const char** okeys, NDArrayHandle* vals, NDArrayHandle* outs, int priority) {
  Gil g;
  return done(call("kv_pushpull", Py_BuildValue("(ONNNNi)", obj(handle), str_list(vnum, vkeys), str_list(onum, okeys),
                                                obj_list(vnum, vals), obj_list(onum, outs), priority)));
}

MXAPI int MXKVStoreGetType(KVStoreHandle handle, const char** type) {
  Gil g;
  Obj* o = static_cast<Obj*>(handle);
  return ret_string(call("kv_type", Py_BuildValue("(O)", o->o)), &o->str, type);
}

MXAPI int MXKVStoreGetRank(KVStoreHandle handle, int* ret) {
  Gil g;
  return ret_int(call("kv_rank", Py_BuildValue("(O)", obj(handle))), ret);
}

MXAPI int MXKVStoreGetGroupSize(KVStoreHandle handle, int* ret) {
  Gil g;
  return ret_int(call("kv_group_size", Py_BuildValue("(O)", obj(handle))), ret);
}

MXAPI int MXKVStoreBarrier(KVStoreHandle handle) {
  Gil g;
  return done(call("kv_barrier", Py_BuildValue("(O)", obj(handle))));
}

// ------------------------------------------------------------------------------------------ runtime
MXAPI int MXRandomSeed(int seed) {
  Gil g;
  return done(call("random_seed", Py_BuildValue("(iii)", seed, -1, 0)));
}

MXAPI int MXRandomSeedContext(int seed, int dev_type, int dev_id) {
  Gil g;
  return done(call("random_seed", Py_BuildValue("(iii)", seed, dev_type, dev_id)));
}

MXAPI int MXNotifyShutdown() {
  Gil g;
  return done(call("notify_shutdown", PyTuple_New(0)));
}

MXAPI int MXSetNumOMPThreads(int thread_num) {
  Gil g;
  return done(call("set_omp_threads", Py_BuildValue("(i)", thread_num)));
}

MXAPI int MXGetGPUCount(int* out) {
  Gil g;
  return ret_int(call("gpu_count", PyTuple_New(0)), out);
}

MXAPI int MXGetGPUMemoryInformation64(int dev, uint64_t* free_mem, uint64_t* total_mem) {
  Gil g;
  PyObject* r = call("gpu_memory", Py_BuildValue("(i)", dev));
  if (!r) return fail_from_python();
  unsigned long long f = 0, t = 0;
  const int ok = PyArg_ParseTuple(r, "KK", &f, &t);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *free_mem = f;
  *total_mem = t;
  return 0;
}

MXAPI int MXEngineSetBulkSize(int bulk_size, int* prev_bulk_size) {
  Gil g;
  return ret_int(call("set_bulk_size", Py_BuildValue("(i)", bulk_size)), prev_bulk_size);
}

MXAPI int MXSetIsNumpyShape(int is_np_shape, int* prev) {
  Gil g;
  return ret_int(call("set_np_shape", Py_BuildValue("(i)", is_np_shape)), prev);
}

MXAPI int MXIsNumpyShape(int* curr) {
  Gil g;
  return ret_int(call("is_np_shape", PyTuple_New(0)), curr);
}

// ----------------------------------------------------------------------------- Symbol / Executor extras
MXAPI int MXSymbolCopy(SymbolHandle symbol, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_copy", Py_BuildValue("(O)", obj(symbol))), out);
}

MXAPI int MXSymbolPrint(SymbolHandle symbol, const char** out_str) {
  Gil g;
  Obj* o = static_cast<Obj*>(symbol);
  return ret_string(call("sym_print", Py_BuildValue("(O)", o->o)), &o->str, out_str);
}

MXAPI int MXSymbolGetAttr(SymbolHandle symbol, const char* key, const char** out, int* success) {
  Gil g;
  Obj* o = static_cast<Obj*>(symbol);
  PyObject* r = call("sym_get_attr", Py_BuildValue("(Os)", o->o, key));
  if (!r) return fail_from_python();
  PyObject* v = nullptr;
  int ok = 0;
  if (!PyArg_ParseTuple(r, "Oi", &v, &ok) || !to_string(v, &o->str)) {
    Py_DECREF(r);
    return fail_from_python();
  }
  Py_DECREF(r);
  *out = ok ? o->str.c_str() : nullptr;
  *success = ok;
  return 0;
}

MXAPI int MXSymbolSetAttr(SymbolHandle symbol, const char* key, const char* value) {
  Gil g;
  return done(call("sym_set_attr", Py_BuildValue("(Oss)", obj(symbol), key, value)));
}

MXAPI int MXSymbolGetInternals(SymbolHandle symbol, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_internals", Py_BuildValue("(O)", obj(symbol))), out);
}

MXAPI int MXSymbolGetChildren(SymbolHandle symbol, SymbolHandle* out) {
  Gil g;
  PyObject* r = call("sym_children", Py_BuildValue("(O)", obj(symbol)));
  if (!r) return fail_from_python();
  if (r == Py_None) {
    Py_DECREF(r);
    *out = nullptr;
    return 0;
  }
  *out = wrap(r);
  return 0;
}

MXAPI int MXSymbolGetOutput(SymbolHandle symbol, uint32_t index, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_output", Py_BuildValue("(OI)", obj(symbol), index)), out);
}

MXAPI int MXSymbolGetNumOutputs(SymbolHandle symbol, uint32_t* output_count) {
  Gil g;
  int n = 0;
  if (ret_int(call("sym_num_outputs", Py_BuildValue("(O)", obj(symbol))), &n) != 0) return -1;
  *output_count = static_cast<uint32_t>(n);
  return 0;
}

MXAPI int MXSymbolCreateGroup(uint32_t num_symbols, SymbolHandle* symbols, SymbolHandle* out) {
  Gil g;
  return new_handle(call("sym_group", Py_BuildValue("(N)", obj_list(num_symbols, symbols))), out);
}

MXAPI int MXSymbolSaveToFile(SymbolHandle symbol, const char* fname) {
  Gil g;
  return done(call("sym_save", Py_BuildValue("(Os)", obj(symbol), fname)));
}

MXAPI int MXExecutorPrint(ExecutorHandle handle, const char** out_str) {
  Gil g;
  Obj* o = static_cast<Obj*>(handle);
  return ret_string(call("exec_print", Py_BuildValue("(O)", o->o)), &o->str, out_str);
}
