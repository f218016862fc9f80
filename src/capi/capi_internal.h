// Helpers shared by the C API translation units (c_api.cc, c_api_more.cc): GIL guard, handle
// objects, conversions between C arrays and Python lists, and the call into c_api_impl.
#pragma once
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace mxamd_capi {
bool ensure_python();
int fail_from_python();
int fail(const char* msg);
}  // namespace mxamd_capi

using mxamd_capi::fail;
using mxamd_capi::fail_from_python;

namespace {

struct Gil {
  PyGILState_STATE st;
  Gil() {
    mxamd_capi::ensure_python();
    st = PyGILState_Ensure();
  }
  ~Gil() { PyGILState_Release(st); }
};

// A handle: one framework object plus the buffers whose pointers the API hands back for it.
struct Obj {
  PyObject* o = nullptr;
  std::vector<uint32_t> u32;
  std::string str;
  std::vector<std::string> strs;
  std::vector<const char*> cstrs;
};

struct OpRec {
  std::string name;
};

// per-thread return storage for calls without a handle (outputs, loads, shape inference)
thread_local std::vector<void*> tl_handles;
thread_local std::vector<std::string> tl_strs;
thread_local std::vector<const char*> tl_cstrs;
thread_local std::vector<std::vector<uint32_t>> tl_shapes[3];
thread_local std::vector<uint32_t> tl_ndim[3];
thread_local std::vector<const uint32_t*> tl_ptr[3];

PyObject* impl() {
  static PyObject* mod = nullptr;
  if (mod == nullptr) mod = PyImport_ImportModule("mxnet_maintenance_amd.c_api_impl");
  return mod;
}

Obj* wrap(PyObject* o) {  // steals the reference
  Obj* h = new Obj();
  h->o = o;
  return h;
}

PyObject* obj(void* h) { return h ? static_cast<Obj*>(h)->o : Py_None; }

// list of the handles' objects (None for null handles)
PyObject* obj_list(uint32_t n, void* const* hs) {
  PyObject* l = PyList_New(n);
  for (uint32_t i = 0; l && i < n; ++i) {
    PyObject* o = hs ? obj(hs[i]) : Py_None;
    Py_INCREF(o);
    PyList_SET_ITEM(l, i, o);
  }
  return l;
}

PyObject* str_list(uint32_t n, const char* const* s) {
  PyObject* l = PyList_New(n);
  for (uint32_t i = 0; l && i < n; ++i) PyList_SET_ITEM(l, i, PyUnicode_FromString(s[i]));
  return l;
}

PyObject* int_list(uint32_t n, const int* v) {
  PyObject* l = PyList_New(n);
  for (uint32_t i = 0; l && i < n; ++i) PyList_SET_ITEM(l, i, PyLong_FromLong(v[i]));
  return l;
}

PyObject* u32_list(uint32_t n, const uint32_t* v) {
  PyObject* l = PyList_New(n);
  for (uint32_t i = 0; l && i < n; ++i) PyList_SET_ITEM(l, i, PyLong_FromUnsignedLong(v ? v[i] : 0));
  return l;
}

// call c_api_impl.<fn>(*args); returns a new reference or nullptr with the Python error set
PyObject* call(const char* fn, PyObject* args) {
  PyObject* mod = impl();
  if (!mod || !args) {
    Py_XDECREF(args);
    return nullptr;
  }
  PyObject* f = PyObject_GetAttrString(mod, fn);
  if (!f) {
    Py_DECREF(args);
    return nullptr;
  }
  PyObject* r = PyObject_CallObject(f, args);
  Py_DECREF(f);
  Py_DECREF(args);
  return r;
}

bool to_u32(PyObject* seq, std::vector<uint32_t>* out) {
  out->clear();
  PyObject* it = PyObject_GetIter(seq);
  if (!it) return false;
  while (PyObject* x = PyIter_Next(it)) {
    out->push_back(static_cast<uint32_t>(PyLong_AsUnsignedLong(x)));
    Py_DECREF(x);
  }
  Py_DECREF(it);
  return !PyErr_Occurred();
}

bool to_strs(PyObject* seq, std::vector<std::string>* strs, std::vector<const char*>* cs) {
  strs->clear();
  cs->clear();
  PyObject* it = PyObject_GetIter(seq);
  if (!it) return false;
  while (PyObject* x = PyIter_Next(it)) {
    const char* c = PyUnicode_AsUTF8(x);
    strs->push_back(c ? c : "");
    Py_DECREF(x);
  }
  Py_DECREF(it);
  for (auto& s : *strs) cs->push_back(s.c_str());
  return !PyErr_Occurred();
}

// list of framework objects -> freshly wrapped handles in tl_handles
bool to_handles(PyObject* seq) {
  tl_handles.clear();
  PyObject* it = PyObject_GetIter(seq);
  if (!it) return false;
  while (PyObject* x = PyIter_Next(it)) tl_handles.push_back(wrap(x));
  Py_DECREF(it);
  return !PyErr_Occurred();
}

int new_handle(PyObject* r, void** out) {
  if (!r) return fail_from_python();
  *out = wrap(r);
  return 0;
}

int done(PyObject* r) {
  if (!r) return fail_from_python();
  Py_DECREF(r);
  return 0;
}

int free_handle(void* h) {
  if (!h) return 0;
  Gil g;
  Obj* o = static_cast<Obj*>(h);
  Py_XDECREF(o->o);
  delete o;
  return 0;
}

int list_strings(void* h, const char* fn, int which, uint32_t* n, const char*** out) {
  Gil g;
  Obj* o = static_cast<Obj*>(h);
  PyObject* r = call(fn, Py_BuildValue("(Oi)", o->o, which));
  if (!r) return fail_from_python();
  const bool ok = to_strs(r, &o->strs, &o->cstrs);
  Py_DECREF(r);
  if (!ok) return fail_from_python();
  *n = static_cast<uint32_t>(o->cstrs.size());
  *out = o->cstrs.data();
  return 0;
}

}  // namespace

#define MXAPI extern "C" __attribute__((visibility("default")))
