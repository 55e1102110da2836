// libsn_core: the C ABI of csrc/core/sn_core.h implemented over an embedded CPython
// interpreter that drives the sparknet_amd engine (sparknet_amd/capi.py).  The compute
// path underneath is the same as for Python callers: HIP kernels from libsn_kernels.so on
// the GPU, RCCL for collectives.  If the interpreter is not running (a C / JVM host
// program) it is started on first use and the package root is derived from this
// library's own location (<root>/sparknet_amd/lib/libsn_core.so).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>

#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "sn_core.h"

namespace {

thread_local std::string g_err;
sn_error_callback_t g_err_cb = nullptr;
PyObject* g_mod = nullptr;  // sparknet_amd.capi (owned)
std::once_flag g_init;

void ensure_interpreter() {
  std::call_once(g_init, [] {
    if (!Py_IsInitialized()) {
      Py_InitializeEx(0);
      PyEval_SaveThread();  // let PyGILState_Ensure work from every thread
    }
  });
}

struct Gil {
  PyGILState_STATE s;
  Gil() : s(PyGILState_Ensure()) {}
  ~Gil() { PyGILState_Release(s); }
};

void fetch_error(const char* where) {
  PyObject *t = nullptr, *v = nullptr, *tb = nullptr;
  PyErr_Fetch(&t, &v, &tb);
  std::string msg = where;
  if (v) {
    PyObject* s = PyObject_Str(v);
    if (s) {
      const char* c = PyUnicode_AsUTF8(s);
      msg += ": ";
      msg += c ? c : "?";
      Py_DECREF(s);
    }
  }
  PyErr_Clear();
  Py_XDECREF(t);
  Py_XDECREF(v);
  Py_XDECREF(tb);
  g_err = msg;
  if (g_err_cb) g_err_cb(g_err.c_str());
}

std::string package_root() {
  Dl_info info;
  if (!dladdr(reinterpret_cast<void*>(&package_root), &info) || !info.dli_fname) return ".";
  std::string p = info.dli_fname;  // <root>/sparknet_amd/lib/libsn_core.so
  for (int i = 0; i < 3; ++i) {
    size_t k = p.find_last_of('/');
    if (k == std::string::npos) return ".";
    p = p.substr(0, k);
  }
  return p.empty() ? "/" : p;
}

bool import_module() {
  if (g_mod) return true;
  PyObject* path = PySys_GetObject("path");  // borrowed
  PyObject* root = PyUnicode_FromString(package_root().c_str());
  if (path && root) PyList_Insert(path, 0, root);
  Py_XDECREF(root);
  g_mod = PyImport_ImportModule("sparknet_amd.capi");
  if (!g_mod) {
    fetch_error("import sparknet_amd.capi");
    return false;
  }
  return true;
}

// Call state.method(*args) built from a Py_BuildValue format; returns a new reference.
PyObject* call(void* state, const char* method, const char* fmt, ...) {
  if (!state) {
    g_err = "null state";
    return nullptr;
  }
  va_list ap;
  va_start(ap, fmt);
  PyObject* args = fmt && *fmt ? Py_VaBuildValue(fmt, ap) : PyTuple_New(0);
  va_end(ap);
  if (!args) {
    fetch_error(method);
    return nullptr;
  }
  if (!PyTuple_Check(args)) {
    PyObject* t = PyTuple_Pack(1, args);
    Py_DECREF(args);
    args = t;
  }
  PyObject* fn = PyObject_GetAttrString(static_cast<PyObject*>(state), method);
  PyObject* r = fn ? PyObject_CallObject(fn, args) : nullptr;
  Py_XDECREF(fn);
  Py_DECREF(args);
  if (!r) fetch_error(method);
  return r;
}

int status(PyObject* r) {
  if (!r) return 1;
  Py_DECREF(r);
  return 0;
}

int parse_file(const char* fn, const char* path, char** out, int* len) {
  ensure_interpreter();
  Gil g;
  if (!import_module()) return 1;
  PyObject* r = PyObject_CallMethod(g_mod, fn, "s", path);
  if (!r) {
    fetch_error(fn);
    return 1;
  }
  char* buf = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(r, &buf, &n) != 0) {
    fetch_error(fn);
    Py_DECREF(r);
    return 1;
  }
  *out = static_cast<char*>(std::malloc(n > 0 ? n : 1));
  std::memcpy(*out, buf, n);
  *len = (int)n;
  Py_DECREF(r);
  return 0;
}

}  // namespace

extern "C" {

const char* sn_last_error(void) { return g_err.c_str(); }

void* sn_create_state(void) {
  ensure_interpreter();
  Gil g;
  if (!import_module()) return nullptr;
  PyObject* st = PyObject_CallMethod(g_mod, "CoreState", nullptr);
  if (!st) fetch_error("CoreState()");
  return st;
}

void sn_destroy_state(void* state) {
  if (!state) return;
  Gil g;
  Py_DECREF(static_cast<PyObject*>(state));
}

int sn_set_device(void* s, int device) {
  Gil g;
  return status(call(s, "set_device", "(i)", device));
}

int sn_load_solver_from_protobuf(void* s, const char* bytes, int len) {
  Gil g;
  return status(call(s, "load_solver", "(y#)", bytes, (Py_ssize_t)len));
}

int sn_load_net_from_protobuf(void* s, const char* bytes, int len) {
  Gil g;
  return status(call(s, "load_net", "(y#)", bytes, (Py_ssize_t)len));
}

static int set_cb(void* s, int test, int layer, sn_data_callback_t cb, void* user) {
  Gil g;
  return status(call(s, "set_data_callback", "(iiKK)", test, layer, (unsigned long long)(uintptr_t)cb,
                     (unsigned long long)(uintptr_t)user));
}

int sn_set_train_data_callback(void* s, int layer, sn_data_callback_t cb, void* user) {
  return set_cb(s, 0, layer, cb, user);
}

int sn_set_test_data_callback(void* s, int layer, sn_data_callback_t cb, void* user) {
  return set_cb(s, 1, layer, cb, user);
}

int sn_forward(void* s, float* loss) {
  Gil g;
  PyObject* r = call(s, "forward", nullptr);
  if (!r) return 1;
  if (loss) *loss = (float)PyFloat_AsDouble(r);
  Py_DECREF(r);
  return 0;
}

int sn_backward(void* s) {
  Gil g;
  return status(call(s, "backward", nullptr));
}

int sn_solver_step(void* s, int iters) {
  Gil g;
  return status(call(s, "step", "(i)", iters));
}

int sn_solver_test(void* s, int iters) {
  Gil g;
  PyObject* r = call(s, "test", "(i)", iters);
  if (!r) return -1;
  long n = PyLong_AsLong(r);
  Py_DECREF(r);
  return (int)n;
}

float sn_get_test_score(void* s, int index) {
  Gil g;
  PyObject* scores = PyObject_GetAttrString(static_cast<PyObject*>(s), "scores");
  float v = 0.f;
  if (scores && index >= 0 && index < PyList_Size(scores)) v = (float)PyFloat_AsDouble(PyList_GetItem(scores, index));
  Py_XDECREF(scores);
  return v;
}

long long sn_num_params(void* s) {
  Gil g;
  PyObject* r = call(s, "num_params", nullptr);
  if (!r) return -1;
  long long n = PyLong_AsLongLong(r);
  Py_DECREF(r);
  return n;
}

int sn_get_weights(void* s, float* out, long long n) {
  Gil g;
  return status(call(s, "get_weights", "(KL)", (unsigned long long)(uintptr_t)out, n));
}

int sn_set_weights(void* s, const float* in, long long n) {
  Gil g;
  return status(call(s, "set_weights", "(KL)", (unsigned long long)(uintptr_t)in, n));
}

void* sn_weights_device_ptr(void* s) {
  Gil g;
  PyObject* r = call(s, "weights_device_ptr", nullptr);
  if (!r) return nullptr;
  void* p = (void*)(uintptr_t)PyLong_AsUnsignedLongLong(r);
  Py_DECREF(r);
  return p;
}

int sn_save_weights_to_file(void* s, const char* path) {
  Gil g;
  return status(call(s, "save_weights", "(s)", path));
}

int sn_load_weights_from_file(void* s, const char* path) {
  Gil g;
  return status(call(s, "load_weights", "(s)", path));
}

int sn_restore_solver_from_file(void* s, const char* path) {
  Gil g;
  return status(call(s, "restore_solver", "(s)", path));
}

int sn_num_layers(void* s) {
  Gil g;
  PyObject* r = call(s, "layer_names", nullptr);
  if (!r) return -1;
  int n = (int)PyList_Size(r);
  Py_DECREF(r);
  return n;
}

int sn_layer_name(void* s, int index, char* buf, int buflen) {
  Gil g;
  PyObject* r = call(s, "layer_names", nullptr);
  if (!r) return 1;
  int rc = 1;
  if (index >= 0 && index < PyList_Size(r) && buflen > 0) {
    const char* c = PyUnicode_AsUTF8(PyList_GetItem(r, index));
    if (c) {
      std::strncpy(buf, c, (size_t)buflen - 1);
      buf[buflen - 1] = 0;
      rc = 0;
    }
  }
  Py_DECREF(r);
  return rc;
}

int sn_parse_net_prototxt(const char* path, char** out, int* len) {
  return parse_file("parse_net_prototxt", path, out, len);
}

int sn_parse_solver_prototxt(const char* path, char** out, int* len) {
  return parse_file("parse_solver_prototxt", path, out, len);
}

void sn_free(void* p) { std::free(p); }

// -- process-level helpers --------------------------------------------------------------------
static int module_call(const char* fn, const char* fmt, ...) {
  ensure_interpreter();
  Gil g;
  if (!import_module()) return 1;
  PyObject* f = PyObject_GetAttrString(g_mod, fn);
  if (!f) {
    fetch_error(fn);
    return 1;
  }
  va_list ap;
  va_start(ap, fmt);
  PyObject* args = Py_VaBuildValue(fmt, ap);
  va_end(ap);
  PyObject* r = args ? PyObject_CallObject(f, args) : nullptr;
  Py_XDECREF(args);
  Py_DECREF(f);
  if (!r) fetch_error(fn);
  return status(r);
}

int sn_init_logging(const char* log_filename, int verbosity) {
  return module_call("init_logging", "(si)", log_filename, verbosity);
}

int sn_set_basepath(const char* path) { return module_call("set_basepath", "(s)", path); }

int sn_get_int_size(void) { return (int)sizeof(int); }
int sn_get_dtype_size(void) { return (int)sizeof(float); }

void sn_set_global_error_callback(sn_error_callback_t cb) { g_err_cb = cb; }

int sn_set_mode_cpu(void* s) { return sn_set_device(s, -1); }
int sn_set_mode_gpu(void* s) { return sn_set_device(s, 0); }

// -- databases ----------------------------------------------------------------------------------
int sn_create_db(void* s, const char* db_name, const char* db_type) {
  Gil g;
  return status(call(s, "create_db", "(ss)", db_name, db_type));
}

int sn_write_to_db(void* s, const char* image, int label, int channels, int height, int width, const char* key) {
  Gil g;
  Py_ssize_t n = (Py_ssize_t)channels * height * width;
  return status(call(s, "write_to_db", "(y#iiiis)", image, n, label, channels, height, width, key ? key : ""));
}

int sn_commit_db_txn(void* s) {
  Gil g;
  return status(call(s, "commit_db_txn", nullptr));
}

int sn_close_db(void* s) {
  Gil g;
  return status(call(s, "close_db", nullptr));
}

int sn_save_mean_image(const float* mean, int channels, int height, int width, const char* filename) {
  return module_call("save_mean_image", "(Kiiis)", (unsigned long long)(uintptr_t)mean, channels, height, width,
                     filename);
}

// -- blobs --------------------------------------------------------------------------------------
static long long int_call(void* s, const char* method, const char* fmt, ...) {
  if (!s) {
    g_err = "null state";
    return -1;
  }
  va_list ap;
  va_start(ap, fmt);
  PyObject* args = fmt && *fmt ? Py_VaBuildValue(fmt, ap) : PyTuple_New(0);
  va_end(ap);
  if (!args) {
    fetch_error(method);
    return -1;
  }
  PyObject* fn = PyObject_GetAttrString(static_cast<PyObject*>(s), method);
  PyObject* r = fn ? PyObject_CallObject(fn, args) : nullptr;
  Py_XDECREF(fn);
  Py_DECREF(args);
  if (!r) {
    fetch_error(method);
    return -1;
  }
  long long v = PyLong_AsLongLong(r);
  Py_DECREF(r);
  return v;
}

int sn_num_layer_weights(void* s, int layer) {
  Gil g;
  return (int)int_call(s, "num_layer_weights", "(i)", layer);
}

int sn_num_data_blobs(void* s) {
  Gil g;
  return (int)int_call(s, "num_data_blobs", "()");
}

int sn_data_blob_name(void* s, int index, char* buf, int buflen) {
  Gil g;
  PyObject* r = call(s, "data_blob_name", "(i)", index);
  if (!r) return 1;
  const char* c = PyUnicode_AsUTF8(r);
  int rc = 1;
  if (c && buflen > 0) {
    std::strncpy(buf, c, (size_t)buflen - 1);
    buf[buflen - 1] = 0;
    rc = 0;
  }
  Py_DECREF(r);
  return rc;
}

int sn_num_output_blobs(void* s) {
  Gil g;
  return (int)int_call(s, "num_output_blobs", "()");
}

int sn_num_test_scores(void* s) {
  Gil g;
  return (int)int_call(s, "num_test_scores", "()");
}

int sn_blob_num_axes(void* s, int layer, int index) {
  Gil g;
  return (int)int_call(s, "blob_num_axes", "(ii)", layer, index);
}

int sn_blob_axis_shape(void* s, int layer, int index, int axis) {
  Gil g;
  return (int)int_call(s, "blob_axis_shape", "(iii)", layer, index, axis);
}

int sn_blob_get(void* s, int layer, int index, int diff, float* out, long long n) {
  Gil g;
  return status(call(s, "blob_get", "(iiiKL)", layer, index, diff, (unsigned long long)(uintptr_t)out, n));
}

int sn_blob_set(void* s, int layer, int index, int diff, const float* in, long long n) {
  Gil g;
  return status(call(s, "blob_set", "(iiiKL)", layer, index, diff, (unsigned long long)(uintptr_t)in, n));
}

}  // extern "C"
