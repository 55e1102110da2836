// libsn_core: the C ABI of csrc/core/sn_core.h.  Construction (net / solver from protobuf),
// the DB verbs and HDF5 weights go through an embedded CPython interpreter that drives the
// sparknet_amd engine (sparknet_amd/capi.py); once a verb's native plan exists, the solver
// step loop (captured hipGraphs), test / forward / backward, flat and per-blob weight and
// activation access and .caffemodel save / load run in C++ without entering it.  The compute
// path underneath is the same as for Python callers: HIP kernels from libsn_kernels.so on
// the GPU, RCCL for collectives.  If the interpreter is not running (a C / JVM host
// program) it is started on first use and the package root is derived from this
// library's own location (<root>/sparknet_amd/lib/libsn_core.so).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>

#include <hip/hip_runtime_api.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

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

// Every entry into the interpreter goes through a Gil; sn_python_entries() reports how many
// there were, so a host test can check that the steady-state verbs never enter Python.
std::atomic<long long> g_py_entries{0};

struct Gil {
  PyGILState_STATE s;
  Gil() : s(PyGILState_Ensure()) { g_py_entries.fetch_add(1, std::memory_order_relaxed); }
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

void sync_python(void* s);

// Call state.method(*args) built from a Py_BuildValue format; returns a new reference.
PyObject* call(void* state, const char* method, const char* fmt, ...) {
  if (!state) {
    g_err = "null state";
    return nullptr;
  }
  sync_python(state);
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

// ---------------------------------------------------------------------------------------
// Native executors.  The reference's verbs run Caffe's C++ Net / Solver directly
// (ccaffe.cpp:181-187 forward / backward, 218-238 solver_test / solver_step, 240-262
// get / set data).  Here, on a GPU state:
//   * sn_solver_step runs its iterations in NativeStep: CoreState.native_plan (capi.py)
//     captures one full training iteration (every kernel from libsn_kernels) into a
//     hipGraph and returns the handles and device buffers; per iteration this code calls
//     the C data callbacks (the JavaData contract, java_data_layer.cpp:37-44), copies each
//     minibatch into its data blob (pinned staging + sn_stage_nchw_f32_bf16 for NHWC image
//     blobs), stages the learning rate (SGDSolver::GetLearningRate, sgd_solver.cpp:27-63)
//     into the solver's hyper-parameter buffer and launches the graph;
//   * sn_forward / sn_solver_test replay a captured forward-only graph of the train / test
//     net (NativeForward, CoreState.forward_plan); the test graph adds each output blob's
//     sum into a device accumulator read once per sn_solver_test (TestAndStoreResult,
//     solver.cpp:413-444);
//   * sn_get_weights / sn_set_weights are a hipMemcpy on the flat fp32 master buffer plus,
//     for set, the sn_cast_f32_bf16 refresh of the bf16 compute shadow (NativeWeights).
// Each plan is built by one Python call on first use; afterwards these verbs never enter
// the interpreter (sn_python_entries counts the entries).  Python is re-entered only for
// display / snapshot iterations, and the solver's iteration counter / the test scores are
// handed back lazily at the next verb that does enter Python (sync_python).

typedef int (*stage_fn_t)(const float*, void*, long long, long long, long long, long long, hipStream_t);
typedef int (*cast_fn_t)(const float*, void*, long long, hipStream_t);

#define HIPOK(x)                                                   \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_);      \
      if (g_err_cb) g_err_cb(g_err.c_str());                       \
      return 1;                                                    \
    }                                                              \
  } while (0)

long long dict_ll(PyObject* d, const char* k) {
  PyObject* v = PyDict_GetItemString(d, k);
  return v ? PyLong_AsLongLong(v) : 0;
}
double dict_f(PyObject* d, const char* k) {
  PyObject* v = PyDict_GetItemString(d, k);
  return v ? PyFloat_AsDouble(v) : 0.0;
}

struct Feed {
  void* dev = nullptr;
  int kind = 0;  // 1: 4-D image blob (bf16 NHWC), 0: fp32 blob copied as is
  std::vector<int> shape;
  long long count = 0;
  sn_data_callback_t cb = nullptr;
  void* user = nullptr;
  float* host = nullptr;     // pinned
  float* staging = nullptr;  // device fp32 NCHW (kind 1)
};

// The data layers' callback feeds of one captured graph.
struct Feeds {
  std::vector<Feed> list;
  hipEvent_t fed = nullptr;
  bool pending = false;
  stage_fn_t stage = nullptr;

  ~Feeds() {
    for (auto& f : list) {
      if (f.host) hipHostFree(f.host);
      if (f.staging) hipFree(f.staging);
    }
    if (fed) hipEventDestroy(fed);
  }

  // from the plan's "feeds" list (GIL held); false with g_err set on failure
  bool build(PyObject* fl) {
    for (Py_ssize_t i = 0; fl && i < PyList_Size(fl); ++i) {
      PyObject* f = PyList_GetItem(fl, i);
      Feed fd;
      fd.dev = (void*)(uintptr_t)dict_ll(f, "dev");
      fd.kind = (int)dict_ll(f, "kind");
      fd.cb = (sn_data_callback_t)(uintptr_t)dict_ll(f, "cb");
      fd.user = (void*)(uintptr_t)dict_ll(f, "user");
      PyObject* sh = PyDict_GetItemString(f, "shape");
      fd.count = 1;
      for (Py_ssize_t k = 0; sh && k < PyTuple_Size(sh); ++k) {
        fd.shape.push_back((int)PyLong_AsLong(PyTuple_GetItem(sh, k)));
        fd.count *= fd.shape.back();
      }
      if (fd.kind == 1 && fd.shape.size() != 4) {
        g_err = "native feed: image blob is not 4-D";
        return false;
      }
      list.push_back(fd);
    }
    stage = (stage_fn_t)dlsym(RTLD_DEFAULT, "sn_stage_nchw_f32_bf16");
    if (!stage) {
      g_err = "native feed: sn_stage_nchw_f32_bf16 not found (libsn_kernels not loaded)";
      return false;
    }
    hipError_t e;
    for (auto& f : list) {
      if ((e = hipHostMalloc((void**)&f.host, sizeof(float) * f.count, 0)) != hipSuccess ||
          (f.kind == 1 && (e = hipMalloc((void**)&f.staging, sizeof(float) * f.count)) != hipSuccess)) {
        g_err = std::string("native feed: allocation: ") + hipGetErrorString(e);
        return false;
      }
    }
    if ((e = hipEventCreateWithFlags(&fed, hipEventDisableTiming)) != hipSuccess) {
      g_err = std::string("native feed: hipEventCreate: ") + hipGetErrorString(e);
      return false;
    }
    return true;
  }

  // call the callbacks and enqueue the copies / staging kernels on `stream`
  int run(hipStream_t stream) {
    // the host staging buffers are reused: the previous iteration's copies must have left
    if (pending) HIPOK(hipEventSynchronize(fed));
    for (auto& f : list) f.cb(f.host, f.shape.empty() ? 0 : f.shape[0], (int)f.shape.size(), f.shape.data(), f.user);
    for (auto& f : list) {
      if (f.kind == 1) {
        HIPOK(hipMemcpyAsync(f.staging, f.host, sizeof(float) * f.count, hipMemcpyHostToDevice, stream));
        if (stage(f.staging, f.dev, f.shape[0], f.shape[1], f.shape[2], f.shape[3], stream)) {
          g_err = "native feed: staging kernel launch failed";
          return 1;
        }
      } else {
        HIPOK(hipMemcpyAsync(f.dev, f.host, sizeof(float) * f.count, hipMemcpyHostToDevice, stream));
      }
    }
    if (!list.empty()) {
      HIPOK(hipEventRecord(fed, stream));
      pending = true;
    }
    return 0;
  }
};

struct NativeStep {
  hipGraphExec_t exec = nullptr;
  hipStream_t stream = nullptr;
  float* hyper_dev = nullptr;
  float hyper[16] = {};
  float last_lr = -1.f;
  static constexpr int RING = 8;
  float* hyper_host = nullptr;  // pinned, RING x 16
  hipEvent_t hyper_ev[RING] = {};
  int ring_pos = 0;
  // host run-ahead bound (engine.GraphStep.max_ahead): iteration k is issued once k - AHEAD
  // has finished, so captured iterations and their feeds are not queued dozens deep (a deep
  // queue runs the device slower for its first ~60 iterations)
  static constexpr int AHEAD = 2;
  hipEvent_t ahead_ev[AHEAD] = {};
  bool ahead_rec[AHEAD] = {};
  float* loss_dev = nullptr;
  float* loss_ring = nullptr;  // device, average_loss slots
  std::vector<float> loss_host;
  Feeds feeds;
  int policy = 0, adam = 0, display = 0, snapshot = 0, average_loss = 1;
  double base_lr = 0, gamma = 0, power = 0, momentum = 0, momentum2 = 0;
  long long stepsize = 0, max_iter = 0, iter = 0, done = 0, synced_iter = 0;
  std::vector<long long> stepvalues;

  ~NativeStep() {
    if (stream) hipStreamSynchronize(stream);
    for (auto& e : hyper_ev)
      if (e) hipEventDestroy(e);
    for (auto& e : ahead_ev)
      if (e) hipEventDestroy(e);
    if (hyper_host) hipHostFree(hyper_host);
    if (loss_ring) hipFree(loss_ring);
  }

  double learning_rate(long long it) const {
    switch (policy) {
      case 0: return base_lr;
      case 1: return base_lr * std::pow(gamma, (double)(it / (stepsize > 0 ? stepsize : 1)));
      case 2: return base_lr * std::pow(gamma, (double)it);
      case 3: return base_lr * std::pow(1.0 + gamma * (double)it, -power);
      case 4: {
        long long cur = 0;
        while (cur < (long long)stepvalues.size() && it >= stepvalues[cur]) ++cur;
        return base_lr * std::pow(gamma, (double)cur);
      }
      case 5: return base_lr * std::pow(1.0 - (double)it / (double)max_iter, power);
      default: return base_lr * (1.0 / (1.0 + std::exp(-gamma * ((double)it - (double)stepsize))));
    }
  }
};

struct NativeForward {
  hipGraphExec_t exec = nullptr;
  hipStream_t stream = nullptr;
  float* loss_dev = nullptr;
  float* acc_dev = nullptr;
  int n_out = 0;
  float* out_host = nullptr;  // pinned: loss + n_out sums
  Feeds feeds;

  ~NativeForward() {
    if (stream) hipStreamSynchronize(stream);
    if (out_host) hipHostFree(out_host);
  }
};

// One layer parameter inside the flat buffers, for the native sn_blob_* verbs (layer >= 0).
struct ParamDesc {
  long long off = 0, count = 0;
  int layout = 0;  // 0: internal order = Caffe's; 1: internal [K][R][S][C], Caffe [K][C][R][S]
  int ndim = 0;
  int cs[6] = {1, 1, 1, 1, 1, 1};  // Caffe shape
  int is[4] = {1, 1, 1, 1};        // internal shape
};

struct NativeWeights {
  float* data = nullptr;  // flat fp32 masters (device or host memory)
  float* diff = nullptr;  // flat fp32 gradients, same offsets
  long long count = 0;
  bool cuda = false;
  void* compute = nullptr;  // bf16 compute shadow (GPU) or null
  long long compute_count = 0;
  hipStream_t stream = nullptr;
  cast_fn_t cast = nullptr;
  std::map<std::pair<int, int>, ParamDesc> params;  // (layer, index)
  std::vector<float> stage;                         // host staging for layout conversion
  // layer names / types / parameter counts (the native .caffemodel IO); `complete` when
  // every parameter of every layer has a descriptor above
  struct Layer {
    std::string name, type;
    int nparams = 0;
  };
  std::vector<Layer> layers;
  std::string net_name;
  bool complete = false;
};

// Per-state native plans.  A plan that could not be built (CPU state, data layers fed
// from Python, solver features the graph cannot hold) is remembered as such until the
// state changes, so an ineligible state costs one Python call, not one per verb.
// Captured backward of the train net (CoreState.backward_plan): sn_backward replays it.
struct NativeBackward {
  hipGraphExec_t exec = nullptr;
  hipStream_t stream = nullptr;
};

// One activation blob (CoreState.blob_table) for the native sn_blob_* verbs on layer < 0:
// device data / gradient pointers (graph-owned memory of the forward / backward plans),
// bf16 or fp32, 4-D image blobs stored NHWC (logical NCHW dims).
struct BlobDesc {
  void* data = nullptr;
  void* diff = nullptr;
  int f32 = 0, image = 0, ndim = 0;
  int dims[6] = {1, 1, 1, 1, 1, 1};
  long long count = 1;
};

// Layer / blob names and counts (CoreState.meta_plan), read once per loaded net.
struct NativeMeta {
  std::vector<std::string> layers, blobs;
  std::vector<int> weights;
  int outputs = 0;
};

struct NativeState {
  std::unique_ptr<NativeStep> step;
  std::unique_ptr<NativeForward> fwd[2];  // [0] train net (sn_forward), [1] test net
  std::unique_ptr<NativeWeights> weights;
  std::unique_ptr<NativeBackward> bwd;
  std::vector<BlobDesc> blobs;  // from the train forward plan; gradients from the backward plan
  std::unique_ptr<NativeMeta> meta;
  bool bwd_failed = false, meta_failed = false;
  std::vector<uint16_t> blob_stage;
  bool step_failed = false, fwd_failed[2] = {false, false}, weights_failed = false;
  std::vector<float> scores;  // last native sn_solver_test
  bool scores_native = false, scores_pending = false;
};

std::mutex g_native_mu;
std::unordered_map<void*, std::unique_ptr<NativeState>> g_native;

NativeState& native_state(void* s) {
  std::lock_guard<std::mutex> lk(g_native_mu);
  auto& p = g_native[s];
  if (!p) p = std::make_unique<NativeState>();
  return *p;
}

NativeState* find_native(void* s) {
  std::lock_guard<std::mutex> lk(g_native_mu);
  auto it = g_native.find(s);
  return it == g_native.end() ? nullptr : it->second.get();
}

void drop_native(void* s) {
  std::lock_guard<std::mutex> lk(g_native_mu);
  g_native.erase(s);
}

bool native_enabled() {
  const char* v = std::getenv("SN_NATIVE_STEP");
  return v == nullptr || std::strcmp(v, "0") != 0;
}

// Hand the native loops' state back to Python before any other Python verb runs on `s`
// (GIL held): the solver's iteration counter and the scores of a native test.
void sync_python(void* s) {
  NativeState* st = find_native(s);
  if (!st) return;
  PyObject* obj = static_cast<PyObject*>(s);
  if (st->step && st->step->synced_iter != st->step->iter) {
    PyObject* r = PyObject_CallMethod(obj, "native_done", "(L)", st->step->iter);
    if (r) st->step->synced_iter = st->step->iter;
    Py_XDECREF(r);
    PyErr_Clear();
  }
  if (st->scores_pending) {
    PyObject* l = PyList_New((Py_ssize_t)st->scores.size());
    for (size_t i = 0; l && i < st->scores.size(); ++i) PyList_SetItem(l, (Py_ssize_t)i, PyFloat_FromDouble(st->scores[i]));
    PyObject* r = l ? PyObject_CallMethod(obj, "set_scores", "(O)", l) : nullptr;
    if (r) st->scores_pending = false;
    Py_XDECREF(r);
    Py_XDECREF(l);
    PyErr_Clear();
  }
}

// Call a plan method without reporting its failure through the error callback (an
// ineligible state simply stays on the Python path).
PyObject* call_quiet(void* s, const char* method, const char* fmt, ...) {
  sync_python(s);
  va_list ap;
  va_start(ap, fmt);
  PyObject* args = fmt && *fmt ? Py_VaBuildValue(fmt, ap) : PyTuple_New(0);
  va_end(ap);
  if (args && !PyTuple_Check(args)) {
    PyObject* t = PyTuple_Pack(1, args);
    Py_DECREF(args);
    args = t;
  }
  PyObject* fn = args ? PyObject_GetAttrString(static_cast<PyObject*>(s), method) : nullptr;
  PyObject* r = fn ? PyObject_CallObject(fn, args) : nullptr;
  Py_XDECREF(fn);
  Py_XDECREF(args);
  if (!r) {
    sn_error_callback_t cb = g_err_cb;
    g_err_cb = nullptr;
    fetch_error(method);
    g_err_cb = cb;
  }
  return r;
}

// Build the step executor from CoreState.native_plan() (GIL held).  Returns the iterations
// the plan's capture already ran, or -1 (g_err set; the caller falls back to Python).
long long build_native_step(void* s, std::unique_ptr<NativeStep>& out) {
  PyObject* r = call_quiet(s, "native_plan", nullptr);
  if (!r) return -1;
  long long ran = PyLong_AsLongLong(PyTuple_GetItem(r, 0));
  PyObject* d = PyTuple_GetItem(r, 1);
  auto ns = std::make_unique<NativeStep>();
  ns->exec = (hipGraphExec_t)(uintptr_t)dict_ll(d, "exec");
  ns->stream = (hipStream_t)(uintptr_t)dict_ll(d, "stream");
  ns->hyper_dev = (float*)(uintptr_t)dict_ll(d, "hyper_dev");
  ns->loss_dev = (float*)(uintptr_t)dict_ll(d, "loss_dev");
  ns->iter = ns->synced_iter = dict_ll(d, "iter");
  ns->policy = (int)dict_ll(d, "policy");
  ns->base_lr = dict_f(d, "base_lr");
  ns->gamma = dict_f(d, "gamma");
  ns->power = dict_f(d, "power");
  ns->stepsize = dict_ll(d, "stepsize");
  ns->max_iter = dict_ll(d, "max_iter");
  ns->adam = (int)dict_ll(d, "adam");
  ns->momentum = dict_f(d, "momentum");
  ns->momentum2 = dict_f(d, "momentum2");
  ns->display = (int)dict_ll(d, "display");
  ns->snapshot = (int)dict_ll(d, "snapshot");
  ns->average_loss = (int)dict_ll(d, "average_loss");
  PyObject* hv = PyDict_GetItemString(d, "hyper");
  for (int i = 0; i < 16 && hv && i < PyList_Size(hv); ++i) ns->hyper[i] = (float)PyFloat_AsDouble(PyList_GetItem(hv, i));
  PyObject* sv = PyDict_GetItemString(d, "stepvalues");
  for (Py_ssize_t i = 0; sv && i < PyList_Size(sv); ++i) ns->stepvalues.push_back(PyLong_AsLongLong(PyList_GetItem(sv, i)));
  const bool fed = ns->feeds.build(PyDict_GetItemString(d, "feeds"));
  Py_DECREF(r);
  if (PyErr_Occurred()) {
    fetch_error("native_plan");
    return -1;
  }
  if (!fed) return -1;
  auto fail = [&](hipError_t e, const char* what) {
    g_err = std::string("native step: ") + what + ": " + hipGetErrorString(e);
    return -1;
  };
  hipError_t e;
  if ((e = hipHostMalloc((void**)&ns->hyper_host, sizeof(float) * 16 * NativeStep::RING, 0)) != hipSuccess)
    return fail(e, "hipHostMalloc");
  for (auto& ev : ns->hyper_ev)
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return fail(e, "hipEventCreate");
  for (auto& ev : ns->ahead_ev)
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return fail(e, "hipEventCreate");
  if ((e = hipMalloc((void**)&ns->loss_ring, sizeof(float) * ns->average_loss)) != hipSuccess) return fail(e, "hipMalloc");
  ns->loss_host.assign(ns->average_loss, 0.f);
  out = std::move(ns);
  return ran;
}

// One training iteration (no GIL needed).
int native_iteration(NativeStep& ns) {
  const int ak = (int)(ns.iter % NativeStep::AHEAD);
  if (ns.ahead_rec[ak]) HIPOK(hipEventSynchronize(ns.ahead_ev[ak]));
  if (ns.feeds.run(ns.stream)) return 1;
  // hyper-parameters (Solver.hyper_values layout: 0 lr, 8 Adam correction)
  const float lr = (float)ns.learning_rate(ns.iter);
  float corr = ns.hyper[8];
  if (ns.adam) {
    const double t = (double)(ns.iter + 1);
    corr = (float)(std::sqrt(1.0 - std::pow(ns.momentum2, t)) / (1.0 - std::pow(ns.momentum, t)));
  }
  if (lr != ns.last_lr || (ns.adam && corr != ns.hyper[8])) {
    const int slot = ns.ring_pos;
    ns.ring_pos = (ns.ring_pos + 1) % NativeStep::RING;
    HIPOK(hipEventSynchronize(ns.hyper_ev[slot]));  // that slot's previous copy has left
    float* h = ns.hyper_host + 16 * slot;
    std::memcpy(h, ns.hyper, sizeof(ns.hyper));
    h[0] = lr;
    h[8] = corr;
    h[9] = 0.f;  // H_T: host-side only
    HIPOK(hipMemcpyAsync(ns.hyper_dev, h, sizeof(float) * 16, hipMemcpyHostToDevice, ns.stream));
    HIPOK(hipEventRecord(ns.hyper_ev[slot], ns.stream));
    ns.last_lr = lr;
    ns.hyper[8] = corr;
  }
  HIPOK(hipGraphLaunch(ns.exec, ns.stream));
  HIPOK(hipMemcpyAsync(ns.loss_ring + (ns.iter % ns.average_loss), ns.loss_dev, sizeof(float),
                       hipMemcpyDeviceToDevice, ns.stream));
  HIPOK(hipEventRecord(ns.ahead_ev[ak], ns.stream));
  ns.ahead_rec[ak] = true;
  ++ns.iter;
  ++ns.done;
  return 0;
}

// The forward executor of the train (test = 0) or test (1) net, if built.
// Parse CoreState.blob_table rows into BlobDesc (GIL held).
bool parse_blobs(PyObject* rows, std::vector<BlobDesc>& out) {
  out.clear();
  if (!rows || !PyList_Check(rows)) return false;
  for (Py_ssize_t i = 0; i < PyList_Size(rows); ++i) {
    PyObject* r = PyList_GetItem(rows, i);
    if (!PyTuple_Check(r) || PyTuple_Size(r) != 11) return false;
    auto at = [&](int k) { return PyLong_AsLongLong(PyTuple_GetItem(r, k)); };
    BlobDesc b;
    b.data = (void*)(uintptr_t)at(0);
    b.diff = (void*)(uintptr_t)at(1);
    b.f32 = (int)at(2);
    b.image = (int)at(3);
    b.ndim = (int)at(4);
    for (int d = 0; d < 6; ++d) {
      b.dims[d] = (int)at(5 + d);
      if (d < b.ndim) b.count *= b.dims[d];
    }
    out.push_back(b);
  }
  return !PyErr_Occurred();
}

NativeForward* native_forward(void* s, int test) {
  NativeState* st = find_native(s);
  return st && native_enabled() ? st->fwd[test].get() : nullptr;
}

// Build it right after the Python verb ran that forward eagerly (GIL held): the capture
// then finds every GEMM tuned, and the first call's side effects happen exactly once.
void build_forward(void* s, int test) {
  if (!native_enabled()) return;
  NativeState& st = native_state(s);
  if (st.fwd[test] || st.fwd_failed[test]) return;
  st.fwd_failed[test] = true;
  PyObject* d = call_quiet(s, "forward_plan", "(i)", test);
  if (!d) return;
  auto nf = std::make_unique<NativeForward>();
  nf->exec = (hipGraphExec_t)(uintptr_t)dict_ll(d, "exec");
  nf->stream = (hipStream_t)(uintptr_t)dict_ll(d, "stream");
  nf->loss_dev = (float*)(uintptr_t)dict_ll(d, "loss_dev");
  nf->acc_dev = (float*)(uintptr_t)dict_ll(d, "acc_dev");
  nf->n_out = (int)dict_ll(d, "n_out");
  const bool fed = nf->feeds.build(PyDict_GetItemString(d, "feeds"));
  if (!test) {
    if (!parse_blobs(PyDict_GetItemString(d, "blobs"), st.blobs)) st.blobs.clear();
    st.bwd.reset();  // it read the blobs this capture rebound
    st.bwd_failed = false;
  }
  Py_DECREF(d);
  if (PyErr_Occurred()) {
    fetch_error("forward_plan");
    return;
  }
  if (!fed || hipHostMalloc((void**)&nf->out_host, sizeof(float) * (1 + nf->n_out), 0) != hipSuccess) return;
  st.fwd_failed[test] = false;
  st.fwd[test] = std::move(nf);
}

NativeBackward* native_backward(void* s) {
  NativeState* st = find_native(s);
  return st && native_enabled() && st->fwd[0] ? st->bwd.get() : nullptr;
}

// Build it right after the Python verb ran a backward (GIL held), on top of the train
// forward plan whose graph memory the blobs are bound to.
void build_backward(void* s) {
  if (!native_enabled()) return;
  NativeState& st = native_state(s);
  if (!st.fwd[0] || st.bwd || st.bwd_failed) return;
  st.bwd_failed = true;
  PyObject* d = call_quiet(s, "backward_plan", nullptr);
  if (!d) return;
  auto nb = std::make_unique<NativeBackward>();
  nb->exec = (hipGraphExec_t)(uintptr_t)dict_ll(d, "exec");
  nb->stream = (hipStream_t)(uintptr_t)dict_ll(d, "stream");
  std::vector<BlobDesc> blobs;
  const bool ok = parse_blobs(PyDict_GetItemString(d, "blobs"), blobs);
  Py_DECREF(d);
  if (PyErr_Occurred()) {
    fetch_error("backward_plan");
    return;
  }
  if (!ok || !nb->exec) return;
  st.blobs = std::move(blobs);
  st.bwd_failed = false;
  st.bwd = std::move(nb);
}

NativeMeta* native_meta(void* s) {
  if (!native_enabled()) return nullptr;
  NativeState& st = native_state(s);
  if (st.meta) return st.meta.get();
  if (st.meta_failed) return nullptr;
  Gil g;
  st.meta_failed = true;
  PyObject* d = call_quiet(s, "meta_plan", nullptr);
  if (!d) return nullptr;
  auto m = std::make_unique<NativeMeta>();
  auto strs = [](PyObject* l, std::vector<std::string>& out) {
    if (!l || !PyList_Check(l)) return false;
    for (Py_ssize_t i = 0; i < PyList_Size(l); ++i) {
      const char* c = PyUnicode_AsUTF8(PyList_GetItem(l, i));
      if (!c) return false;
      out.emplace_back(c);
    }
    return true;
  };
  bool ok = strs(PyDict_GetItemString(d, "layers"), m->layers) && strs(PyDict_GetItemString(d, "blobs"), m->blobs);
  PyObject* w = PyDict_GetItemString(d, "weights");
  ok = ok && w && PyList_Check(w);
  for (Py_ssize_t i = 0; ok && i < PyList_Size(w); ++i) m->weights.push_back((int)PyLong_AsLong(PyList_GetItem(w, i)));
  m->outputs = (int)dict_ll(d, "outputs");
  Py_DECREF(d);
  if (PyErr_Occurred() || !ok) {
    PyErr_Clear();
    return nullptr;
  }
  st.meta_failed = false;
  st.meta = std::move(m);
  return st.meta.get();
}

// The activation blob `index` with a native pointer for data (diff = 0) or gradient (1).
const BlobDesc* native_blob(void* s, int index, int diff, hipStream_t* stream) {
  NativeState* st = find_native(s);
  if (!st || !native_enabled() || !st->fwd[0] || index < 0 || index >= (int)st->blobs.size()) return nullptr;
  const BlobDesc& b = st->blobs[(size_t)index];
  if (!(diff ? b.diff : b.data)) return nullptr;
  if (diff && !st->bwd) return nullptr;
  *stream = st->fwd[0]->stream;
  return &b;
}

// logical (NCHW) element index -> storage index of an NHWC image blob
inline long long nhwc_index(const BlobDesc& b, long long i) {
  const long long W = b.dims[3], H = b.dims[2], Cc = b.dims[1];
  const long long w = i % W, h = (i / W) % H, c = (i / (W * H)) % Cc, n = i / (W * H * Cc);
  return ((n * H + h) * W + w) * Cc + c;
}

int blob_get_native(NativeState& st, const BlobDesc& b, hipStream_t stream, int diff, float* out, long long n) {
  if (!out || n < b.count) {
    g_err = "sn_blob_get: buffer smaller than the blob";
    return 1;
  }
  const void* src = diff ? b.diff : b.data;
  const size_t es = b.f32 ? 4 : 2;
  st.blob_stage.resize((size_t)(b.count * es + 1) / 2);
  void* tmp = st.blob_stage.data();
  HIPOK(hipMemcpyAsync(tmp, src, es * b.count, hipMemcpyDeviceToHost, stream));
  HIPOK(hipStreamSynchronize(stream));
  for (long long i = 0; i < b.count; ++i) {
    const long long j = b.image ? nhwc_index(b, i) : i;
    if (b.f32) {
      out[i] = static_cast<const float*>(tmp)[j];
    } else {
      const uint32_t u = (uint32_t)static_cast<const uint16_t*>(tmp)[j] << 16;
      std::memcpy(&out[i], &u, 4);
    }
  }
  return 0;
}

int blob_set_native(NativeState& st, const BlobDesc& b, hipStream_t stream, int diff, const float* in, long long n) {
  if (!in || n < b.count) {
    g_err = "sn_blob_set: buffer smaller than the blob";
    return 1;
  }
  void* dst = diff ? b.diff : b.data;
  const size_t es = b.f32 ? 4 : 2;
  st.blob_stage.resize((size_t)(b.count * es + 1) / 2);
  void* tmp = st.blob_stage.data();
  for (long long i = 0; i < b.count; ++i) {
    const long long j = b.image ? nhwc_index(b, i) : i;
    if (b.f32) {
      static_cast<float*>(tmp)[j] = in[i];
    } else {  // round to nearest even, as the device casts
      uint32_t u;
      std::memcpy(&u, &in[i], 4);
      const uint32_t r = ((u >> 16) & 1u) + 0x7fffu;
      static_cast<uint16_t*>(tmp)[j] = (uint16_t)((u + r) >> 16);
    }
  }
  HIPOK(hipMemcpyAsync(dst, tmp, es * b.count, hipMemcpyHostToDevice, stream));
  HIPOK(hipStreamSynchronize(stream));
  return 0;
}

NativeWeights* native_weights(void* s) {
  if (!native_enabled()) return nullptr;
  NativeState& st = native_state(s);
  if (st.weights) return st.weights.get();
  if (st.weights_failed) return nullptr;
  Gil g;
  st.weights_failed = true;
  PyObject* d = call_quiet(s, "weights_plan", nullptr);
  if (!d) return nullptr;
  auto w = std::make_unique<NativeWeights>();
  w->data = (float*)(uintptr_t)dict_ll(d, "data");
  w->count = dict_ll(d, "count");
  w->cuda = dict_ll(d, "cuda") != 0;
  w->compute = (void*)(uintptr_t)dict_ll(d, "compute");
  w->compute_count = dict_ll(d, "compute_count");
  w->stream = (hipStream_t)(uintptr_t)dict_ll(d, "stream");
  w->diff = (float*)(uintptr_t)dict_ll(d, "diff");
  if (PyObject* rows = PyDict_GetItemString(d, "params")) {  // borrowed
    const Py_ssize_t nr = PySequence_Size(rows);
    for (Py_ssize_t i = 0; i < nr && !PyErr_Occurred(); ++i) {
      PyObject* row = PySequence_GetItem(rows, i);
      long long v[16];
      bool ok = row && PySequence_Size(row) == 16;
      for (int j = 0; ok && j < 16; ++j) {
        PyObject* x = PySequence_GetItem(row, j);
        v[j] = x ? PyLong_AsLongLong(x) : -1;
        Py_XDECREF(x);
        ok = x != nullptr && !PyErr_Occurred();
      }
      Py_XDECREF(row);
      if (!ok) break;
      ParamDesc p;
      p.off = v[2];
      p.count = v[3];
      p.layout = (int)v[4];
      p.ndim = (int)v[5];
      for (int j = 0; j < 6; ++j) p.cs[j] = (int)v[6 + j];
      for (int j = 0; j < 4; ++j) p.is[j] = (int)v[12 + j];
      w->params[{(int)v[0], (int)v[1]}] = p;
    }
  }
  if (PyObject* ls = PyDict_GetItemString(d, "layers")) {  // borrowed
    const Py_ssize_t nl = PySequence_Size(ls);
    for (Py_ssize_t i = 0; i < nl && !PyErr_Occurred(); ++i) {
      PyObject* row = PySequence_GetItem(ls, i);
      const char* nm = nullptr;
      const char* ty = nullptr;
      int np = 0;
      if (row && PyArg_ParseTuple(row, "ssi", &nm, &ty, &np)) w->layers.push_back({nm, ty, np});
      Py_XDECREF(row);
    }
    w->complete = !PyErr_Occurred();
    for (size_t li = 0; w->complete && li < w->layers.size(); ++li)
      for (int pi = 0; pi < w->layers[li].nparams; ++pi)
        if (!w->params.count({(int)li, pi})) w->complete = false;
  }
  if (PyObject* nn = PyDict_GetItemString(d, "net_name")) {  // borrowed
    if (const char* c = PyUnicode_AsUTF8(nn)) w->net_name = c;
  }
  Py_DECREF(d);
  if (PyErr_Occurred()) {
    fetch_error("weights_plan");
    return nullptr;
  }
  if (w->compute) {
    w->cast = (cast_fn_t)dlsym(RTLD_DEFAULT, "sn_cast_f32_bf16");
    if (!w->cast) return nullptr;
  }
  st.weights_failed = false;
  st.weights = std::move(w);
  return st.weights.get();
}

// Forget the plans that depend on what a verb is about to change.
enum : unsigned { P_STEP = 1, P_FWD_TRAIN = 2, P_FWD_TEST = 4, P_WEIGHTS = 8, P_SCORES = 16, P_META = 32 };

void invalidate(void* s, unsigned what) {
  NativeState* st = find_native(s);
  if (!st) return;
  if (what & P_STEP) st->step.reset(), st->step_failed = false;
  if (what & P_FWD_TRAIN) {  // the backward plan and the blob table hang off the forward plan
    st->fwd[0].reset(), st->fwd_failed[0] = false;
    st->bwd.reset(), st->bwd_failed = false;
    st->blobs.clear();
  }
  if (what & P_META) st->meta.reset(), st->meta_failed = false;
  if (what & P_FWD_TEST) st->fwd[1].reset(), st->fwd_failed[1] = false;
  if (what & P_WEIGHTS) st->weights.reset(), st->weights_failed = false;
  if (what & P_SCORES) st->scores_native = st->scores_pending = false;
}

// The native weights plan's descriptor of parameter `index` of layer `layer`, or null
// (activation blobs, params outside the flat buffers, no plan: the Python path).
const ParamDesc* native_param(void* s, int layer, int index, NativeWeights** wo) {
  if (layer < 0) return nullptr;
  NativeWeights* w = native_weights(s);
  if (!w) return nullptr;
  auto it = w->params.find({layer, index});
  if (it == w->params.end()) return nullptr;
  *wo = w;
  return &it->second;
}

// internal [K][R][S][C] <-> Caffe [K][C][R][S]
void krsc_to_kcrs(const float* src, float* dst, const int* is, bool to_caffe) {
  const long long K = is[0], R = is[1], S = is[2], Cc = is[3];
  for (long long k = 0; k < K; ++k)
    for (long long r = 0; r < R; ++r)
      for (long long q = 0; q < S; ++q)
        for (long long c = 0; c < Cc; ++c) {
          const long long a = ((k * R + r) * S + q) * Cc + c, b = ((k * Cc + c) * R + r) * S + q;
          if (to_caffe) dst[b] = src[a];
          else dst[a] = src[b];
        }
}

bool param_buffer_ok(const ParamDesc& p, long long n, const void* buf) {
  if (n < p.count || (p.count > 0 && !buf)) {
    g_err = "buffer holds " + std::to_string(n) + " floats, blob has " + std::to_string(p.count);
    return false;
  }
  return true;
}

int param_get(NativeWeights* w, const ParamDesc& p, int diff, float* out, long long n) {
  if (!param_buffer_ok(p, n, out)) return 1;
  const float* src = (diff ? w->diff : w->data) + p.off;
  float* dst = out;
  if (p.layout) {
    w->stage.resize((size_t)p.count);
    dst = w->stage.data();
  }
  if (w->cuda) {
    HIPOK(hipMemcpyAsync(dst, src, sizeof(float) * p.count, hipMemcpyDeviceToHost, w->stream));
    HIPOK(hipStreamSynchronize(w->stream));
  } else {
    std::memcpy(dst, src, sizeof(float) * p.count);
  }
  if (p.layout) krsc_to_kcrs(dst, out, p.is, true);
  return 0;
}

int param_set(NativeWeights* w, const ParamDesc& p, int diff, const float* in, long long n) {
  if (!param_buffer_ok(p, n, in)) return 1;
  float* dst = (diff ? w->diff : w->data) + p.off;
  const float* src = in;
  if (p.layout) {
    w->stage.resize((size_t)p.count);
    krsc_to_kcrs(in, w->stage.data(), p.is, false);
    src = w->stage.data();
  }
  if (!w->cuda) {
    std::memcpy(dst, src, sizeof(float) * p.count);
    return 0;
  }
  HIPOK(hipMemcpyAsync(dst, src, sizeof(float) * p.count, hipMemcpyHostToDevice, w->stream));
  // the master changed: refresh its slice of the bf16 compute shadow (Net.sync_compute)
  if (!diff && w->compute && w->cast(dst, static_cast<char*>(w->compute) + 2 * p.off, p.count, w->stream)) {
    g_err = "sn_blob_set: sn_cast_f32_bf16 launch failed";
    return 1;
  }
  HIPOK(hipStreamSynchronize(w->stream));  // `in` may be reused as soon as this returns
  return 0;
}

// ---- native .caffemodel IO (Net::ToProto / Net::CopyTrainedLayersFrom, caffe/src/caffe/net.cpp:
// 816-858, 953-961; blob.cpp:463-530) over the protobuf wire format: NetParameter { name = 1;
// layer = 100 (LayerParameter { name = 1; type = 2; blobs = 7 }); legacy layers = 2
// (V1LayerParameter { name = 4; blobs = 6 }) }, BlobProto { num..width = 1..4 (legacy 4-D);
// data = 5 (packed float); double_data = 8; shape = 7 (BlobShape { dim = 1, packed int64 }) }.

void pb_varint(std::string& o, unsigned long long v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}

void pb_bytes(std::string& o, int field, const std::string& b) {
  pb_varint(o, ((unsigned long long)field << 3) | 2);
  pb_varint(o, b.size());
  o += b;
}

// BlobProto of one parameter (Caffe layout, fp32 data)
int pb_blob(NativeWeights* w, const ParamDesc& p, std::string& out) {
  std::vector<float> v((size_t)p.count);
  if (param_get(w, p, 0, v.data(), p.count)) return 1;
  std::string shape, dims;
  for (int a = 0; a < p.ndim; ++a) pb_varint(dims, (unsigned long long)(long long)p.cs[a]);
  pb_bytes(shape, 1, dims);
  out.clear();
  pb_bytes(out, 7, shape);
  std::string data(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(float));  // little endian
  pb_bytes(out, 5, data);
  return 0;
}

int save_caffemodel_native(NativeWeights* w, const char* path) {
  std::string net, layer, blob;
  if (!w->net_name.empty()) pb_bytes(net, 1, w->net_name);
  for (size_t li = 0; li < w->layers.size(); ++li) {
    layer.clear();
    pb_bytes(layer, 1, w->layers[li].name);
    pb_bytes(layer, 2, w->layers[li].type);
    for (int pi = 0; pi < w->layers[li].nparams; ++pi) {
      if (pb_blob(w, w->params.at({(int)li, pi}), blob)) return 1;
      pb_bytes(layer, 7, blob);
    }
    pb_bytes(net, 100, layer);
  }
  FILE* f = std::fopen(path, "wb");
  if (!f) {
    g_err = std::string("cannot open ") + path + " for writing";
    return 1;
  }
  const bool ok = std::fwrite(net.data(), 1, net.size(), f) == net.size();
  if (std::fclose(f) != 0 || !ok) {
    g_err = std::string("short write to ") + path;
    return 1;
  }
  return 0;
}

// A bounds-checked reader over one message.
struct PbReader {
  const unsigned char* p;
  const unsigned char* end;
  bool bad = false;
  bool more() const { return !bad && p < end; }
  unsigned long long varint() {
    unsigned long long v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (p >= end) break;
      const unsigned char b = *p++;
      v |= (unsigned long long)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    bad = true;
    return 0;
  }
  // next field: number and wire type; a length-delimited payload in [*lp, *lp + *ln)
  bool field(int* num, int* wt, const unsigned char** lp, size_t* ln) {
    const unsigned long long key = varint();
    *num = (int)(key >> 3);
    *wt = (int)(key & 7);
    switch (*wt) {
      case 0: *ln = (size_t)varint(); return !bad;  // the value, for varints
      case 1: *lp = p; *ln = 8; break;
      case 2: *ln = (size_t)varint(); *lp = p; break;
      case 5: *lp = p; *ln = 4; break;
      default: bad = true; return false;
    }
    if (bad || (size_t)(end - p) < *ln) {
      bad = true;
      return false;
    }
    p += *ln;
    return true;
  }
};

struct PbBlob {
  std::vector<long long> shape;
  bool legacy = false;
  long long leg[4] = {0, 0, 0, 0};  // num, channels, height, width (proto2 default 0)
  std::vector<float> data;
};

bool parse_blob(const unsigned char* b, size_t n, PbBlob* out) {
  PbReader r{b, b + n};
  std::vector<double> dd;
  while (r.more()) {
    int num, wt;
    const unsigned char* lp = nullptr;
    size_t ln = 0;
    if (!r.field(&num, &wt, &lp, &ln)) return false;
    if (num >= 1 && num <= 4 && wt == 0) {
      out->legacy = true;
      out->leg[num - 1] = (long long)(int)ln;
    } else if (num == 5 && wt == 2) {  // packed floats
      const size_t k = out->data.size();
      out->data.resize(k + ln / 4);
      std::memcpy(out->data.data() + k, lp, (ln / 4) * 4);
    } else if (num == 5 && wt == 5) {
      float f;
      std::memcpy(&f, lp, 4);
      out->data.push_back(f);
    } else if (num == 8 && (wt == 2 || wt == 1)) {
      const size_t k = dd.size();
      dd.resize(k + ln / 8);
      std::memcpy(dd.data() + k, lp, (ln / 8) * 8);
    } else if (num == 7 && wt == 2) {  // BlobShape
      PbReader sr{lp, lp + ln};
      while (sr.more()) {
        int sn, swt;
        const unsigned char* slp = nullptr;
        size_t sln = 0;
        if (!sr.field(&sn, &swt, &slp, &sln)) return false;
        if (sn != 1) continue;
        if (swt == 0) {
          out->shape.push_back((long long)sln);
        } else if (swt == 2) {
          PbReader dr{slp, slp + sln};
          while (dr.more()) out->shape.push_back((long long)dr.varint());
          if (dr.bad) return false;
        }
      }
    }
  }
  if (out->data.empty() && !dd.empty()) out->data.assign(dd.begin(), dd.end());
  return !r.bad;
}

// Blob::ShapeEquals (blob.cpp:463-478): legacy 4-D dims compare against the target padded to 4 axes
bool blob_shape_equals(const PbBlob& b, const ParamDesc& p) {
  if (b.legacy) {
    if (p.ndim > 4) return false;
    long long t[4] = {1, 1, 1, 1};
    for (int a = 0; a < p.ndim; ++a) t[4 - p.ndim + a] = p.cs[a];
    return t[0] == b.leg[0] && t[1] == b.leg[1] && t[2] == b.leg[2] && t[3] == b.leg[3];
  }
  if ((int)b.shape.size() != p.ndim) return false;
  for (int a = 0; a < p.ndim; ++a)
    if (b.shape[a] != p.cs[a]) return false;
  return true;
}

std::string shape_str(const PbBlob& b) {
  std::string s = "(";
  if (b.legacy) {
    for (int a = 0; a < 4; ++a) s += std::to_string(b.leg[a]) + (a < 3 ? ", " : "");
  } else {
    for (size_t a = 0; a < b.shape.size(); ++a) s += std::to_string(b.shape[a]) + (a + 1 < b.shape.size() ? ", " : "");
  }
  return s + ")";
}

// 1: error (g_err set), 2: a form this reader leaves to the Python path (V0 layers)
int load_caffemodel_native(NativeWeights* w, const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    g_err = std::string("cannot open ") + path;
    return 1;
  }
  std::vector<unsigned char> buf;
  unsigned char chunk[1 << 16];
  size_t k;
  while ((k = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + k);
  std::fclose(f);
  std::map<std::string, int> index;
  for (size_t li = 0; li < w->layers.size(); ++li) index.emplace(w->layers[li].name, (int)li);  // first wins
  PbReader r{buf.data(), buf.data() + buf.size()};
  while (r.more()) {
    int num, wt;
    const unsigned char* lp = nullptr;
    size_t ln = 0;
    if (!r.field(&num, &wt, &lp, &ln)) break;
    if (wt != 2 || (num != 100 && num != 2)) continue;
    const bool v1 = num == 2;
    PbReader lr{lp, lp + ln};
    std::string name;
    std::vector<std::pair<const unsigned char*, size_t>> blobs;
    while (lr.more()) {
      int fn, fwt;
      const unsigned char* flp = nullptr;
      size_t fln = 0;
      if (!lr.field(&fn, &fwt, &flp, &fln)) break;
      if (fwt != 2) continue;
      if (v1 && fn == 1) return 2;  // a V0 layer inside: upgrade on the Python path
      if (fn == (v1 ? 4 : 1)) name.assign(reinterpret_cast<const char*>(flp), fln);
      if (fn == (v1 ? 6 : 7)) blobs.emplace_back(flp, fln);
    }
    if (lr.bad) break;
    auto it = index.find(name);
    if (it == index.end()) continue;  // "Ignoring source layer"
    const int li = it->second;
    if ((int)blobs.size() != w->layers[li].nparams) {
      g_err = "Incompatible number of blobs for layer '" + name + "'";
      return 1;
    }
    for (int pi = 0; pi < (int)blobs.size(); ++pi) {
      PbBlob b;
      if (!parse_blob(blobs[pi].first, blobs[pi].second, &b)) {
        r.bad = true;
        break;
      }
      const ParamDesc& p = w->params.at({li, pi});
      std::string ts = "(";
      for (int a = 0; a < p.ndim; ++a) ts += std::to_string(p.cs[a]) + (a + 1 < p.ndim ? ", " : "");
      ts += ")";
      if (!blob_shape_equals(b, p) || (long long)b.data.size() != p.count) {
        g_err = "Cannot copy param of layer '" + name + "'; shape mismatch. Source " + shape_str(b) +
                " (" + std::to_string(b.data.size()) + " values), target " + ts;
        return 1;
      }
      if (param_set(w, p, 0, b.data.data(), p.count)) return 1;
    }
  }
  if (r.bad) {
    g_err = std::string("malformed NetParameter in ") + path;
    return 1;
  }
  return 0;
}

// ---- native record databases (ccaffe.cpp:51-81 create_db / write_to_db / commit_db_txn /
// close_db; caffe/src/caffe/util/db_lmdb.cpp): Datum records into an LMDB environment (the
// bulk-loaded B+tree of sparknet_amd/data/lmdb.py write_lmdb, page for page) or the sndb
// record file; LevelDB stays on the Python path (sparknet_amd/data/leveldb.py).
struct NativeDB {
  std::string path;
  bool lmdb = false;
  FILE* f = nullptr;  // sndb
  std::map<std::string, std::string> all;  // lmdb: committed records, key order (memcmp order)
  std::vector<std::pair<std::string, std::string>> txn;
  long long count = 0;
};

std::mutex g_db_mu;
std::unordered_map<void*, std::unique_ptr<NativeDB>> g_dbs;

NativeDB* find_db(void* s) {
  std::lock_guard<std::mutex> lk(g_db_mu);
  auto it = g_dbs.find(s);
  return it == g_dbs.end() ? nullptr : it->second.get();
}

// Datum { channels = 1; height = 2; width = 3; data = 4; label = 5; encoded = 7 }, every field
// present, in field order (what Python's SerializeToString writes for capi.write_to_db)
std::string datum_bytes(const char* image, int label, int c, int h, int w) {
  std::string o;
  pb_varint(o, 1 << 3), pb_varint(o, (unsigned long long)(long long)c);
  pb_varint(o, 2 << 3), pb_varint(o, (unsigned long long)(long long)h);
  pb_varint(o, 3 << 3), pb_varint(o, (unsigned long long)(long long)w);
  pb_bytes(o, 4, std::string(image, (size_t)c * h * w));
  pb_varint(o, 5 << 3), pb_varint(o, (unsigned long long)(long long)label);
  pb_varint(o, 7 << 3), pb_varint(o, 0);
  return o;
}

constexpr int kPage = 4096, kPageHdr = 16, kMaxKey = 511;
constexpr uint16_t MDB_P_BRANCH = 0x01, MDB_P_LEAF = 0x02, MDB_P_OVERFLOW = 0x04, MDB_P_META = 0x08, MDB_F_BIGDATA = 0x01;
constexpr unsigned long long MDB_P_INVALID = ~0ull;

template <typename T>
void put_le(std::string& o, T v) {
  o.append(reinterpret_cast<const char*>(&v), sizeof v);
}

std::string lmdb_node(const std::string& key, uint16_t lo, uint16_t hi, uint16_t flags, const std::string& payload) {
  std::string b;
  put_le<uint16_t>(b, lo), put_le<uint16_t>(b, hi), put_le<uint16_t>(b, flags), put_le<uint16_t>(b, (uint16_t)key.size());
  b += key;
  b += payload;
  if (b.size() & 1) b.push_back('\0');
  return b;
}

struct LmdbPages {
  FILE* f;
  unsigned long long next = 2, branch = 0, leaf = 0, overflow = 0;
  bool ok = true;
  void put(unsigned long long pg, const std::string& data) {
    ok = ok && fseeko(f, (off_t)(pg * kPage), SEEK_SET) == 0 && std::fwrite(data.data(), 1, data.size(), f) == data.size();
  }
  unsigned long long over(const std::string& v) {
    const unsigned long long n = (kPageHdr + v.size() + kPage - 1) / kPage, pg = next;
    next += n;
    std::string b;
    put_le<unsigned long long>(b, pg), put_le<uint16_t>(b, 0), put_le<uint16_t>(b, MDB_P_OVERFLOW), put_le<uint32_t>(b, (uint32_t)n);
    b += v;
    b.resize((size_t)(n * kPage), '\0');
    put(pg, b);
    overflow += n;
    return pg;
  }
  unsigned long long page(const std::vector<std::string>& nodes, uint16_t flags) {
    const unsigned long long pg = next++;
    std::string b((size_t)kPage, '\0');
    size_t upper = kPage;
    for (size_t i = 0; i < nodes.size(); ++i) {
      upper -= nodes[i].size();
      std::memcpy(&b[upper], nodes[i].data(), nodes[i].size());
      const uint16_t u = (uint16_t)upper;
      std::memcpy(&b[kPageHdr + 2 * i], &u, 2);
    }
    std::string h;
    put_le<unsigned long long>(h, pg), put_le<uint16_t>(h, 0), put_le<uint16_t>(h, flags);
    put_le<uint16_t>(h, (uint16_t)(kPageHdr + 2 * nodes.size())), put_le<uint16_t>(h, (uint16_t)upper);
    std::memcpy(&b[0], h.data(), h.size());
    put(pg, b);
    ++(flags & MDB_P_BRANCH ? branch : leaf);
    return pg;
  }
};

// MDB_db: pad, flags, depth, branch / leaf / overflow page counts, entries, root
void db_meta(std::string& b, uint32_t pad, uint16_t depth, unsigned long long branch, unsigned long long leaf,
             unsigned long long overflow, unsigned long long entries, unsigned long long root) {
  put_le<uint32_t>(b, pad), put_le<uint16_t>(b, 0), put_le<uint16_t>(b, depth);
  put_le<unsigned long long>(b, branch), put_le<unsigned long long>(b, leaf), put_le<unsigned long long>(b, overflow);
  put_le<unsigned long long>(b, entries), put_le<unsigned long long>(b, root);
}

int write_lmdb_native(const std::string& dir, const std::map<std::string, std::string>& data) {
  std::error_code ec;
  std::filesystem::create_directories(dir, ec);
  const std::string fname = dir + "/data.mdb";
  FILE* f = std::fopen((fname + ".tmp").c_str(), "w+b");
  if (!f) {
    g_err = "cannot create " + fname;
    return 1;
  }
  const size_t nodemax = (size_t)((((kPage - kPageHdr) / 2) & ~1) - 2);
  LmdbPages w{f};
  std::vector<std::pair<std::string, unsigned long long>> level;  // (first key, page) of each page
  std::vector<std::string> cur;
  size_t used = kPageHdr;
  std::string first;
  for (const auto& kv : data) {
    const std::string& k = kv.first;
    const std::string& v = kv.second;
    const uint16_t lo = (uint16_t)(v.size() & 0xFFFF), hi = (uint16_t)(v.size() >> 16);
    std::string nd;
    if (8 + k.size() + v.size() > nodemax) {
      std::string pgb;
      put_le<unsigned long long>(pgb, w.over(v));
      nd = lmdb_node(k, lo, hi, MDB_F_BIGDATA, pgb);
    } else {
      nd = lmdb_node(k, lo, hi, 0, v);
    }
    if (!cur.empty() && used + 2 + nd.size() > (size_t)kPage) {
      level.emplace_back(first, w.page(cur, MDB_P_LEAF));
      cur.clear(), used = kPageHdr;
    }
    if (cur.empty()) first = k;
    cur.push_back(std::move(nd));
    used += 2 + cur.back().size();
  }
  if (!cur.empty()) level.emplace_back(first, w.page(cur, MDB_P_LEAF));
  uint16_t depth = level.empty() ? 0 : 1;
  while (level.size() > 1) {
    std::vector<std::pair<std::string, unsigned long long>> nxt;
    cur.clear(), used = kPageHdr;
    for (const auto& kp : level) {
      const unsigned long long pg = kp.second;
      const uint16_t lo = (uint16_t)(pg & 0xFFFF), hi = (uint16_t)((pg >> 16) & 0xFFFF), fl = (uint16_t)((pg >> 32) & 0xFFFF);
      std::string nd = lmdb_node(cur.empty() ? std::string() : kp.first, lo, hi, fl, std::string());
      if (!cur.empty() && used + 2 + nd.size() > (size_t)kPage) {
        nxt.emplace_back(first, w.page(cur, MDB_P_BRANCH));
        cur.clear(), used = kPageHdr;
        nd = lmdb_node(std::string(), lo, hi, fl, std::string());  // leftmost key of a branch page is implicit
      }
      if (cur.empty()) first = kp.first;
      cur.push_back(std::move(nd));
      used += 2 + cur.back().size();
    }
    nxt.emplace_back(first, w.page(cur, MDB_P_BRANCH));
    level.swap(nxt);
    ++depth;
  }
  const unsigned long long root = level.empty() ? MDB_P_INVALID : level[0].second, last_pg = w.next - 1;
  const unsigned long long mapsize = std::max<unsigned long long>(w.next * kPage, 1ull << 20);
  for (unsigned long long pg = 0; pg < 2; ++pg) {
    std::string m;
    put_le<unsigned long long>(m, pg), put_le<uint16_t>(m, 0), put_le<uint16_t>(m, MDB_P_META);
    put_le<uint16_t>(m, 0), put_le<uint16_t>(m, 0);
    put_le<uint32_t>(m, 0xBEEFC0DEu), put_le<uint32_t>(m, 1), put_le<unsigned long long>(m, 0);
    put_le<unsigned long long>(m, mapsize);
    db_meta(m, (uint32_t)kPage, 0, 0, 0, 0, 0, MDB_P_INVALID);  // free DB (md_pad holds the page size)
    db_meta(m, 0, depth, w.branch, w.leaf, w.overflow, data.size(), root);
    put_le<unsigned long long>(m, last_pg), put_le<unsigned long long>(m, 1);
    m.resize(kPage, '\0');
    w.put(pg, m);
  }
  bool ok = w.ok && std::fflush(f) == 0 && ftruncate(fileno(f), (off_t)(w.next * kPage)) == 0;
  ok = std::fclose(f) == 0 && ok;
  if (!ok || std::rename((fname + ".tmp").c_str(), fname.c_str()) != 0) {
    g_err = "write error on " + fname;
    return 1;
  }
  return 0;
}

bool native_model_path(const char* path) {
  const size_t n = std::strlen(path);
  return !(n >= 3 && std::strcmp(path + n - 3, ".h5") == 0);
}

}  // namespace

extern "C" {

const char* sn_last_error(void) { return g_err.c_str(); }

long long sn_native_iterations(void* s) {
  NativeState* st = find_native(s);
  return st && st->step ? st->step->done : 0;
}

long long sn_python_entries(void) { return g_py_entries.load(std::memory_order_relaxed); }

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
  if (NativeDB* db = find_db(state)) {  // an unclosed native DB: its sndb file handle
    if (db->f) std::fclose(db->f);
    std::lock_guard<std::mutex> lk(g_db_mu);
    g_dbs.erase(state);
  }
  drop_native(state);  // before the Python state (which owns the captured graphs)
  Gil g;
  Py_DECREF(static_cast<PyObject*>(state));
}

int sn_set_device(void* s, int device) {
  Gil g;
  sync_python(s);
  drop_native(s);
  return status(call(s, "set_device", "(i)", device));
}

int sn_load_solver_from_protobuf(void* s, const char* bytes, int len) {
  Gil g;
  sync_python(s);
  drop_native(s);
  return status(call(s, "load_solver", "(y#)", bytes, (Py_ssize_t)len));
}

int sn_load_net_from_protobuf(void* s, const char* bytes, int len) {
  Gil g;
  sync_python(s);
  invalidate(s, P_FWD_TRAIN | P_FWD_TEST | P_WEIGHTS | P_SCORES | P_META);
  return status(call(s, "load_net", "(y#)", bytes, (Py_ssize_t)len));
}

static int set_cb(void* s, int test, int layer, sn_data_callback_t cb, void* user) {
  Gil g;
  sync_python(s);
  // the native executors bind the callbacks they were built with
  invalidate(s, test ? P_FWD_TEST : (P_STEP | P_FWD_TRAIN));
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
  if (!s) {
    g_err = "null state";
    return 1;
  }
  if (NativeForward* nf = native_forward(s, 0)) {
    if (nf->feeds.run(nf->stream)) return 1;
    HIPOK(hipGraphLaunch(nf->exec, nf->stream));
    HIPOK(hipMemcpyAsync(nf->out_host, nf->loss_dev, sizeof(float), hipMemcpyDeviceToHost, nf->stream));
    HIPOK(hipStreamSynchronize(nf->stream));
    if (loss) *loss = nf->out_host[0];
    return 0;
  }
  Gil g;
  PyObject* r = call(s, "forward", nullptr);
  if (!r) return 1;
  if (loss) *loss = (float)PyFloat_AsDouble(r);
  Py_DECREF(r);
  build_forward(s, 0);
  if (NativeForward* nf = native_forward(s, 0)) {
    // forward_plan replayed the captured graph once, so the net's blobs hold THAT forward:
    // report its loss (differs from the eager one only through fresh dropout draws)
    HIPOK(hipMemcpyAsync(nf->out_host, nf->loss_dev, sizeof(float), hipMemcpyDeviceToHost, nf->stream));
    HIPOK(hipStreamSynchronize(nf->stream));
    if (loss) *loss = nf->out_host[0];
  }
  return 0;
}

int sn_backward(void* s) {
  if (!s) {
    g_err = "null state";
    return 1;
  }
  if (NativeBackward* nb = native_backward(s)) {
    HIPOK(hipGraphLaunch(nb->exec, nb->stream));
    HIPOK(hipStreamSynchronize(nb->stream));
    return 0;
  }
  Gil g;
  const int rc = status(call(s, "backward", nullptr));
  if (rc == 0) build_backward(s);
  return rc;
}

int sn_solver_step(void* s, int iters) {
  if (iters <= 0) return 0;
  if (!s) {
    g_err = "null state";
    return 1;
  }
  NativeState& st = native_state(s);
  NativeStep* ns = st.step.get();
  if (!ns) {
    // steps through Python (eager iterations, or the step graph's capture) rebind the train
    // net's blobs: a forward plan's buffers are no longer what the net (sn_backward,
    // sn_blob_get) sees.  Native replays of the step graph write only the step graph's own
    // buffers and update the weights in place, so a forward plan stays valid across them.
    invalidate(s, P_FWD_TRAIN);
    Gil g;
    if (native_enabled() && !st.step_failed && iters > 3) {
      PyObject* ok = call_quiet(s, "native_eligible", nullptr);
      const bool eligible = ok && PyObject_IsTrue(ok) == 1;
      Py_XDECREF(ok);
      PyErr_Clear();
      std::unique_ptr<NativeStep> built;
      const long long ran = eligible ? build_native_step(s, built) : -1;
      if (ran >= 0) {
        ns = built.get();
        st.step = std::move(built);
        iters -= (int)ran;
      } else {
        st.step_failed = true;
        // a capture that failed after its warmup iterations already advanced the solver
        PyObject* nr = PyObject_GetAttrString(static_cast<PyObject*>(s), "native_ran");
        if (nr) iters -= (int)PyLong_AsLong(nr);
        Py_XDECREF(nr);
        PyErr_Clear();
        if (iters <= 0) return 0;
      }
    }
    if (!ns) return status(call(s, "step", "(i)", iters));
  }
  // native loop: no GIL; Python only for display / snapshot iterations
  for (int i = 0; i < iters; ++i) {
    if (native_iteration(*ns)) return 1;
    const long long it = ns->iter;
    const bool disp = ns->display && (it - 1) % ns->display == 0;
    const bool snap = ns->snapshot && it % ns->snapshot == 0;
    if (disp || snap) {
      HIPOK(hipStreamSynchronize(ns->stream));
      float smoothed = -1.f;
      if (disp) {
        const long long n = ns->done < ns->average_loss ? ns->done : ns->average_loss;
        HIPOK(hipMemcpy(ns->loss_host.data(), ns->loss_ring, sizeof(float) * ns->average_loss, hipMemcpyDeviceToHost));
        double acc = 0;
        for (long long k = 0; k < n; ++k) acc += ns->loss_host[(it - 1 - k) % ns->average_loss];
        smoothed = (float)(acc / (double)(n > 0 ? n : 1));
      }
      Gil g;
      if (status(call(s, "native_event", "(Ldi)", it, (double)smoothed, (int)snap))) return 1;
      ns->synced_iter = it;
    }
  }
  HIPOK(hipStreamSynchronize(ns->stream));
  return 0;  // the solver's iteration counter reaches Python at its next entry (sync_python)
}

int sn_solver_test(void* s, int iters) {
  if (!s) {
    g_err = "null state";
    return -1;
  }
  if (NativeForward* nf = native_forward(s, 1)) {
    NativeState& st = native_state(s);
    st.scores.clear();
    if (iters > 0) {
      auto check = [&](hipError_t e, const char* what) {
        if (e == hipSuccess) return true;
        g_err = std::string("native test: ") + what + ": " + hipGetErrorString(e);
        if (g_err_cb) g_err_cb(g_err.c_str());
        return false;
      };
      if (!check(hipMemsetAsync(nf->acc_dev, 0, sizeof(float) * (nf->n_out > 0 ? nf->n_out : 1), nf->stream), "memset"))
        return -1;
      for (int i = 0; i < iters; ++i) {
        if (nf->feeds.run(nf->stream)) return -1;
        if (!check(hipGraphLaunch(nf->exec, nf->stream), "hipGraphLaunch")) return -1;
      }
      if (!check(hipMemcpyAsync(nf->out_host + 1, nf->acc_dev, sizeof(float) * nf->n_out, hipMemcpyDeviceToHost,
                                nf->stream), "hipMemcpyAsync") ||
          !check(hipStreamSynchronize(nf->stream), "hipStreamSynchronize"))
        return -1;
      st.scores.assign(nf->out_host + 1, nf->out_host + 1 + nf->n_out);
    }
    st.scores_native = st.scores_pending = true;
    return (int)st.scores.size();
  }
  Gil g;
  invalidate(s, P_SCORES);
  PyObject* r = call(s, "test", "(i)", iters);
  if (!r) return -1;
  long n = PyLong_AsLong(r);
  Py_DECREF(r);
  if (iters > 0) build_forward(s, 1);
  return (int)n;
}

float sn_get_test_score(void* s, int index) {
  NativeState* st = find_native(s);
  if (st && st->scores_native) return index >= 0 && index < (int)st->scores.size() ? st->scores[index] : 0.f;
  Gil g;
  sync_python(s);
  PyObject* scores = PyObject_GetAttrString(static_cast<PyObject*>(s), "scores");
  float v = 0.f;
  if (scores && index >= 0 && index < PyList_Size(scores)) v = (float)PyFloat_AsDouble(PyList_GetItem(scores, index));
  Py_XDECREF(scores);
  PyErr_Clear();
  return v;
}

long long sn_num_params(void* s) {
  if (NativeWeights* w = native_weights(s)) return w->count;
  Gil g;
  PyObject* r = call(s, "num_params", nullptr);
  if (!r) return -1;
  long long n = PyLong_AsLongLong(r);
  Py_DECREF(r);
  return n;
}

int sn_get_weights(void* s, float* out, long long n) {
  if (NativeWeights* w = native_weights(s)) {
    if (n < 0 || n > w->count || (n > 0 && !out)) {
      g_err = "sn_get_weights: buffer size " + std::to_string(n) + " vs " + std::to_string(w->count) + " parameters";
      return 1;
    }
    if (!w->cuda) {
      std::memcpy(out, w->data, sizeof(float) * n);
      return 0;
    }
    HIPOK(hipMemcpyAsync(out, w->data, sizeof(float) * n, hipMemcpyDeviceToHost, w->stream));
    HIPOK(hipStreamSynchronize(w->stream));
    return 0;
  }
  Gil g;
  return status(call(s, "get_weights", "(KL)", (unsigned long long)(uintptr_t)out, n));
}

int sn_set_weights(void* s, const float* in, long long n) {
  if (NativeWeights* w = native_weights(s)) {
    if (n < 0 || n > w->count || (n > 0 && !in)) {
      g_err = "sn_set_weights: buffer size " + std::to_string(n) + " vs " + std::to_string(w->count) + " parameters";
      return 1;
    }
    if (!w->cuda) {
      std::memcpy(w->data, in, sizeof(float) * n);
      return 0;
    }
    HIPOK(hipMemcpyAsync(w->data, in, sizeof(float) * n, hipMemcpyHostToDevice, w->stream));
    if (w->compute && w->cast(w->data, w->compute, w->compute_count, w->stream)) {
      g_err = "sn_set_weights: sn_cast_f32_bf16 launch failed";
      return 1;
    }
    HIPOK(hipStreamSynchronize(w->stream));  // `in` may be reused as soon as this returns
    return 0;
  }
  Gil g;
  return status(call(s, "set_weights", "(KL)", (unsigned long long)(uintptr_t)in, n));
}

void* sn_weights_device_ptr(void* s) {
  if (NativeWeights* w = native_weights(s)) return w->data;
  Gil g;
  PyObject* r = call(s, "weights_device_ptr", nullptr);
  if (!r) return nullptr;
  void* p = (void*)(uintptr_t)PyLong_AsUnsignedLongLong(r);
  Py_DECREF(r);
  return p;
}

// .caffemodel files are written and read natively once the weights plan exists and covers
// every parameter (HDF5 files, V0 nets and parameters outside the flat buffers: the Python path)
int sn_save_weights_to_file(void* s, const char* path) {
  NativeWeights* w = native_weights(s);
  if (w && w->complete && native_model_path(path)) return save_caffemodel_native(w, path);
  Gil g;
  return status(call(s, "save_weights", "(s)", path));
}

int sn_load_weights_from_file(void* s, const char* path) {
  NativeWeights* w = native_weights(s);
  if (w && w->complete && native_model_path(path)) {
    const int rc = load_caffemodel_native(w, path);
    if (rc != 2) return rc;
  }
  Gil g;
  return status(call(s, "load_weights", "(s)", path));
}

int sn_restore_solver_from_file(void* s, const char* path) {
  Gil g;
  sync_python(s);
  invalidate(s, P_STEP);  // the iteration counter and schedule position change
  return status(call(s, "restore_solver", "(s)", path));
}

int sn_num_layers(void* s) {
  if (NativeMeta* m = native_meta(s)) return (int)m->layers.size();
  Gil g;
  PyObject* r = call(s, "layer_names", nullptr);
  if (!r) return -1;
  int n = (int)PyList_Size(r);
  Py_DECREF(r);
  return n;
}

int copy_name(const std::string& v, char* buf, int buflen) {
  if (!buf || buflen <= 0) return 1;
  std::strncpy(buf, v.c_str(), (size_t)buflen - 1);
  buf[buflen - 1] = 0;
  return 0;
}

int sn_layer_name(void* s, int index, char* buf, int buflen) {
  if (NativeMeta* m = native_meta(s))
    return index >= 0 && index < (int)m->layers.size() ? copy_name(m->layers[(size_t)index], buf, buflen) : 1;
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
  std::string t(db_type ? db_type : "");
  for (auto& ch : t) ch = (char)std::tolower((unsigned char)ch);
  {
    std::lock_guard<std::mutex> lk(g_db_mu);
    g_dbs.erase(s);
  }
  if (native_enabled() && (t == "lmdb" || t == "sndb")) {
    std::error_code ec;
    if (std::filesystem::is_directory(db_name, ec)) std::filesystem::remove_all(db_name, ec);
    auto db = std::make_unique<NativeDB>();
    db->path = db_name;
    db->lmdb = t == "lmdb";
    if (!db->lmdb) {
      db->f = std::fopen(db_name, "wb");
      if (!db->f || std::fwrite("SNDB1\n", 1, 6, db->f) != 6) {
        if (db->f) std::fclose(db->f);
        g_err = std::string("cannot create ") + db_name;
        return 1;
      }
    }
    std::lock_guard<std::mutex> lk(g_db_mu);
    g_dbs[s] = std::move(db);
    return 0;
  }
  Gil g;
  return status(call(s, "create_db", "(ss)", db_name, db_type));
}

int sn_write_to_db(void* s, const char* image, int label, int channels, int height, int width, const char* key) {
  if (NativeDB* db = find_db(s)) {
    const std::string rec = datum_bytes(image, label, channels, height, width);
    if (!db->lmdb) {
      const uint32_t n = (uint32_t)rec.size();
      if (std::fwrite(&n, 4, 1, db->f) != 1 || std::fwrite(rec.data(), 1, rec.size(), db->f) != rec.size()) {
        g_err = "sn_write_to_db: write error on " + db->path;
        return 1;
      }
    } else {
      char auto_key[32];
      std::snprintf(auto_key, sizeof auto_key, "%08lld", db->count);
      std::string k = key && *key ? std::string(key) : std::string(auto_key);
      if (k.empty() || k.size() > (size_t)kMaxKey) {
        g_err = "LMDB keys must be 1..511 bytes";
        return 1;
      }
      db->txn.emplace_back(std::move(k), rec);
    }
    ++db->count;
    return 0;
  }
  Gil g;
  Py_ssize_t n = (Py_ssize_t)channels * height * width;
  return status(call(s, "write_to_db", "(y#iiiis)", image, n, label, channels, height, width, key ? key : ""));
}

int sn_commit_db_txn(void* s) {
  if (NativeDB* db = find_db(s)) {
    if (!db->lmdb) return std::fflush(db->f) == 0 ? 0 : 1;
    for (auto& kv : db->txn) db->all[kv.first] = std::move(kv.second);  // a later put of a key wins
    db->txn.clear();
    return 0;
  }
  Gil g;
  return status(call(s, "commit_db_txn", nullptr));
}

int sn_close_db(void* s) {
  if (NativeDB* db = find_db(s)) {
    int rc = sn_commit_db_txn(s);
    if (!db->lmdb) {
      rc = std::fclose(db->f) == 0 ? rc : 1;
    } else if (rc == 0) {
      rc = write_lmdb_native(db->path, db->all);
    }
    std::lock_guard<std::mutex> lk(g_db_mu);
    g_dbs.erase(s);
    return rc;
  }
  Gil g;
  return status(call(s, "close_db", nullptr));
}

// BlobProto { num = 1, channels, height, width, data (packed) } (ccaffe.cpp:83-97), written natively
int sn_save_mean_image(const float* mean, int channels, int height, int width, const char* filename) {
  std::string o;
  pb_varint(o, 1 << 3), pb_varint(o, 1);
  pb_varint(o, 2 << 3), pb_varint(o, (unsigned long long)(long long)channels);
  pb_varint(o, 3 << 3), pb_varint(o, (unsigned long long)(long long)height);
  pb_varint(o, 4 << 3), pb_varint(o, (unsigned long long)(long long)width);
  const size_t n = (size_t)channels * height * width;
  pb_bytes(o, 5, std::string(reinterpret_cast<const char*>(mean), n * sizeof(float)));
  FILE* f = std::fopen(filename, "wb");
  if (!f) {
    g_err = std::string("cannot open ") + filename + " for writing";
    return 1;
  }
  const bool ok = std::fwrite(o.data(), 1, o.size(), f) == o.size();
  if (std::fclose(f) != 0 || !ok) {
    g_err = std::string("short write to ") + filename;
    return 1;
  }
  return 0;
}

// -- blobs --------------------------------------------------------------------------------------
static long long int_call(void* s, const char* method, const char* fmt, ...) {
  if (!s) {
    g_err = "null state";
    return -1;
  }
  sync_python(s);
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
  if (NativeMeta* m = native_meta(s))
    if (layer >= 0 && layer < (int)m->weights.size()) return m->weights[(size_t)layer];
  Gil g;
  return (int)int_call(s, "num_layer_weights", "(i)", layer);
}

int sn_num_data_blobs(void* s) {
  if (NativeMeta* m = native_meta(s)) return (int)m->blobs.size();
  Gil g;
  return (int)int_call(s, "num_data_blobs", "()");
}

int sn_data_blob_name(void* s, int index, char* buf, int buflen) {
  if (NativeMeta* m = native_meta(s))
    return index >= 0 && index < (int)m->blobs.size() ? copy_name(m->blobs[(size_t)index], buf, buflen) : 1;
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
  if (NativeMeta* m = native_meta(s)) return m->outputs;
  Gil g;
  return (int)int_call(s, "num_output_blobs", "()");
}

int sn_num_test_scores(void* s) {
  NativeState* st = find_native(s);
  if (st && st->scores_native) return (int)st->scores.size();
  Gil g;
  return (int)int_call(s, "num_test_scores", "()");
}

int sn_blob_num_axes(void* s, int layer, int index) {
  NativeWeights* w = nullptr;
  if (const ParamDesc* p = native_param(s, layer, index, &w)) return p->ndim;
  hipStream_t bs;
  if (layer < 0)
    if (const BlobDesc* b = native_blob(s, index, 0, &bs)) return b->ndim;
  Gil g;
  return (int)int_call(s, "blob_num_axes", "(ii)", layer, index);
}

int sn_blob_axis_shape(void* s, int layer, int index, int axis) {
  NativeWeights* w = nullptr;
  if (const ParamDesc* p = native_param(s, layer, index, &w))
    if (axis >= 0 && axis < p->ndim) return p->cs[axis];
  hipStream_t bs;
  if (layer < 0)
    if (const BlobDesc* b = native_blob(s, index, 0, &bs))
      if (axis >= 0 && axis < b->ndim) return b->dims[axis];
  Gil g;
  return (int)int_call(s, "blob_axis_shape", "(iii)", layer, index, axis);
}

int sn_blob_get(void* s, int layer, int index, int diff, float* out, long long n) {
  NativeWeights* w = nullptr;
  if (const ParamDesc* p = native_param(s, layer, index, &w)) return param_get(w, *p, diff, out, n);
  hipStream_t bs;
  if (layer < 0)
    if (const BlobDesc* b = native_blob(s, index, diff, &bs)) return blob_get_native(native_state(s), *b, bs, diff, out, n);
  Gil g;
  return status(call(s, "blob_get", "(iiiKL)", layer, index, diff, (unsigned long long)(uintptr_t)out, n));
}

int sn_blob_set(void* s, int layer, int index, int diff, const float* in, long long n) {
  NativeWeights* w = nullptr;
  if (const ParamDesc* p = native_param(s, layer, index, &w)) return param_set(w, *p, diff, in, n);
  hipStream_t bs;
  if (layer < 0)
    if (const BlobDesc* b = native_blob(s, index, diff, &bs)) return blob_set_native(native_state(s), *b, bs, diff, in, n);
  Gil g;
  return status(call(s, "blob_set", "(iiiKL)", layer, index, diff, (unsigned long long)(uintptr_t)in, n));
}

}  // extern "C"
