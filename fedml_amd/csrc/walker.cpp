// walker.cpp — host-side native helper of the device-resident FedAvg path.
//
// FedML's GPU server hands the aggregator K state dicts whose tensors were
// moved to the device one by one (ml_engine_adapter.py:234-254), so a ResNet-50
// round at K = 128 is 40,960 separate device tensors.  Reading their dtype,
// shape, device, contiguity and data pointer through Python costs ~0.4 us per
// attribute per tensor (~20 ms per round, ten times the reduction itself).
// This module walks the dicts in C++ and returns, per dtype, the flat [T][K]
// table of client pointers that fedagg_wsum_multi consumes, and optionally
// allocates the T output tensors (at::empty, the caching allocator) so the
// caller launches without touching any tensor from Python.
//
// It only ever takes the fast path: any irregularity (a missing key, a host or
// non-contiguous tensor, mismatched shapes/dtypes/devices, a dtype the
// multi-tensor kernel does not take, a pointer that is not 16-byte aligned, a
// dict type that overrides lookup) returns None, and the caller falls back to
// the Python walk, which raises the reference's exceptions
// (agg_operator.py:36-44: KeyError for a missing key, torch's errors for
// shape/dtype mismatches).  No arithmetic happens here.

#include <Python.h>

#include <ATen/ATen.h>
#include <torch/csrc/autograd/python_variable.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// FEDAGG_DT_* codes of include/fedagg.h for the dtypes fedagg_wsum_multi takes
int multi_code(c10::ScalarType s) {
  switch (s) {
    case c10::ScalarType::Float: return 0;
    case c10::ScalarType::BFloat16: return 1;
    case c10::ScalarType::Half: return 2;
    case c10::ScalarType::Long: return 4;
    default: return -1;
  }
}

// A small persistent pool for the validation pass (spawning threads per call
// would cost more than the pass).  Workers never touch Python objects: they
// only read at::Tensor metadata, while the calling thread holds the GIL, so
// no Python code can mutate the dicts meanwhile.  Re-created after a fork.
class Pool {
 public:
  static Pool& get() {
    static Pool* p = nullptr;
    static pid_t owner = 0;
    if (!p || owner != getpid()) {  // a forked child inherits no workers: leak the old object, start anew
      p = new Pool(std::max(1u, std::min(8u, std::thread::hardware_concurrency())) - 1);
      owner = getpid();
    }
    return *p;
  }
  // fn(lo, hi) over [0, n) in `parts` contiguous ranges; the caller works too
  void run(int64_t n, int parts, const std::function<void(int64_t, int64_t)>& fn) {
    parts = std::max(1, std::min<int>(parts, int(workers_.size()) + 1));
    if (parts == 1 || n < 2) {
      fn(0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &fn;
      n_ = n;
      parts_ = parts;
      next_.store(0);
      pending_ = parts;
      ++gen_;
    }
    cv_.notify_all();
    const int done = work(fn, n, parts);
    std::unique_lock<std::mutex> lk(mu_);
    pending_ -= done;
    // every part finished AND every worker out of its part loop, so none can
    // take a part index of the next job with this job's function
    done_cv_.wait(lk, [&] { return pending_ == 0 && active_ == 0; });
    job_ = nullptr;
  }

 private:
  explicit Pool(unsigned nworkers) {
    for (unsigned w = 0; w < nworkers; ++w) workers_.emplace_back([this] { loop(); });
    for (auto& t : workers_) t.detach();
  }
  int work(const std::function<void(int64_t, int64_t)>& fn, int64_t n, int parts) {
    int done = 0;
    const int64_t per = (n + parts - 1) / parts;
    for (int part = next_.fetch_add(1); part < parts; part = next_.fetch_add(1), ++done) {
      const int64_t lo = part * per;
      if (lo < n) fn(lo, std::min(n, lo + per));
    }
    return done;
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (!job_) continue;  // woke after that job was already finished
      const std::function<void(int64_t, int64_t)>* fn = job_;
      const int64_t n = n_;
      const int parts = parts_;
      ++active_;
      lk.unlock();
      const int done = work(*fn, n, parts);
      lk.lock();
      pending_ -= done;
      --active_;
      if (pending_ == 0 && active_ == 0) done_cv_.notify_one();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t, int64_t)>* job_ = nullptr;
  int64_t n_ = 0;
  int parts_ = 0, pending_ = 0, active_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
};

// FEDAGG_DT_* codes of the row dtypes a ClientBucket stores without
// conversion (the host walk feeds a byte-for-byte pack)
int row_code(c10::ScalarType s) {
  switch (s) {
    case c10::ScalarType::Float: return 0;
    case c10::ScalarType::BFloat16: return 1;
    case c10::ScalarType::Half: return 2;
    case c10::ScalarType::Double: return 3;
    case c10::ScalarType::Long: return 4;
    default: return -1;
  }
}

// dict and OrderedDict share dict's lookup; anything overriding __getitem__
// goes through the Python walk so that its own semantics apply.
bool plain_lookup(PyObject* d) {
  if (!PyDict_Check(d)) return false;
  return Py_TYPE(d)->tp_as_mapping && Py_TYPE(d)->tp_as_mapping->mp_subscript == PyDict_Type.tp_as_mapping->mp_subscript;
}

// walk(dicts: list, keys: list, alloc: bool = False)
//     -> None | (device_index, codes, numels, tables[, outs, out_tables])
//   codes[t]   : FEDAGG_DT_* of key t
//   numels[t]  : elements of key t
//   tables     : {code: bytes}, the int64 pointer table [T_code][K] of the keys
//                of that dtype in key order, clients in list order
//   outs[t]    : (alloc) a new contiguous tensor shaped like client 0's key t,
//                float32 for int64 keys (the reference's int64 * float
//                promotion), the dtype otherwise, on the inputs' device
//   out_tables : (alloc) {code: bytes}, the output pointers [T_code]
PyObject* walk_impl(PyObject* dicts, PyObject* keys, bool alloc, bool host);

PyObject* walk(PyObject*, PyObject* args) {
  PyObject* dicts;
  PyObject* keys;
  int alloc = 0;
  if (!PyArg_ParseTuple(args, "O!O!|p", &PyList_Type, &dicts, &PyList_Type, &keys, &alloc)) return nullptr;
  try {
    return walk_impl(dicts, keys, alloc != 0, false);
  } catch (const std::exception&) {  // a tensor torch itself would refuse here: let the Python walk report it
    PyErr_Clear();
    Py_RETURN_NONE;
  }
}

// walk_host(dicts: list, keys: list) -> None | (codes, numels, tables)
//   as walk() for host (CPU) tensors of the bucket's row dtypes (fp32, bf16,
//   f16, f64, int64): the pointer tables feed one fedagg_host_pack per dtype
//   that stages every client of a small round at once.  No alignment needed.
PyObject* walk_host(PyObject*, PyObject* args) {
  PyObject* dicts;
  PyObject* keys;
  if (!PyArg_ParseTuple(args, "O!O!", &PyList_Type, &dicts, &PyList_Type, &keys)) return nullptr;
  try {
    return walk_impl(dicts, keys, false, true);
  } catch (const std::exception&) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
}

// order_by_size(d: dict, keys: list) -> None | list of key indices, largest
// tensor first (stable).  The pipelined reduction walks and launches the big
// keys first, so the GPU starts on most of the bytes while the host is still
// walking the many small ones.
PyObject* order_by_size(PyObject*, PyObject* args) {
  PyObject* d;
  PyObject* keys;
  if (!PyArg_ParseTuple(args, "OO!", &d, &PyList_Type, &keys)) return nullptr;
  if (!plain_lookup(d)) Py_RETURN_NONE;
  const Py_ssize_t T = PyList_GET_SIZE(keys);
  std::vector<std::pair<int64_t, Py_ssize_t>> sz(T);
  for (Py_ssize_t t = 0; t < T; ++t) {
    PyObject* v = PyDict_GetItemWithError(d, PyList_GET_ITEM(keys, t));
    if (!v) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_NONE;
    }
    if (!THPVariable_Check(v)) Py_RETURN_NONE;
    sz[t] = {-THPVariable_Unpack(v).numel(), t};
  }
  std::stable_sort(sz.begin(), sz.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  PyObject* out = PyList_New(T);
  if (!out) return nullptr;
  for (Py_ssize_t t = 0; t < T; ++t) PyList_SET_ITEM(out, t, PyLong_FromSsize_t(sz[t].second));
  return out;
}

// {code: bytes of the int64 table} for every non-empty code; -1 on error
int add_tables(PyObject* dict, const std::vector<int64_t> (&tab)[5]) {
  for (int c = 0; c < 5; ++c) {
    if (tab[c].empty()) continue;
    PyObject* k = PyLong_FromLong(c);
    PyObject* b = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(tab[c].data()),
                                            Py_ssize_t(tab[c].size() * sizeof(int64_t)));
    const int rc = (k && b) ? PyDict_SetItem(dict, k, b) : -1;
    Py_XDECREF(k);
    Py_XDECREF(b);
    if (rc) return -1;
  }
  return 0;
}

PyObject* walk_impl(PyObject* dicts, PyObject* keys, bool alloc, bool host) {
  const Py_ssize_t K = PyList_GET_SIZE(dicts), T = PyList_GET_SIZE(keys);
  if (K < 1) Py_RETURN_NONE;
  for (Py_ssize_t i = 0; i < K; ++i)
    if (!plain_lookup(PyList_GET_ITEM(dicts, i))) Py_RETURN_NONE;

  // Lookups, client-major so each client's hash table stays hot while its T
  // keys are found (twice as fast as key-major at K = 128, T = 320).  Only
  // exact torch.Tensor objects go on: a subclass may route its metadata
  // through Python, which the validation threads below must not call.
  std::vector<const at::Tensor*> ts(size_t(T) * K);
  for (Py_ssize_t i = 0; i < K; ++i) {
    PyObject* d = PyList_GET_ITEM(dicts, i);
    for (Py_ssize_t t = 0; t < T; ++t) {
      PyObject* v = PyDict_GetItemWithError(d, PyList_GET_ITEM(keys, t));  // borrowed
      if (!v) {
        if (PyErr_Occurred()) return nullptr;  // e.g. an unhashable key
        Py_RETURN_NONE;
      }
      if (Py_TYPE(v) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) Py_RETURN_NONE;
      ts[size_t(t) * K + i] = &THPVariable_Unpack(v);
    }
  }

  // Validation and pointer tables, key by key, on the pool for big walks.
  std::vector<int> codes(T), devs(T);
  std::vector<int64_t> numels(T), ptrs(size_t(T) * K);
  std::vector<uint8_t> ok(T, 0);
  auto check = [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) {
      const at::Tensor* const* row = ts.data() + size_t(t) * K;
      const at::Tensor& x0 = *row[0];
      const c10::DeviceType want = host ? c10::DeviceType::CPU : c10::DeviceType::CUDA;
      if (!x0.defined() || x0.layout() != c10::kStrided || x0.device().type() != want) continue;
      const int code = host ? row_code(x0.scalar_type()) : multi_code(x0.scalar_type());
      if (code < 0) continue;
      const int dev = host ? -1 : x0.get_device();
      bool good = true;
      for (Py_ssize_t i = 0; i < K && good; ++i) {
        const at::Tensor& x = *row[i];
        good = x.defined() && x.layout() == c10::kStrided && x.device().type() == want && x.is_contiguous() &&
               x.scalar_type() == x0.scalar_type() && (host || x.get_device() == dev) && x.sizes() == x0.sizes();
        if (good) {
          const auto p = reinterpret_cast<intptr_t>(x.data_ptr());
          good = host || (p & 15) == 0;
          ptrs[size_t(t) * K + i] = static_cast<int64_t>(p);
        }
      }
      codes[t] = code;
      devs[t] = dev;
      numels[t] = x0.numel();
      ok[t] = good;
    }
  };
  if (int64_t(T) * K >= 4096)
    Pool::get().run(T, 8, check);
  else
    check(0, T);

  std::vector<int64_t> tab[5];
  const int device = T ? devs[0] : -1;  // -1 for a host walk
  for (Py_ssize_t t = 0; t < T; ++t) {
    if (!ok[t] || devs[t] != device) Py_RETURN_NONE;
    tab[codes[t]].insert(tab[codes[t]].end(), ptrs.begin() + size_t(t) * K, ptrs.begin() + size_t(t + 1) * K);
  }

  // outputs only once every key has passed, so a declined walk allocates nothing
  std::vector<at::Tensor> outs;
  std::vector<int64_t> otab[5];
  if (alloc) {
    outs.reserve(T);
    for (Py_ssize_t t = 0; t < T; ++t) {
      const at::Tensor& x0 = THPVariable_Unpack(PyDict_GetItem(PyList_GET_ITEM(dicts, 0), PyList_GET_ITEM(keys, t)));
      outs.push_back(at::empty(x0.sizes(), x0.options().dtype(codes[t] == 4 ? at::kFloat : x0.scalar_type())));
      const auto p = reinterpret_cast<intptr_t>(outs.back().data_ptr());
      if (p & 15) Py_RETURN_NONE;  // the caching allocator never does this
      otab[codes[t]].push_back(static_cast<int64_t>(p));
    }
  }

  PyObject* py_codes = PyList_New(T);
  PyObject* py_numels = PyList_New(T);
  PyObject* tables = PyDict_New();
  PyObject* py_outs = nullptr;
  PyObject* out_tables = nullptr;
  if (!py_codes || !py_numels || !tables) goto fail;
  for (Py_ssize_t t = 0; t < T; ++t) {
    PyList_SET_ITEM(py_codes, t, PyLong_FromLong(codes[t]));
    PyList_SET_ITEM(py_numels, t, PyLong_FromLongLong(numels[t]));
  }
  if (add_tables(tables, tab)) goto fail;
  if (alloc) {
    py_outs = PyList_New(T);
    out_tables = PyDict_New();
    if (!py_outs || !out_tables || add_tables(out_tables, otab)) goto fail;
    for (Py_ssize_t t = 0; t < T; ++t) {
      PyObject* o = THPVariable_Wrap(std::move(outs[t]));
      if (!o) goto fail;
      PyList_SET_ITEM(py_outs, t, o);
    }
    return Py_BuildValue("(iNNNNN)", device, py_codes, py_numels, tables, py_outs, out_tables);
  }
  if (host) return Py_BuildValue("(NNN)", py_codes, py_numels, tables);
  return Py_BuildValue("(iNNN)", device, py_codes, py_numels, tables);
fail:
  Py_XDECREF(py_codes);
  Py_XDECREF(py_numels);
  Py_XDECREF(tables);
  Py_XDECREF(py_outs);
  Py_XDECREF(out_tables);
  return nullptr;
}

// host_round(dicts: list, keys: list, weights: list of float, fn: int, stream: int,
//            max_bytes: int) -> None | (rc, outs)
//   One small host round through libfedagg's fedagg_host_round_f32 (fn is
//   its address): every key of every client a contiguous CPU tensor of fp32
//   or int64, same shapes across clients, K <= 256.  outs[t] is a new fp32
//   host tensor shaped like client 0's key t (the reference's result dtype
//   for both), filled when rc == 0.  None for anything else, or for rounds
//   of more than max_bytes of client elements (as fp32) (the caller's
//   general path then runs and raises the reference's errors).  The GIL is
//   released while the round runs.
using HostRoundFn = int (*)(const void* const*, const int32_t*, const int64_t*, int32_t, int32_t, const float*,
                            void* const*, void*);

PyObject* host_round(PyObject*, PyObject* args) {
  PyObject* dicts;
  PyObject* keys;
  PyObject* weights;
  unsigned long long fn_addr = 0, stream = 0;
  long long max_bytes = 0;
  if (!PyArg_ParseTuple(args, "O!O!O!KKL", &PyList_Type, &dicts, &PyList_Type, &keys, &PyList_Type, &weights,
                        &fn_addr, &stream, &max_bytes))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(dicts), T = PyList_GET_SIZE(keys);
  if (K < 1 || K > 256 || PyList_GET_SIZE(weights) != K || !fn_addr) Py_RETURN_NONE;
  try {
    for (Py_ssize_t i = 0; i < K; ++i)
      if (!plain_lookup(PyList_GET_ITEM(dicts, i))) Py_RETURN_NONE;
    std::vector<float> w(static_cast<size_t>(K));
    for (Py_ssize_t i = 0; i < K; ++i) {
      const double v = PyFloat_AsDouble(PyList_GET_ITEM(weights, i));  // a Python float: n_i / sum n
      if (v == -1.0 && PyErr_Occurred()) {
        PyErr_Clear();
        Py_RETURN_NONE;
      }
      w[size_t(i)] = static_cast<float>(v);  // RNE, as torch rounds the scalar of p * w
    }
    std::vector<const void*> src(size_t(T) * K);
    // every source tensor, held (a handle copy holds its storage) until the
    // native call returns: the GIL is released around it, and another thread
    // (e.g. a transport's receive thread) may rebind or drop a dict entry
    std::vector<at::Tensor> keep;
    keep.reserve(size_t(T) * K);
    std::vector<int32_t> codes(T);
    std::vector<int64_t> numels(T);
    std::vector<at::Tensor> outs;
    std::vector<void*> optr(T);
    outs.reserve(T);
    int64_t total = 0;
    for (Py_ssize_t t = 0; t < T; ++t) {
      const at::Tensor* x0 = nullptr;
      for (Py_ssize_t i = 0; i < K; ++i) {
        PyObject* v = PyDict_GetItemWithError(PyList_GET_ITEM(dicts, i), PyList_GET_ITEM(keys, t));
        if (!v) {
          if (PyErr_Occurred()) return nullptr;
          Py_RETURN_NONE;
        }
        if (Py_TYPE(v) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) Py_RETURN_NONE;
        const at::Tensor& x = THPVariable_Unpack(v);
        if (!x.defined() || x.layout() != c10::kStrided || x.device().type() != c10::DeviceType::CPU ||
            !x.is_contiguous())
          Py_RETURN_NONE;
        if (i == 0) {
          x0 = &x;
          const auto st = x.scalar_type();
          if (st != c10::ScalarType::Float && st != c10::ScalarType::Long) Py_RETURN_NONE;
          codes[t] = st == c10::ScalarType::Float ? 0 : 4;
          numels[t] = x.numel();
        } else if (x.scalar_type() != x0->scalar_type() || x.sizes() != x0->sizes()) {
          Py_RETURN_NONE;
        }
        src[size_t(t) * K + i] = x.data_ptr();
        keep.push_back(x);
      }
      total += numels[t];
      if (total * 4 * K > max_bytes) Py_RETURN_NONE;  // a big round: the staging-ring path
    }
    for (Py_ssize_t t = 0; t < T; ++t) {  // outputs only once every key has passed
      const at::Tensor& x0 = THPVariable_Unpack(PyDict_GetItem(PyList_GET_ITEM(dicts, 0), PyList_GET_ITEM(keys, t)));
      outs.push_back(at::empty(x0.sizes(), x0.options().dtype(at::kFloat)));
      optr[t] = outs.back().data_ptr();
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = reinterpret_cast<HostRoundFn>(fn_addr)(src.data(), codes.data(), numels.data(), int32_t(T), int32_t(K),
                                                 w.data(), optr.data(), reinterpret_cast<void*>(stream));
    Py_END_ALLOW_THREADS
    PyObject* py_outs = PyList_New(T);
    if (!py_outs) return nullptr;
    for (Py_ssize_t t = 0; t < T; ++t) {
      PyObject* o = THPVariable_Wrap(std::move(outs[t]));
      if (!o) {
        Py_DECREF(py_outs);
        return nullptr;
      }
      PyList_SET_ITEM(py_outs, t, o);
    }
    return Py_BuildValue("(iN)", rc, py_outs);
  } catch (const std::exception&) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
}

// device_round(dicts: list, keys: list, weights: list of float, fn: int,
//              stream_of: callable) -> None | (rc, outs)
//   One small round of device tensors through libfedagg's
//   fedagg_device_round_f32 (fn is its address): every key of every client a
//   contiguous, 16-byte aligned tensor of fp32 or int64 on ONE CUDA device,
//   same shapes across clients, at most 16 keys and 128 client tensors.
//   outs[t] is a new fp32 tensor on that device shaped like client 0's key t
//   (the caching allocator, on the device's current stream), written by the
//   launch on stream_of(device_index) (torch's current raw stream there).
//   None for anything else (the caller's general path then runs and raises
//   the reference's errors).  Asynchronous, like every device path.
using DeviceRoundFn = HostRoundFn;
constexpr Py_ssize_t kDevRoundMaxKeys = 16, kDevRoundMaxPtrs = 128;

PyObject* device_round(PyObject*, PyObject* args) {
  PyObject* dicts;
  PyObject* keys;
  PyObject* weights;
  PyObject* stream_of;
  unsigned long long fn_addr = 0;
  if (!PyArg_ParseTuple(args, "O!O!O!KO", &PyList_Type, &dicts, &PyList_Type, &keys, &PyList_Type, &weights,
                        &fn_addr, &stream_of))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(dicts), T = PyList_GET_SIZE(keys);
  if (K < 1 || T < 1 || T > kDevRoundMaxKeys || T * K > kDevRoundMaxPtrs || PyList_GET_SIZE(weights) != K ||
      !fn_addr)
    Py_RETURN_NONE;
  try {
    for (Py_ssize_t i = 0; i < K; ++i)
      if (!plain_lookup(PyList_GET_ITEM(dicts, i))) Py_RETURN_NONE;
    float w[kDevRoundMaxPtrs];
    for (Py_ssize_t i = 0; i < K; ++i) {
      const double v = PyFloat_AsDouble(PyList_GET_ITEM(weights, i));  // a Python float: n_i / sum n
      if (v == -1.0 && PyErr_Occurred()) {
        PyErr_Clear();
        Py_RETURN_NONE;
      }
      w[i] = static_cast<float>(v);  // RNE, as torch rounds the scalar of p * w
    }
    const void* src[kDevRoundMaxPtrs];
    int32_t codes[kDevRoundMaxKeys];
    int64_t numels[kDevRoundMaxKeys];
    const at::Tensor* first[kDevRoundMaxKeys];
    int dev = -1;
    for (Py_ssize_t t = 0; t < T; ++t) {
      const at::Tensor* x0 = nullptr;
      for (Py_ssize_t i = 0; i < K; ++i) {
        PyObject* v = PyDict_GetItemWithError(PyList_GET_ITEM(dicts, i), PyList_GET_ITEM(keys, t));
        if (!v) {
          if (PyErr_Occurred()) return nullptr;
          Py_RETURN_NONE;
        }
        if (Py_TYPE(v) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) Py_RETURN_NONE;
        const at::Tensor& x = THPVariable_Unpack(v);
        if (!x.defined() || x.layout() != c10::kStrided || x.device().type() != c10::DeviceType::CUDA ||
            !x.is_contiguous())
          Py_RETURN_NONE;
        if (i == 0) {
          x0 = &x;
          const auto st = x.scalar_type();
          if (st != c10::ScalarType::Float && st != c10::ScalarType::Long) Py_RETURN_NONE;
          if (t == 0) dev = x.get_device();
          if (x.get_device() != dev) Py_RETURN_NONE;
          codes[t] = st == c10::ScalarType::Float ? 0 : 4;
          numels[t] = x.numel();
          first[t] = x0;
        } else if (x.scalar_type() != x0->scalar_type() || x.sizes() != x0->sizes() || x.get_device() != dev) {
          Py_RETURN_NONE;
        }
        const void* p = x.data_ptr();
        if (numels[t] && (reinterpret_cast<uintptr_t>(p) & 15)) Py_RETURN_NONE;
        src[t * K + i] = p;
      }
    }
    PyObject* sobj = PyObject_CallFunction(stream_of, "i", dev);
    if (!sobj) return nullptr;
    const unsigned long long stream = PyLong_AsUnsignedLongLong(sobj);
    Py_DECREF(sobj);
    if (stream == static_cast<unsigned long long>(-1) && PyErr_Occurred()) return nullptr;
    std::vector<at::Tensor> outs;  // only once every key has passed
    outs.reserve(size_t(T));
    void* optr[kDevRoundMaxKeys];
    for (Py_ssize_t t = 0; t < T; ++t) {
      outs.push_back(at::empty(first[t]->sizes(), first[t]->options().dtype(at::kFloat)));
      optr[t] = outs.back().data_ptr();
      if (reinterpret_cast<uintptr_t>(optr[t]) & 15) Py_RETURN_NONE;  // the caching allocator never does this
    }
    const int rc = reinterpret_cast<DeviceRoundFn>(fn_addr)(src, codes, numels, int32_t(T), int32_t(K), w, optr,
                                                            reinterpret_cast<void*>(stream));
    PyObject* py_outs = PyList_New(T);
    if (!py_outs) return nullptr;
    for (Py_ssize_t t = 0; t < T; ++t) {
      PyObject* o = THPVariable_Wrap(std::move(outs[t]));
      if (!o) {
        Py_DECREF(py_outs);
        return nullptr;
      }
      PyList_SET_ITEM(py_outs, t, o);
    }
    return Py_BuildValue("(iN)", rc, py_outs);
  } catch (const std::exception&) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
}

// group_by_device(d: dict, keys: list) -> None | [(device, [key indices])]
//   The keys of one state dict grouped by the CUDA device their tensor lives
//   on (devices in order of first appearance), each group largest tensor
//   first (stable).  A multi-device bucket (fedml_amd.multidev) leaves a
//   round's keys spread over several GPUs; the pipelined device reduction
//   walks and launches each device's keys as their own chunks.  None if a
//   value is not a plain tensor on a CUDA device (the caller's general path
//   handles it).
PyObject* group_by_device(PyObject*, PyObject* args) {
  PyObject* d;
  PyObject* keys;
  if (!PyArg_ParseTuple(args, "OO!", &d, &PyList_Type, &keys)) return nullptr;
  if (!plain_lookup(d)) Py_RETURN_NONE;
  const Py_ssize_t T = PyList_GET_SIZE(keys);
  std::vector<int> dev_order;
  std::vector<std::vector<std::pair<int64_t, Py_ssize_t>>> groups;
  for (Py_ssize_t t = 0; t < T; ++t) {
    PyObject* v = PyDict_GetItemWithError(d, PyList_GET_ITEM(keys, t));
    if (!v) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_NONE;
    }
    if (Py_TYPE(v) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) Py_RETURN_NONE;
    const at::Tensor& x = THPVariable_Unpack(v);
    if (!x.defined() || x.device().type() != c10::DeviceType::CUDA) Py_RETURN_NONE;
    const int dev = x.get_device();
    size_t g = 0;
    while (g < dev_order.size() && dev_order[g] != dev) ++g;
    if (g == dev_order.size()) {
      dev_order.push_back(dev);
      groups.emplace_back();
    }
    groups[g].push_back({-x.numel(), t});
  }
  PyObject* out = PyList_New(Py_ssize_t(groups.size()));
  if (!out) return nullptr;
  for (size_t g = 0; g < groups.size(); ++g) {
    auto& sz = groups[g];
    std::stable_sort(sz.begin(), sz.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    PyObject* idx = PyList_New(Py_ssize_t(sz.size()));
    if (!idx) {
      Py_DECREF(out);
      return nullptr;
    }
    for (size_t j = 0; j < sz.size(); ++j) {
      PyObject* v = PyLong_FromSsize_t(sz[j].second);
      if (!v) {
        Py_DECREF(idx);
        Py_DECREF(out);
        return nullptr;
      }
      PyList_SET_ITEM(idx, Py_ssize_t(j), v);
    }
    // (device, indices): built by hand so a failed allocation drops both
    // references and raises, instead of leaving a NULL item in the list
    PyObject* d = PyLong_FromLong(dev_order[g]);
    PyObject* pair = d ? PyTuple_New(2) : nullptr;
    if (!pair) {
      Py_XDECREF(d);
      Py_DECREF(idx);
      Py_DECREF(out);
      return nullptr;
    }
    PyTuple_SET_ITEM(pair, 0, d);
    PyTuple_SET_ITEM(pair, 1, idx);
    PyList_SET_ITEM(out, Py_ssize_t(g), pair);
  }
  return out;
}

// same_values(dicts: list, views: list, keys: list) -> bool
// True when every dicts[i] is a plain-lookup dict whose value under every key
// IS views[i]'s value (object identity): the round's dicts are still the
// bucket views the cross-silo ingest bound them to, so the reduction can run
// over the bucket's rows (agg_operator._reduce_resident).  No allocation; a
// missing key is simply False.
PyObject* same_values(PyObject*, PyObject* args) {
  PyObject *dicts, *views, *keys;
  if (!PyArg_ParseTuple(args, "O!O!O!", &PyList_Type, &dicts, &PyList_Type, &views, &PyList_Type, &keys))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(dicts), T = PyList_GET_SIZE(keys);
  if (PyList_GET_SIZE(views) != K) Py_RETURN_FALSE;
  for (Py_ssize_t i = 0; i < K; ++i) {
    PyObject* d = PyList_GET_ITEM(dicts, i);
    PyObject* v = PyList_GET_ITEM(views, i);
    if (!plain_lookup(d) || !PyDict_Check(v)) Py_RETURN_FALSE;
    for (Py_ssize_t t = 0; t < T; ++t) {
      PyObject* k = PyList_GET_ITEM(keys, t);
      PyObject* a = PyDict_GetItemWithError(d, k);
      if (!a) {
        if (PyErr_Occurred()) return nullptr;
        Py_RETURN_FALSE;
      }
      PyObject* b = PyDict_GetItemWithError(v, k);
      if (!b) {
        if (PyErr_Occurred()) return nullptr;
        Py_RETURN_FALSE;
      }
      if (a != b) Py_RETURN_FALSE;
    }
  }
  Py_RETURN_TRUE;
}

PyMethodDef kMethods[] = {
    {"group_by_device", group_by_device, METH_VARARGS,
     "Key indices of a state dict grouped by CUDA device, largest first, or None."},
    {"host_round", host_round, METH_VARARGS, "One small host round through fedagg_host_round_f32, or None."},
    {"device_round", device_round, METH_VARARGS, "One small device round through fedagg_device_round_f32, or None."},
    {"walk", walk, METH_VARARGS, "Pointer tables of K device state dicts for fedagg_wsum_multi, or None."},
    {"order_by_size", order_by_size, METH_VARARGS, "Key indices of a state dict, largest tensor first, or None."},
    {"walk_host", walk_host, METH_VARARGS, "Host pointer tables of K CPU state dicts for one batched pack, or None."},
    {"same_values", same_values, METH_VARARGS, "Every dict's values are the given views' objects (identity)."},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fedagg_walker", nullptr, -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fedagg_walker(void) { return PyModule_Create(&kModule); }
