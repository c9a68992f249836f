// One API token bucket shared by every process of a replica (the parent's watch hub and
// its shard workers), kept as a single 64-bit word in a shared mapping.
//
// A replica split into K shard-worker processes used to give each worker a fixed
// kube-qps / K: under skew (one worker holding most of a failure wave) that worker was
// capped at qps / K while the others' shares went unused, and the parent's own client
// took another share on top.  Here the replica's kube-qps / kube-burst is one generic
// cell-rate (GCRA) schedule: the word is the "theoretical arrival time" (TAT) of the next
// request in CLOCK_MONOTONIC nanoseconds, which every process of the host reads the same.
//
//   reserve(now):  t = max(TAT, now); TAT' = t + T; the request may go at t - tau
//   (T = 1 / qps, tau = (burst - 1) * T — the tolerance that lets `burst` requests pass at
//   once).  The slot is committed by one compare-and-swap; the caller sleeps the returned
//   delay, so processes are served in reservation order and a process with no demand
//   takes nothing: the split adapts to the load.
//   try_take(now): the same, but only when the slot is due now (no commitment otherwise).
//   give_back():   return an unused reservation (TAT -= T, never below now - tau).
//
// Lock-free 64-bit atomics on x86-64 are address-free, so the same instructions are
// correct between processes mapping one memfd.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <ctime>

namespace {

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// The word: an 8-byte aligned int64 at offset 0 of a writable buffer.
int64_t* word(PyObject* obj, Py_buffer* view) {
  if (PyObject_GetBuffer(obj, view, PyBUF_WRITABLE) < 0) return nullptr;
  if (view->len < 8 || (reinterpret_cast<uintptr_t>(view->buf) & 7u) != 0) {
    PyBuffer_Release(view);
    PyErr_SetString(PyExc_ValueError, "shared bucket needs an 8-byte aligned writable buffer of >= 8 bytes");
    return nullptr;
  }
  return static_cast<int64_t*>(view->buf);
}

bool parse(PyObject* const* args, Py_ssize_t n, const char* name, int64_t* interval, int64_t* tolerance) {
  if (n != 3) {
    PyErr_Format(PyExc_TypeError, "%s(buffer, interval_ns, tolerance_ns)", name);
    return false;
  }
  *interval = PyLong_AsLongLong(args[1]);
  *tolerance = PyLong_AsLongLong(args[2]);
  if (PyErr_Occurred()) return false;
  if (*interval <= 0 || *tolerance < 0) {
    PyErr_SetString(PyExc_ValueError, "interval_ns must be > 0 and tolerance_ns >= 0");
    return false;
  }
  return true;
}

// reserve(buffer, interval_ns, tolerance_ns) -> delay_ns (>= 0): the slot is committed.
PyObject* bucket_reserve(PyObject*, PyObject* const* args, Py_ssize_t n) {
  int64_t T, tau;
  if (!parse(args, n, "reserve", &T, &tau)) return nullptr;
  Py_buffer view;
  int64_t* w = word(args[0], &view);
  if (!w) return nullptr;
  const int64_t now = mono_ns();
  int64_t tat = __atomic_load_n(w, __ATOMIC_ACQUIRE);
  int64_t t;
  do {
    t = tat > now ? tat : now;
  } while (!__atomic_compare_exchange_n(w, &tat, t + T, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE));
  PyBuffer_Release(&view);
  const int64_t at = t - tau;
  return PyLong_FromLongLong(at > now ? at - now : 0);
}

// try_take(buffer, interval_ns, tolerance_ns) -> bool: a slot due now was taken.
PyObject* bucket_try_take(PyObject*, PyObject* const* args, Py_ssize_t n) {
  int64_t T, tau;
  if (!parse(args, n, "try_take", &T, &tau)) return nullptr;
  Py_buffer view;
  int64_t* w = word(args[0], &view);
  if (!w) return nullptr;
  const int64_t now = mono_ns();
  int64_t tat = __atomic_load_n(w, __ATOMIC_ACQUIRE);
  bool took = false;
  for (;;) {
    const int64_t t = tat > now ? tat : now;
    if (t - tau > now) break;  // not due: take nothing
    if (__atomic_compare_exchange_n(w, &tat, t + T, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
      took = true;
      break;
    }
  }
  PyBuffer_Release(&view);
  return PyBool_FromLong(took);
}

// give_back(buffer, interval_ns, tolerance_ns): undo one reservation that was not used.
PyObject* bucket_give_back(PyObject*, PyObject* const* args, Py_ssize_t n) {
  int64_t T, tau;
  if (!parse(args, n, "give_back", &T, &tau)) return nullptr;
  Py_buffer view;
  int64_t* w = word(args[0], &view);
  if (!w) return nullptr;
  const int64_t floor = mono_ns() - tau;
  int64_t tat = __atomic_load_n(w, __ATOMIC_ACQUIRE);
  for (;;) {
    int64_t next = tat - T;
    if (next < floor) next = floor;
    if (next >= tat) break;
    if (__atomic_compare_exchange_n(w, &tat, next, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) break;
  }
  PyBuffer_Release(&view);
  Py_RETURN_NONE;
}

// backlog_ns(buffer) -> how far the schedule runs ahead of now (0 = idle).
PyObject* bucket_backlog(PyObject*, PyObject* obj) {
  Py_buffer view;
  int64_t* w = word(obj, &view);
  if (!w) return nullptr;
  const int64_t tat = __atomic_load_n(w, __ATOMIC_ACQUIRE);
  PyBuffer_Release(&view);
  const int64_t now = mono_ns();
  return PyLong_FromLongLong(tat > now ? tat - now : 0);
}

PyObject* bucket_now(PyObject*, PyObject*) { return PyLong_FromLongLong(mono_ns()); }

}  // namespace

extern "C" int nexus_register_shared_bucket(PyObject* m) {
  static PyMethodDef methods[] = {
      {"bucket_reserve", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(bucket_reserve)),
       METH_FASTCALL, "bucket_reserve(buffer, interval_ns, tolerance_ns) -> delay_ns (slot committed)"},
      {"bucket_try_take", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(bucket_try_take)),
       METH_FASTCALL, "bucket_try_take(buffer, interval_ns, tolerance_ns) -> bool"},
      {"bucket_give_back", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(bucket_give_back)),
       METH_FASTCALL, "bucket_give_back(buffer, interval_ns, tolerance_ns)"},
      {"bucket_backlog", bucket_backlog, METH_O, "bucket_backlog(buffer) -> ns the schedule runs ahead of now"},
      {"bucket_now", bucket_now, METH_NOARGS, "bucket_now() -> CLOCK_MONOTONIC ns"},
      {nullptr, nullptr, 0, nullptr}};
  for (PyMethodDef* d = methods; d->ml_name; ++d) {
    PyObject* f = PyCFunction_New(d, nullptr);
    if (!f || PyModule_AddObject(m, d->ml_name, f) < 0) {
      Py_XDECREF(f);
      return -1;
    }
  }
  return 0;
}
