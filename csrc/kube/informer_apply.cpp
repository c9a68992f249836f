// Native informer apply: one watch batch into the informer's cache (``informer.store.Indexer``)
// and out to the event handlers, in one C loop.
//
// client-go's reflector hands every watch event to its DeltaFIFO / indexer in Go
// (/root/reference/services/supervisor.go:73-75 builds the informers).  Here the decoded
// batch (``ProjectedDecoder.feed_events``: a list of ``(type, object)``) was applied by a
// Python loop (``SharedInformer._apply_lines``): per line a key string, a dict get/set, the
// job-name label index upkeep and the handler dispatch — about an eighth of a shard
// worker's CPU under the benchmark's churn (profiles/r4_prof2).  ``apply_lines`` does the
// same work, in the same order, with the same results:
//
//   apply_lines(batch, start, end, items, labels, indices, adds, updates, deletes, on_error)
//     -> (error_object_or_None, lines_seen, last_resource_version_or_None)
//
//   items    the Indexer's {key: object} dict (key "ns/name", or "name" without a namespace)
//   labels   [(index_name, label_key)] — the single-label indices (Indexer._labels) or None
//   indices  {index_name: {label_value: set(keys)}}
//   adds / updates / deletes   handler callables (lists); on_error(kind, exc) logs a
//            handler's exception (a handler bug must not kill the informer)
//
// An ERROR event stops the batch and is returned (the lines before it are applied);
// BOOKMARKs only advance the resourceVersion.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

namespace {

PyObject* K_METADATA;
PyObject* K_NAMESPACE;
PyObject* K_NAME;
PyObject* K_RV;
PyObject* K_LABELS;
PyObject* T_ERROR;
PyObject* T_BOOKMARK;
PyObject* T_DELETED;
PyObject* S_EMPTY;

bool init_strings() {
  if (K_METADATA) return true;
  K_METADATA = PyUnicode_InternFromString("metadata");
  K_NAMESPACE = PyUnicode_InternFromString("namespace");
  K_NAME = PyUnicode_InternFromString("name");
  K_RV = PyUnicode_InternFromString("resourceVersion");
  K_LABELS = PyUnicode_InternFromString("labels");
  T_ERROR = PyUnicode_InternFromString("ERROR");
  T_BOOKMARK = PyUnicode_InternFromString("BOOKMARK");
  T_DELETED = PyUnicode_InternFromString("DELETED");
  S_EMPTY = PyUnicode_InternFromString("");
  return K_METADATA && K_NAMESPACE && K_NAME && K_RV && K_LABELS && T_ERROR && T_BOOKMARK && T_DELETED && S_EMPTY;
}

// borrowed dict item, nullptr when absent or not a dict
PyObject* dget(PyObject* d, PyObject* k) {
  if (!d || !PyDict_Check(d)) return nullptr;
  return PyDict_GetItem(d, k);  // borrowed; never raises for str keys
}

bool truthy_str(PyObject* v) { return v && PyUnicode_Check(v) && PyUnicode_GET_LENGTH(v) > 0; }

// type equality for interned / ordinary str
bool is_type(PyObject* t, PyObject* want) {
  if (t == want) return true;
  return PyUnicode_Check(t) && PyUnicode_Compare(t, want) == 0;
}

// "ns/name" or "name" (new reference)
PyObject* object_key(PyObject* meta) {
  PyObject* ns = dget(meta, K_NAMESPACE);
  PyObject* name = dget(meta, K_NAME);
  if (!name || !PyUnicode_Check(name)) name = S_EMPTY;
  if (truthy_str(ns)) return PyUnicode_FromFormat("%U/%U", ns, name);
  Py_INCREF(name);
  return name;
}

// remove `key` from idx[value] (dropping the set when it empties)
int unindex(PyObject* idx, PyObject* value, PyObject* key) {
  PyObject* st = PyDict_GetItemWithError(idx, value);
  if (!st) return PyErr_Occurred() ? -1 : 0;
  if (PySet_Discard(st, key) < 0) return -1;
  if (PySet_GET_SIZE(st) == 0 && PyDict_DelItem(idx, value) < 0) return -1;
  return 0;
}

int index_add(PyObject* idx, PyObject* value, PyObject* key) {
  PyObject* st = PyDict_GetItemWithError(idx, value);
  if (!st) {
    if (PyErr_Occurred()) return -1;
    PyObject* s = PySet_New(nullptr);
    if (!s) return -1;
    if (PySet_Add(s, key) < 0 || PyDict_SetItem(idx, value, s) < 0) {
      Py_DECREF(s);
      return -1;
    }
    Py_DECREF(s);
    return 0;
  }
  return PySet_Add(st, key);
}

// label-index upkeep of one upsert (old may be null) or delete (obj null); -1 on error
int update_indices(PyObject* labels, PyObject* indices, PyObject* key, PyObject* old, PyObject* obj) {
  if (labels == Py_None || !indices || indices == Py_None) return 0;
  PyObject* new_l = obj ? dget(dget(obj, K_METADATA), K_LABELS) : nullptr;
  PyObject* old_l = old ? dget(dget(old, K_METADATA), K_LABELS) : nullptr;
  Py_ssize_t n = PyList_GET_SIZE(labels);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* pair = PyList_GET_ITEM(labels, i);
    PyObject* name = PyTuple_GET_ITEM(pair, 0);
    PyObject* label = PyTuple_GET_ITEM(pair, 1);
    PyObject* v = new_l ? dget(new_l, label) : nullptr;
    PyObject* ov = old_l ? dget(old_l, label) : nullptr;
    if (v == ov) continue;
    if (v && ov) {
      int eq = PyObject_RichCompareBool(v, ov, Py_EQ);
      if (eq < 0) return -1;
      if (eq) continue;
    }
    PyObject* idx = PyDict_GetItemWithError(indices, name);
    if (!idx) {
      if (PyErr_Occurred()) return -1;
      continue;
    }
    if (ov && PyObject_IsTrue(ov) == 1 && unindex(idx, ov, key) < 0) return -1;
    if (v && PyObject_IsTrue(v) == 1 && index_add(idx, v, key) < 0) return -1;
  }
  return 0;
}

// call every handler in `hs` with (a) or (a, b); a raising handler goes to on_error
int dispatch(PyObject* hs, PyObject* a, PyObject* b, PyObject* on_error, PyObject* kind) {
  Py_ssize_t n = PyList_GET_SIZE(hs);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* f = PyList_GET_ITEM(hs, i);
    PyObject* r = b ? PyObject_CallFunctionObjArgs(f, a, b, nullptr) : PyObject_CallFunctionObjArgs(f, a, nullptr);
    if (r) {
      Py_DECREF(r);
      continue;
    }
    if (!PyErr_ExceptionMatches(PyExc_Exception)) return -1;  // KeyboardInterrupt / SystemExit propagate
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyErr_NormalizeException(&et, &ev, &tb);
    if (tb) PyException_SetTraceback(ev, tb);
    PyObject* lr = PyObject_CallFunctionObjArgs(on_error, kind, ev ? ev : Py_None, nullptr);
    Py_XDECREF(et);
    Py_XDECREF(ev);
    Py_XDECREF(tb);
    if (!lr) return -1;
    Py_DECREF(lr);
  }
  return 0;
}

}  // namespace

extern "C" PyObject* nexus_apply_lines(PyObject*, PyObject* args) {
  PyObject *batch, *items, *labels, *indices, *adds, *updates, *deletes, *on_error, *kind;
  Py_ssize_t start, end;
  if (!PyArg_ParseTuple(args, "O!nnO!OOO!O!O!OO", &PyList_Type, &batch, &start, &end, &PyDict_Type, &items, &labels,
                        &indices, &PyList_Type, &adds, &PyList_Type, &updates, &PyList_Type, &deletes, &on_error, &kind))
    return nullptr;
  if (!init_strings()) return nullptr;
  if (labels != Py_None && !PyList_Check(labels)) {
    PyErr_SetString(PyExc_TypeError, "labels must be a list of (index, label) or None");
    return nullptr;
  }
  Py_ssize_t n = PyList_GET_SIZE(batch);
  if (start < 0) start = 0;
  if (end > n) end = n;
  PyObject* rv = nullptr;  // borrowed from a line's metadata (kept alive by the batch)
  Py_ssize_t seen = 0;
  PyObject* err = Py_None;
  for (Py_ssize_t i = start; i < end; ++i) {
    PyObject* ev = PyList_GET_ITEM(batch, i);
    if (!PyTuple_Check(ev) || PyTuple_GET_SIZE(ev) != 2) {
      PyErr_SetString(PyExc_TypeError, "watch batch entries must be (type, object)");
      return nullptr;
    }
    PyObject* etype = PyTuple_GET_ITEM(ev, 0);
    PyObject* obj = PyTuple_GET_ITEM(ev, 1);
    if (is_type(etype, T_ERROR)) {
      err = obj;
      break;
    }
    ++seen;
    PyObject* meta = dget(obj, K_METADATA);
    if (meta && PyDict_Check(meta) && PyDict_GET_SIZE(meta)) {
      PyObject* v = dget(meta, K_RV);
      if (v && PyObject_IsTrue(v) == 1) rv = v;
    }
    if (is_type(etype, T_BOOKMARK)) continue;
    PyObject* key = object_key(meta);
    if (!key) return nullptr;
    if (is_type(etype, T_DELETED)) {
      // Indexer.delete: pop the cached object, unindex it; the handlers see the cached
      // version (the DELETED line's projection carries only the identity)
      PyObject* old = PyDict_GetItemWithError(items, key);
      if (!old && PyErr_Occurred()) {
        Py_DECREF(key);
        return nullptr;
      }
      Py_XINCREF(old);
      if (old && PyDict_DelItem(items, key) < 0) {
        Py_DECREF(old);
        Py_DECREF(key);
        return nullptr;
      }
      int rc = old ? update_indices(labels, indices, key, old, nullptr) : 0;
      Py_DECREF(key);
      if (rc == 0 && PyList_GET_SIZE(deletes)) rc = dispatch(deletes, old ? old : obj, nullptr, on_error, kind);
      Py_XDECREF(old);
      if (rc < 0) return nullptr;
      continue;
    }
    PyObject* old = PyDict_GetItemWithError(items, key);
    if (!old && PyErr_Occurred()) {
      Py_DECREF(key);
      return nullptr;
    }
    Py_XINCREF(old);
    int rc = PyDict_SetItem(items, key, obj);
    if (rc == 0) rc = update_indices(labels, indices, key, old, obj);
    Py_DECREF(key);
    if (rc == 0) rc = old ? dispatch(updates, old, obj, on_error, kind) : dispatch(adds, obj, nullptr, on_error, kind);
    Py_XDECREF(old);
    if (rc < 0) return nullptr;
  }
  return Py_BuildValue("(OnO)", err, seen, rv ? rv : Py_None);
}
