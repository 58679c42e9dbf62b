/*
 * _csgjson: json.dumps(obj, indent=2, ensure_ascii=False) in C, for the
 * generator's per-frame label files (save_label_json,
 * generate_construction_data.py:608-613).  With an indent, the standard
 * library's json encoder runs in pure Python (its C accelerator serves only
 * the compact form): ~4 ms of GIL per 80-KB label at 1080p C3, which capped
 * a pool of writer threads near 250 frames/s.  This produces the same bytes
 * (UTF-8) for the types json encodes: dict (insertion order; str, int,
 * float, bool and None keys), list, tuple, str, int, float (repr; NaN,
 * Infinity, -Infinity), bool, None.  Anything else raises TypeError, as
 * json does.  Floats: the shortest round-trip digits (std::to_chars, as
 * Python's repr) laid out by repr's rules -- exponent form when the decimal
 * point is more than 16 places right or 4 places left of the first digit,
 * else fixed with at least one fractional digit.
 *
 *   dumps_indent2(obj) -> bytes
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <string.h>

#include <charconv>

#include "csg_repr.h"

typedef struct {
  char* p;
  Py_ssize_t n, cap;
} Buf;

static int grow(Buf* b, Py_ssize_t add) {
  if (b->n + add <= b->cap) return 0;
  Py_ssize_t cap = b->cap ? b->cap : 65536;
  while (cap < b->n + add) cap *= 2;
  char* q = static_cast<char*>(PyMem_Realloc(b->p, (size_t)cap));
  if (!q) {
    PyErr_NoMemory();
    return -1;
  }
  b->p = q;
  b->cap = cap;
  return 0;
}

static int put(Buf* b, const char* s, Py_ssize_t n) {
  if (grow(b, n)) return -1;
  memcpy(b->p + b->n, s, (size_t)n);
  b->n += n;
  return 0;
}

static int newline(Buf* b, int level) {
  if (grow(b, 1 + 2 * (Py_ssize_t)level)) return -1;
  b->p[b->n++] = '\n';
  memset(b->p + b->n, ' ', (size_t)(2 * level));
  b->n += 2 * level;
  return 0;
}

/* JSON string, ensure_ascii=False: escape '"', '\\' and control characters */
static int put_str(Buf* b, PyObject* s) {
  Py_ssize_t n;
  const char* u = PyUnicode_AsUTF8AndSize(s, &n);
  if (!u) return -1;
  if (grow(b, 2 + 6 * n)) return -1;
  char* o = b->p + b->n;
  *o++ = '"';
  for (Py_ssize_t i = 0; i < n; ++i) {
    const unsigned char c = (unsigned char)u[i];
    if (c == '"' || c == '\\') {
      *o++ = '\\';
      *o++ = (char)c;
    } else if (c < 0x20) {
      *o++ = '\\';
      switch (c) {
        case '\n': *o++ = 'n'; break;
        case '\r': *o++ = 'r'; break;
        case '\t': *o++ = 't'; break;
        case '\b': *o++ = 'b'; break;
        case '\f': *o++ = 'f'; break;
        default: {
          static const char hex[] = "0123456789abcdef";
          *o++ = 'u';
          *o++ = '0';
          *o++ = '0';
          *o++ = hex[c >> 4];
          *o++ = hex[c & 15];
        }
      }
    } else {
      *o++ = (char)c;
    }
  }
  *o++ = '"';
  b->n = o - b->p;
  return 0;
}

static int put_obj_str(Buf* b, PyObject* s) {   /* a str object's text as-is */
  Py_ssize_t n;
  const char* u = PyUnicode_AsUTF8AndSize(s, &n);
  if (!u) return -1;
  return put(b, u, n);
}

/* repr(float) of a finite double (csg_repr.h) */
static int put_repr_double(Buf* b, double x) {
  if (grow(b, 48)) return -1;
  b->n = csg::repr_double(b->p + b->n, x) - b->p;
  return 0;
}

static int put_float(Buf* b, PyObject* o) {
  const double x = PyFloat_AS_DOUBLE(o);
  if (isnan(x)) return put(b, "NaN", 3);
  if (isinf(x)) return x > 0 ? put(b, "Infinity", 8) : put(b, "-Infinity", 9);
  return put_repr_double(b, x);
}

static int put_int(Buf* b, PyObject* o) {   /* int.__repr__, as json (bool handled before) */
  int overflow = 0;
  const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
  if (!overflow) {
    if (v == -1 && PyErr_Occurred()) return -1;
    if (grow(b, 24)) return -1;
    b->n = std::to_chars(b->p + b->n, b->p + b->n + 24, v).ptr - b->p;
    return 0;
  }
  PyObject* r = PyLong_Type.tp_repr(o);
  if (!r) return -1;
  const int rc = put_obj_str(b, r);
  Py_DECREF(r);
  return rc;
}

static int enc(Buf* b, PyObject* o, int level);

static int put_key(Buf* b, PyObject* k) {
  if (PyUnicode_Check(k)) return put_str(b, k);
  if (k == Py_True) return put(b, "\"true\"", 6);
  if (k == Py_False) return put(b, "\"false\"", 7);
  if (k == Py_None) return put(b, "\"null\"", 6);
  if (put(b, "\"", 1)) return -1;
  int rc;
  if (PyFloat_Check(k)) rc = put_float(b, k);
  else if (PyLong_Check(k)) rc = put_int(b, k);
  else {
    PyErr_Format(PyExc_TypeError, "keys must be str, int, float, bool or None, not %.100s", Py_TYPE(k)->tp_name);
    return -1;
  }
  if (rc) return -1;
  return put(b, "\"", 1);
}

static int enc(Buf* b, PyObject* o, int level) {
  if (o == Py_None) return put(b, "null", 4);
  if (o == Py_True) return put(b, "true", 4);
  if (o == Py_False) return put(b, "false", 5);
  if (PyUnicode_Check(o)) return put_str(b, o);
  if (PyLong_Check(o)) return put_int(b, o);
  if (PyFloat_Check(o)) return put_float(b, o);
  if (Py_EnterRecursiveCall(" while encoding a JSON object")) return -1;
  int rc = 0;
  if (PyList_Check(o) || PyTuple_Check(o)) {
    PyObject* seq = PySequence_Fast(o, "");
    const Py_ssize_t n = seq ? PySequence_Fast_GET_SIZE(seq) : 0;
    if (!seq) rc = -1;
    else if (n == 0) rc = put(b, "[]", 2);
    else {
      rc = put(b, "[", 1);
      PyObject** it = PySequence_Fast_ITEMS(seq);
      for (Py_ssize_t i = 0; !rc && i < n; ++i) {
        rc = (i ? put(b, ",", 1) : 0) || newline(b, level + 1) || enc(b, it[i], level + 1);
      }
      if (!rc) rc = newline(b, level) || put(b, "]", 1);
    }
    Py_XDECREF(seq);
  } else if (PyDict_Check(o)) {
    if (PyDict_GET_SIZE(o) == 0) rc = put(b, "{}", 2);
    else {
      rc = put(b, "{", 1);
      Py_ssize_t pos = 0, i = 0;
      PyObject *k, *v;
      while (!rc && PyDict_Next(o, &pos, &k, &v)) {
        rc = (i++ ? put(b, ",", 1) : 0) || newline(b, level + 1) || put_key(b, k) || put(b, ": ", 2) ||
             enc(b, v, level + 1);
      }
      if (!rc) rc = newline(b, level) || put(b, "}", 1);
    }
  } else {
    PyErr_Format(PyExc_TypeError, "Object of type %.100s is not JSON serializable", Py_TYPE(o)->tp_name);
    rc = -1;
  }
  Py_LeaveRecursiveCall();
  return rc;
}

static PyObject* repr_float(PyObject* self, PyObject* obj) {   /* test hook: repr(float(obj)) */
  (void)self;
  const double x = PyFloat_AsDouble(obj);
  if (x == -1.0 && PyErr_Occurred()) return NULL;
  Buf b = {NULL, 0, 0};
  if (!isfinite(x) ? put(&b, "nan", 3) : put_repr_double(&b, x)) {
    PyMem_Free(b.p);
    return NULL;
  }
  PyObject* r = PyUnicode_FromStringAndSize(b.p, b.n);
  PyMem_Free(b.p);
  return r;
}

static PyObject* dumps_indent2(PyObject* self, PyObject* obj) {
  (void)self;
  Buf b = {NULL, 0, 0};
  if (enc(&b, obj, 0)) {
    PyMem_Free(b.p);
    return NULL;
  }
  PyObject* r = PyBytes_FromStringAndSize(b.p, b.n);
  PyMem_Free(b.p);
  return r;
}

static PyMethodDef methods[] = {
    {"dumps_indent2", dumps_indent2, METH_O,
     "json.dumps(obj, indent=2, ensure_ascii=False).encode('utf-8'), in C."},
    {"repr_float", repr_float, METH_O, "repr(float(x)) for finite x (test hook)."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_csgjson", NULL, -1, methods, NULL, NULL, NULL, NULL};

extern "C" PyMODINIT_FUNC PyInit__csgjson(void) { return PyModule_Create(&module); }
