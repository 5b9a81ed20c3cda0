/* CPython extension of the batching layer (fsdkr/batch.py): writes Python ints
 * straight into the little-endian u32-limb SoA buffers of struct
 * fsdkr_collect_batch (include/fsdkr/fsdkr.h), without a bytes object per value.
 * This is the gather step north_star's job (4) places in the Rust crate
 * (mpz_export of each curv BigInt into the batch); here the messages are
 * Python objects with the reference's field names.
 *
 *   maxbits(objs, attr)              -> max bit length of getattr(o, attr) (attr None: o itself);
 *                                       raises ValueError on a negative value
 *   pack(objs, attr, buffer, limbs)  -> fills buffer[len(objs)][limbs] (uint32, little-endian);
 *                                       raises ValueError / OverflowError (negative / too wide)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <longintrepr.h>
#include <stdint.h>
#include <string.h>

/* CPython stores |v| in Py_SIZE(v) digits of PyLong_SHIFT bits (sign in the size):
 * re-slice those digits into 32-bit limbs directly (no per-value bytes object). */
static int long_to_limbs(PyObject* v, uint32_t* out, size_t limbs) {
  const Py_ssize_t nd = Py_SIZE(v);
  if (nd < 0) {
    PyErr_SetString(PyExc_ValueError, "negative big integer in a proof field");
    return -1;
  }
  const digit* d = ((PyLongObject*)v)->ob_digit;
  uint64_t acc = 0;
  int have = 0;
  size_t k = 0;
  for (Py_ssize_t i = 0; i < nd; ++i) {
    acc |= (uint64_t)d[i] << have;
    have += PyLong_SHIFT;
    while (have >= 32) {
      if (k >= limbs) {
        if ((uint32_t)acc != 0 || (acc >> 32) != 0) goto overflow;
      } else {
        out[k] = (uint32_t)acc;
      }
      ++k;
      acc >>= 32;
      have -= 32;
    }
  }
  if (have > 0 || acc) {
    if (k >= limbs) {
      if (acc) goto overflow;
    } else {
      out[k++] = (uint32_t)acc;
    }
  }
  if (k < limbs) memset(out + k, 0, (limbs - k) * 4);
  return 0;
overflow:
  /* a zero digit run past the slot is fine only if every remaining digit is zero:
   * CPython normalises (no leading zero digits), so any spill is a real overflow */
  PyErr_SetString(PyExc_OverflowError, "value exceeds the slot");
  return -1;
}

static PyObject* item_value(PyObject* o, PyObject* attr) {
  if (attr == Py_None) {
    Py_INCREF(o);
    return o;
  }
  return PyObject_GetAttr(o, attr);
}

static PyObject* py_maxbits(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  if (!PyArg_ParseTuple(args, "OO", &seq, &attr)) return NULL;
  PyObject* fast = PySequence_Fast(seq, "objs must be a sequence");
  if (!fast) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  PyObject** items = PySequence_Fast_ITEMS(fast);
  size_t best = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* v = item_value(items[i], attr);
    if (!v) goto fail;
    if (!PyLong_Check(v)) {
      Py_DECREF(v);
      PyErr_SetString(PyExc_TypeError, "big integer field is not an int");
      goto fail;
    }
    if (_PyLong_Sign(v) < 0) {
      Py_DECREF(v);
      PyErr_SetString(PyExc_ValueError, "negative big integer in a proof field");
      goto fail;
    }
    const size_t b = _PyLong_NumBits(v);
    Py_DECREF(v);
    if (b == (size_t)-1 && PyErr_Occurred()) goto fail;
    if (b > best) best = b;
  }
  Py_DECREF(fast);
  return PyLong_FromSize_t(best);
fail:
  Py_DECREF(fast);
  return NULL;
}

static PyObject* py_pack(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  Py_buffer buf;
  int limbs;
  if (!PyArg_ParseTuple(args, "OOw*i", &seq, &attr, &buf, &limbs)) return NULL;
  PyObject* fast = PySequence_Fast(seq, "objs must be a sequence");
  if (!fast) {
    PyBuffer_Release(&buf);
    return NULL;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  PyObject** items = PySequence_Fast_ITEMS(fast);
  const size_t row = (size_t)limbs * 4;
  if (limbs <= 0 || (size_t)buf.len < (size_t)n * row) {
    PyErr_SetString(PyExc_ValueError, "buffer too small");
    goto fail;
  }
  unsigned char* out = (unsigned char*)buf.buf;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* v = item_value(items[i], attr);
    if (!v) goto fail;
    if (!PyLong_Check(v)) {
      Py_DECREF(v);
      PyErr_SetString(PyExc_TypeError, "big integer field is not an int");
      goto fail;
    }
    const int rc = long_to_limbs(v, (uint32_t*)(out + (size_t)i * row), (size_t)limbs);
    Py_DECREF(v);
    if (rc < 0) goto fail;
  }
  Py_DECREF(fast);
  PyBuffer_Release(&buf);
  Py_RETURN_NONE;
fail:
  Py_DECREF(fast);
  PyBuffer_Release(&buf);
  return NULL;
}

static PyMethodDef methods[] = {
    {"maxbits", py_maxbits, METH_VARARGS, "max bit length of getattr(o, attr) over objs"},
    {"pack", py_pack, METH_VARARGS, "pack ints into a u32-limb buffer"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_pack", NULL, -1, methods};

PyMODINIT_FUNC PyInit__pack(void) { return PyModule_Create(&moddef); }
