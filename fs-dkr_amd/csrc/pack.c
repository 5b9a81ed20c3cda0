/* CPython extension of the batching layer (fsdkr/batch.py): writes Python ints
 * straight into the little-endian u32-limb SoA buffers of struct
 * fsdkr_collect_batch (include/fsdkr/fsdkr.h), without a bytes object per value.
 * This is the gather step north_star's job (4) places in the Rust crate
 * (mpz_export of each curv BigInt into the batch); here the messages are
 * Python objects with the reference's field names.
 *
 * Two phases, so one collect() walks every proof object once and converts on
 * many cores:
 *   gather(objs, attr)        -> (handle, maxbits): holds a reference to getattr(o, attr)
 *                                (attr None: o itself) of every object, max bit length;
 *                                ValueError on a negative value, TypeError on a non-int
 *   gather_rows(objs, attr, take) -> (handle, maxbits) of the first `take` items of every
 *                                getattr(o, attr) sequence, flattened (the ring-Pedersen
 *                                A / Z and sigma vectors without a Python list per call);
 *                                IndexError when a sequence is shorter than `take`
 *   convert(jobs, threads)    -> jobs = [(handle, buffer, limbs), ...]: fills every
 *                                buffer[len][limbs] (uint32, little-endian) with the GIL
 *                                released, `threads` workers; OverflowError if a value
 *                                exceeds its slot (names the job index)
 *   points(objs, attr, buffer)-> affine (x, y) tuples or None -> buffer[len][16]
 *                                (x | y << 256, (0,0) = infinity)
 *   maxbits / pack            -> one-shot forms of gather / gather+convert
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <longintrepr.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* CPython stores |v| in Py_SIZE(v) digits of PyLong_SHIFT bits (sign in the size):
 * re-slice those digits into 32-bit limbs directly.  Needs no GIL (reads an
 * immutable int kept alive by the caller).  Returns -1 when v exceeds `limbs`. */
static int long_to_limbs(PyObject* v, uint32_t* out, size_t limbs) {
  const Py_ssize_t nd = Py_SIZE(v);
  const digit* d = ((PyLongObject*)v)->ob_digit;
  uint64_t acc = 0;
  int have = 0;
  size_t k = 0;
  if ((size_t)nd * PyLong_SHIFT <= limbs * 32) {
    /* fits by digit count: no bounds checks in the loop */
    Py_ssize_t i = 0;
#if PyLong_SHIFT == 30
    /* 16 digits of 30 bits are 15 limbs of 32: whole blocks without a data-
     * dependent branch (the n = 64 stage-1 pack converts ~8k 2048-bit values on
     * the call's critical path, before GA starts) */
    for (; i + 16 <= nd; i += 16) {
      const digit* q = d + i;
#define FSDKR_LIMB(j) out[k + (j)] = (uint32_t)((((uint64_t)q[(32 * (j)) / 30] >> ((32 * (j)) % 30)) | \
                                               ((uint64_t)q[(32 * (j)) / 30 + 1] << (30 - (32 * (j)) % 30)) | \
                                               (((32 * (j)) % 30 > 28) ? ((uint64_t)q[(32 * (j)) / 30 + 2] << (60 - (32 * (j)) % 30)) : 0)))
      FSDKR_LIMB(0); FSDKR_LIMB(1); FSDKR_LIMB(2); FSDKR_LIMB(3); FSDKR_LIMB(4);
      FSDKR_LIMB(5); FSDKR_LIMB(6); FSDKR_LIMB(7); FSDKR_LIMB(8); FSDKR_LIMB(9);
      FSDKR_LIMB(10); FSDKR_LIMB(11); FSDKR_LIMB(12); FSDKR_LIMB(13); FSDKR_LIMB(14);
#undef FSDKR_LIMB
      k += 15;
    }
#endif
    for (; i < nd; ++i) {
      acc |= (uint64_t)d[i] << have;
      have += PyLong_SHIFT;
      if (have >= 32) {
        out[k++] = (uint32_t)acc;
        acc >>= 32;
        have -= 32;
      }
    }
    if (have > 0) out[k++] = (uint32_t)acc;
  } else {
    for (Py_ssize_t i = 0; i < nd; ++i) {
      acc |= (uint64_t)d[i] << have;
      have += PyLong_SHIFT;
      while (have >= 32) {
        if (k >= limbs) {
          if ((uint32_t)acc != 0) return -1;
        } else {
          out[k] = (uint32_t)acc;
        }
        ++k;
        acc >>= 32;
        have -= 32;
      }
    }
    /* CPython normalises (no leading zero digits), so a non-zero spill past the
     * slot is a real overflow */
    if (have > 0 || acc) {
      if (k >= limbs) {
        if (acc) return -1;
      } else {
        out[k++] = (uint32_t)acc;
      }
    }
  }
  if (k < limbs) memset(out + k, 0, (limbs - k) * 4);
  return 0;
}

/* ---- gathered handle: owned references to the values of one field ---- */
typedef struct {
  Py_ssize_t n;
  PyObject** v;
} Gathered;

static const char* CAP = "fsdkr._pack.gathered";

static void gathered_free(PyObject* cap) {
  Gathered* g = (Gathered*)PyCapsule_GetPointer(cap, CAP);
  if (!g) return;
  for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(g->v[i]);
  free(g->v);
  free(g);
}

static PyObject* item_value(PyObject* o, PyObject* attr) {
  if (attr == Py_None) {
    Py_INCREF(o);
    return o;
  }
  return PyObject_GetAttr(o, attr);
}

/* gather the field values; *best = max bit length.  NULL on error. */
static Gathered* do_gather(PyObject* seq, PyObject* attr, size_t* best) {
  PyObject* fast = PySequence_Fast(seq, "objs must be a sequence");
  if (!fast) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  PyObject** items = PySequence_Fast_ITEMS(fast);
  Gathered* g = (Gathered*)calloc(1, sizeof(Gathered));
  PyObject** v = (PyObject**)calloc(n ? (size_t)n : 1, sizeof(PyObject*));
  if (!g || !v) {
    free(g);
    free(v);
    Py_DECREF(fast);
    PyErr_NoMemory();
    return NULL;
  }
  g->v = v;
  *best = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = item_value(items[i], attr);
    if (!x) goto fail;
    g->n = i + 1;
    v[i] = x;
    if (!PyLong_Check(x)) {
      PyErr_SetString(PyExc_TypeError, "big integer field is not an int");
      goto fail;
    }
    if (Py_SIZE(x) < 0) {
      PyErr_SetString(PyExc_ValueError, "negative big integer in a proof field");
      goto fail;
    }
    const size_t b = _PyLong_NumBits(x);
    if (b == (size_t)-1 && PyErr_Occurred()) goto fail;
    if (b > *best) *best = b;
  }
  g->n = n;
  Py_DECREF(fast);
  return g;
fail:
  for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(v[i]);
  free(v);
  free(g);
  Py_DECREF(fast);
  return NULL;
}

/* one value of a gather: owned reference stored in v[i], checked, bit length folded into *best */
static int take_value(PyObject* x, PyObject** slot, size_t* best) {
  *slot = x;
  if (!PyLong_Check(x)) {
    PyErr_SetString(PyExc_TypeError, "big integer field is not an int");
    return -1;
  }
  if (Py_SIZE(x) < 0) {
    PyErr_SetString(PyExc_ValueError, "negative big integer in a proof field");
    return -1;
  }
  const size_t b = _PyLong_NumBits(x);
  if (b == (size_t)-1 && PyErr_Occurred()) return -1;
  if (b > *best) *best = b;
  return 0;
}

static PyObject* py_gather_rows(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  Py_ssize_t take;
  if (!PyArg_ParseTuple(args, "OOn", &seq, &attr, &take)) return NULL;
  if (take < 0) {
    PyErr_SetString(PyExc_ValueError, "take < 0");
    return NULL;
  }
  PyObject* fast = PySequence_Fast(seq, "objs must be a sequence");
  if (!fast) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  PyObject** items = PySequence_Fast_ITEMS(fast);
  const size_t total = (size_t)n * (size_t)take;
  Gathered* g = (Gathered*)calloc(1, sizeof(Gathered));
  PyObject** v = (PyObject**)calloc(total ? total : 1, sizeof(PyObject*));
  size_t best = 0;
  if (!g || !v) {
    free(g);
    free(v);
    Py_DECREF(fast);
    return PyErr_NoMemory();
  }
  g->v = v;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* row = item_value(items[i], attr);
    if (!row) goto fail;
    PyObject* rf = PySequence_Fast(row, "row must be a sequence");
    Py_DECREF(row);
    if (!rf) goto fail;
    if (PySequence_Fast_GET_SIZE(rf) < take) {
      PyErr_Format(PyExc_IndexError, "row %zd holds %zd values, %zd needed", i, PySequence_Fast_GET_SIZE(rf), take);
      Py_DECREF(rf);
      goto fail;
    }
    PyObject** ri = PySequence_Fast_ITEMS(rf);
    for (Py_ssize_t k = 0; k < take; ++k) {
      PyObject* x = ri[k];
      Py_INCREF(x);
      g->n += 1;
      if (take_value(x, &v[g->n - 1], &best)) {
        Py_DECREF(rf);
        goto fail;
      }
    }
    Py_DECREF(rf);
  }
  Py_DECREF(fast);
  PyObject* cap = PyCapsule_New(g, CAP, gathered_free);
  if (!cap) {
    for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(g->v[i]);
    free(g->v);
    free(g);
    return NULL;
  }
  return Py_BuildValue("(Nn)", cap, (Py_ssize_t)best);
fail:
  for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(v[i]);
  free(v);
  free(g);
  Py_DECREF(fast);
  return NULL;
}

static PyObject* py_gather(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  if (!PyArg_ParseTuple(args, "OO", &seq, &attr)) return NULL;
  size_t best;
  Gathered* g = do_gather(seq, attr, &best);
  if (!g) return NULL;
  PyObject* cap = PyCapsule_New(g, CAP, gathered_free);
  if (!cap) {
    for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(g->v[i]);
    free(g->v);
    free(g);
    return NULL;
  }
  return Py_BuildValue("(Nn)", cap, (Py_ssize_t)best);
}

static PyObject* py_maxbits(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  if (!PyArg_ParseTuple(args, "OO", &seq, &attr)) return NULL;
  size_t best;
  Gathered* g = do_gather(seq, attr, &best);
  if (!g) return NULL;
  for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(g->v[i]);
  free(g->v);
  free(g);
  return PyLong_FromSize_t(best);
}

/* ---- conversion: (value, destination row) units spread over worker threads ---- */
typedef struct {
  PyObject* v;
  uint32_t* out;
  uint32_t limbs;
  uint32_t job;
} Unit;

typedef struct {
  Unit* u;
  size_t n;
  atomic_size_t next;
  atomic_long bad; /* lowest failing job index + 1, 0 = none */
} Work;

enum { CHUNK = 512 };

static void* worker(void* arg) {
  Work* w = (Work*)arg;
  for (;;) {
    const size_t s = atomic_fetch_add(&w->next, CHUNK);
    if (s >= w->n) break;
    const size_t e = s + CHUNK < w->n ? s + CHUNK : w->n;
    for (size_t i = s; i < e; ++i) {
      if (long_to_limbs(w->u[i].v, w->u[i].out, w->u[i].limbs) < 0) {
        long want = (long)w->u[i].job + 1, cur = atomic_load(&w->bad);
        while ((cur == 0 || want < cur) && !atomic_compare_exchange_weak(&w->bad, &cur, want)) {
        }
      }
    }
  }
  return NULL;
}

static void run_work(Work* w, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  /* a worker per >= 4 chunks of 512 values (thread start ~ tens of us): n = 64
   * whole call 45.9 -> 44.5 ms against one per 16 chunks, interleaved A/B
   * (profiles/r05/r05q_ab_pack_chunks) */
  const int per = 4;
  if ((size_t)threads > w->n / ((size_t)per * CHUNK) + 1) threads = (int)(w->n / ((size_t)per * CHUNK) + 1);
  pthread_t tid[64];
  int started = 0;
  for (int i = 1; i < threads; ++i)
    if (pthread_create(&tid[started], NULL, worker, w) == 0) ++started;
  worker(w);
  for (int i = 0; i < started; ++i) pthread_join(tid[i], NULL);
}

static PyObject* py_convert(PyObject* self, PyObject* args) {
  PyObject* jobs;
  int threads;
  if (!PyArg_ParseTuple(args, "Oi", &jobs, &threads)) return NULL;
  PyObject* fast = PySequence_Fast(jobs, "jobs must be a sequence");
  if (!fast) return NULL;
  const Py_ssize_t nj = PySequence_Fast_GET_SIZE(fast);
  PyObject** items = PySequence_Fast_ITEMS(fast);
  Py_buffer* bufs = (Py_buffer*)calloc(nj ? (size_t)nj : 1, sizeof(Py_buffer));
  Gathered** gs = (Gathered**)calloc(nj ? (size_t)nj : 1, sizeof(Gathered*));
  int* lim = (int*)calloc(nj ? (size_t)nj : 1, sizeof(int));
  Py_ssize_t got = 0;
  Unit* units = NULL;
  PyObject* ret = NULL;
  if (!bufs || !gs || !lim) {
    PyErr_NoMemory();
    goto done;
  }
  size_t total = 0;
  for (Py_ssize_t j = 0; j < nj; ++j) {
    PyObject* cap;
    if (!PyArg_ParseTuple(items[j], "Ow*i", &cap, &bufs[j], &lim[j])) goto done;
    got = j + 1;
    gs[j] = (Gathered*)PyCapsule_GetPointer(cap, CAP);
    if (!gs[j]) goto done;
    if (lim[j] <= 0 || (size_t)bufs[j].len < (size_t)gs[j]->n * (size_t)lim[j] * 4) {
      PyErr_Format(PyExc_ValueError, "job %zd: buffer too small", j);
      goto done;
    }
    total += (size_t)gs[j]->n;
  }
  units = (Unit*)malloc((total ? total : 1) * sizeof(Unit));
  if (!units) {
    PyErr_NoMemory();
    goto done;
  }
  size_t k = 0;
  for (Py_ssize_t j = 0; j < nj; ++j) {
    uint32_t* base = (uint32_t*)bufs[j].buf;
    for (Py_ssize_t i = 0; i < gs[j]->n; ++i) {
      units[k].v = gs[j]->v[i];
      units[k].out = base + (size_t)i * lim[j];
      units[k].limbs = (uint32_t)lim[j];
      units[k].job = (uint32_t)j;
      ++k;
    }
  }
  Work w;
  w.u = units;
  w.n = total;
  atomic_init(&w.next, 0);
  atomic_init(&w.bad, 0);
  Py_BEGIN_ALLOW_THREADS run_work(&w, threads);
  Py_END_ALLOW_THREADS
  const long bad = atomic_load(&w.bad);
  if (bad) {
    PyErr_Format(PyExc_OverflowError, "job %ld: value exceeds the %d-bit slot", bad - 1, 32 * lim[bad - 1]);
    goto done;
  }
  Py_INCREF(Py_None);
  ret = Py_None;
done:
  for (Py_ssize_t j = 0; j < got; ++j) PyBuffer_Release(&bufs[j]);
  free(units);
  free(bufs);
  free(gs);
  free(lim);
  Py_DECREF(fast);
  return ret;
}

static PyObject* py_pack(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  Py_buffer buf;
  int limbs;
  if (!PyArg_ParseTuple(args, "OOw*i", &seq, &attr, &buf, &limbs)) return NULL;
  size_t best;
  Gathered* g = do_gather(seq, attr, &best);
  PyObject* ret = NULL;
  if (!g) goto out;
  if (limbs <= 0 || (size_t)buf.len < (size_t)g->n * (size_t)limbs * 4) {
    PyErr_SetString(PyExc_ValueError, "buffer too small");
  } else if (best > (size_t)limbs * 32) {
    PyErr_SetString(PyExc_OverflowError, "value exceeds the slot");
  } else {
    for (Py_ssize_t i = 0; i < g->n; ++i) long_to_limbs(g->v[i], (uint32_t*)buf.buf + (size_t)i * limbs, limbs);
    Py_INCREF(Py_None);
    ret = Py_None;
  }
  for (Py_ssize_t i = 0; i < g->n; ++i) Py_XDECREF(g->v[i]);
  free(g->v);
  free(g);
out:
  PyBuffer_Release(&buf);
  return ret;
}

/* one affine coordinate: a non-negative int below 2^256 */
static int coord(PyObject* c, uint32_t* out) {
  if (!PyLong_Check(c)) {
    PyErr_SetString(PyExc_TypeError, "point coordinate is not an int");
    return -1;
  }
  if (Py_SIZE(c) < 0) {
    PyErr_SetString(PyExc_ValueError, "negative point coordinate");
    return -1;
  }
  if (long_to_limbs(c, out, 8) < 0) {
    PyErr_SetString(PyExc_OverflowError, "point coordinate exceeds 256 bits");
    return -1;
  }
  return 0;
}

static PyObject* py_points(PyObject* self, PyObject* args) {
  PyObject *seq, *attr;
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "OOw*", &seq, &attr, &buf)) return NULL;
  PyObject* fast = PySequence_Fast(seq, "objs must be a sequence");
  PyObject* ret = NULL;
  if (!fast) goto out;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  PyObject** items = PySequence_Fast_ITEMS(fast);
  if ((size_t)buf.len < (size_t)n * 64) {
    PyErr_SetString(PyExc_ValueError, "buffer too small");
    goto fail;
  }
  uint32_t* o = (uint32_t*)buf.buf;
  for (Py_ssize_t i = 0; i < n; ++i, o += 16) {
    PyObject* p = item_value(items[i], attr);
    if (!p) goto fail;
    int rc = 0;
    if (p == Py_None) {
      memset(o, 0, 64);
    } else if (PyTuple_Check(p) && PyTuple_GET_SIZE(p) == 2) {
      rc = coord(PyTuple_GET_ITEM(p, 0), o) || coord(PyTuple_GET_ITEM(p, 1), o + 8) ? -1 : 0;
    } else {
      PyObject* x = PySequence_GetItem(p, 0);
      PyObject* y = x ? PySequence_GetItem(p, 1) : NULL;
      rc = (!x || !y || coord(x, o) || coord(y, o + 8)) ? -1 : 0;
      Py_XDECREF(x);
      Py_XDECREF(y);
    }
    Py_DECREF(p);
    if (rc) goto fail;
  }
  Py_INCREF(Py_None);
  ret = Py_None;
fail:
  Py_DECREF(fast);
out:
  PyBuffer_Release(&buf);
  return ret;
}

static PyMethodDef methods[] = {
    {"gather", py_gather, METH_VARARGS, "(handle, maxbits) of getattr(o, attr) over objs"},
    {"gather_rows", py_gather_rows, METH_VARARGS, "(handle, maxbits) of getattr(o, attr)[:take] over objs, flattened"},
    {"convert", py_convert, METH_VARARGS, "fill [(handle, buffer, limbs), ...] on `threads` workers"},
    {"points", py_points, METH_VARARGS, "affine points (or None) -> [len][16] uint32"},
    {"maxbits", py_maxbits, METH_VARARGS, "max bit length of getattr(o, attr) over objs"},
    {"pack", py_pack, METH_VARARGS, "pack ints into a u32-limb buffer"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_pack", NULL, -1, methods};

PyMODINIT_FUNC PyInit__pack(void) { return PyModule_Create(&moddef); }
