/* _pystr -- host-side helpers for the Python drivers (CPython C API, no GPU code).
 *
 * The drivers hand batches of ~10^5 Python objects to the engine: NanoporeRead objects and their
 * seq strs. Each Python-level pass over such a batch (a list comprehension, map(len, ...), one
 * ctypes call per str for its buffer address) costs 20-60 ms per 100k objects, mostly cache
 * misses on the scattered objects plus the interpreter's per-item overhead; the end-trim driver
 * made five such passes before its GPU call. These helpers make one C pass each:
 *
 *   ascii_buffers(strs, addr, lens) -> bool
 *       For a list of str: addr[k] = the address of strs[k]'s characters (a compact ASCII str
 *       keeps its bytes inside the object: PyUnicode_AsUTF8 is that address, no copy), lens[k] =
 *       its length. addr: writable uint64 buffer, lens: writable int64 buffer, len(strs) entries
 *       each. Returns False (buffers partly filled) at the first item that is not an ASCII str:
 *       the caller takes its slicing path. The addresses are valid while the strs live.
 *   attr_list(objs, name) -> list
 *       [getattr(o, name) for o in objs].
 *   append_rows(reads, name, objs, read, obj, f1, f2, i1, i2)
 *       Alignment tuples appended to each read's list attribute (below).
 *   int_attrs(objs, name, out)
 *       out[k] = getattr(objs[k], name) for int attributes (out: writable int64 buffer) -- the
 *       middle driver's trim amounts without a list of ints and its numpy conversion.
 *   raise_trims(reads, start, end)
 *       For each read k: read.start_trim_amount = max(read.start_trim_amount, start[k]), the same
 *       for end_trim_amount (start / end: int32 buffers) -- the end-trim driver's update of the
 *       reference's NanoporeRead fields (nanopore_read.py:175-217, find_start_trim /
 *       find_end_trim keep the largest trim).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

/* Software prefetch of an object's instance attributes, in three stages a few items apart (the
 * drivers walk 10^5 NanoporeRead objects scattered over the heap: each getattr / setattr waits on
 * the object, its __dict__ and the dict's value array in turn, ~3 misses per read):
 *   stage 0: the object;  stage 1: its instance dict;  stage 2: the dict's values (split table). */
static inline void pf_attrs(PyObject *o, int stage) {
    if (stage == 0) {
        __builtin_prefetch(o);
        return;
    }
#if PY_VERSION_HEX >= 0x030B0000
    /* 3.11+: objects with managed / inline-values dicts have no dict until one is asked for, and
     * _PyObject_GetDictPtr would create it from the inline values -- an allocation per object
     * ahead of the cursor that also turns off the inline-values fast path. Only the
     * object itself is prefetched there. */
    (void)o;
    return;
#else
    PyObject **dp = _PyObject_GetDictPtr(o);
    if (!dp || !*dp) return;
    if (stage == 1) {
        __builtin_prefetch(*dp);
        return;
    }
    PyDictObject *d = (PyDictObject *)*dp;
    if (d->ma_values) {
        __builtin_prefetch(d->ma_values);
        __builtin_prefetch((const char *)d->ma_values + 64);
        __builtin_prefetch((const char *)d->ma_values + 128);
    }
#endif
}
/* The value slot of attribute value v in o's split-table dict (-1 if none): the drivers' objects
 * share one key table, so the slot locates the attribute's value in every one of them -- the
 * fourth stage (the value object itself, e.g. a read's str header that getattr's INCREF touches). */
static Py_ssize_t value_slot(PyObject *o, PyObject *v, void **keys) {
#if PY_VERSION_HEX < 0x030B0000
    PyObject **dp = _PyObject_GetDictPtr(o);
    if (!dp || !*dp) return -1;
    PyDictObject *d = (PyDictObject *)*dp;
    if (!d->ma_values) return -1;
    for (Py_ssize_t i = 0; i < d->ma_used; ++i)
        if (d->ma_values[i] == v) {
            *keys = d->ma_keys;
            return i;
        }
#endif
    return -1;
}
static inline void pf_value(PyObject *o, Py_ssize_t slot, void *keys) {
#if PY_VERSION_HEX < 0x030B0000
    PyObject **dp = _PyObject_GetDictPtr(o);
    if (!dp || !*dp) return;
    PyDictObject *d = (PyDictObject *)*dp;
    if (d->ma_values && (void *)d->ma_keys == keys) __builtin_prefetch(d->ma_values[slot]);
#endif
}
#define PF_AHEAD(items, k, n)                                 \
    do {                                                      \
        if ((k) + 12 < (n)) pf_attrs((items)[(k) + 12], 0);   \
        if ((k) + 8 < (n)) pf_attrs((items)[(k) + 8], 1);     \
        if ((k) + 4 < (n)) pf_attrs((items)[(k) + 4], 2);     \
    } while (0)

static PyObject *ascii_buffers(PyObject *self, PyObject *args) {
    PyObject *seq;
    Py_buffer ab, lb;
    if (!PyArg_ParseTuple(args, "Ow*w*", &seq, &ab, &lb)) return NULL;
    PyObject *fast = PySequence_Fast(seq, "ascii_buffers: a sequence of str");
    PyObject *ret = NULL;
    if (!fast) goto done;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    if (ab.len < n * (Py_ssize_t)sizeof(uint64_t) || lb.len < n * (Py_ssize_t)sizeof(int64_t)) {
        PyErr_SetString(PyExc_ValueError, "ascii_buffers: buffers too small");
        goto done;
    }
    uint64_t *addr = (uint64_t *)ab.buf;
    int64_t *lens = (int64_t *)lb.buf;
    PyObject **items = PySequence_Fast_ITEMS(fast);
    int ok = 1;
    for (Py_ssize_t k = 0; k < n; ++k) {
        PyObject *s = items[k];
        if (!PyUnicode_Check(s) || PyUnicode_READY(s) != 0 || !PyUnicode_IS_ASCII(s)) {
            PyErr_Clear();
            ok = 0;
            break;
        }
        const char *p = PyUnicode_AsUTF8(s);   /* compact ASCII: the object's own bytes */
        if (!p) {
            PyErr_Clear();
            ok = 0;
            break;
        }
        addr[k] = (uint64_t)(uintptr_t)p;
        lens[k] = (int64_t)PyUnicode_GET_LENGTH(s);
    }
    ret = PyBool_FromLong(ok);
done:
    Py_XDECREF(fast);
    PyBuffer_Release(&ab);
    PyBuffer_Release(&lb);
    return ret;
}

static PyObject *attr_list(PyObject *self, PyObject *args) {
    PyObject *seq, *name;
    if (!PyArg_ParseTuple(args, "OU", &seq, &name)) return NULL;
    PyObject *fast = PySequence_Fast(seq, "attr_list: a sequence");
    if (!fast) return NULL;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    PyObject **items = PySequence_Fast_ITEMS(fast);
    PyObject *out = PyList_New(n);
    if (!out) {
        Py_DECREF(fast);
        return NULL;
    }
    Py_ssize_t slot = -1;
    void *keys = NULL;
    for (Py_ssize_t k = 0; k < n; ++k) {
        PF_AHEAD(items, k, n);
        if (slot >= 0 && k + 2 < n) pf_value(items[k + 2], slot, keys);
        PyObject *v = PyObject_GetAttr(items[k], name);
        if (!v) {
            Py_DECREF(out);
            Py_DECREF(fast);
            return NULL;
        }
        if (k == 0) slot = value_slot(items[0], v, &keys);
        PyList_SET_ITEM(out, k, v);
    }
    Py_DECREF(fast);
    return out;
}

static PyObject *int_attrs(PyObject *self, PyObject *args) {
    PyObject *seq, *name;
    Py_buffer ob;
    if (!PyArg_ParseTuple(args, "OUw*", &seq, &name, &ob)) return NULL;
    PyObject *ret = NULL;
    PyObject *fast = PySequence_Fast(seq, "int_attrs: a sequence");
    if (!fast) goto done;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    if (ob.len < n * (Py_ssize_t)sizeof(int64_t)) {
        PyErr_SetString(PyExc_ValueError, "int_attrs: buffer too small");
        goto done;
    }
    int64_t *out = (int64_t *)ob.buf;
    PyObject **items = PySequence_Fast_ITEMS(fast);
    for (Py_ssize_t k = 0; k < n; ++k) {
        PF_AHEAD(items, k, n);
        PyObject *v = PyObject_GetAttr(items[k], name);
        if (!v) goto done;
        const long long x = PyLong_AsLongLong(v);   /* an int (or __index__): as int(...) would */
        Py_DECREF(v);
        if (x == -1 && PyErr_Occurred()) goto done;
        out[k] = (int64_t)x;
    }
    Py_INCREF(Py_None);
    ret = Py_None;
done:
    Py_XDECREF(fast);
    PyBuffer_Release(&ob);
    return ret;
}

static int raise_field(PyObject *o, PyObject *name, long v) {
    PyObject *cur = PyObject_GetAttr(o, name);
    if (!cur) return -1;
    int gt = 0;
    PyObject *nv = PyLong_FromLong(v);
    if (!nv) {
        Py_DECREF(cur);
        return -1;
    }
    gt = PyObject_RichCompareBool(nv, cur, Py_GT);   /* v > current, as the driver's `if a > r.x` */
    Py_DECREF(cur);
    int rc = gt < 0 ? -1 : 0;
    if (gt > 0) rc = PyObject_SetAttr(o, name, nv);
    Py_DECREF(nv);
    return rc;
}

static PyObject *raise_trims(PyObject *self, PyObject *args) {
    PyObject *seq;
    Py_buffer sb, eb;
    if (!PyArg_ParseTuple(args, "Oy*y*", &seq, &sb, &eb)) return NULL;
    PyObject *ret = NULL, *fast = NULL;
    PyObject *ns = PyUnicode_InternFromString("start_trim_amount");
    PyObject *ne = PyUnicode_InternFromString("end_trim_amount");
    if (!ns || !ne) goto done;
    fast = PySequence_Fast(seq, "raise_trims: a sequence of reads");
    if (!fast) goto done;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    if (sb.len < n * 4 || eb.len < n * 4) {
        PyErr_SetString(PyExc_ValueError, "raise_trims: buffers too small");
        goto done;
    }
    const int32_t *st = (const int32_t *)sb.buf, *et = (const int32_t *)eb.buf;
    PyObject **items = PySequence_Fast_ITEMS(fast);
    for (Py_ssize_t k = 0; k < n; ++k) {
        PF_AHEAD(items, k, n);
        if (raise_field(items[k], ns, st[k]) < 0 || raise_field(items[k], ne, et[k]) < 0) goto done;
    }
    Py_INCREF(Py_None);
    ret = Py_None;
done:
    Py_XDECREF(fast);
    Py_XDECREF(ns);
    Py_XDECREF(ne);
    PyBuffer_Release(&sb);
    PyBuffer_Release(&eb);
    return ret;
}

/* append_rows(reads, name, objs, read, obj, f1, f2, i1, i2): for every row k (rows grouped by read,
 * in the order they are to be appended), getattr(reads[read[k]], name).append(
 * (objs[obj[k]], f1[k], f2[k], i1[k], i2[k])) -- the end-trim driver's alignment lists
 * (nanopore_read.py:186-188, 208-210: (adapter, full identity, partial identity, read start,
 * read end)). read / obj / i1 / i2: int64 buffers, f1 / f2: float64 buffers. */
static PyObject *append_rows(PyObject *self, PyObject *args) {
    PyObject *reads, *name, *objs;
    Py_buffer rb, ob, f1b, f2b, i1b, i2b;
    if (!PyArg_ParseTuple(args, "OUOy*y*y*y*y*y*", &reads, &name, &objs, &rb, &ob, &f1b, &f2b, &i1b, &i2b))
        return NULL;
    PyObject *ret = NULL, *fr = NULL, *fo = NULL, *lst = NULL;
    int gc_was = 0;
    /* the identities are pid6 values of small (matches, length) pairs: a few hundred distinct
     * doubles over 10^5 rows, so their float objects are shared through a small cache (direct
     * mapped on the value's bits) instead of two allocations per row */
    enum { kFC = 4096 };
    PyObject *fcache[kFC];
    uint64_t fkey[kFC];
    memset(fcache, 0, sizeof(fcache));
    memset(fkey, 0, sizeof(fkey));
    fr = PySequence_Fast(reads, "append_rows: a sequence of reads");
    fo = fr ? PySequence_Fast(objs, "append_rows: a sequence of objects") : NULL;
    if (!fo) goto done;
    const Py_ssize_t m = rb.len / 8;
    if (ob.len / 8 < m || f1b.len / 8 < m || f2b.len / 8 < m || i1b.len / 8 < m || i2b.len / 8 < m) {
        PyErr_SetString(PyExc_ValueError, "append_rows: buffers of different lengths");
        goto done;
    }
    const int64_t *rd = (const int64_t *)rb.buf, *oi = (const int64_t *)ob.buf;
    const double *f1 = (const double *)f1b.buf, *f2 = (const double *)f2b.buf;
    const int64_t *i1 = (const int64_t *)i1b.buf, *i2 = (const int64_t *)i2b.buf;
    const Py_ssize_t nr = PySequence_Fast_GET_SIZE(fr), no = PySequence_Fast_GET_SIZE(fo);
    PyObject **ri = PySequence_Fast_ITEMS(fr), **oo = PySequence_Fast_ITEMS(fo);
#define CACHED_FLOAT(dst, val)                                                           \
    do {                                                                                 \
        uint64_t b_;                                                                     \
        const double v_ = (val);                                                         \
        memcpy(&b_, &v_, 8);                                                             \
        const unsigned h_ = (unsigned)((b_ * 0x9E3779B97F4A7C15ull) >> 52) & (kFC - 1);  \
        if (!fcache[h_] || fkey[h_] != b_) {                                             \
            PyObject *f_ = PyFloat_FromDouble(v_);                                       \
            if (!f_) goto done;                                                          \
            Py_XDECREF(fcache[h_]);                                                      \
            fcache[h_] = f_;                                                             \
            fkey[h_] = b_;                                                               \
        }                                                                                \
        (dst) = fcache[h_];                                                              \
    } while (0)
    /* no cyclic collection while the rows are made: every ~700 new tuples would start one, and
     * the older generations' passes walk the tuples made so far (half of this call's time at 10^5
     * rows). The call holds the GIL throughout, so only its own allocations see the pause. */
#if PY_VERSION_HEX >= 0x030A0000
    gc_was = PyGC_Disable();
#endif
    int64_t cur = -1;
    for (Py_ssize_t k = 0; k < m; ++k) {
        if (rd[k] < 0 || rd[k] >= nr || oi[k] < 0 || oi[k] >= no) {
            PyErr_SetString(PyExc_IndexError, "append_rows: index out of range");
            goto done;
        }
        /* the reads of the rows ahead (rows come grouped by read, a few per read) */
        if (k + 12 < m && rd[k + 12] >= 0 && rd[k + 12] < nr) pf_attrs(ri[rd[k + 12]], 0);
        if (k + 8 < m && rd[k + 8] >= 0 && rd[k + 8] < nr) pf_attrs(ri[rd[k + 8]], 1);
        if (k + 4 < m && rd[k + 4] >= 0 && rd[k + 4] < nr) pf_attrs(ri[rd[k + 4]], 2);
        if (rd[k] != cur) {
            Py_XDECREF(lst);
            lst = PyObject_GetAttr(ri[rd[k]], name);
            if (!lst) goto done;
            cur = rd[k];
        }
        PyObject *a1, *a2;
        CACHED_FLOAT(a1, f1[k]);
        CACHED_FLOAT(a2, f2[k]);
        PyObject *t = PyTuple_New(5);
        if (!t) goto done;
        PyObject *x1 = PyLong_FromLongLong(i1[k]), *x2 = PyLong_FromLongLong(i2[k]);
        if (!x1 || !x2) {
            Py_XDECREF(x1);
            Py_XDECREF(x2);
            Py_DECREF(t);
            goto done;
        }
        Py_INCREF(oo[oi[k]]);
        Py_INCREF(a1);
        Py_INCREF(a2);
        PyTuple_SET_ITEM(t, 0, oo[oi[k]]);
        PyTuple_SET_ITEM(t, 1, a1);
        PyTuple_SET_ITEM(t, 2, a2);
        PyTuple_SET_ITEM(t, 3, x1);
        PyTuple_SET_ITEM(t, 4, x2);
        const int rc = PyList_Check(lst) ? PyList_Append(lst, t) : -1;
        if (rc < 0 && !PyErr_Occurred()) {
            PyObject *r = PyObject_CallMethod(lst, "append", "O", t);   /* not a list: its append */
            Py_DECREF(t);
            if (!r) goto done;
            Py_DECREF(r);
            continue;
        }
        Py_DECREF(t);
        if (rc < 0) goto done;
    }
    Py_INCREF(Py_None);
    ret = Py_None;
done:
#if PY_VERSION_HEX >= 0x030A0000
    if (gc_was) PyGC_Enable();
#endif
    for (int h = 0; h < kFC; ++h) Py_XDECREF(fcache[h]);
#undef CACHED_FLOAT
    Py_XDECREF(lst);
    Py_XDECREF(fr);
    Py_XDECREF(fo);
    PyBuffer_Release(&rb);
    PyBuffer_Release(&ob);
    PyBuffer_Release(&f1b);
    PyBuffer_Release(&f2b);
    PyBuffer_Release(&i1b);
    PyBuffer_Release(&i2b);
    return ret;
}

static PyMethodDef methods[] = {
    {"append_rows", append_rows, METH_VARARGS, "append alignment tuples to the reads' lists"},
    {"ascii_buffers", ascii_buffers, METH_VARARGS, "addresses and lengths of ASCII strs"},
    {"attr_list", attr_list, METH_VARARGS, "[getattr(o, name) for o in objs]"},
    {"int_attrs", int_attrs, METH_VARARGS, "int attributes of objs into an int64 buffer"},
    {"raise_trims", raise_trims, METH_VARARGS, "raise the reads' trim amounts to the given ones"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pystr", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pystr(void) { return PyModule_Create(&module); }
