/* dcol_amd._fastpair: the drop-in's per-call host glue in C (Engine.solve_pair).
 *
 * proximity_mrp / proximity_gradient are called one pair at a time by an unchanged
 * reference ALTRO loop (systems/cluttered_hallway_quadrotor.py:131-133, :155), so the
 * Python around the library call is part of every call's latency: staging the four 3-vectors
 * (prim.r / prim.p: ndarrays or lists), the ctypes argument conversion and the output
 * copies cost ~8-12 us per call, a third of the call.  Here they are one C function: the
 * poses are read straight from the objects' buffers (float64, 3 contiguous values) or, for
 * lists and other sequences, item by item; dcol_prox_pair (include/dcol.h) is called through
 * the address ctypes resolved, with the GIL released; the outputs come back as fresh numpy
 * arrays.  No numerics here -- the solve is the HIP library's.
 *
 * solve(fn, table, s1, s2, r1, p1, r2, p2, tol, max_iter, flags, want_contact)
 *   -> (rc, alpha: np.float64, contact (3,) | None, grad (12,) | None, iters, status)
 *   or None when a pose is not 3 numbers (the caller then takes its Python path).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_2_0_API_VERSION
#include <numpy/arrayobject.h>
#include <numpy/arrayscalars.h>
#include <stdint.h>
#include <string.h>

#include "../../include/dcol.h"

typedef int (*prox_pair_fn)(const dcol_table*, int32_t, int32_t, const double*, const double*, double, int32_t,
                            int32_t, double*, double*, double*, int32_t*, int32_t*);

/* three doubles from a float64 buffer of exactly 3 contiguous values, or a sequence of 3
 * numbers; 0 on success, -1 (no exception set) when the object is neither */
static int read3(PyObject* o, double* out) {
    if (PyObject_CheckBuffer(o)) {
        Py_buffer v;
        if (PyObject_GetBuffer(o, &v, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) == 0) {
            const int ok = v.len == 3 * (Py_ssize_t)sizeof(double) && v.itemsize == (Py_ssize_t)sizeof(double) &&
                           v.format && (strcmp(v.format, "d") == 0 || strcmp(v.format, "<d") == 0 ||
                                        strcmp(v.format, "=d") == 0);
            if (ok) memcpy(out, v.buf, 3 * sizeof(double));
            PyBuffer_Release(&v);
            if (ok) return 0;
        } else {
            PyErr_Clear();
        }
    }
    PyObject* seq = PySequence_Fast(o, "");
    if (!seq) {
        PyErr_Clear();
        return -1;
    }
    int rc = -1;
    if (PySequence_Fast_GET_SIZE(seq) == 3) {
        PyObject** it = PySequence_Fast_ITEMS(seq);
        rc = 0;
        for (int k = 0; k < 3 && rc == 0; ++k) {
            if (PyFloat_CheckExact(it[k])) {
                out[k] = PyFloat_AS_DOUBLE(it[k]);
            } else if (PyFloat_Check(it[k]) || PyLong_Check(it[k]) || PyArray_IsScalar(it[k], Floating) ||
                       PyArray_IsScalar(it[k], Integer)) {
                out[k] = PyFloat_AsDouble(it[k]);
                if (out[k] == -1.0 && PyErr_Occurred()) {
                    PyErr_Clear();
                    rc = -1;
                }
            } else {
                rc = -1;   /* nested sequences ((3, 1) arrays ...): the Python path reshapes */
            }
        }
    }
    Py_DECREF(seq);
    return rc;
}

static PyObject* new_vec(const double* v, npy_intp n) {
    PyObject* a = PyArray_SimpleNew(1, &n, NPY_FLOAT64);
    if (a) memcpy(PyArray_DATA((PyArrayObject*)a), v, (size_t)n * sizeof(double));
    return a;
}

static PyObject* solve(PyObject* self, PyObject* args) {
    (void)self;
    unsigned long long fn_addr, table;
    int s1, s2, max_iter, flags, want_contact;
    PyObject *r1, *p1, *r2, *p2;
    double tol;
    if (!PyArg_ParseTuple(args, "KKiiOOOOdiip", &fn_addr, &table, &s1, &s2, &r1, &p1, &r2, &p2, &tol, &max_iter,
                          &flags, &want_contact))
        return NULL;
    double pose[12];
    if (read3(r1, pose) || read3(p1, pose + 3) || read3(r2, pose + 6) || read3(p2, pose + 9)) Py_RETURN_NONE;
    double alpha = 0.0, contact[3], grad[12];
    int32_t iters = 0, status = 0;
    const prox_pair_fn fn = (prox_pair_fn)(uintptr_t)fn_addr;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn((const dcol_table*)(uintptr_t)table, s1, s2, pose, pose + 6, tol, max_iter, flags, &alpha, contact, grad,
            &iters, &status);
    Py_END_ALLOW_THREADS
    PyObject* a = PyArrayScalar_New(Double);
    if (!a) return NULL;
    PyArrayScalar_ASSIGN(a, Double, alpha);
    PyObject* c = Py_None;
    PyObject* g = Py_None;
    Py_INCREF(Py_None);
    Py_INCREF(Py_None);
    if (rc == 0 && want_contact) {
        Py_DECREF(c);
        if (!(c = new_vec(contact, 3))) goto fail;
    }
    if (rc == 0 && (flags & DCOL_GRAD_ANY)) {
        Py_DECREF(g);
        if (!(g = new_vec(grad, 12))) goto fail;
    }
    return Py_BuildValue("(iNNNii)", rc, a, c, g, (int)iters, (int)status);
fail:
    Py_DECREF(a);
    Py_XDECREF(c);
    Py_XDECREF(g);
    return NULL;
}

static PyMethodDef methods[] = {
    {"solve", solve, METH_VARARGS, "dcol_prox_pair for one pair of primitive poses (see module docstring)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fastpair", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fastpair(void) {
    import_array();
    return PyModule_Create(&module);
}
