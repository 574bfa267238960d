/* CPython binding of hm_project_scalar (include/heatmap_amd.h) for the
 * per-record Tile calls (reference tile.py:9-21): a ctypes call costs ~1.5 us
 * of argument conversion, more than the projection; this METH_FASTCALL module
 * costs ~0.1 us.  It holds no arithmetic of its own: it calls the library's
 * C-ABI entry point (libheatmap_amd.so, found next to it through the rpath).
 *
 *   project(lat, lon, zoom) -> (status, row, col)
 *   tile_id(lat, lon, zoom) -> (status, "zoom_row_col" or None)
 * status as hm_project_scalar's: HM_BIGCOL gives the column as the bits of an
 * integer-valued double (the caller makes the unbounded int). */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stdint.h>

int hm_project_scalar(double lat, double lon, int zoom, int64_t* row_col);

static int args3(PyObject* const* args, Py_ssize_t n, double* lat, double* lon, int* zoom)
{
    if (n != 3) {
        PyErr_SetString(PyExc_TypeError, "expected (lat, lon, zoom)");
        return -1;
    }
    *lat = PyFloat_AsDouble(args[0]);
    if (*lat == -1.0 && PyErr_Occurred()) return -1;
    *lon = PyFloat_AsDouble(args[1]);
    if (*lon == -1.0 && PyErr_Occurred()) return -1;
    /* zoom: an int (or any index type), or an integral float (the
     * reference's 2 ** zoom takes floats); out of range, huge or non-integral:
     * 1000, which hm_project_scalar answers with HM_E_ARG (ValueError in
     * tile.py) */
    PyObject* o = args[2];
    long z = 1000;
    if (PyFloat_Check(o)) {
        const double d = PyFloat_AS_DOUBLE(o);
        if (d == floor(d) && fabs(d) <= 1000.0) z = (long)d;
    } else {
        PyObject* i = PyNumber_Index(o);   /* TypeError for non-numbers, as int(zoom) */
        if (!i) return -1;
        int overflow = 0;
        z = PyLong_AsLongAndOverflow(i, &overflow);
        Py_DECREF(i);
        if (z == -1 && PyErr_Occurred()) return -1;
        if (overflow) z = 1000;
    }
    *zoom = (z < -1000 || z > 1000) ? 1000 : (int)z;   /* out of range: HM_E_ARG below */
    return 0;
}

static PyObject* project(PyObject* self, PyObject* const* args, Py_ssize_t n)
{
    double lat, lon;
    int zoom;
    if (args3(args, n, &lat, &lon, &zoom)) return NULL;
    int64_t rc[2];
    const int st = hm_project_scalar(lat, lon, zoom, rc);
    return Py_BuildValue("(iLL)", st, (long long)rc[0], (long long)rc[1]);
}

static PyObject* tile_id(PyObject* self, PyObject* const* args, Py_ssize_t n)
{
    double lat, lon;
    int zoom;
    if (args3(args, n, &lat, &lon, &zoom)) return NULL;
    int64_t rc[2];
    const int st = hm_project_scalar(lat, lon, zoom, rc);
    if (st != 0) return Py_BuildValue("(iO)", st, Py_None);
    PyObject* s = PyUnicode_FromFormat("%d_%lld_%lld", zoom, (long long)rc[0], (long long)rc[1]);
    if (!s) return NULL;
    PyObject* t = Py_BuildValue("(iN)", 0, s);
    return t;
}

static PyMethodDef methods[] = {
    {"project", (PyCFunction)(void (*)(void))project, METH_FASTCALL, "(status, row, col) of one point"},
    {"tile_id", (PyCFunction)(void (*)(void))tile_id, METH_FASTCALL, "(status, tile id or None) of one point"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_hm_scalar", NULL, -1, methods};

PyMODINIT_FUNC PyInit__hm_scalar(void) { return PyModule_Create(&mod); }
