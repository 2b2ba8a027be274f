/* Host-side helper of the N = 1 drop-in (FJSPSimulation.py facade): one env's observation
 * columns from the pinned step record -> the reference's dict of numpy arrays, built with the
 * CPython / numpy C APIs in one call (spec.obs_dicts is the same function in Python, and the
 * definition the tests compare this one with).
 *
 * Reference dict layout: PickupStationAgent.py:87-96, AGVAgent.py:60-75, MachineAgent.py:64-69,
 * PackagingAgent.py:266-271 — every field a 0-d array of its dtype (np.array(x, dtype=...)),
 * the AGV's position a 2-vector, every action mask its own int8 array (get_action_mask().astype).
 *
 * Inputs are the record's column views: i32 [20] int32, i8 [12] int8, f32 [6] float32,
 * mask [29] int8 (any objects exporting C-contiguous buffers of at least those sizes).
 * No GPU code: this module never touches the device. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <string.h>

#define N_AG 8
#define N_PICK 7
#define N_AGV 12
static const char* AGENTS[N_AG] = {"pickup_station", "agv", "small_machine", "big_machine",
                                   "packaging_blue_1", "packaging_blue_2", "packaging_red", "packaging_green"};
static const char* PICK[N_PICK] = {"order_size", "products_remaining", "next_product_type", "next_product_color",
                                   "current_tray_type", "current_tray_color", "current_tray_count"};
static const char* AGV[N_AGV] = {"position", "carrying_tray", "tray_product_count", "tray_type",
                                 "tray_needs_processing", "tray_needs_packaging", "pickup_ready_trays",
                                 "small_machine_busy", "big_machine_busy", "small_machine_ready",
                                 "big_machine_ready", "storage_tray_count"};
static const int MASK_OFF[N_AG + 1] = {0, 3, 11, 14, 17, 20, 23, 26, 29};

static PyObject *s_agents[N_AG], *s_pick[N_PICK], *s_agv[N_AGV];
static PyObject *s_busy, *s_prog, *s_queue, *s_mask;

static PyObject* scalar(int type, const void* v, size_t bytes) {
    PyObject* a = PyArray_SimpleNew(0, NULL, type);
    if (a) memcpy(PyArray_DATA((PyArrayObject*)a), v, bytes);
    return a;
}

static PyObject* vec(int type, npy_intp n, const void* v, size_t bytes) {
    PyObject* a = PyArray_SimpleNew(1, &n, type);
    if (a) memcpy(PyArray_DATA((PyArrayObject*)a), v, bytes);
    return a;
}

/* d[key] = value, stealing the value reference; 0 on success */
static int put(PyObject* d, PyObject* key, PyObject* v) {
    if (!v) return -1;
    const int r = PyDict_SetItem(d, key, v);
    Py_DECREF(v);
    return r;
}

static int get_buf(PyObject* o, Py_buffer* b, Py_ssize_t need, const char* what) {
    if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS) != 0) return -1;
    if (b->len < need) {
        PyBuffer_Release(b);
        PyErr_Format(PyExc_ValueError, "obs_dicts: %s holds %zd bytes, needs %zd", what, b->len, need);
        return -1;
    }
    return 0;
}

static PyObject* obs_dicts(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *o32, *o8, *of, *om;
    if (!PyArg_ParseTuple(args, "OOOO", &o32, &o8, &of, &om)) return NULL;
    Py_buffer b32, b8, bf, bm;
    if (get_buf(o32, &b32, 20 * 4, "i32")) return NULL;
    if (get_buf(o8, &b8, 12, "i8")) { PyBuffer_Release(&b32); return NULL; }
    if (get_buf(of, &bf, 6 * 4, "f32")) { PyBuffer_Release(&b32); PyBuffer_Release(&b8); return NULL; }
    if (get_buf(om, &bm, 29, "mask")) { PyBuffer_Release(&b32); PyBuffer_Release(&b8); PyBuffer_Release(&bf); return NULL; }
    /* the values are copied out first (the record may be rewritten by the next step only) */
    int32_t a[20];
    int8_t b[12], m[29];
    float c[6];
    memcpy(a, b32.buf, sizeof a);
    memcpy(b, b8.buf, sizeof b);
    memcpy(c, bf.buf, sizeof c);
    memcpy(m, bm.buf, sizeof m);
    PyBuffer_Release(&b32); PyBuffer_Release(&b8); PyBuffer_Release(&bf); PyBuffer_Release(&bm);

    PyObject* obs = PyDict_New();
    if (!obs) return NULL;
    PyObject* d = NULL;
    /* pickup station */
    if (!(d = PyDict_New())) goto fail;
    for (int i = 0; i < N_PICK; i++)
        if (put(d, s_pick[i], scalar(NPY_INT32, &a[i], 4))) goto fail_d;
    if (put(d, s_mask, vec(NPY_INT8, 3, m, 3))) goto fail_d;
    if (put(obs, s_agents[0], d)) goto fail;
    /* AGV: position = i32[7:9], the other fields i32[9..19] */
    if (!(d = PyDict_New())) goto fail;
    if (put(d, s_agv[0], vec(NPY_INT32, 2, &a[7], 8))) goto fail_d;
    for (int j = 1; j < N_AGV; j++)
        if (put(d, s_agv[j], scalar(NPY_INT32, &a[8 + j], 4))) goto fail_d;
    if (put(d, s_mask, vec(NPY_INT8, 8, &m[3], 8))) goto fail_d;
    if (put(obs, s_agents[1], d)) goto fail;
    /* machines and packaging stations: is_busy i8[2s], processing_progress f32[s], queue_length i8[2s+1] */
    for (int s = 0; s < 6; s++) {
        if (!(d = PyDict_New())) goto fail;
        if (put(d, s_busy, scalar(NPY_INT8, &b[2 * s], 1))) goto fail_d;
        if (put(d, s_prog, scalar(NPY_FLOAT32, &c[s], 4))) goto fail_d;
        if (put(d, s_queue, scalar(NPY_INT8, &b[2 * s + 1], 1))) goto fail_d;
        if (put(d, s_mask, vec(NPY_INT8, 3, &m[MASK_OFF[2 + s]], 3))) goto fail_d;
        if (put(obs, s_agents[2 + s], d)) goto fail;
    }
    return obs;
fail_d:
    Py_DECREF(d);
fail:
    Py_DECREF(obs);
    return NULL;
}

static PyMethodDef methods[] = {
    {"obs_dicts", obs_dicts, METH_VARARGS,
     "obs_dicts(i32, i8, f32, mask) -> the reference's observation dict of one env (spec.obs_dicts)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_facade", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__facade(void) {
    import_array();
    for (int i = 0; i < N_AG; i++)
        if (!(s_agents[i] = PyUnicode_InternFromString(AGENTS[i]))) return NULL;
    for (int i = 0; i < N_PICK; i++)
        if (!(s_pick[i] = PyUnicode_InternFromString(PICK[i]))) return NULL;
    for (int i = 0; i < N_AGV; i++)
        if (!(s_agv[i] = PyUnicode_InternFromString(AGV[i]))) return NULL;
    if (!(s_busy = PyUnicode_InternFromString("is_busy")) || !(s_prog = PyUnicode_InternFromString("processing_progress")) ||
        !(s_queue = PyUnicode_InternFromString("queue_length")) || !(s_mask = PyUnicode_InternFromString("action_mask")))
        return NULL;
    return PyModule_Create(&module);
}
